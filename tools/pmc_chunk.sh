#!/bin/bash
# Counters of the chunk-persistent rollout kernel (tools/mb_chunk_pmc.py: 13 launches of 20 steps at 4096 x 8,
# GRU-64): three SQ passes (8 SQ + GRBM each) -> tools/pmc_fwd_sum.py, and two HBM passes (FETCH_SIZE, WRITE_SIZE)
# -> tools/pmc_traffic.py. Each pass its own rocprofv3 run. usage: bash tools/pmc_chunk.sh <outdir>
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_chunk}
rm -rf $O && mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $P -d $O/p$i -- python3 tools/mb_chunk_pmc.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_fwd_sum.py $O rollout_chunk_kernel "rollout_chunk_kernel<64,64,64,1> (20 rollout steps per launch; grid 262144 = 256 blocks x 1024)" > $O/summary_sq.json || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/fetch -- python3 tools/mb_chunk_pmc.py > $O/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/write -- python3 tools/mb_chunk_pmc.py > $O/write.log 2>&1 || { echo "write pass failed"; exit 1; }
# algorithmic bytes of one 20-step launch at 4096 x 8 (D 47, H 64, 12 x 8 grid), bench.py's formula (hidden states
# in / out once per launch): 20 (32768 (188 + 16) + 4096 x 9) + 32768 (1024 + 12) + 4096 (192 + 24)
python3 tools/pmc_traffic.py $O/fetch $O/write rollout_chunk_kernel 262144 169263104 $O/pmc_rollout_chunk.json \
  "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace --output-format csv -- python3 tools/mb_chunk_pmc.py (two separate passes)"
