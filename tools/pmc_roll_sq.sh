#!/bin/bash
# SQ / GRBM counters of the fused rollout step (tools/mb_roll.py: 60 eager fused steps at 4096 x 8, GRU-64),
# three separate --pmc passes (8 SQ + 1 GRBM each), then tools/pmc_fwd_sum.py -> one JSON summary of
# the fused launches (grid 262144 = 256 blocks x 1024).
export TMPDIR=/tmp
O=gpurun_out/pmc_roll_sq
rm -rf $O && mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $P -d $O/p$i -- python3 tools/mb_roll.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_fwd_sum.py $O rollout_step_kernel "rollout_step_kernel<64,64,64,1> (env step + dual forward; grid 262144 = 256 blocks x 1024)" > $O/summary.json && cat $O/summary.json
