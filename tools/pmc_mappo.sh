# HBM traffic (FETCH_SIZE / WRITE_SIZE, one rocprofv3 pass each) of every mappo_* kernel over one MAPPO
# episode at cfg3 (tools/mb_mappo.py, 2 PPO epochs) + one SQ pass with its kernel trace for both gradient passes
# (tools/pmc_fwd_sum.py: clock = SQ_BUSY_CYCLES / 32 SEs / duration per dispatch, MFMA busy from the same dispatch).
# usage: bash tools/pmc_mappo.sh <outdir>
set -e
export TMPDIR=/tmp
O=$1
rm -rf $O && mkdir -p $O
CMD="tools/mb_mappo.py --episodes 1 --epochs 2"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/fetch -- python3 $CMD > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/write -- python3 $CMD > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/sq/p1 -- python3 $CMD > $O/sq.log 2>&1
python3 tools/pmc_mappo_sum.py $O
python3 tools/pmc_fwd_sum.py $O/sq mappo_grad_gru_kernel "mappo_grad_gru_kernel<47,5> (recurrent pass, 128 x 2 blocks x 256)" 0 > $O/sq_gru.json
python3 tools/pmc_fwd_sum.py $O/sq mappo_grad_mlp_kernel "mappo_grad_mlp_kernel<47,5> (MLP pass, 128 x 2 blocks x 512)" 0 > $O/sq_mlp.json
