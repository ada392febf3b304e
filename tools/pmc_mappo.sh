# HBM traffic (FETCH_SIZE / WRITE_SIZE, one rocprofv3 pass each) of every mappo_* kernel over one MAPPO
# episode at cfg3 (tools/mb_mappo.py, 2 PPO epochs) + SQ counters of the fused gradient kernel.
# usage: bash tools/pmc_mappo.sh <outdir>
set -e
export TMPDIR=/tmp
O=$1
mkdir -p $O
CMD="tools/mb_mappo.py --episodes 1 --epochs 2"
timeout -s KILL 120 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $O/fetch -- python3 $CMD > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --output-format csv --pmc WRITE_SIZE -d $O/write -- python3 $CMD > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/sq -- python3 $CMD > $O/sq.log 2>&1
python3 tools/pmc_mappo_sum.py $O
