#!/bin/bash
# Round-4 profile on the GPU box (via gpurun from the repo root): kernel stats of the bench (fused rollout step,
# learner, MAPPO episode), HBM bytes of the fused rollout step from two separate PMC passes, and the MAPPO
# gradient kernels' traffic + SQ counters. Outputs under gpurun_out/prof4/; copy the summaries into profiles/.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof4
mkdir -p $OUT
Q="--steps 40 --warmup 10 --repeats 1 --learner-steps 2 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -- \
  python3 bench.py --steps 200 --warmup 20 --learner-steps 50 --no-cpu-baseline --mappo-episodes 1 > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -- python3 bench.py $Q > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -- python3 bench.py $Q > $OUT/write.log 2>&1
python3 profiles/summarize.py $OUT/stats > $OUT/kernel_stats.txt
cp $(find $OUT/stats -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
# algorithmic bytes of one fused launch at 4096 x 8 (D 47, H 64, 12 x 8 grid): 32768 x 1240 + 4096 x 225
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write rollout_step_kernel 262144 41553920 $OUT/pmc_rollout_step.json \
  "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace --output-format csv -- python3 bench.py $Q (two separate passes)"
timeout -k 10 400 bash tools/pmc_mappo.sh $OUT/mappo > $OUT/mappo.log 2>&1
tail -1 $OUT/stats.log
