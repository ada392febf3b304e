#!/bin/bash
# Round profile on the GPU box (run via gpurun from the repo root): kernel stats of the bench
# (QMIX rollout + learner + MAPPO episode) and the HBM bytes of the dual agent forward from two
# separate PMC passes. Outputs under gpurun_out/prof/; copy the summaries into profiles/.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -- \
  python3 bench.py --steps 200 --warmup 20 --learner-steps 50 --no-cpu-baseline --mappo-episodes 1 > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -- \
  python3 bench.py --steps 40 --warmup 10 --repeats 1 --learner-steps 2 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -- \
  python3 bench.py --steps 40 --warmup 10 --repeats 1 --learner-steps 2 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline > $OUT/write.log 2>&1
python3 profiles/summarize.py $OUT/stats > $OUT/kernel_stats.txt
cp $(find $OUT/stats -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write agent_q_fwd_h3_kernel 262144 46268416 $OUT/pmc_agent_fwd.json \
  "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace --output-format csv -- python3 bench.py --steps 40 --warmup 10 --repeats 1 --learner-steps 2 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline (two separate passes)"
tail -1 $OUT/stats.log
