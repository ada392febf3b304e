# HBM bytes per dispatch of the dual agent forward (two separate PMC passes) -> gpurun_out/prof/pmc_agent_fwd.json
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -- \
  python3 bench.py --steps 40 --warmup 10 --repeats 1 --learner-steps 2 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -- \
  python3 bench.py --steps 40 --warmup 10 --repeats 1 --learner-steps 2 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline > $OUT/write.log 2>&1
python3 tools/pmc_traffic.py $OUT/fetch $OUT/write agent_q_fwd_h3_kernel 262144 46268416 $OUT/pmc_agent_fwd.json \
  "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-trace --output-format csv -- python3 bench.py --steps 40 --warmup 10 --repeats 1 --learner-steps 2 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline (two separate passes)"
