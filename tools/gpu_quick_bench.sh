# headline-only bench (no side lines) for quick A/B on the GPU box
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cfg5 --mappo-episodes 0 --learner-big-steps 0 --offq-updates 0 \
  --train-episodes 0 --cfg1-episodes 0 --no-cpu-baseline "$@" > gpurun_out/quick_bench.log 2>&1
rc=$?
tail -3 gpurun_out/quick_bench.log
exit $rc
