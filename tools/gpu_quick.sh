# quick GPU check: gpu tests (optionally -k filter in $1), env microbench, short bench
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 60 python tools/mb_env.py > gpurun_out/mb_env.log 2>&1 && cat gpurun_out/mb_env.log | tail -1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --mappo-episodes 0 > gpurun_out/bench.log 2>&1
rc=$?
tail -1 gpurun_out/bench.log | cut -c1-330
exit $rc
