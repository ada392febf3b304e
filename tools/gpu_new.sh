# GPU check of a test subset ($1 = -k expression) + the default bench line
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${1:+-k "$1"} \
  > gpurun_out/new_tests.log 2>&1
rc=$?
tail -25 gpurun_out/new_tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/new_bench.log 2>&1
rc=$?
tail -3 gpurun_out/new_bench.log | cut -c1-3000
exit $rc
