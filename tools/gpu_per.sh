set -o pipefail
mkdir -p gpurun_out/per
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rollout.py -k "per_" > gpurun_out/per/test.log 2>&1
rc=$?; tail -4 gpurun_out/per/test.log; exit $rc
