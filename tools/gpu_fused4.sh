set -o pipefail
mkdir -p gpurun_out/fused4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fused_step.py tests/test_gpu_rollout.py tests/test_gpu_train.py > gpurun_out/fused4/test.log 2>&1
rc=$?; tail -5 gpurun_out/fused4/test.log; exit $rc
