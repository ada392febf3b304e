set -o pipefail
mkdir -p gpurun_out/fused1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fused_step.py > gpurun_out/fused1/test.log 2>&1
