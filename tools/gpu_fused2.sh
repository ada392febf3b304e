set -o pipefail
mkdir -p gpurun_out/fused2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fused_step.py > gpurun_out/fused2/test.log 2>&1 &&
timeout -k 10 120 python -u tools/roll_trace.py > gpurun_out/fused2/trace.txt 2>&1 &&
timeout -k 10 120 python -u tools/roll_probe.py > gpurun_out/fused2/probe.json 2>&1
rc=$?; tail -3 gpurun_out/fused2/test.log; cat gpurun_out/fused2/trace.txt | tail -10; cat gpurun_out/fused2/probe.json; exit $rc
