# GPU tests selected by -k expression ($1), verbose log (per-test progress), no -x
mkdir -p gpurun_out
timeout -k 10 ${2:-500} python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread ${1:+-k "$1"} -s > gpurun_out/gpu_k.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_k.log | tail -40
exit $rc
