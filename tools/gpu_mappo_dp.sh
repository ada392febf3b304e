mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mappo.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mappo_dp.log 2>&1; rc=$?
tail -15 gpurun_out/mappo_dp.log
exit $rc
