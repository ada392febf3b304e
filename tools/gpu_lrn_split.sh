set -o pipefail
mkdir -p gpurun_out/lrn
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learner.py tests/test_gpu_headline.py tests/test_gpu_train.py tests/test_gpu_adapters.py tests/test_gpu_checkpoint.py tests/test_gpu_dist.py > gpurun_out/lrn/test.log 2>&1
rc=$?; tail -3 gpurun_out/lrn/test.log; [ $rc -eq 0 ] || exit $rc
MB_E=4096 MB_CAP=65536 timeout -k 10 300 python -u tools/mb_learner.py > gpurun_out/lrn/mb.log 2>&1; rc=$?; tail -2 gpurun_out/lrn/mb.log; exit $rc
