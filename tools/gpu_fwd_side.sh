# Learner forward: mixer state projection + recurrence on the side stream (MM_LRN_FWD_SIDE=1) or in line (0):
# learner-path tests, then an interleaved B=32 update A/B.
set -o pipefail
mkdir -p gpurun_out/fside
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learner.py tests/test_gpu_headline.py tests/test_gpu_train.py tests/test_gpu_adapters.py tests/test_gpu_dist.py tests/test_gpu_checkpoint.py > gpurun_out/fside/test.log 2>&1
rc=$?; tail -3 gpurun_out/fside/test.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    MM_LRN_FWD_SIDE=$v MB_E=4096 MB_CAP=65536 timeout -k 10 300 python -u tools/mb_learner.py > gpurun_out/fside/mb_${v}_$i.log 2>&1 || exit 1
    echo "fwd_side=$v: $(tail -1 gpurun_out/fside/mb_${v}_$i.log)"
  done
done
