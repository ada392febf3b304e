# Agent BPTT + mixer recurrence backward in one launch (mm_agent_mixer_bwd_seq): learner-path tests, then an
# interleaved B=32 update A/B against the side-stream version (MM_LRN_PAIR_BWD=0).
set -o pipefail
mkdir -p gpurun_out/pair
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learner.py tests/test_gpu_headline.py tests/test_gpu_train.py tests/test_gpu_adapters.py tests/test_gpu_dist.py tests/test_gpu_checkpoint.py > gpurun_out/pair/test.log 2>&1
rc=$?; tail -3 gpurun_out/pair/test.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    MM_LRN_PAIR_BWD=$v MB_E=4096 MB_CAP=65536 timeout -k 10 300 python -u tools/mb_learner.py > gpurun_out/pair/mb_${v}_$i.log 2>&1 || exit 1
    echo "pair=$v: $(tail -1 gpurun_out/pair/mb_${v}_$i.log)"
  done
done
