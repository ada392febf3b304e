# paired forward launches: learner tests, update time, timeline
mkdir -p gpurun_out/lrn
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/lrn/t.log 2>&1
rc=$?; tail -3 gpurun_out/lrn/t.log; grep "^E  " gpurun_out/lrn/t.log | head -5; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  MB_E=4096 MB_CAP=65536 timeout -k 10 200 python -u tools/mb_learner.py 2> gpurun_out/lrn/mb.err || { tail -5 gpurun_out/lrn/mb.err; exit 1; }
done
MB_E=4096 MB_CAP=65536 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lrn/kt3 -- python3 tools/mb_learner.py > gpurun_out/lrn/kt3.log 2>&1 || { tail -5 gpurun_out/lrn/kt3.log; exit 1; }
python3 tools/ktimeline.py gpurun_out/lrn/kt3 per_sample_kernel 18
