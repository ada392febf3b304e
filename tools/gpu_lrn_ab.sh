# B=32 learner A/B (interleaved): update time per knob setting, then the kernel timeline of the default
mkdir -p gpurun_out/lrn
export TMPDIR=/tmp
for r in 1 2; do
  for ps in 1 0; do
    MB_PER_SIDE=$ps MB_E=4096 MB_CAP=65536 timeout -k 10 200 python -u tools/mb_learner.py 2> gpurun_out/lrn/mb.err || { tail -5 gpurun_out/lrn/mb.err; exit 1; }
  done
done
MB_E=4096 MB_CAP=65536 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lrn/kt2 -- python3 tools/mb_learner.py > gpurun_out/lrn/kt2.log 2>&1 || { tail -5 gpurun_out/lrn/kt2.log; exit 1; }
python3 tools/ktimeline.py gpurun_out/lrn/kt2 per_sample_kernel 19
