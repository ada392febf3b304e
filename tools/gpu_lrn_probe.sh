# B=32 learner: update time, REC sequence phase trace, kernel timeline of the replayed update graph
mkdir -p gpurun_out/lrn
export TMPDIR=/tmp
MB_E=4096 MB_CAP=65536 timeout -k 10 200 python -u tools/mb_learner.py > gpurun_out/lrn/mb.json 2> gpurun_out/lrn/mb.err || { tail -5 gpurun_out/lrn/mb.err; exit 1; }
cat gpurun_out/lrn/mb.json
timeout -k 10 200 python -u tools/trace_rec.py > gpurun_out/lrn/rec.json 2> gpurun_out/lrn/rec.err || { tail -5 gpurun_out/lrn/rec.err; exit 1; }
cat gpurun_out/lrn/rec.json
MB_E=4096 MB_CAP=65536 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lrn/kt -- python3 tools/mb_learner.py > gpurun_out/lrn/kt.log 2>&1 || { tail -5 gpurun_out/lrn/kt.log; exit 1; }
python3 tools/ktimeline.py gpurun_out/lrn/kt per_sample_kernel 22
