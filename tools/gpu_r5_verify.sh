# full GPU suite, then the chunk kernel's debug-build timeline and the 20 / 200-step headline lines
mkdir -p gpurun_out/vf
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/vf/t.log 2>&1
rc=$?; tail -2 gpurun_out/vf/t.log; grep "^E  \|FAILED" gpurun_out/vf/t.log | head -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/chunk_trace.py > gpurun_out/vf/trace.txt 2>&1 || { tail -5 gpurun_out/vf/trace.txt; exit 1; }
head -12 gpurun_out/vf/trace.txt
for K in 20 200; do
timeout -k 10 300 python3 -u bench.py --no-cfg5 --mappo-episodes 0 --learner-big-steps 0 --offq-updates 0 \
  --train-episodes 0 --cfg1-episodes 0 --no-cpu-baseline --steps $K --warmup 5 > gpurun_out/vf/qb$K.log 2>&1 || { tail -5 gpurun_out/vf/qb$K.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/vf/qb$K.log').read().strip().split('\n')[-1]); print($K, d['ms_per_step'], d['ms_per_step_min'], d['ms_per_step_max'], d['roofline']['kernel_us_per_step'], d['roofline']['frac'])"
done
