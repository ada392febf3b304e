# chunk kernel hand-off / TD fold change: parity tests, microbenchmark, 20- and 200-step quick benches, kernel stats
mkdir -p gpurun_out/ho
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests ${TESTS:--m gpu} -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/ho/t.log 2>&1
rc=$?; tail -3 gpurun_out/ho/t.log; grep "^E  \|FAILED" gpurun_out/ho/t.log | head -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mb_chunk.py chunk > gpurun_out/ho/mb_chunk.json 2> gpurun_out/ho/mb_chunk.err || { tail -5 gpurun_out/ho/mb_chunk.err; exit 1; }
cat gpurun_out/ho/mb_chunk.json
for K in 20 200; do
timeout -k 10 300 python3 -u bench.py --no-cfg5 --mappo-episodes 0 --learner-big-steps 0 --offq-updates 0 \
  --train-episodes 0 --cfg1-episodes 0 --no-cpu-baseline --steps $K --warmup 5 > gpurun_out/ho/qb$K.log 2>&1 || { tail -5 gpurun_out/ho/qb$K.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/ho/qb$K.log').read().strip().split('\n')[-1]); print($K, d['ms_per_step'], d['ms_per_step_min'], d['ms_per_step_max'], d['roofline']['kernel_us_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ho/st -- python3 bench.py --no-cfg5 --mappo-episodes 0 --learner-big-steps 0 --offq-updates 0 --train-episodes 0 --cfg1-episodes 0 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/ho/st.log 2>&1 || { tail -5 gpurun_out/ho/st.log; exit 1; }
python3 profiles/summarize.py gpurun_out/ho/st > gpurun_out/ho/stats.txt; head -14 gpurun_out/ho/stats.txt
