mkdir -p gpurun_out/vf
timeout -k 10 200 python -u tools/chunk_trace.py > gpurun_out/vf/trace.txt 2>&1 || { tail -5 gpurun_out/vf/trace.txt; exit 1; }
head -9 gpurun_out/vf/trace.txt | tail -4
for K in 20 200; do
timeout -k 10 300 python3 -u bench.py --no-cfg5 --mappo-episodes 0 --learner-big-steps 0 --offq-updates 0 \
  --train-episodes 0 --cfg1-episodes 0 --no-cpu-baseline --steps $K --warmup 5 > gpurun_out/vf/qb$K.log 2>&1 || { tail -5 gpurun_out/vf/qb$K.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/vf/qb$K.log').read().strip().split('\n')[-1]); print($K, d['ms_per_step'], d['ms_per_step_min'], d['ms_per_step_max'], d['roofline']['kernel_us_per_step'], d['roofline']['frac'])"
done
timeout -k 10 200 python -u tools/mb_chunk.py chunk > gpurun_out/mbc.json 2>&1; tail -c 300 gpurun_out/mbc.json
