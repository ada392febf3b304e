#!/bin/bash
# Round-5 profile on the GPU box (via gpurun from the repo root). Each step bounded, chained with &&.
# Outputs under gpurun_out/prof5/; the summaries are copied into profiles/r05_*.
export TMPDIR=/tmp
O=${O:-gpurun_out/prof5}
mkdir -p $O
Q="--steps 40 --warmup 10 --repeats 1 --learner-steps 10 --learner-big-steps 0 --train-episodes 0 --cfg1-episodes 0 --mappo-episodes 0 --offq-updates 0 --no-cfg5 --no-cpu-baseline"
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2> $O/bench_default.err && \
grep '^{"metric"' $O/bench_default.log | tail -1 > $O/bench_default.json && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- \
  python3 bench.py --steps 200 --warmup 20 --learner-steps 50 --no-cpu-baseline --mappo-episodes 1 > $O/stats.log 2>&1 && \
python3 profiles/summarize.py $O/stats > $O/kernel_stats.txt && \
cp $(find $O/stats -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv && \
bash tools/pmc_chunk.sh $O/pmc_chunk > $O/pmc_chunk.log 2>&1 && \
timeout -k 10 200 python -u tools/chunk_trace.py > $O/chunk_trace.txt 2>&1 && \
MB_K=1 MB_E=4096 MB_CAP=65536 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/lrn -- python3 tools/mb_learner.py > $O/lrn.log 2>&1 && \
python3 tools/ktimeline.py $O/lrn per_sample_kernel 16 > $O/learner_timeline.txt && \
timeout -k 10 600 bash tools/pmc_mappo.sh $O/mappo > $O/mappo.log 2>&1
rc=$?
tail -2 $O/bench_default.json; tail -3 $O/kernel_stats.txt
exit $rc
