#!/bin/bash
# Round-6 profile on the GPU box (via gpurun from the repo root). Each step bounded, chained with &&.
# Outputs under gpurun_out/prof6/; the summaries are copied into profiles/r06_*.
export TMPDIR=/tmp
O=${O:-gpurun_out/prof6}
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 20 > $O/bench_default.log 2> $O/bench_default.err && \
grep '^{"metric"' $O/bench_default.log | tail -1 > $O/bench_default.json && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- \
  python3 bench.py --steps 20 --warmup 20 --learner-steps 50 --no-cpu-baseline --mappo-episodes 1 > $O/stats.log 2>&1 && \
python3 profiles/summarize.py $O/stats > $O/kernel_stats.txt && \
cp $(find $O/stats -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv && \
bash tools/pmc_chunk.sh $O/pmc_chunk > $O/pmc_chunk.log 2>&1 && \
timeout -k 10 200 python -u tools/chunk_trace.py > $O/chunk_trace.txt 2>&1 && \
MB_LIB=mini-marl_amd/lib_ptr/libminimarl.so timeout -k 10 200 python3 tools/mb_per_trace.py > $O/per_trace.txt 2>&1 && \
timeout -k 10 600 bash tools/pmc_mappo.sh $O/mappo > $O/mappo.log 2>&1 && \
O2=$O bash tools/prof_mappo_r6.sh > $O/mappo_stats.txt 2>&1 && \
bash tools/prof_lrn_big.sh > $O/lrn_big.txt 2>&1
rc=$?
cp -r gpurun_out/prof_mappo $O/ 2>/dev/null; cp -r gpurun_out/plrnb $O/ 2>/dev/null
tail -2 $O/bench_default.json; tail -3 $O/kernel_stats.txt
exit $rc
