# kernel stats of a short rollout+learner bench (no MAPPO) -> gpurun_out/pb/k.txt
export TMPDIR=/tmp
mkdir -p gpurun_out/pb
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pb/p -- python3 bench.py --no-cpu-baseline --mappo-episodes 0 --learner-steps 20 > gpurun_out/pb/b.log 2>&1 || exit 1
python3 profiles/summarize.py gpurun_out/pb/p > gpurun_out/pb/k.txt
head -12 gpurun_out/pb/k.txt
tail -1 gpurun_out/pb/b.log | cut -c1-300
