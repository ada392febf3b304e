# rehearsal of bench.py --gpus 2 on a one-GPU box (both ranks on cuda:0, gloo collectives)
mkdir -p gpurun_out
MM_BENCH_SHARED_GPU=1 timeout -k 10 500 python bench.py --gpus 2 --steps 20 --warmup 5 --learner-steps 10 --no-cpu-baseline --mappo-episodes 1 --no-cfg5 --train-episodes 2 > gpurun_out/dist2.log 2>&1
rc=$?
tail -c 3000 gpurun_out/dist2.log
exit $rc
