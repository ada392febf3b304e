# the bench's RCCL branch at world size 1 on a one-GPU box (torch.distributed.run, backend "nccl" = RCCL)
mkdir -p gpurun_out
export MM_BENCH_DIST1=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 1 --steps 20 --warmup 5 --learner-steps 10 --no-cpu-baseline --mappo-episodes 1 --no-cfg5 \
  --train-episodes 2 --cfg1-episodes 0 --offq-updates 0 --learner-big-steps 0 > gpurun_out/rccl_ws1.log 2>&1
rc=$?
grep '^{"metric"' gpurun_out/rccl_ws1.log | tail -1 > gpurun_out/rccl_ws1.json
python3 -c "import json; d=json.load(open('gpurun_out/rccl_ws1.json')); print(d['rccl_world_size'], d['ms_per_step'], d['replica_checksums'], d['learner'].get('grad_allreduce'), d['train_loop'].get('grad_allreduce'), d['mappo'].get('grad_allreduce'))" || tail -20 gpurun_out/rccl_ws1.log
exit $rc
