"""GPU: the data-parallel path through a REAL collective (verdict r03 item 7).

bench.py --gpus 2 is started as a fresh child process with MM_BENCH_SHARED_GPU=1: both ranks run on the one
GPU of the box and their collectives go over gloo (RCCL refuses two ranks on one device; the 8-GPU RCCL run is
the driver's). This exercises, with real inter-process all-reduces: the rank-0 parameter broadcast, the
QMIX learner's flat-gradient all-reduce inside replay_update (QLearner.replay_update(allreduce)), the
integrated train loop's learner, and MAPPO's per-epoch gradient all-reduce plus the all-reduced advantage /
return statistics (MappoRunner(grad_allreduce=...)). After the updates every replica's parameters must be
bit-identical (exact int64 checksums of the parameter bytes, all-gathered by bench.py). Each rank runs cfg4's shard:
4096 envs x 8 agents (the rollout in one-launch-per-step mode: two processes share the GPU)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(420)
def test_bench_two_ranks_replicas_stay_identical():
    env = dict(os.environ, MM_BENCH_SHARED_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
           "--repeats", "1", "--envs", "4096", "--learner-steps", "5", "--learner-big-steps", "0",
           "--train-episodes", "1", "--cfg1-episodes", "0", "--mappo-episodes", "1", "--offq-updates", "0",
           "--no-cfg5", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["rccl_world_size"] == 2 and line["n_gpus"] == 2
    reps = line["replica_checksums"]
    assert set(reps) == {"qmix_learner_params", "train_loop_learner_params", "mappo_actor", "mappo_critic"}
    for name, cks in reps.items():
        assert len(cks) == 2 and cks[0] == cks[1], (name, cks)
    assert line["learner"]["grad_allreduce"] == "gloo"
    assert line["mappo"]["grad_allreduce"] == "gloo"
    assert all(np.isfinite(v) for v in line["mappo"]["train_info"].values()), line["mappo"]["train_info"]
    assert line["value"] > 0 and np.isfinite(line["train_loop"]["ms_per_episode"])


@pytest.mark.timeout(300)
def test_bench_rccl_branch_world_size_one():
    """The RCCL branch itself on the box's one GPU: bench.py under torch.distributed.run with one rank and
    MM_BENCH_DIST1=1 initialises the "nccl" (= RCCL) process group with device_id and runs every collective of the
    N > 1 path (parameter broadcast, barriers, max-over-ranks timing, the learner / train-loop / MAPPO gradient
    all-reduces, the all-gathered replica checksums) through RCCL."""
    env = dict(os.environ, MM_BENCH_DIST1="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", "29531", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "10",
           "--warmup", "2", "--repeats", "1", "--learner-steps", "3", "--learner-big-steps", "0", "--train-episodes",
           "1", "--cfg1-episodes", "0", "--mappo-episodes", "1", "--offq-updates", "0", "--no-cfg5", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["rccl_world_size"] == 1 and line["n_gpus"] == 1
    assert set(line["replica_checksums"]) == {"qmix_learner_params", "train_loop_learner_params", "mappo_actor",
                                              "mappo_critic"}
    assert line["learner"]["grad_allreduce"] == "rccl" and line["mappo"]["grad_allreduce"] == "rccl"
    assert line["train_loop"]["grad_allreduce"] == "rccl"
    assert all(np.isfinite(v) for v in line["mappo"]["train_info"].values()), line["mappo"]["train_info"]
