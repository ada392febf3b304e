"""CPU: bench.py's own multi-rank launcher (``--gpus N`` spawns N ranks with torch.distributed.run
before any GPU call) and the typed trainer configuration."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def test_bench_gpus_2_spawns_two_ranks():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--probe-ranks"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["world"] == 2
    assert sorted(r["rank"] for r in rec["ranks"]) == [0, 1]
    assert sorted(r["local_rank"] for r in rec["ranks"]) == [0, 1]
    assert len({r["pid"] for r in rec["ranks"]}) == 2


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--probe-ranks"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "launcher started 1 ranks" in out.stderr


def test_trainer_config_schedule_and_presets():
    from minimarl.config import QTrainConfig, presets, qmix_reference, vdn_reference
    c = vdn_reference()
    # vdn/main.py:133-134 with the vdn/_config.py defaults (0.8 -> 0.05 over 15000 episodes)
    assert c.epsilon(0) == 0.8
    assert abs(c.epsilon(7500) - (0.8 - 0.75 * 0.5)) < 1e-12
    assert abs(c.epsilon(15000) - 0.05) < 1e-12 and c.epsilon(30000) == 0.05
    q = qmix_reference()
    assert (q.alpha, q.beta, q.buffer_limit, q.max_epsilon, q.epsilon_anneal_episode) == (0.8, 0.2, 1000, 0.9, 60000)
    assert q.per_flavor == "qmix" and c.per_flavor == "vdn"
    # env_name defaults: vdn Checkers-v0 (vdn/_config.py:19-24), qmix Switch2-v0 (qmix/_config.py:14-19)
    assert c.env == "checkers" and q.env == "switch" and q.n_agents == 2
    p = presets()
    assert set(p) == {"cfg1", "cfg2", "cfg3", "cfg4", "cfg5"}
    assert p["cfg2"].q.n_envs == 4096 and p["cfg2"].q.n_agents == 8 and p["cfg2"].q.h == 64
    assert p["cfg2"].q.env == "checkers" and p["cfg1"].q.env == "checkers"
    assert p["cfg4"].gpus == 8 and p["cfg3"].mappo.ppo_epoch == 15
    assert isinstance(p["cfg1"].q, QTrainConfig) and p["cfg1"].q.full_observable
