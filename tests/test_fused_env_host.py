"""CPU check of the fused rollout step's per-env pieces (mini-marl_amd/csrc/fused_env.h, used by
agent_fwd.hip rollout_step_h3_kernel) against oracle/env.py: the 2-bit grid packing (dword and byte
loads), the 45-bit obs masks and the features built from them, the dynamics (positions, rewards, done,
eaten fruit), the dword grid write-back and the reset obs from the initial state — bit for bit over random
rollouts. The helpers are compiled for the host by hipcc (no GPU needed)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle.env import EnvSpec, VecEnvOracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("fec") / "fused_env_check")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "mini-marl_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "fused_env_check.cpp"), "-o", out], check=True)
    return out


def _write(path, spec, E, steps, seed):
    rng = np.random.default_rng(seed)
    ora = VecEnvOracle(spec, E)
    # start from scattered states: a few random steps first
    for _ in range(int(rng.integers(0, 30))):
        ora.step(rng.integers(0, 5, (E, spec.n_agents)))
    with open(path, "wb") as fp:
        N, R, C = spec.n_agents, spec.rows, spec.cols
        np.array([E, N, R, C, spec.obs_dim, int(spec.full_observable), spec.max_steps, steps], np.int32).tofile(fp)
        np.array([spec.step_cost, spec.inv_r, spec.inv_c], np.float32).tofile(fp)
        spec.init_pos.astype(np.int32).tofile(fp)
        spec.init_grid.astype(np.int8).tofile(fp)
        init = VecEnvOracle(spec, 1)
        init.observe()[0].astype(np.float32).tofile(fp)
        for _ in range(steps):
            ora.pos.astype(np.int32).tofile(fp)
            ora.grid.astype(np.int8).tofile(fp)
            ora.steps.astype(np.int32).tofile(fp)
            ora.apples.astype(np.int32).tofile(fp)
            ora.observe().astype(np.float32).tofile(fp)
            act = rng.integers(0, 5, (E, N)).astype(np.int32)
            act.tofile(fp)
            nxt, rew, done = ora.step(act)
            nxt.astype(np.float32).tofile(fp)
            rew.astype(np.float32).tofile(fp)
            done.astype(np.uint8).tofile(fp)
            ora.pos.astype(np.int32).tofile(fp)
            ora.grid.astype(np.int8).tofile(fp)
            ora.reset_envs(done)


@pytest.mark.parametrize("n,full,cols,max_steps", [(2, False, 8, 100), (2, True, 8, 100), (3, False, 8, 25),
                                                    (8, False, 8, 100), (4, True, 8, 40), (2, False, 5, 30),
                                                    (5, False, 7, 60)])
def test_fused_env_helpers_vs_oracle(checker, tmp_path, n, full, cols, max_steps):
    spec = EnvSpec(n, max_steps, full_observable=full, cols=cols)
    path = str(tmp_path / "rec.bin")
    _write(path, spec, 48, 60, seed=n * 100 + cols)
    r = subprocess.run([checker, path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
