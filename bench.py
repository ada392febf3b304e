"""Headline benchmark: agent-env-steps/s (+ learner updates/s) at 4096 envs x 8 agents per GPU.

Workload (BASELINE.json configs[1]): QMIX 8-agent gridworld, 4096 envs per GPU, agent
Q-net GRU-64 (F1 = G = H = 64), chunk 10, device PER. One "step" = one lockstep
rollout step of every env on every rank: behavior Q forward + eps-greedy, env step,
target Q forward on the next obs, TD error + transition store, and every 10th step
the chunk insert into the prioritized replay. Synthetic data = the build's own
gridworld (the reference's ma_gym env is absent); random-init weights.

The JSON line also carries the QMIX learner (updates/s, configs[1]) and the MAPPO episode
(configs[2]: rollout + GAE + 15 PPO epochs; agent-env-steps/s including training).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 the driver uses
torch.distributed.run (one process per GPU, RCCL). Envs shard across ranks with no
data-path collective (weak scaling); rank 0 prints ONE JSON line.
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "mini-marl_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (vector = f32 MFMA), MI355X_MICROARCH.md
PEAK_F16_TFLOPS = 16 * PEAK_FP32_TFLOPS   # dense f16/bf16 MFMA (= 16x the f32 MFMA rate), ~2.5 PF
PEAK_HBM_GBS = 8000.0


def qnet_flops_per_agent_step(D, F1, G, H, A):
    return 2 * (D * F1 + F1 * G + 3 * G * H + 3 * H * H + H * A)


def cpu_baseline(E, N, F1, G, H, budget_s=12.0):
    """Oracle (CPU port) of the same rollout step on the host cores: numpy env + torch-CPU nets."""
    import numpy as np
    from oracle import nets
    from oracle.env import EnvSpec, VecEnvOracle
    torch.manual_seed(0)
    spec = EnvSpec(N, 100)
    D = spec.obs_dim
    P = {"W1": torch.randn(N, F1, D) * 0.1, "b1": torch.zeros(N, F1), "W2": torch.randn(N, G, F1) * 0.1,
         "b2": torch.zeros(N, G), "Wih": torch.randn(N, 3 * H, G) * 0.1, "Whh": torch.randn(N, 3 * H, H) * 0.1,
         "bih": torch.zeros(N, 3 * H), "bhh": torch.zeros(N, 3 * H), "Wq": torch.randn(N, 5, H) * 0.1,
         "bq": torch.zeros(N, 5)}
    env = VecEnvOracle(spec, E)
    obs = torch.tensor(env.observe())
    h = torch.zeros(E, N, H)
    ht = torch.zeros(E, N, H)
    rng = np.random.default_rng(0)
    steps = 0
    t0 = time.perf_counter()
    with torch.no_grad():
        while True:
            q, h = nets.agent_forward(P, obs, h)
            act = q.argmax(2).numpy()
            rnd = rng.random(E) < 0.1
            act[rnd] = rng.integers(0, 5, (int(rnd.sum()), N))
            nxt, rew, done = env.step(act)
            tq, ht = nets.agent_forward(P, torch.tensor(nxt), ht)
            qs = q.gather(2, torch.tensor(act).long().unsqueeze(-1)).squeeze(-1)
            _td = (torch.tensor(rew).sum(1) + (1 - torch.tensor(done).float()) * 0.99 * tq.max(2)[0].sum(1)
                   - qs.sum(1)).abs()
            env.reset_envs(done)
            keep = torch.tensor(~done).float().view(E, 1, 1)
            h, ht = h * keep, ht * keep
            obs = torch.tensor(env.observe())
            steps += 1
            if time.perf_counter() - t0 > budget_s:
                break
    dt = time.perf_counter() - t0
    return {"value": steps * E * N / dt, "unit": "agent-env-steps/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle rollout step (numpy env + torch-CPU GRU-{H} nets, behavior+target, TD) at "
                      f"{E} envs x {N} agents, {steps} steps in {dt:.1f}s"}


def time_kernel(fn, iters=50):
    """Average device time of fn() via events on torch's current stream (our launch stream)."""
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    start.record()
    for _ in range(iters):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--epsilon", type=float, default=0.1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--learner-steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--mappo-episodes", type=int, default=2, help="timed MAPPO episodes (0 = skip)")
    ap.add_argument("--cfg5", action="store_true",
                    help="also time the cfg5 dual agent forward (E=8192, N=27, D=300, A=36); off by default so "
                         "the default run's h3 dispatches are all the roofline's cfg2 launch")
    ap.add_argument("--learner-big-steps", type=int, default=10,
                    help="timed QMIX updates at B=4096 chunks (0 = skip; single-GPU runs only)")
    ap.add_argument("--offq-updates", type=int, default=30,
                    help="timed offpolicy episode-QMix updates on one GPU (0 = skip; single-GPU runs only)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from minimarl.engine import RolloutEngine
    E, N, Hh = args.envs, args.agents, args.hidden
    F1, G = 64, Hh
    eng = RolloutEngine(E, N, f1=F1, g=G, h=Hh, chunk=10, capacity=16 * E, seed=1234 + rank, device=dev)
    D = eng.D
    from minimarl.learner import Mixer, QLearner
    mix = Mixer(N, N * D, 64, 32, dev, seed=7)
    tmix = Mixer(N, N * D, 64, 32, dev, seed=7)
    learner = QLearner(eng.behavior, eng.target, mix, tmix, batch=args.batch, chunk=10, mode="qmix", device=dev)
    if dist:   # identical replicas: rank 0's parameters everywhere
        dist.broadcast(learner.P, 0)
        eng.sync_target()
        tmix.flat.copy_(mix.flat)
        eng.behavior.mark_dirty()
    GS = eng.graph_steps()                      # one HIP graph = one chunk of GS lockstep steps
    warm_rep = max(1, -(-args.warmup // GS))
    n_rep = max(1, -(-args.steps // GS))
    steps = n_rep * GS
    for _ in range(warm_rep):
        eng.run_graph(args.epsilon)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_rep):
        eng.run_graph(args.epsilon)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = steps * E * N * world / elapsed

    # learner: one QMIX update = PER sample (B chunks) -> C-step fwd/BPTT -> [RCCL all-reduce of the
    # flat grads] -> clip/Adam -> reprioritize; replayed as two HIP graphs
    allreduce = None
    if dist:
        def allreduce(g):
            dist.all_reduce(g)
            return world
        learner._graph_scale = 1.0 / world
    learner.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=99 + rank)
    for _ in range(5):
        learner.replay_update(allreduce)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.learner_steps):
        learner.replay_update(allreduce)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el_l = time.perf_counter() - t1
    if dist:
        t = torch.tensor([el_l], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el_l = float(t.item())
    upd_per_s = args.learner_steps / el_l

    # the same QMIX update at SURVEY 8(d)'s throughput batch (B = 4096 chunks of C = 10), single GPU
    big = None
    if args.learner_big_steps > 0 and world == 1:
        mixb, tmixb = Mixer(N, N * D, 64, 32, dev, seed=7), Mixer(N, N * D, 64, 32, dev, seed=7)
        lb = QLearner(eng.behavior, eng.target, mixb, tmixb, batch=4096, chunk=10, mode="qmix", device=dev)
        lb.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=5)
        for _ in range(2):
            lb.replay_update()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        for _ in range(args.learner_big_steps):
            lb.replay_update()
        torch.cuda.synchronize()
        el_b = time.perf_counter() - t4
        big = {"batch_chunks": 4096, "chunk": 10, "ms_per_update": round(el_b / args.learner_big_steps * 1e3, 3),
               "updates_per_s": round(args.learner_big_steps / el_b, 1),
               "chunk_samples_per_s": round(4096 * args.learner_big_steps / el_b, 1)}
        del lb, mixb, tmixb
        torch.cuda.empty_cache()

    # MAPPO (BASELINE configs[2]): 4096 envs x 8 agents per GPU, T=100 rollout steps with the fused
    # actor/critic kernel, device GAE, then 15 PPO epochs of chunked (L=5) BPTT on the whole buffer
    mappo = None
    if args.mappo_episodes > 0:
        from minimarl.env import VecEnv
        from minimarl.mappo import MappoPolicy, MappoRunner
        menv = VecEnv(E, N, max_steps=100, device=dev)
        mpol = MappoPolicy(menv.obs_dim, 5, 32, dev, seed=3)
        if dist:
            dist.broadcast(mpol.actor.flat, 0)
            dist.broadcast(mpol.critic.flat, 0)
        mr = MappoRunner(menv, mpol, T=100, L=5, ppo_epoch=15, seed=11 + rank, grad_allreduce=allreduce)
        mr.warmup()
        mr.run_episode()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t_ro = t_tr = 0.0
        t2 = time.perf_counter()
        for _ in range(args.mappo_episodes):
            ev[0].record()
            mr.rollout()
            mr.compute()
            ev[1].record()
            info = mr.train()
            ev[2].record()
            torch.cuda.synchronize()
            t_ro += ev[0].elapsed_time(ev[1])
            t_tr += ev[1].elapsed_time(ev[2])
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        el_m = time.perf_counter() - t2
        if dist:
            t = torch.tensor([el_m], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_m = float(t.item())
        k = args.mappo_episodes
        mappo = {"algo": "rmappo shared policy (MLP-LN + GRU-32 actor/critic, ValueNorm, GAE, 15 PPO epochs)",
                 "envs_per_gpu": E, "agents": N, "episode_length": 100, "data_chunk_length": 5, "ppo_epoch": 15,
                 "ms_per_episode": round(el_m / k * 1e3, 3),
                 "agent_env_steps_per_s_incl_train": round(E * N * 100 * world * k / el_m, 1),
                 "rollout_ms_per_step": round(t_ro / k / 100, 4), "train_ms": round(t_tr / k, 3),
                 "ppo_updates_per_s": round(15 * k / el_m, 2),
                 "train_info": {kk: round(float(v), 6) for kk, v in info.items()},
                 "grad_allreduce": "rccl" if dist else None}
        del mr, menv, mpol
        torch.cuda.empty_cache()

    # offpolicy episode-level QMix (offpolicy/algorithms/qmix/qmix.py:80-210):
    # train_policy_on_batch + soft target update on a device batch of B = 32 episodes x T = 100
    # steps, 8 agents, QMixer with 2-layer hypernets, double Q, PER priorities
    offq = None
    if args.offq_updates > 0 and world == 1:
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from make_golden_offq import make_batch
        from minimarl.offq import OffQMix
        oT, oB = 100, 32
        otr = OffQMix(N, D, 5, oT, oB, seed=5, device=dev)
        rng = np.random.default_rng(0)
        obs, share, acts, rew, dones, dn = make_batch(rng, N, oT, oB, D, 5)
        to = lambda x: torch.as_tensor(x).to(dev).contiguous()  # noqa: E731
        pid = "policy_0"
        ob = ({pid: to(obs)}, {pid: to(share)}, {pid: to(acts)}, {pid: to(rew)}, {pid: to(dones)}, {pid: to(dn)},
              {pid: None}, to((0.5 + rng.random(oB)).astype(np.float32)), None)
        for _ in range(3):
            otr.train_policy_on_batch(ob)
            otr.soft_target_updates()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        for _ in range(args.offq_updates):
            otr.train_policy_on_batch(ob)
            otr.soft_target_updates()
        torch.cuda.synchronize()
        el_o = time.perf_counter() - t3
        offq = {"algo": "offpolicy QMix.train_policy_on_batch + soft_update (episode BPTT, QMixer hypernets, "
                        "double Q, R2D2 priorities)", "agents": N, "episode_length": oT, "batch_episodes": oB,
                "ms_per_update": round(el_o / args.offq_updates * 1e3, 4),
                "updates_per_s": round(args.offq_updates / el_o, 1),
                "reference_cpu_ms_per_update": 115.8,
                "reference_cpu_note": "reference train_policy_on_batch, same shapes, 8 threads of the build "
                                      "container (tools/ref_time_offq.py)"}
        del otr
        torch.cuda.empty_cache()

    # cfg5 (SMAC 27m_vs_30m-like shapes, no env of that shape exists here): the dual agent
    # forward (target + behavior) at E = 8192, N = 27, D = 300, A = 36, GRU-32 on synthetic obs
    cfg5 = None
    if rank == 0 and args.cfg5:
        import ctypes
        from minimarl._lib import MM_Q_ACT, MM_Q_MAX, lib
        from minimarl.qnet import AgentQNet, ptr, stream_handle
        E5, N5, D5, A5, H5 = 8192, 27, 300, 36, 32
        n5 = [AgentQNet(N5, D5, A5, 64, 32, H5, dev, seed=s) for s in (1, 2)]
        for n in n5:
            n.pack()
        g5 = torch.Generator(device=dev).manual_seed(5)
        o5 = [(torch.rand(E5, N5, D5, device=dev, generator=g5) < 0.2).float() for _ in range(2)]
        h5 = [torch.zeros(N5, H5, E5, device=dev).permute(2, 0, 1) for _ in range(2)]
        hq = [torch.empty(N5, H5, E5, device=dev).permute(2, 0, 1) for _ in range(2)]
        qs5 = [torch.empty(E5, N5, device=dev) for _ in range(2)]
        act5 = torch.empty(E5, N5, dtype=torch.int32, device=dev)
        io5 = []
        for k, mode in enumerate((MM_Q_MAX, MM_Q_ACT)):
            io = n5[k].make_io(o5[k], h5[k], hq[k], None, mode)
            io.qsel_out = qs5[k].data_ptr()
            if mode == MM_Q_ACT:
                io.act_out, io.epsilon = act5.data_ptr(), 0.05
            io5.append(io)
        L5, st5 = lib(), stream_handle(dev)

        def dual5():
            L5.mm_agent_q_fwd2(ctypes.byref(n5[0].dims), ptr(n5[0].packed), ctypes.byref(io5[0]), E5,
                               ptr(n5[1].packed), ctypes.byref(io5[1]), E5, st5)
        t5 = time_kernel(dual5)
        f5 = 2 * qnet_flops_per_agent_step(D5, 64, 32, H5, A5) * E5 * N5
        cfg5 = {"workload": "cfg5 dual agent forward (target + behavior), synthetic obs", "envs": E5, "agents": N5,
                "obs_dim": D5, "n_actions": A5, "gru": H5, "dual_us": round(t5 * 1e6, 2),
                "agent_steps_per_s": round(2 * E5 * N5 / t5, 1), "tflops_fp32_equiv": round(f5 / t5 / 1e12, 2)}
        del n5, o5, h5, hq
        torch.cuda.empty_cache()

    # roofline of the dominant kernel: the fused agent Q forward (one launch = target net on s'_t +
    # behavior net on s_{t+1}: 2 nets x E x N agent-steps). At E >= 2048 it runs the fp16x3-split
    # kernel: every fp32 product as 3 f16 MFMAs, so its MFMA ceiling for the network's fp32 FLOPs
    # is the dense f16 peak / 3; the native f32-MFMA peak is reported beside it.
    t_fwd = time_kernel(eng.fused_forward)
    flops = 2 * qnet_flops_per_agent_step(D, F1, G, Hh, 5) * E * N
    achieved = flops / t_fwd / 1e12
    h3 = E >= 2048 and not os.environ.get("MM_FWD_F32")
    peak = PEAK_F16_TFLOPS / 3 if h3 else PEAK_FP32_TFLOPS
    # algorithmic HBM bytes per launch: per agent-step obs 4D + hidden in/out 8H + outputs (act/q 8 or max 4)
    alg_bytes = E * N * ((4 * D + 8 * Hh + 8) + (4 * D + 8 * Hh + 4))
    traffic = None
    prof = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_agent_fwd.json")))
    if prof and E == 4096 and N == 8 and Hh == 64:
        pm = json.load(open(prof[-1]))
        if pm.get("kernel", "").startswith("agent_q_fwd_h3_kernel" if h3 else "agent_q_fwd_lds_kernel"):
            traffic = int(pm["traffic_bytes_corrected"])
    kname = "agent_q_fwd_h3_kernel" if h3 else "agent_q_fwd_lds_kernel"
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "traffic_source": os.path.basename(prof[-1]) if traffic else None,
                "kernel": f"{kname}<64,64,64,1> (dual: target+behavior)", "kernel_us": round(t_fwd * 1e6, 2),
                "arith": "fp32 network FLOPs as fp16x3-split MFMA (v_mfma_f32_16x16x32_f16 x3, fp32 accumulate)"
                         if h3 else "exact f32 MFMA (v_mfma_f32_32x32x2_f32)",
                "fp32_native_peak": PEAK_FP32_TFLOPS, "frac_of_fp32_native_peak": round(achieved / PEAK_FP32_TFLOPS, 4),
                "flop_per_launch": flops, "alg_bytes_per_launch": alg_bytes,
                "hbm_frac": round(alg_bytes / t_fwd / (PEAK_HBM_GBS * 1e9), 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(E, N, F1, G, Hh)

    if rank == 0:
        line = {
            "metric": "agent-env-steps/sec (4096 envs x 8 agents per GPU, QMIX GRU-64 rollout step)",
            "value": round(value, 1), "unit": "agent-env-steps/s", "n_gpus": world, "steps": steps,
            "warmup": warm_rep * GS, "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic (build's gridworld, random init)",
            "config": {"workload": "QMIX 8-agent gridworld rollout, 4096 envs/GPU, GRU-64 agents, chunk 10, PER",
                       "envs_per_gpu": E, "agents": N, "obs_dim": D, "f1": F1, "gru": Hh, "chunk": 10,
                       "parallelism": f"env-shard x{world}"},
            "learner_updates_per_s": round(upd_per_s, 1),
            "learner": {"algo": "QMIX Train_dqn update", "batch_chunks": args.batch, "chunk": 10,
                        "mixer_hidden": 64, "ms_per_update": round(el_l / args.learner_steps * 1e3, 4),
                        "updates": args.learner_steps, "grad_allreduce": "rccl" if dist else None,
                        "reference_cpu_updates_per_s": 12.0, "throughput_batch": big},
            "mappo": mappo,
            "offpolicy_qmix": offq,
            "cfg5_forward": cfg5,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
