"""Headline benchmark: agent-env-steps/s (+ learner updates/s) at 4096 envs x 8 agents per GPU.

Workload (BASELINE.json configs[1]): QMIX 8-agent gridworld, 4096 envs per GPU, agent
Q-net GRU-64 (F1 = G = H = 64), chunk 10, device PER. One "step" = one lockstep
rollout step of every env on every rank: behavior Q forward + eps-greedy, env step,
target Q forward on the next obs, TD error + transition store, and every 10th step
the chunk insert into the prioritized replay. Env = ma_gym Checkers-v0 restated (oracle/env.py; ma-gym
itself is absent), 8 agents as 4 stacked 3x8 boards; random-init weights.

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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _cpu_rollout_rate(E, N, F1, G, H, budget_s):
    """Oracle (CPU port) of the same rollout step: numpy env + torch-CPU nets, behavior + target + TD."""
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
    return steps * E * N / dt, steps, dt


def cpu_baseline(E, N, F1, G, H, budget_s=8.0):
    """The oracle's rollout step on the host cores, at torch's default thread count and at 1 thread;
    the better of the two is the baseline."""
    nthreads = torch.get_num_threads()
    runs = []
    for th in (nthreads, 1):
        torch.set_num_threads(th)
        rate, steps, dt = _cpu_rollout_rate(E, N, F1, G, H, budget_s)
        runs.append({"threads": th, "value": round(rate, 1), "steps": steps, "seconds": round(dt, 2)})
    torch.set_num_threads(nthreads)
    best = max(runs, key=lambda r: r["value"])
    return {"value": best["value"], "unit": "agent-env-steps/s", "cores": best["threads"], "kind": "port",
            "nproc": os.cpu_count(), "cpu_model": cpu_model(), "runs": runs,
            "sample": f"oracle rollout step (numpy env + torch-CPU GRU-{H} nets, behavior+target, TD) at "
                      f"{E} envs x {N} agents, ~{budget_s:.0f} s per thread setting; best of {nthreads} threads "
                      f"and 1 thread"}


def cpu_learner_baseline(N, D, B=32, C=10, H=64, Hm=64, budget_s=6.0):
    """The oracle's Train_dqn update (qmix/_train.py:19-121 restated in oracle/nets.py) at the bench
    learner's shapes, timed on the host cores: the port's updates/s beside the GPU's."""
    from oracle import nets
    torch.manual_seed(0)
    F1, G, A, K1 = 64, H, 5, 32
    r = lambda *s: torch.randn(*s) * 0.1  # noqa: E731
    P = {"W1": r(N, F1, D), "b1": r(N, F1), "W2": r(N, G, F1), "b2": r(N, G), "Wih": r(N, 3 * H, G),
         "Whh": r(N, 3 * H, H), "bih": r(N, 3 * H), "bhh": r(N, 3 * H), "Wq": r(N, A, H), "bq": r(N, A)}
    S = N * D
    M = {"gWih": r(3 * Hm, S), "gWhh": r(3 * Hm, Hm), "gbih": r(3 * Hm), "gbhh": r(3 * Hm), "w1W": r(N * K1, Hm),
         "w1b": r(N * K1), "w2W": r(K1, Hm), "w2b": r(K1), "b1W": r(K1, Hm), "b1b": r(K1), "b2aW": r(K1, Hm),
         "b2ab": r(K1), "b2bW": r(1, K1), "b2bb": r(1)}
    g = torch.Generator().manual_seed(1)
    batch = (torch.rand(B, C, N, D, generator=g), torch.randint(0, A, (B, C, N), generator=g).float(),
             torch.randn(B, C, N, generator=g), torch.rand(B, C, N, D, generator=g),
             (torch.rand(B, C, 1, generator=g) < 0.1).float(), torch.ones(B, 1))
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        P, M, _, _, _ = nets.qmix_train_step(P, M, P, M, batch, 0.99, 1e-3, 5.0, hidden_dim=K1)
        P = {k: v.detach() for k, v in P.items()}
        M = {k: v.detach() for k, v in M.items()}
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 2), "unit": "updates/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle Train_dqn update (torch-CPU autograd) at B={B}, C={C}, N={N}, GRU-{H}, Hm={Hm}: "
                      f"{n} updates in {dt:.1f} s"}


def cpu_offq_baseline(otr, batch_np, budget_s=6.0):
    """The oracle's offpolicy QMix.train_policy_on_batch (qmix.py:80-210 restated in oracle/offq.py) at
    the bench's shapes, on the host cores, from the GPU trainer's initial parameters."""
    from oracle import offq as ref
    q, m = otr.state_dict()
    qt, mt = otr.state_dict(target=True)
    P = ref.agent_from_state({"q." + k: v.numpy() for k, v in q.items()})
    M = ref.mixer_from_state({"m." + k: v.numpy() for k, v in m.items()})
    PT = ref.agent_from_state({"q." + k: v.numpy() for k, v in qt.items()})
    MT = ref.mixer_from_state({"m." + k: v.numpy() for k, v in mt.items()})
    n, st = 0, {}
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        P, M, _ = ref.train_batch(P, M, PT, MT, batch_np, mixer="qmix", double_q=True, use_per=True,
                                  adam_state=st)
        PT, MT = ref.soft_update(PT, P, 0.005), ref.soft_update(MT, M, 0.005)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(dt / n * 1e3, 2), "unit": "ms/update", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle train_policy_on_batch + soft update (torch-CPU autograd), same shapes: {n} updates "
                      f"in {dt:.1f} s"}


def time_kernel(fn, iters=50):
    """Average device time of fn(): `iters` back-to-back launches captured in one HIP graph and replayed
    between events on torch's current stream (our launch stream), so host launch latency does not pad
    the kernel time (rocprofv3's per-dispatch durations are the cross-check, profiles/)."""
    from minimarl.qnet import graph_capture
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with graph_capture(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    start.record()
    g.replay()
    end.record()
    torch.cuda.synchronize()
    del g
    return start.elapsed_time(end) / iters / 1e3


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n):
    """``--gpus N`` without an outer launcher: start N ranks (one process per GPU) with
    torch.distributed.run as a CHILD process, before this process makes any GPU call, and return its
    exit code. An outer torchrun (WORLD_SIZE set) runs main() directly instead."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def replica_checksums(dist, tensors):
    """{name: [exact int64 checksum of the tensor's bytes on every rank]} (data-parallel replicas must stay
    bit-identical after every update); an all-gather over the process group."""
    out = {}
    for name, t in tensors.items():
        ck = t.detach().contiguous().view(torch.int32).to(torch.int64).sum().reshape(1)
        if dist is None:
            out[name] = [int(ck.item())]
            continue
        ck = ck.to(t.device) if dist.get_backend() == "nccl" else ck.cpu()
        parts = [torch.zeros_like(ck) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, ck)
        out[name] = [int(x.item()) for x in parts]
    return out


def probe_ranks(world, rank):
    """``--probe-ranks``: rendezvous over gloo (no GPU), gather every rank id, rank 0 prints one JSON line."""
    import torch.distributed as dist
    dist.init_process_group("gloo")
    ids = [None] * world
    dist.all_gather_object(ids, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                                 "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"probe": "ranks", "world": dist.get_world_size(), "ranks": ids}))
    dist.destroy_process_group()


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
    ap.add_argument("--no-cfg5", action="store_true",
                    help="skip the cfg5 lines (dual agent forward at E=8192, N=27, D=300, A=36 and the cfg5 "
                         "QMIX update with the fp16 mixer state projection)")
    ap.add_argument("--cfg5-batch", type=int, default=4096, help="cfg5 learner batch (chunks of C=10)")
    ap.add_argument("--learner-big-steps", type=int, default=10,
                    help="timed QMIX updates at B=4096 chunks (0 = skip; single-GPU runs only)")
    ap.add_argument("--offq-updates", type=int, default=30,
                    help="timed offpolicy episode-QMix updates on one GPU (0 = skip; single-GPU runs only)")
    ap.add_argument("--train-episodes", type=int, default=3,
                    help="timed episodes of the integrated QMIX train loop (0 = skip)")
    ap.add_argument("--repeats", type=int, default=10,
                    help="timed regions of exactly --steps steps each; ms_per_step is their median (min / max beside)")
    ap.add_argument("--cfg1-episodes", type=int, default=20,
                    help="timed training episodes of the cfg1 VDN trainer lines (0 = skip; single-GPU runs only)")
    ap.add_argument("--probe-ranks", action="store_true", help="launcher check: gloo rendezvous only, no GPU")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    if args.probe_ranks:
        probe_ranks(world, rank)
        return
    # MM_BENCH_SHARED_GPU=1 (rehearsal of the N > 1 path on a one-GPU box): every rank on cuda:0 and the
    # collectives over gloo instead of RCCL (RCCL refuses two ranks on one device); numbers then are not
    # a scaling measurement
    shared = os.environ.get("MM_BENCH_SHARED_GPU", "0") == "1"
    if shared:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    # MM_BENCH_DIST1=1 (with a launcher's RANK / WORLD_SIZE / MASTER_*): the collective path at world size 1 — on a
    # one-GPU box this runs the RCCL branch (init with device_id, barriers, the max-over-ranks timing, the gradient
    # all-reduce, the replica checksums) on the hardware; the numbers equal the N = 1 line's
    if world > 1 or (os.environ.get("MM_BENCH_DIST1", "0") == "1" and "WORLD_SIZE" in os.environ):
        import torch.distributed as dist
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from minimarl.engine import RolloutEngine
    E, N, Hh = args.envs, args.agents, args.hidden
    F1, G = 64, Hh
    cap = 16 * E
    # (ranks sharing one GPU: one launch per step, the chunk-persistent kernel needs every CU for its own blocks)
    eng = RolloutEngine(E, N, f1=F1, g=G, h=Hh, chunk=10, capacity=cap, seed=1234 + rank, device=dev,
                        persistent=False if shared else None)
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
    # setup (untimed, not counted as warm-up): fill the PER to capacity so every timed chunk insert
    # is a steady-state evicting insert
    fill_chunks = cap // E
    for _ in range(fill_chunks):
        eng.run_graph(args.epsilon)
    eng.capture_steps()
    assert len(eng.per) == cap
    # warm-up, then R timed regions of exactly K lockstep steps each (chunk graphs + single-step graphs),
    # each bracketed by barrier + synchronize and maxed over ranks; the median region is the result
    eng.run_steps(args.warmup, args.epsilon)
    # each timed region of K steps replays ONE captured K-step graph (captured here, untimed, for every graph
    # phase a region starts at): consecutive graph launches leave the GPU idle ~9 us each (region
    # fixed cost), which a run of chunk + single-step graph replays per region would pay ~10 times
    n_phase = eng.graph_steps()
    for i in range(min(n_phase, max(1, args.repeats))):
        eng.capture_region(args.steps, start=eng.t + i * args.steps)
    reps = []
    for _ in range(max(1, args.repeats)):
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run_steps(args.steps, args.epsilon)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        reps.append(el)
    elapsed = float(np.median(reps))
    steps = args.steps
    # the device error words of the timed rollout (untimed poll): bit 0 a staging row outside the chunk store, bit 1 a
    # chunk-persistent hand-off wait that expired (its blocks were not co-resident), bit 8 a PER tree-node guard; any
    # set bit means the timed regions did not run the path as specified, and the line is not printed
    errors = int(eng.err.item()) | (eng.per.error_word(clear=False) << 8)
    if errors:
        raise SystemExit(f"bench.py: rollout device error bits {errors:#x} after the timed regions")
    value = steps * E * N * world / elapsed

    # learner: one QMIX update = PER sample (B chunks) -> C-step fwd/BPTT -> [RCCL all-reduce of the
    # flat grads] -> clip/Adam -> reprioritize; replayed as two HIP graphs
    allreduce = None
    if dist:
        def allreduce(g):
            dist.all_reduce(g)
            return world
        learner._graph_scale = 1.0 / world
    # single-replica: the trainer's update_iter = 10 consecutive updates per graph launch (QTrainer.learn)
    per_replay = 10 if allreduce is None else 1
    learner.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=99 + rank, per_replay=per_replay)
    learner.replay_updates(10, allreduce)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    learner.replay_updates(args.learner_steps, allreduce)
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
    replicas = replica_checksums(dist, {"qmix_learner_params": learner.P}) if dist else None

    # the same QMIX update at SURVEY 8(d)'s throughput batch (B = 4096 chunks of C = 10), single GPU
    big = None
    if args.learner_big_steps > 0 and world == 1:
        from minimarl.qnet import AgentQNet
        mixb, tmixb = Mixer(N, N * D, 64, 32, dev, seed=7), Mixer(N, N * D, 64, 32, dev, seed=7)
        behb, tgtb = (AgentQNet(N, D, 5, F1, G, Hh, dev) for _ in range(2))
        behb.copy_from(eng.behavior)
        tgtb.copy_from(eng.target)
        lb = QLearner(behb, tgtb, mixb, tmixb, batch=4096, chunk=10, mode="qmix", device=dev)
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
        del lb, mixb, tmixb, behb, tgtb
        torch.cuda.empty_cache()

    # integrated QMIX rollout-and-learn (minimarl/train.py; vdn/main.py:127-186, qmix/main.py:172-262):
    # per training episode 100 lockstep steps of all envs, then update_iter = 10 learner updates of
    # B = 32 chunks (the reference's 10 updates per episode), hard target sync every 20 episodes;
    # the replay is filled to capacity by the (untimed) epsilon = 1 warm-up
    trainer = None
    if args.train_episodes > 0:
        from minimarl.config import presets
        from minimarl.train import QTrainer
        tcfg = presets()["cfg2"].q
        tcfg.n_envs, tcfg.n_agents, tcfg.buffer_limit, tcfg.test_interval = E, N, cap, 0
        tcfg.persistent = False if shared else None
        tcfg.seed = 17
        tr = QTrainer(tcfg, device=dev, rank=rank, grad_allreduce=allreduce, world=world, track_score=True)
        if dist:
            dist.broadcast(tr.learner.P, 0)
            tr.eng.behavior.mark_dirty()
            tr.eng.sync_target()
            tr.tmix.flat.copy_(tr.mix.flat)
        tr.warmup()
        tr.train_episode()                       # captures the learner graphs
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        el_t = tr.timed(args.train_episodes)
        if dist:
            dist.barrier()
            t = torch.tensor([el_t], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_t = float(t.item())
        k = args.train_episodes
        if dist:
            replicas.update(replica_checksums(dist, {"train_loop_learner_params": tr.learner.P}))
        trainer = {"algo": "QMIX train loop (rollout + 10 Train_dqn updates per episode + target sync)",
                   "envs_per_gpu": E, "agents": N, "episode_steps": tcfg.max_step, "updates_per_episode":
                   tcfg.update_iter, "batch_chunks": tcfg.batch_size, "episodes": k,
                   "ms_per_episode": round(el_t / k * 1e3, 3),
                   "agent_env_steps_per_s_incl_learning": round(E * N * tcfg.max_step * world * k / el_t, 1),
                   "learner_updates_per_s": round(tcfg.update_iter * k / el_t, 1),
                   "train_score": tr.train_score(), "grad_allreduce": (("gloo" if shared else "rccl") if dist else None)}
        del tr
        torch.cuda.empty_cache()

    # cfg1 (BASELINE configs[0]): VDN, 2 agents, full obs (D = 94), GRU-32, the vdn/_config.py learner (B = 32
    # chunks of 10, 10 updates per episode, PER 10000 chunks, alpha = beta = 0.4) and the logged run's test cadence
    # (test_interval 10, test_episodes 20; vdn/logs/vdn-1710766189.log:30-31). Two shapes: 32 lockstep envs (the
    # BASELINE config; one training iteration = 100 steps of all 32 envs + 10 updates) and ONE env, the
    # reference's own runner shape (an iteration = one episode + 10 updates), whose episodes/s sits beside the
    # reference's logged 2.43 episodes/s (vdn/logs/vdn-1710766189.log:41,16539: 15000 episodes in 6160 s on a
    # desktop CPU) and warm-up 2968 agent-env-steps/s (wandb run tw6w4mqv output.log:36)
    cfg1 = None
    if args.cfg1_episodes > 0 and world == 1:
        from minimarl.config import presets
        from minimarl.train import QTrainer
        cfg1 = {"workload": "VDN 2-agent gridworld (full obs D = 94), GRU-32, B = 32 x C = 10, 10 updates/episode, "
                            "PER 10000 chunks, 20 greedy test episodes every 10 episodes",
                "reference_cpu": {"episodes_per_s": 2.43, "warmup_agent_env_steps_per_s": 2968.0,
                                  "source": "reference's own logged run on a desktop CPU (12 cores / 24 threads): "
                                            "vdn/logs/vdn-1710766189.log:41,16539 (15000 episodes in 6160 s); "
                                            "warm-up 148.4 chunks/s, vdn/wandb/run-20240318_214947-tw6w4mqv/files/"
                                            "output.log:36"}}
        for envs in (32, 1):
            c1 = presets()["cfg1"].q
            c1.n_envs, c1.test_interval, c1.test_envs, c1.seed = envs, 10, 20, 23
            tr1 = QTrainer(c1, device=dev, track_score=True)
            torch.cuda.synchronize()
            tw = time.perf_counter()
            tr1.warmup()                          # epsilon = 1 rollout until the replay holds 10000 chunks
            torch.cuda.synchronize()
            el_w = time.perf_counter() - tw
            tr1.train(10)                         # captures the learner graphs, runs the first test
            torch.cuda.synchronize()
            t7 = time.perf_counter()
            tr1.train(args.cfg1_episodes)
            torch.cuda.synchronize()
            el7 = time.perf_counter() - t7
            k7 = args.cfg1_episodes
            cfg1[f"envs_{envs}"] = {
                "training_iterations_per_s": round(k7 / el7, 2), "env_episodes_per_s": round(k7 * envs / el7, 1),
                "agent_env_steps_per_s_incl_learning": round(envs * 2 * c1.max_step * k7 / el7, 1),
                "learner_updates_per_s": round(c1.update_iter * k7 / el7, 1), "ms_per_iteration": round(el7 / k7 * 1e3, 3),
                "warmup_agent_env_steps_per_s": round(c1.buffer_limit * c1.chunk_size * 2 / el_w, 1),
                "timed_iterations": k7, "test_score": tr1.history[-1]["test_score"] if tr1.history else None}
            del tr1
            torch.cuda.empty_cache()
        r1 = cfg1["envs_1"]
        cfg1["vs_reference_cpu"] = {"episodes_per_s (1 env)": round(r1["env_episodes_per_s"] / 2.43, 1),
                                    "warmup agent-env-steps/s (1 env)": round(r1["warmup_agent_env_steps_per_s"] / 2968.0, 1)}

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
        if dist:
            replicas.update(replica_checksums(dist, {"mappo_actor": mpol.actor.flat, "mappo_critic": mpol.critic.flat}))
        Dm, Hm_ = menv.obs_dim, 32
        macs = sum(Hm_ * Dm + Hm_ * Hm_ + 6 * Hm_ * Hm_ + o * Hm_ for o in (5, 1))
        mflop = 6.0 * macs * E * N * 100
        mappo = {"algo": "rmappo shared policy (MLP-LN + GRU-32 actor/critic, ValueNorm, GAE, 15 PPO epochs)",
                 "envs_per_gpu": E, "agents": N, "episode_length": 100, "data_chunk_length": 5, "ppo_epoch": 15,
                 "ms_per_episode": round(el_m / k * 1e3, 3),
                 "agent_env_steps_per_s_incl_train": round(E * N * 100 * world * k / el_m, 1),
                 "rollout_ms_per_step": round(t_ro / k / 100, 4), "train_ms": round(t_tr / k, 3),
                 "train_ms_per_epoch": round(t_tr / k / 15, 3),
                 # algorithmic fp32 work of one epoch's gradients (forward + data backward + weight
                 # gradients = 3 x 2 x MACs per row-step of both nets; the fused pass also recomputes the forward)
                 "grad_gflop_per_epoch": round(mflop / 1e9, 1),
                 "grad_tflops_fp32": round(mflop / (t_tr / k / 15 * 1e-3) / 1e12, 2),
                 "grad_path": "mm_mappo_grad: recurrent + MLP passes on fp16x3-split v_mfma_f32_32x32x16_f16 with power-of-two operand scaling (fp32-level products, f32 accumulate), forward recomputed from chunk-start hiddens",
                 "ppo_updates_per_s": round(15 * k / el_m, 2),
                 "train_info": {kk: round(float(v), 6) for kk, v in info.items()},
                 "grad_allreduce": (("gloo" if shared else "rccl") if dist else None)}
        del mr, menv, mpol
        torch.cuda.empty_cache()

    # offpolicy episode-level QMix (offpolicy/algorithms/qmix/qmix.py:80-210):
    # train_policy_on_batch + soft target update on a device batch of B = 32 episodes x T = 100
    # steps, 8 agents, QMixer with 2-layer hypernets, double Q, PER priorities
    offq = None
    if args.offq_updates > 0 and world == 1:
        from minimarl.offq import OffQMix
        from minimarl.synth import offq_episode_batch as make_batch
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
        # the same update fed by the device episode replay (PrioritizedRecReplayBuffer, rec_buffer.py:243-324,
        # the reference's default buffer_size 10000 episodes): sample(B, beta) -> train_policy_on_batch ->
        # update_priorities -> soft update, nothing leaves the GPU
        from minimarl.recbuf import PrioritizedRecReplayBuffer

        box = lambda n: type("Box", (), {"shape": (n,)})()  # noqa: E731  (gym.spaces stand-ins: .shape / .n)
        pinfo = {pid: {"obs_space": box(D), "share_obs_space": box(N * D),
                       "act_space": type("Discrete", (), {"n": 5})()}}
        rb = PrioritizedRecReplayBuffer(0.6, pinfo, {pid: list(range(N))}, 10000, oT, True, False, device=dev,
                                        seed=7, leaf_mode="slots")
        ins = [to(np.ascontiguousarray(np.moveaxis(x, 0, 2))) for x in (obs, acts, rew, dones)]   # -> [L, n, N, X]
        sh_in = to(np.ascontiguousarray(np.repeat(share[:, :, None], N, axis=2)))                 # [T+1, n, N, S]
        dn_in = to(dn)
        for _ in range(10000 // oB + 1):
            rb.insert(oB, {pid: ins[0]}, {pid: sh_in}, {pid: ins[1]}, {pid: ins[2]}, {pid: ins[3]}, {pid: dn_in})
        ev_r = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(3):
            smp = rb.sample(oB, 0.4, pid)
            _, pr, ix = otr.train_policy_on_batch(smp)
            rb.update_priorities(ix, pr, pid)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        for _ in range(args.offq_updates):
            smp = rb.sample(oB, 0.4, pid)
            _, pr, ix = otr.train_policy_on_batch(smp)
            rb.update_priorities(ix, pr, pid)
            otr.soft_target_updates()
        torch.cuda.synchronize()
        el_r = time.perf_counter() - t4
        ev_r[0].record()
        for _ in range(args.offq_updates):
            smp = rb.sample(oB, 0.4, pid)
            rb.update_priorities(smp[8], torch.ones(oB, device=dev), pid)
        ev_r[1].record()
        torch.cuda.synchronize()
        gb = sum(t.numel() * 4 for t in (smp[0][pid], smp[1][pid], smp[2][pid], smp[3][pid], smp[4][pid],
                                         smp[5][pid])) * 2 / 1e9           # gathered bytes read + written
        ms_buf = ev_r[0].elapsed_time(ev_r[1]) / args.offq_updates
        offq["with_episode_replay"] = {
            "buffer": "PrioritizedRecReplayBuffer (device, 10000 episodes, sum/min segment trees)",
            "ms_per_update": round(el_r / args.offq_updates * 1e3, 4),
            "buffer_ms_per_sample_and_update": round(ms_buf, 4),
            "gather_bytes_per_sample": int(gb * 1e9),
            "gather_GBps_incl_tree_ops": round(gb / (ms_buf * 1e-3), 1)}
        del rb
        if not args.no_cpu_baseline:
            bnp = {"obs": obs, "share_obs": share, "acts": acts, "rewards": rew, "dones_env": dn,
                   "is_weight": (0.5 + np.random.default_rng(1).random(oB)).astype(np.float32)}
            offq["cpu_baseline"] = cpu_offq_baseline(otr, bnp)
        del otr
        torch.cuda.empty_cache()

    # cfg5 (SMAC 27m_vs_30m-like shapes, no env of that shape exists here): the dual agent
    # forward (target + behavior) at E = 8192, N = 27, D = 300, A = 36, GRU-32 on synthetic obs
    cfg5 = None
    if rank == 0 and not args.no_cfg5 and world == 1:
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
                               ptr(n5[1].packed), ctypes.byref(io5[1]), E5, stream_handle(dev))
        t5 = time_kernel(dual5)
        f5 = 2 * qnet_flops_per_agent_step(D5, 64, 32, H5, A5) * E5 * N5
        cfg5 = {"workload": "cfg5 dual agent forward (target + behavior), synthetic obs", "envs": E5, "agents": N5,
                "parity_test": "tests/test_gpu_headline.py::test_cfg5_dual_forward_vs_oracle",
                "obs_dim": D5, "n_actions": A5, "gru": H5, "dual_us": round(t5 * 1e6, 2),
                "agent_steps_per_s": round(2 * E5 * N5 / t5, 1), "tflops_fp32_equiv": round(f5 / t5 / 1e12, 2)}
        # cfg5 QMIX update at the throughput batch: agent nets GRU-32, Hm = 32 mixer over the 8100-wide
        # state, the state projection on fp16 MFMA (SURVEY 8c tolerance: rtol 2e-3 on Q_tot, tested in
        # test_gpu_learner.py); synthetic batch resident in HBM
        B5, C5 = args.cfg5_batch, 10
        m5 = [Mixer(N5, N5 * D5, 32, 32, dev, seed=7 + k) for k in range(2)]
        l5 = QLearner(n5[1], n5[0], m5[0], m5[1], batch=B5, chunk=C5, mode="qmix", device=dev, mixer_fp16=True)
        st5 = (torch.rand(B5, C5, N5, D5, device=dev, generator=g5) < 0.2).float()
        ns5 = (torch.rand(B5, C5, N5, D5, device=dev, generator=g5) < 0.2).float()
        act5b = torch.randint(0, A5, (B5, C5, N5), device=dev, generator=g5).float()
        rew5 = torch.randn(B5, C5, N5, device=dev, generator=g5) * 0.5
        dn5 = (torch.rand(B5, C5, 1, device=dev, generator=g5) < 0.1).float()
        w5 = torch.rand(B5, 1, device=dev, generator=g5) * 0.5 + 0.5
        l5.load_batch(st5, act5b, rew5, ns5, dn5, w5)
        del st5, ns5
        l5.capture_update(None, None, None)
        l5.replay_update()
        torch.cuda.synchronize()
        k5 = 3
        t6 = time.perf_counter()
        for _ in range(k5):
            l5.replay_update()
        torch.cuda.synchronize()
        el5 = (time.perf_counter() - t6) / k5
        cfg5["learner"] = {"batch_chunks": B5, "chunk": C5, "mixer_state_projection": "fp16 MFMA (rtol 2e-3 on Q_tot)",
                           "agent_path": "exact f32 MFMA (forward, BPTT and weight gradients)",
                           "mixer_weight_gradients": "bf16x3-split MFMA products (~2^-16 relative per product)"
                           if l5.mixer_bf3 else "exact f32 MFMA",
                           "parity_test": "tests/test_gpu_learner.py::test_learner_cfg5_benched_path_vs_oracle (same "
                                          "graphs at B = 512: Q_tot / loss / TD, every gradient, post-Adam params)",
                           "ms_per_update": round(el5 * 1e3, 3), "chunk_samples_per_s": round(B5 / el5, 1),
                           "loss_finite": bool(torch.isfinite(l5.loss).all().item())}
        del n5, o5, h5, hq, l5, m5
        torch.cuda.empty_cache()

    # roofline of the dominant kernel. Fused mode (E >= 2048, the default here): the ONE launch of a rollout step,
    # mm_rollout_step = env step + target net on s'_t + behavior net on s_{t+1} (2 nets x E x N agent-steps of
    # network FLOPs; the env step is integer work on top). Otherwise the dual forward launch of the two-launch
    # step. At E >= 2048 the network runs as fp16x3-split MFMAs (every fp32 product as 3 f16 MFMAs), so the
    # MFMA ceiling for the network's fp32 FLOPs is the dense f16 peak / 3; the native f32-MFMA peak beside it.
    flops = 2 * qnet_flops_per_agent_step(D, F1, G, Hh, 5) * E * N
    h3 = E >= 2048
    peak = PEAK_F16_TFLOPS / 3 if h3 else PEAK_FP32_TFLOPS
    per_launch_steps = 1
    if eng.chunked:
        # chunk mode (the default at the headline shape): ONE launch runs the C steps of a chunk, mm_rollout_chunk =
        # per step the env step + target net on s'_t + behavior net on s_{t+1}; its FLOPs per launch = C steps' worth
        # (the timed regions run launches of up to (S - 1) C steps across chunk boundaries: the roofline times a launch
        # of the region's length)
        per_launch_steps = L = min(args.steps, (eng.S - 1) * eng.C)
        t_fwd = t_iso = time_kernel(lambda: eng.chunk_only(L))
        flops *= L
        kname = "rollout_chunk_kernel"
        RC = eng.env.rows * eng.env.cols
        # algorithmic HBM bytes per launch: per step and agent-step the stored s'_t 4D, behavior act / Q(a) out 8,
        # max Q' out 4, reward out 4; per step and env done 1 + cur_row 8; per launch and agent-step the hidden
        # states of both nets in / out 16H (register-resident across the launch's steps), the first actions in 4 and
        # the position word in / out 8; per launch and env the grid in / out 2RC, step / apple counters in / out 16,
        # store row in 8 (the weight images, LDS-resident for the launch, and the tile-local action hand-off,
        # <= 2N bytes per agent-step, are not counted)
        alg_bytes = L * (E * N * (4 * D + 16) + E * 9) + E * N * (16 * Hh + 12) + E * (2 * RC + 24)
        kdesc = (f"{kname}<64,64,64,1> ({L} rollout steps per launch, chunk {eng.C}: env step + dual forward, "
                 "chunk-persistent)")
    elif eng.fused:
        t_fwd = t_iso = time_kernel(eng.fused_step_only)
        kname = "rollout_step_kernel"
        RC = eng.env.rows * eng.env.cols
        # algorithmic HBM bytes per launch: per agent-step the stored s'_t 4D, hidden in/out of both nets 16H,
        # action in 4, behavior act / Q(a) out 8, max Q' out 4, reward out 4, position word in / out 8; per env
        # the grid in / out 2RC, step / apple counters in / out 16, done 1, store row in 8, cur_row out 8
        alg_bytes = E * N * (4 * D + 16 * Hh + 28) + E * (2 * RC + 33)
        kdesc = f"{kname}<64,64,64,1> (env step + dual forward: target+behavior, one launch per rollout step)"
    else:
        t_iso = time_kernel(eng.fused_forward)
        # in its rollout context: graphs of K x (env + dual forward) and K x env, the difference per step (the
        # forward then reads the obs the env launch just wrote, as in the timed rollout; back-to-back forwards
        # alone re-read cold obs and take longer, reported as kernel_us_isolated)
        t_fwd = time_kernel(lambda: (eng.env_only(), eng.fused_forward())) - time_kernel(eng.env_only)
        kname = "agent_q_fwd_h3_kernel" if h3 else "agent_q_fwd_lds_kernel"
        # algorithmic HBM bytes per launch: per agent-step obs 4D + hidden in/out 8H + outputs (act/q 8 or max 4)
        alg_bytes = E * N * ((4 * D + 8 * Hh + 8) + (4 * D + 8 * Hh + 4))
        kdesc = f"{kname}<64,64,64,1> (dual: target+behavior)"
    achieved = flops / t_fwd / 1e12
    traffic = None
    prof = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_rollout_chunk.json" if eng.chunked else
                                         "r*_pmc_rollout_step.json" if eng.fused else "r*_pmc_agent_fwd.json")))
    if prof and E == 4096 and N == 8 and Hh == 64:
        pm = json.load(open(prof[-1]))
        if pm.get("kernel", "").startswith(kname):
            traffic = int(pm["traffic_bytes_corrected"])
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "traffic_source": os.path.basename(prof[-1]) if traffic else None,
                "kernel": kdesc,
                "kernel_us": round(t_fwd * 1e6, 2), "kernel_us_isolated": round(t_iso * 1e6, 2),
                "rollout_steps_per_launch": per_launch_steps,
                "kernel_us_per_step": round(t_fwd * 1e6 / per_launch_steps, 2),
                "arith": "fp32 network FLOPs as fp16x3-split MFMA (v_mfma_f32_16x16x32_f16 x3, fp32 accumulate)"
                         if h3 else "exact f32 MFMA (v_mfma_f32_32x32x2_f32)",
                "fp32_native_peak": PEAK_FP32_TFLOPS, "frac_of_fp32_native_peak": round(achieved / PEAK_FP32_TFLOPS, 4),
                "flop_per_launch": flops, "alg_bytes_per_launch": alg_bytes,
                "hbm_frac": round(alg_bytes / t_fwd / (PEAK_HBM_GBS * 1e9), 4)}

    cpu = cpu_l = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(E, N, F1, G, Hh)
        cpu_l = cpu_learner_baseline(N, D, B=args.batch, C=10, H=Hh, Hm=64)

    errors |= int(eng.err.item()) | (eng.per.error_word(clear=False) << 8)   # (the learner's PER updates too)
    if errors:
        raise SystemExit(f"bench.py: device error bits {errors:#x} after the learner / other lines")
    if rank == 0:
        line = {
            "metric": "agent-env-steps/sec (4096 envs x 8 agents per GPU, QMIX GRU-64 rollout step)",
            "value": round(value, 1), "unit": "agent-env-steps/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True,
            "repeats": len(reps), "ms_per_step_min": round(min(reps) / steps * 1e3, 4),
            "ms_per_step_max": round(max(reps) / steps * 1e3, 4),
            "scaling": "weak", "vs_baseline": None,
            "dtype": "f32 (agent forward: fp16x3-split MFMA emulating f32 products, f32 accumulate)",
            "data": "synthetic (restated ma_gym Checkers, 4 bands for 8 agents; random init)",
            "config": {"workload": "QMIX 8-agent gridworld rollout, 4096 envs/GPU, GRU-64 agents, chunk 10, PER",
                       "envs_per_gpu": E, "agents": N, "obs_dim": D, "f1": F1, "gru": Hh, "chunk": 10,
                       "per_capacity_chunks": cap, "per_prefilled_chunks": fill_chunks * E,
                       "step_launches": ("chunk-persistent launches of up to (S - 1) C = "
                                         f"{(eng.S - 1) * eng.C} steps across chunk boundaries (env step + dual forward "
                                         "of each step; S = 4 staging row sets), then per chunk the TD fold" if eng.chunked else
                                         "ONE fused launch (env step + dual forward) per step" if eng.fused else
                                         "env + dual forward per step") + " + PER insert every chunk; one captured "
                                                                            "graph per timed region",
                       "parallelism": f"env-shard x{world}"},
            "rccl_world_size": world,
            "errors": errors,
            "replica_checksums": replicas,
            "learner_updates_per_s": round(upd_per_s, 1),
            "learner": {"algo": "QMIX Train_dqn update", "batch_chunks": args.batch, "chunk": 10,
                        "mixer_hidden": 64, "ms_per_update": round(el_l / args.learner_steps * 1e3, 4),
                        "updates": args.learner_steps, "updates_per_graph_launch": per_replay, "grad_allreduce": (("gloo" if shared else "rccl") if dist else None),
                        "reference_cpu_updates_per_s": 12.0,
                        "reference_cpu_note": "reference Train_dqn.train at its own shapes (GRU-32), 8 threads of "
                                              "the build container (BASELINE.md)",
                        "cpu_baseline": cpu_l, "throughput_batch": big},
            "train_loop": trainer,
            "cfg1_vdn": cfg1,
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
