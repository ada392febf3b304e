"""GPU: the PyTorch custom ops (torch.ops.minimarl.*, torch.classes.minimarl.*; csrc/torch_ops.cpp)
against the oracle and the golden vectors, their argument checks and HIP-graph capture."""
import numpy as np
import pytest
import torch

from oracle import nets
from oracle.env import EnvSpec, VecEnvOracle
from oracle.sumtree import SumTreeOracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from minimarl.ops import load
    return load()


def _net(N=8, D=47, A=5, f1=64, g=64, h=64, seed=3):
    from minimarl.qnet import AgentQNet
    net = AgentQNet(N, D, A, f1, g, h, DEV, seed=seed)
    return net, {k: v.detach().cpu().clone() for k, v in net.params().items()}


@pytest.mark.parametrize("E", [96, 2304])
def test_agent_q_ops_vs_oracle(ops, E):
    from minimarl.ops import dims
    net, P = _net()
    packed = torch.empty_like(net.packed)
    ops.qnet_pack(net.flat, dims(net), packed)
    g = torch.Generator().manual_seed(2)
    obs, hid = torch.rand(E, 8, 47, generator=g), torch.randn(E, 8, 64, generator=g) * 0.5
    o, h = obs.to(DEV), hid.to(DEV)
    q, h2 = torch.empty(E, 8, 5, device=DEV), torch.empty(E, 8, 64, device=DEV)
    ops.agent_q_fwd(packed, dims(net), o, h, h2, q)
    qo, ho = nets.agent_forward(P, obs, hid)
    np.testing.assert_allclose(q.cpu().numpy(), qo.numpy(), rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(h2.cpu().numpy(), ho.numpy(), rtol=1e-5, atol=2e-5)
    mq = torch.empty(E, 8, device=DEV)
    ops.agent_q_max(packed, dims(net), o, h, h2, mq)
    np.testing.assert_allclose(mq.cpu().numpy(), qo.max(2)[0].numpy(), rtol=1e-5, atol=2e-5)
    # injected draws: the reference's epsilon_greedy (vdn/_network.py:52-58) exactly
    u = torch.rand(E, generator=g)
    ra = torch.randint(0, 5, (E, 8), generator=g, dtype=torch.int32)
    act, qt = torch.empty(E, 8, dtype=torch.int32, device=DEV), torch.empty(E, 8, device=DEV)
    q2 = torch.empty_like(q)
    ops.agent_q_act(packed, dims(net), o, h, 0.3, u.to(DEV), ra.to(DEV), 0, 0, h2, act, qt, q2)
    ref = nets.epsilon_greedy(qo, 0.3, u, ra).long()
    a = act.cpu().long()
    greedy = (u > 0.3)
    np.testing.assert_array_equal(a[~greedy].numpy(), ref[~greedy].numpy())
    gap = qo.max(2)[0] - qo.gather(2, a.unsqueeze(-1)).squeeze(-1)
    assert float(gap[greedy].max()) <= 2e-5
    np.testing.assert_allclose(q2.cpu().numpy(), qo.numpy(), rtol=1e-5, atol=2e-5)


def test_td_error_op(ops):
    E, N = 300, 8
    g = torch.Generator().manual_seed(4)
    rew, qt, mq = (torch.randn(E, N, generator=g) for _ in range(3))
    done = (torch.rand(E, generator=g) < 0.2).to(torch.uint8)
    td = torch.empty(E, device=DEV)
    ops.td_error(rew.to(DEV), done.to(DEV), qt.to(DEV), mq.to(DEV), 0.99, td)
    ref = (rew.sum(1) + (1 - done.float()) * 0.99 * mq.sum(1) - qt.sum(1)).abs()     # vdn/_utils.py:44-52
    np.testing.assert_allclose(td.cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-5)


def test_gae_scan_op_golden(ops, golden):
    fx = golden("mappo_gae")
    T, E, N = fx["rewards"].shape[:3]
    vp = fx["value_preds"].copy()
    vp[-1] = fx["next_value"]
    vn = torch.tensor([float(fx["vn_mean"][0]), float(fx["vn_mean_sq"][0]), float(fx["vn_debias"])], device=DEV)
    ret = torch.zeros(T + 1, E * N, device=DEV)
    ops.gae_scan(torch.from_numpy(fx["rewards"].reshape(T, E * N)).to(DEV), torch.from_numpy(vp.reshape(T + 1, -1)).to(DEV),
                 torch.from_numpy(fx["masks"].reshape(T + 1, -1)).to(DEV), vn, float(fx["gamma"]),
                 float(fx["gae_lambda"]), ret)
    np.testing.assert_allclose(ret[:T].cpu().numpy(), fx["returns"][:T].reshape(T, E * N), rtol=1e-6, atol=1e-6)


def test_env_class_bit_exact(ops):
    from minimarl.ops import Env
    E, N = 200, 8
    env = Env(E, N, 100, -0.01, False, DEV)
    D = env.obs_dim()
    ora = VecEnvOracle(EnvSpec(N, 100), E)
    obs = torch.empty(E, N, D, device=DEV)
    env.reset(obs)
    np.testing.assert_array_equal(obs.cpu().numpy(), ora.observe())
    nxt, cur = torch.empty_like(obs), torch.empty_like(obs)
    rew, done = torch.empty(E, N, device=DEV), torch.empty(E, dtype=torch.uint8, device=DEV)
    rng = np.random.default_rng(0)
    for _ in range(130):
        a = rng.integers(0, 5, (E, N)).astype(np.int32)
        env.step(torch.from_numpy(a).to(DEV), nxt, cur, rew, done)
        on, orew, od = ora.step(a)
        np.testing.assert_array_equal(nxt.cpu().numpy(), on)
        np.testing.assert_array_equal(rew.cpu().numpy(), orew)
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), od)
        ora.reset_envs(od)
        np.testing.assert_array_equal(cur.cpu().numpy(), ora.observe())


def test_per_class_vs_oracle(ops):
    from minimarl.ops import PER
    cap = 4096
    per = PER(cap, "vdn", 0.4, 0.4, 1e-6, 0.99, True, 0.0, 0.0, DEV)
    ora = SumTreeOracle(cap, "vdn", 0.4, 0.4)
    rng = np.random.default_rng(3)
    for _ in range(5):
        td = (rng.random(1500) * 2).astype(np.float32)
        slots = torch.empty(1500, dtype=torch.int64, device=DEV)
        per.insert(torch.from_numpy(td).to(DEV), slots)
        np.testing.assert_array_equal(slots.cpu().numpy(), ora.add_batch([float(x) for x in td]))
        fr = rng.random(64)
        nodes, s2, w = (torch.empty(64, dtype=torch.int64, device=DEV), torch.empty(64, dtype=torch.int64, device=DEV),
                        torch.empty(64, device=DEV))
        per.sample(torch.from_numpy(fr).to(DEV), 0, 0, nodes, s2, w)
        on, _, _, ow = ora.sample(64, fr)
        np.testing.assert_array_equal(nodes.cpu().numpy(), on)
        np.testing.assert_allclose(w.cpu().numpy(), ow, rtol=1e-5)
        np.testing.assert_allclose(per.tree().cpu().numpy(), ora.tree, rtol=1e-6, atol=1e-9)
    assert per.size() == cap and per.capacity() == cap


def test_ops_argument_errors(ops):
    from minimarl.ops import dims
    net, _ = _net(N=2, D=47, A=5, g=32, h=32)
    o = torch.rand(4, 2, 47, device=DEV)
    h = torch.zeros(4, 2, 32, device=DEV)
    with pytest.raises(RuntimeError, match="obs shape"):
        ops.agent_q_fwd(net.packed, dims(net), torch.rand(4, 3, 47, device=DEV), h, h.clone(),
                        torch.empty(4, 3, 5, device=DEV))
    with pytest.raises(RuntimeError, match="must be float"):
        ops.agent_q_fwd(net.packed, dims(net), o, h.double(), h, torch.empty(4, 2, 5, device=DEV))
    with pytest.raises(RuntimeError, match="'CPU' backend"):   # no CPU kernel is registered: no fallback
        ops.td_error(torch.zeros(4, 2), torch.zeros(4, dtype=torch.uint8), torch.zeros(4, 2), torch.zeros(4, 2), 0.99,
                     torch.zeros(4))


def test_ops_capture_in_hip_graph(ops):
    """The ops enqueue on torch's current stream: a captured forward replays like an eager one."""
    from minimarl.ops import dims
    net, _ = _net()
    packed = net.packed
    net.pack()
    E = 512
    o = torch.rand(E, 8, 47, device=DEV)
    h = torch.randn(E, 8, 64, device=DEV)
    q1, h1 = torch.empty(E, 8, 5, device=DEV), torch.empty(E, 8, 64, device=DEV)
    ops.agent_q_fwd(packed, dims(net), o, h, h1, q1)
    q2, h2 = torch.zeros_like(q1), torch.zeros_like(h1)
    gph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(gph):
            ops.agent_q_fwd(packed, dims(net), o, h, h2, q2)
    torch.cuda.current_stream().wait_stream(s)
    gph.replay()
    torch.cuda.synchronize()
    assert torch.equal(q1, q2) and torch.equal(h1, h2)
