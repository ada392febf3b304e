"""Debug: two-launch vs chunk engines step by step: next actions / Q(a) right after each step, counters."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402

kw = dict(f1=64, g=64, h=64, chunk=10, capacity=4 * 2048, seed=21, device="cuda")
ref = RolloutEngine(2048, 8, fused=False, **kw)
ch = RolloutEngine(2048, 8, persistent=True, **kw)
for t in range(10):
    ref.step(0.3)
    ch.step(0.3)
    torch.cuda.synchronize()
    k = (t + 1) % 2
    na_ref, nq_ref = ref.act_buf[k], ref.qsel_buf[k]
    i1 = ch._act_idx(t + 1)
    na, nq = ch.act_r[i1], ch.qsel_r[i1]
    dq = (nq - nq_ref).abs().max().item()
    print(f"t={t} next-act diff {(na != na_ref).sum().item()} next-qsel maxdiff {dq:.3g} "
          f"h eq {torch.equal(ref.h, ch.h)} ctr ref {ref.counter_dev.tolist()} ch {ch.counter_dev.tolist()} "
          f"ctl {ch.ctl.tolist()} eps {ch.eps_dev.item()} err {ch.err.item()}", flush=True)
    for j in range(10):
        a = ch.act_r[j]
        print("   ring", j, "sum", int(a.sum().item()), "nz", int((a != 0).sum().item()))
    if t >= 8:
        break
