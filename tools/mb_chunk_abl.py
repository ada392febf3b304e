"""Chunk kernel alone (10- and 20-step launches, event-timed) for one library build (MB_LIB): the same-box timing of
ablation / A/B builds (tools/gpu_abl.sh). GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
import minimarl._lib as _L  # noqa: E402

if os.environ.get("MB_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["MB_LIB"])
from minimarl.engine import RolloutEngine  # noqa: E402

eng = RolloutEngine(4096, 8, f1=64, g=64, h=64, chunk=10, capacity=65536, seed=1, device="cuda", persistent=True)
for _ in range(30):
    eng.step(0.1)


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for _ in range(60):   # (clock ramp: the first hundreds of microseconds of launches run slower)
    eng.chunk_only(20)
res = {"lib": os.environ.get("MB_LIB", "lib"), "us10": [], "us20": []}
for _ in range(5):
    res["us10"].append(round(1000 * timed(lambda: eng.chunk_only(10), 20), 2))
    res["us20"].append(round(1000 * timed(lambda: eng.chunk_only(20), 10), 2))
res["us20_min"] = min(res["us20"])
import hashlib  # noqa: E402
hs = hashlib.sha1()
for tsr in (eng.h, eng.ht, eng.act_r, eng.qsel_r, eng.maxq_r, eng.rew_r, eng.store.obs):
    hs.update(tsr.contiguous().cpu().numpy().tobytes())
res["state_sha1"] = hs.hexdigest()[:16]   # (builds with identical arithmetic agree on it)
print(json.dumps(res), flush=True)
