"""Microbenchmark of the batched PER insert at the bench shape (cap 65536, 4096 chunks per insert)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl.replay import DevicePER  # noqa: E402

cap, K = int(os.environ.get("MB_CAP", 65536)), int(os.environ.get("MB_K", 4096))
per = DevicePER(cap, "qmix", device="cuda")
g = torch.Generator(device="cuda").manual_seed(0)
tds = [torch.rand(K, device="cuda", generator=g) * 3 for _ in range(8)]
rows = torch.arange(cap, cap + K, device="cuda")
for i in range(cap // K + 2):          # fill the tree, then time steady-state (evicting) inserts
    per.add(tds[i % 8], rows)
torch.cuda.synchronize()
a, b = torch.cuda.Event(True), torch.cuda.Event(True)
n = 50
a.record()
for i in range(n):
    per.add(tds[i % 8], rows)
b.record()
torch.cuda.synchronize()
print(json.dumps({"cap": cap, "K": K, "dbg": os.environ.get("MM_PER_DBG", "0"), "insert_us": a.elapsed_time(b) / n * 1e3}))
