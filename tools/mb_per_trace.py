"""Phase timeline of the multi-block PER insert inside the bench's rollout region (4096 envs x 8 agents, chunk 10, PER
full, eager 20-step regions) from a trace build (make variant VAR=ptr VFLAGS=-DMM_PER_TRACE=1; MB_LIB=that library):
per launch the workgroups' start / phase / end stamps (s_memrealtime, 10 ns), the gaps between the launches, and the
candidate-list sizes of the threshold select.

usage: MB_LIB=mini-marl_amd/lib_ptr/libminimarl.so python3 tools/mb_per_trace.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mini-marl_amd"))
import minimarl._lib as _L  # noqa: E402

if os.environ.get("MB_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["MB_LIB"])
import torch  # noqa: E402

from minimarl.engine import RolloutEngine  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    eng = RolloutEngine(4096, 8, f1=64, g=64, h=64, chunk=10, capacity=16 * 4096, seed=1234, device=dev)
    eng.set_epsilon(0.1)
    eng._advance(16 * 10 + 20)
    torch.cuda.synchronize()
    L = _L.lib()
    L.mm_per_trace_copy.argtypes = [ctypes.c_void_p]
    buf = np.zeros((4, 64, 16), dtype=np.uint64)
    tick = 10e-3   # us per s_memrealtime tick
    for rep in range(6):
        eng._advance(20)
        torch.cuda.synchronize()
        assert L.mm_per_trace_copy(buf.ctypes.data) == 0
        b = buf.astype(np.int64)
        t0 = b[0, :, 0].min()
        sel1_end = b[0, :, 1].max()
        s2 = b[1, :, :3]
        ap = b[3]
        last = int(np.argmax(ap[:, 7]))
        line = {
            "m_listed": int(buf[0, 0, 6]), "n_36bit": int(buf[0, 0, 7]),
            "sel1_us": (sel1_end - t0) * tick,
            "gap12": (s2[:, 0].min() - sel1_end) * tick,
            "sel2_pick": np.median(s2[:, 1] - s2[:, 0]) * tick, "sel2_rest": np.median(s2[:, 2] - s2[:, 1]) * tick,
            "sel2_us": (s2[:, 2].max() - s2[:, 0].min()) * tick,
            "gap2a": (ap[:, 0].min() - s2[:, 2].max()) * tick,
        }
        names = ["pick", "scan", "radix", "offs", "write", "subtree"]
        for i, nm in enumerate(names):
            line["ap_" + nm] = np.median(ap[:, i + 1] - ap[:, i]) * tick
            line["ap_" + nm + "_max"] = np.max(ap[:, i + 1] - ap[:, i]) * tick
        for nm, (i0, i1) in {"w_scans": (4, 8), "w_jload": (8, 9), "w_powst": (9, 10), "w_sync": (10, 5)}.items():
            line[nm] = np.median(ap[:, i1] - ap[:, i0]) * tick
            line[nm + "_max"] = np.max(ap[:, i1] - ap[:, i0]) * tick
        line["ap_spread_start"] = (ap[:, 0].max() - ap[:, 0].min()) * tick
        line["ap_top_last"] = (ap[last, 7] - ap[last, 6]) * tick
        line["ap_ticket_wait"] = (ap[last, 6] - ap[:, 6].min()) * tick
        line["apply_us"] = (ap[:, 7].max() - ap[:, 0].min()) * tick
        line["total_us"] = (ap[:, 7].max() - t0) * tick
        print({k: (round(float(v), 2) if isinstance(v, (float, np.floating)) else v) for k, v in line.items()})
        if os.environ.get("MB_BLOCKS"):
            tot = (ap[:, 6] - ap[:, 0]) * tick
            o = np.argsort(tot)
            print("  apply blocks 0->6 us (sorted):", [(int(i), round(float(tot[i]), 2)) for i in o[::8]], "max",
                  (int(o[-1]), round(float(tot[o[-1]]), 2)))
            for nm, (i0, i1) in {"pick": (0, 1), "scan": (1, 2), "offs": (3, 4), "scans": (4, 8), "jload": (8, 9),
                                 "powst": (9, 10), "sync": (10, 5), "sub": (5, 6)}.items():
                d = (ap[:, i1] - ap[:, i0]) * tick
                print("   ", nm, "slowest block", round(float(d[o[-1]]), 2), "median", round(float(np.median(d)), 2))


if __name__ == "__main__":
    main()
