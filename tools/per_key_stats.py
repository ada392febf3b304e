"""Distribution of the PER leaf keys at the bench's steady state (4096 envs x 8 agents, chunk 10, PER of 65536 chunks
full, epsilon 0.1): for the next insert's threshold T (the 4096-th smallest leaf), how many leaves share T's top b bits
(the candidate-list sizes a b-bit first selection level would leave). Host analysis of the device tree."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mini-marl_amd"))
import torch  # noqa: E402

from minimarl.engine import RolloutEngine  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    eng = RolloutEngine(4096, 8, f1=64, g=64, h=64, chunk=10, capacity=16 * 4096, seed=1234, device=dev)
    eng.set_epsilon(0.1)
    eng._advance(16 * 10 + 20)
    for rep in range(4):
        eng._advance(20)
        torch.cuda.synchronize()
        cap = eng.per.capacity
        leaves = eng.per.tree()[cap - 1:].cpu().numpy()
        keys = leaves.view(np.uint64)
        T = np.sort(keys)[4095]
        out = {"T": float(np.frombuffer(np.uint64(T).tobytes(), np.float64)[0]),
               "exp_range": [int(((keys >> np.uint64(52)) & np.uint64(2047)).min()) - 1023,
                             int(((keys >> np.uint64(52)) & np.uint64(2047)).max()) - 1023],
               "n_eq_T": int((keys == T).sum())}
        for b in (12, 16, 20, 24, 28, 36):
            sh = np.uint64(64 - b)
            out[f"share{b}"] = int(((keys >> sh) == (T >> sh)).sum())
        print(out)


if __name__ == "__main__":
    main()
