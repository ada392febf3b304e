"""Extract the per-episode train scores of the reference's logged VDN run (Checkers-v0, 2 agents, full obs,
max_step 100, step_cost -0.01) into tests/golden/vdn_log_scores.npy: data only (the scores printed by
vdn/main.py:182 into vdn/logs/vdn-1710766189.log), used as an end-to-end anchor of the restated env
(tests/test_env_checkers.py). Run in the build container: python tests/golden/make_golden_vdn_log.py"""
import os
import re

import numpy as np

LOG = "/root/reference/vdn/logs/vdn-1710766189.log"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vdn_log_scores.npy")

scores = []
with open(LOG) as f:
    for line in f:
        m = re.search(r"(\d+)\s*/15000\s+episodes \| train score: (-?[\d.]+)", line)
        if m:
            assert int(m.group(1)) == len(scores) + 1
            scores.append(float(m.group(2)))
np.save(OUT, np.array(scores, np.float64))
print(len(scores), "scores ->", OUT)
