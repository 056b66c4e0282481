"""Host-side (Python) cost of the rollout loop: cProfile of 200 rollout steps (GPU box)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
pr = cProfile.Profile()
r = bench.rollout_rate(4096, dev, steps=200, warmup=24, prof=pr)
print(r)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
