"""Micro-benchmark of the PPO update's reductions (GPU): the split-K weight-gradient sum over 16 chunks and the
bias-gradient column sum, as torch .sum(0) against a ones-vector GEMV (hipBLASLt).  python tools/reduce_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_tracking_amd import rollout as R  # noqa: E402


def bench(f, it=200):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def main():
    dev = torch.device("cuda", 0)
    for shape in [(16, 512, 263), (16, 256, 512), (16, 128, 256), (16, 256, 261)]:
        x = torch.randn(shape, device=dev)
        ones = torch.ones(1, shape[0], device=dev)
        v = x.view(shape[0], -1)
        ref = x.sum(0)
        alt = (ones @ v).view(shape[1:])
        print(f"chunk sum {shape}: sum(0) {bench(lambda: x.sum(0)):.1f} us, ones@ {bench(lambda: ones @ v):.1f} us, "
              f"max rel diff {((alt - ref).abs().max() / ref.abs().max()).item():.1e}")
    for shape in [(24576, 512), (24576, 256), (24576, 128), (24576, 12)]:
        g = torch.randn(shape, device=dev)
        ones = torch.ones(1, shape[0], device=dev)
        print(f"column sum {shape}: sum(0) {bench(lambda: g.sum(0)):.1f} us, ones@ {bench(lambda: ones @ g):.1f} us, "
              f"go1_colsum {bench(lambda: R._colsum(g)):.1f} us")


if __name__ == "__main__":
    main()
