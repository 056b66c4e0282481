"""Per-workgroup phase times of the engine's xw GEMM (diagnostic build with -DPPO_STAMPS):
python tools/xw_stamps.py lib_with_stamps.so

Stamps are s_memrealtime (100 MHz) at kernel start, after the first staged group, after the K loop and after
the epilogue; printed per shape: the launch span, the start-time spread (dispatch rounds) and the median /
p90 of each phase per workgroup."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_tracking_amd import ppo_engine as PE  # noqa: E402

SHAPES = [("acL1 k264 n512", 24576, 264, 512), ("acL2 k512 n256", 24576, 512, 256), ("acL3 k256 n128", 24576, 256, 128)]


def main():
    lib = PE.load_library(sys.argv[1])
    lib.go1_ppo_xw_stamps.argtypes = [C.c_void_p]
    g = torch.Generator(device="cuda").manual_seed(0)
    work = torch.zeros(512 << 20, dtype=torch.uint8, device="cuda")
    base = (work.data_ptr() + 255) // 256 * 256
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    buf = np.zeros((8192, 4), dtype=np.uint64)
    for name, rows, k, n in SHAPES:
        x = torch.randn(rows, k, device="cuda", generator=g)
        w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
        b = torch.zeros(n, device="cuda")
        y = torch.empty(rows, n, device="cuda")
        for _ in range(3):  # warm: the last launch's stamps are read
            lib.go1_ppo_test_linear(x.data_ptr(), rows, k, w.data_ptr(), b.data_ptr(), n, 1, y.data_ptr(), base,
                                    work.numel() - 256, 1, s)
        torch.cuda.synchronize()
        assert lib.go1_ppo_xw_stamps(buf.ctypes.data) == 0
        nb = (rows + 127) // 128 * (n // 128)
        st = buf[:nb].astype(np.int64)
        t0 = st[:, 0].min()
        rel = (st - t0) * 10e-3  # us
        span = rel[:, 3].max()
        ph = np.diff(rel, axis=1)
        print(f"{name}: {nb} workgroups, span {span:.1f} us; start spread p50 {np.median(rel[:, 0]):.1f} "
              f"p90 {np.percentile(rel[:, 0], 90):.1f} max {rel[:, 0].max():.1f} us")
        ev = sorted([(a, 1) for a in rel[:, 0]] + [(b, -1) for b in rel[:, 3]])
        cur = peak = 0
        for _, d in ev:
            cur += d
            peak = max(peak, cur)
        print(f"    peak concurrent workgroups {peak}")
        for i, nm in enumerate(("prologue", "k-loop", "epilogue")):
            print(f"    {nm:9s} p10 {np.percentile(ph[:, i], 10):6.2f}  p50 {np.median(ph[:, i]):6.2f}  "
                  f"p90 {np.percentile(ph[:, i], 90):6.2f}  max {ph[:, i].max():6.2f} us")


if __name__ == "__main__":
    main()
