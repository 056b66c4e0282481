"""Time the PPO engine's two GEMM kernels (csrc/ppo_update.hip xw_kernel, wgrad_kernel) at the update's shapes,
for one or more builds of the library: python tools/ppo_gemm_bench.py [lib.so ...]

Per shape: (time of 1 + R launches - time of 1 launch) / R with HIP events, and the f16-MFMA rate of the 3xF16
products (3 MFMAs per product) against the 2.5 PFLOP/s dense peak."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_tracking_amd import ppo_engine as PE  # noqa: E402

R = 20
LIN = [("acL1 k264 n512", 24576, 264, 512), ("acL2 k512 n256", 24576, 512, 256), ("acL3 k256 n128", 24576, 256, 128),
       ("dL2 k256 n512", 24576, 256, 512), ("dL3 k128 n256", 24576, 128, 256)]
WG = [("wL1 k264 n512", 24576, 264, 512), ("wL2 k512 n256", 24576, 512, 256), ("wL3 k256 n128", 24576, 256, 128)]


def timed(fn):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(1)
    torch.cuda.synchronize()
    out = []
    for reps in (1, R + 1):
        e0.record(st)
        fn(reps)
        e1.record(st)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return (out[1] - out[0]) / R * 1e3  # us


def main():
    libs = sys.argv[1:] or [PE.LIB_PATH]
    g = torch.Generator(device="cuda").manual_seed(0)
    work = torch.zeros(512 << 20, dtype=torch.uint8, device="cuda")
    base = (work.data_ptr() + 255) // 256 * 256
    nb = work.numel() - 256
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for path in libs:
        lib = PE.load_library(path)
        print(f"== {os.path.basename(path)}")
        for name, rows, k, n in LIN:
            x = torch.randn(rows, k, device="cuda", generator=g)
            w = torch.randn(n, k, device="cuda", generator=g) / k ** 0.5
            b = torch.zeros(n, device="cuda")
            y = torch.empty(rows, n, device="cuda")
            us = timed(lambda r: lib.go1_ppo_test_linear(x.data_ptr(), rows, k, w.data_ptr(), b.data_ptr(), n, 1,
                                                         y.data_ptr(), base, nb, r, s))
            tf = 2.0 * rows * k * n * 3 / us / 1e6
            print(f"  xw    {name:18s} {us:8.1f} us  {tf:7.1f} TF f16 ({tf / 2500:.2f} of peak)  {tf / 3:6.1f} TF f32-equiv")
        for name, rows, k, n in WG:
            x = torch.randn(rows, k, device="cuda", generator=g)
            d = torch.randn(rows, n, device="cuda", generator=g) * 1e-5
            dw = torch.empty(n, k, device="cuda")
            us = timed(lambda r: lib.go1_ppo_test_wgrad(x.data_ptr(), d.data_ptr(), rows, k, n, dw.data_ptr(), base,
                                                        nb, r, s))
            tf = 2.0 * rows * k * n * 3 / us / 1e6
            print(f"  wgrad {name:18s} {us:8.1f} us  {tf:7.1f} TF f16 ({tf / 2500:.2f} of peak)  {tf / 3:6.1f} TF f32-equiv")


if __name__ == "__main__":
    main()
