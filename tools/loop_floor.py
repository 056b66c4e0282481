"""Per-step wall time of the fused step at 4096 envs, from the leanest host loop to the bench's
VecEnv.step loop (GPU box):

  raw       ctypes go1_step on one prepared argument block, nothing else (the GPU-bound floor:
            kernel + launch gap)
  raw+ev    the same with a HIP event pair around every 4th kernel (bench.py's timing method)
  vecenv    HistoryWrapper(TrajectoryTrackingEnv).step, the bench headline loop

  python tools/loop_floor.py [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 4096
    env = bench.make_env(n, 0, 1, dev)
    env.reset()
    base = env.env
    sim = base._sim
    ring = torch.randn((64, n, 12), device=dev)
    out = dict(obs=sim.obs, priv=sim.priv, rew=sim.rew, reset=sim.reset, time_out=sim.time_out)
    args = sim.prepare(out)
    ck, gvec, sgrav, scales = base._step_consts()
    ev = bench.EventPairs(steps // 4 + 1)

    def raw(k0, events):
        for k in range(steps):
            e = ev.pair(k // 4) if events and k % 4 == 0 else None
            sim.step_prepared(args, ring[k % 64], gvec, sgrav, scales, ck, 7, k0 + k, events=e)

    for name, fn in (("raw", lambda: raw(1 << 40, False)), ("raw+ev", lambda: raw(2 << 40, True)),
                     ("vecenv", lambda: [env.step(ring[k % 64]) for k in range(steps)])):
        fn()  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        print(f"{name:7s} {t / steps * 1e6:6.1f} us/step wall  (host enqueue {th / steps * 1e6:5.1f} us/step)")
    kt = [ev.ms(i) for i in range(steps // 4)]
    print(f"event-bracketed kernel (raw+ev): {sum(kt) / len(kt) * 1e3:.1f} us")
    env.close()


if __name__ == "__main__":
    main()
