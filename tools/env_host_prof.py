"""Host-side cost of the env-only VecEnv.step loop (bench.py's headline loop), GPU box.

  python tools/env_host_prof.py [steps] [--velocity]   (--velocity: HistoryWrapper(VelocityTrackingEasyEnv))

Prints the loop's wall time per step, the host enqueue time per step (the loop with the
GPU kept busy by a long queue: time until the Python loop returns), and a cProfile of
the loop sorted by own time."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[0]) if args else 512
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 4096
    if "--velocity" in sys.argv:
        from legged_tracking_amd import env as E, velocity as VEL
        env = E.HistoryWrapper(VEL.VelocityTrackingEasyEnv(sim_device=str(dev), num_envs=n, seed=11))
        env.close = env.env.close
    else:
        env = bench.make_env(n, 0, 1, dev)
    env.reset()
    ring = torch.randn((64, n, 12), device=dev)
    for k in range(64):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        env.step(ring[k % 64])
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"loop: {t_all / steps * 1e6:.1f} us/step wall, host returns after {t_host / steps * 1e6:.1f} us/step")
    pr = cProfile.Profile()
    pr.enable()
    for k in range(steps):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    env.close()


if __name__ == "__main__":
    main()
