"""A/B cost of the native contact model's options on the step kernel (bench.py's workload: 4096 envs, single_path,
README config, N(0, 1) actions): python tools/physics_ab.py [steps]

Arms: self-collision on (asset.self_collisions = 0, the reference scene) / off (= 1); restitution drawn in
[0, 1] per env / 0.  Kernel time per step from the HIP events of bench.kernel_loop, arms alternated twice."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from legged_tracking_amd import config as CF, env as E  # noqa: E402


def make(self_on, rest_on, n=4096):
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=32, cols=32)
    cfg.asset.self_collisions = 0 if self_on else 1
    env = E.HistoryWrapper(E.TrajectoryTrackingEnv(sim_device="cuda:0", cfg=cfg, seed=11))
    st = env.env._sim.state
    if rest_on:
        st["restitution"].copy_(torch.rand(n, 1, device="cuda:0"))
    else:
        st["restitution"].zero_()
    return env


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    g = torch.Generator(device="cuda:0").manual_seed(0)
    ring = [torch.randn(4096, 12, device="cuda:0", generator=g) for _ in range(8)]
    arms = [("self+rest", True, True), ("self only", True, False), ("rest only", False, True), ("neither", False, False)]
    res = {a[0]: [] for a in arms}
    for rep in range(2):
        for name, s, r in arms:
            env = make(s, r)
            out = bench.kernel_loop(env, ring, steps, 50)
            res[name].append(out[1])
            del env
            torch.cuda.synchronize()
    for name, v in res.items():
        print(f"{name:10s} kernel {np.mean(v) * 1e3:7.2f} us  ({', '.join(f'{x * 1e3:.2f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
