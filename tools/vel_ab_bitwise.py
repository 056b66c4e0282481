"""Bitwise A/B of two velocity-library builds in Philox mode (the bench's draws, which the fixture tests do not
cover): python tools/vel_ab_bitwise.py OUT.npz [steps] with GO1_VEL_LIB_OVERRIDE naming the build; then
python tools/vel_ab_bitwise.py --compare A.npz B.npz."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out, steps):
    import torch
    from legged_tracking_amd import env as E, velocity as VEL
    n = 4096
    dev = torch.device("cuda", 0)
    env = E.HistoryWrapper(VEL.VelocityTrackingEasyEnv(sim_device=str(dev), num_envs=n, seed=11))
    env.reset()
    gen = torch.Generator(device=dev).manual_seed(5)
    rec = {}
    for t in range(steps):
        o, r, d, _ = env.step(torch.randn((n, 12), device=dev, generator=gen))
        if t % 10 == 9 or t == steps - 1:
            rec[f"obs{t}"] = o["obs"].cpu().numpy()
            rec[f"rew{t}"] = r.cpu().numpy()
            rec[f"done{t}"] = d.cpu().numpy()
    st = env.env._sim.state
    for k, v in st.items():
        rec["state_" + k] = v.cpu().numpy()
    np.savez(out, **rec)
    env.env.close()


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
        print("bitwise equal" if not bad else f"DIFFER: {bad[:10]}")
        cat_changes = sum(int((a[k] != 0).sum()) for k in a.files if k.startswith("state_command_bins"))
        print("keys", len(a.files), "nonzero command bins", cat_changes)
        sys.exit(1 if bad else 0)
    run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 300)
