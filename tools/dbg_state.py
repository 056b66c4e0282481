"""Diagnostic: the bench workload's state after K kernel steps (GO1_LIB_OVERRIDE picks the build): finite
fraction, base heights, the envs whose sphere geometry overlaps (self-contact classes), reset rate."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
import tests.self_geom as TS

dev = torch.device("cuda", 0)
n = 4096
env = bench.make_env(n, 0, 1, dev)
env.reset()
ring = torch.randn((64, n, 12), device=dev)
sim = env.env._sim
base = env.env
grav, gvec = base._sim_gravity, base._gravity_vec
scales = base._scale_vector()
for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 300):
    sim.step(ring[k % 64], gvec, grav, scales, rng_seed=7, rng_step=(1 << 40) + k)
    if k % 100 == 99:
        torch.cuda.synchronize()
        st = sim.state.numpy() if hasattr(sim, "state") else base._state.numpy()
        q = st["dof_pos"].astype(np.float64)
        root = st["root"]
        P, r = TS.spheres(q)
        flags, names = TS.pair_classes(P, r)
        fin = np.isfinite(q).all(1) & np.isfinite(root).all(1)
        cf = base.contact_forces.float().cpu().numpy() if hasattr(base, "contact_forces") else None
        print(f"step {k+1}: finite {fin.mean():.4f} z mean {np.nanmean(root[:,2]):.3f} min {np.nanmin(root[:,2]):.3f} "
              f"self-overlap envs {flags.any(1).mean():.3f} ep_len mean {st['episode_length'][:,0].mean():.1f}")
        fr = flags.mean(0)
        top = np.argsort(-fr)[:8]
        print("   classes:", int((fr > 0).sum()), {str(names[i]): round(float(fr[i]), 4) for i in top if fr[i] > 0})
        vmax = np.nanmax(np.abs(root[:, 7:13]), axis=1)
        print(f"   |v| p50 {np.nanpercentile(vmax,50):.2f} p99 {np.nanpercentile(vmax,99):.2f} max {np.nanmax(vmax):.2f}",
              f" |qd| max {np.nanmax(np.abs(st['dof_vel'])):.1f}")
