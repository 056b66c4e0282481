"""Debug: one full-size step, HIP vs f64 oracle -- which envs / bodies change their contact set."""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_full_size import _setup, _handle, N  # noqa: E402
from legged_tracking_amd import config as CF  # noqa: E402
from oracle import oracle as O  # noqa: E402

terrain = sys.argv[1] if len(sys.argv) > 1 else "single_path"
cfg, td, dr, ep, rng = _setup(seed=9, terrain=terrain)
dec1 = len(sys.argv) > 2
if dec1:  # one sim step only
    from legged_tracking_amd import native
    c = CF.build_abi_config(cfg, n_envs=N)
    c.decimation = 1
    g = native.Go1Native(c, "cuda:0")
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    for k, v in dr.items():
        g.state[k].copy_(torch.from_numpy(v.astype(np.float32)))
    keep = g.reset_envs(torch.ones(N, dtype=torch.bool, device="cuda:0"), rng_seed=11, rng_step=0)
    g.state["episode_length"].copy_(torch.from_numpy(ep))
else:
    c, g, keep = _handle(cfg, td, dr, ep, 0, N)
torch.cuda.synchronize()
st = O.NpState(N, g.state.numpy(), c)
st0 = O.NpState(N, g.state.numpy(), c)
ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
grav, gvec = CF.gravity_state([0.2, -0.1, 0.3])
act = rng.normal(0, 1, (N, 12)).astype(np.float32)
g.step(torch.from_numpy(act).to("cuda:0"), gvec, grav, scales, rng_seed=3, rng_step=1)
torch.cuda.synchronize()
out = O.step(c, st, ter, act, gvec, grav, scales, rng_seed=3, rng_step=1, debug=False)
gs = g.state.numpy()
cg, co = g.contact_forces.cpu().numpy(), out["contact_forces"]
ng, no = np.linalg.norm(cg, axis=2), np.linalg.norm(co, axis=2)
flipb = (ng > 0) != (no > 0)
flip = flipb.any(axis=1)
print("flipped envs", flip.sum(), "bodies flipped per index", flipb.sum(axis=0))
mag = np.where(flipb, np.maximum(ng, no), 0).max(axis=1)
print("force on the active side of flips: pct 50/90/max", np.percentile(mag[flip], [50, 90, 100]) if flip.any() else None)
for k in ("dof_pos", "dof_vel", "root"):
    err = (np.abs(gs[k] - st[k]) / np.maximum(1.0, np.abs(st[k]))).max(axis=1)
    print(k, "err non-flip max", err[~flip].max(), "p99", np.percentile(err[~flip], 99), "flip median",
          np.median(err[flip]) if flip.any() else None)
both = (ng > 0) & (no > 0)
rel = np.abs(ng - no)[both] / np.maximum(no[both], 1.0)
print("force rel err where both active: p50/p99/max", np.percentile(rel, [50, 99, 100]))
print("reset diff", (g.reset.cpu().numpy().astype(bool) != out["reset"].astype(bool)).sum())
print("base z before", np.percentile(st0["root"][:, 2], [0, 50, 100]))
e = int(np.argmax(mag))
print("worst env", e, "bodies", np.nonzero(flipb[e])[0], "\n hip", ng[e], "\n orc", no[e])

err = (np.abs(gs["dof_vel"] - st["dof_vel"])).max(axis=1)
ncon = (no > 0).sum(axis=1)
for lo, hi in ((0, 1e-3), (1e-3, 1e-2), (1e-2, 1e9)):
    m = (err >= lo) & (err < hi)
    if m.any():
        print(f"dof_vel err [{lo},{hi}): {m.sum()} envs; mean payload {st0['payload'][m, 0].mean():.2f} friction "
              f"{st0['friction'][m, 0].mean():.2f} n_contacts {ncon[m].mean():.2f} motor_strength "
              f"{np.abs(st0['motor_strength'][m]).mean():.3f}")
e = int(np.argmax(err))
print("worst dof_vel env", e, err[e], "payload", st0["payload"][e], "friction", st0["friction"][e])
print(" hip cf", ng[e]); print(" orc cf", no[e])
print(" hip qd", gs["dof_vel"][e]); print(" orc qd", st["dof_vel"][e])
