"""GPU step vs the f64 and f32 oracles on the trunk-face / self-collision scenarios of tests/test_gpu_self_collision.py:
per step, the envs over the integrator bound, and for the worst one the per-body contact forces of all three (GPU box).
  python tools/dbg_capsule.py [faces|selfc]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from legged_tracking_amd import config as CF, layout as L, native  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_parity import DEV, INTEGRATOR_MAX_ERR, _dev, _sim_setup  # noqa: E402


def faces():
    n = 256
    cfg, c, td, ter, st, rng = _sim_setup(n, "single_path")
    hs = float(c.horizontal_scale)
    tiles = td.tiles.copy()
    tiles[:, 1] = 0.0
    tiles[:, 0] = 0.5
    i0, j0 = 40, 20
    for di, dj in ((0, 0), (3, 0), (-3, 1)):
        tiles[:, 0, i0 + di, j0 + dj] = 0.395
    tiles[:, 1, i0 - 1:i0 + 2, j0] = 0.255
    td.tiles[:] = tiles
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    root = st["root"]
    root[:, 0] = td.env_terrain_origin[:, 0] + i0 * hs + rng.uniform(-0.02, 0.02, n)
    root[:, 1] = td.env_terrain_origin[:, 1] + j0 * hs + rng.uniform(-0.02, 0.02, n)
    root[:, 2] = rng.uniform(0.30, 0.35, n)
    yaw, pitch, roll = rng.uniform(-0.5, 0.5, n), rng.uniform(-0.1, 0.1, n), rng.uniform(-0.1, 0.1, n)
    cy, sy, cp, sp, cr, sr = (np.cos(yaw / 2), np.sin(yaw / 2), np.cos(pitch / 2), np.sin(pitch / 2),
                              np.cos(roll / 2), np.sin(roll / 2))
    root[:, 3] = sr * cp * cy - cr * sp * sy
    root[:, 4] = cr * sp * cy + sr * cp * sy
    root[:, 5] = cr * cp * sy - sr * sp * cy
    root[:, 6] = cr * cp * cy + sr * sp * sy
    root[:, 7:13] = rng.normal(0, 0.1, (n, 6))
    st["episode_length"][:, 0] = 10
    grav, gvec = CF.gravity_state([0.0, 0.0, 0.0])
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    acts = [rng.normal(0, 0.3, (n, 12)).astype(np.float32) for _ in range(3)]
    return c, td, ter, st, acts, gvec, grav, scales, 4, 400


def main():
    c, td, ter, st, acts, gvec, grav, scales, seed, step0 = faces()
    n = c.n_envs
    g = native.Go1Native(c, DEV)
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    for t, a in enumerate(acts):
        g.state.load(st.arrays)
        g.step(_dev(a), gvec, grav, scales, rng_seed=seed, rng_step=step0 + t)
        torch.cuda.synchronize()
        gs = g.state.numpy()
        cfg_ = g.contact_forces.cpu().numpy()
        s64, s32 = st.copy(), st.copy()
        o64 = O.step(c, s64, ter, a, gvec, grav, scales, rng_seed=seed, rng_step=step0 + t, debug=False)
        o32 = O.step(c, s32, ter, a, gvec, grav, scales, rng_seed=seed, rng_step=step0 + t, debug=False,
                     precision="f32")
        for name, s in (("gpu", gs), ("f32", s32)):
            err = np.zeros(n)
            for k, tol in INTEGRATOR_MAX_ERR.items():
                e = (np.abs(s[k] - s64[k]) / np.maximum(1.0, np.abs(s64[k]))).max(axis=1) / tol
                err = np.maximum(err, e)
            bad = np.nonzero(err > 1)[0]
            print(f"step {t} {name}: envs over the bound {list(bad)}")
            if name == "gpu":
                for e in bad[:3]:
                    print(f" env {e}: dof_pos err {np.abs(gs['dof_pos'][e] - s64['dof_pos'][e]).round(6)}")
                    print(f"  root gpu {gs['root'][e].round(4)}\n  root f64 {s64['root'][e].round(4)}")
                    for b in range(17):
                        x, y, z = cfg_[e, b], o64["contact_forces"][e, b], o32["contact_forces"][e, b]
                        if np.abs(x).max() + np.abs(y).max() > 0:
                            print(f"  body {b:2d} gpu {x.round(3)} f64 {y.round(3)} f32 {z.round(3)}")
        st = O.NpState(n, gs, c)


if __name__ == "__main__":
    main()
