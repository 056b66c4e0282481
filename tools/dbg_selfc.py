"""Diagnostic: GPU vs oracle self-contact forces of colliding states (tests/test_gpu_self_collision.py), with and
without velocities, error per body."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tests.self_geom as TS
from legged_tracking_amd import config as CF, layout as L, native, terrain as T
from oracle import oracle as O
from tests.test_gpu_parity import DEV, _dev

n = 512
cfg = CF.readme_config(n_envs=n, terrain="plane", rows=2, cols=4)
cfg.control.decimation = 1
c = CF.build_abi_config(cfg)
c.camera_zero = 0
td = T.build(cfg, n, np.random.RandomState(11))
ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
rng = np.random.default_rng(21)
lim = np.array([L.JOINT_LIMITS[j % 3] for j in range(12)])
pool = rng.uniform(lim[:, 0], lim[:, 1], (60000, 12))
inward = rng.random(60000) < 0.5
sgn = np.array([-1.0, 1.0, -1.0, 1.0])
for l in range(4):
    pool[inward, 3 * l] = sgn[l] * rng.uniform(0.2, 0.8, inward.sum())
P, r = TS.spheres(pool)
flags, names = TS.pair_classes(P, r)
idx = np.nonzero(flags.any(1))[0][:n]
q = pool[idx].astype(np.float32)
for vel in (0.0, 1.0):
    st = O.NpState(n, cfg=c)
    O.reset_envs(c, st, ter, np.ones(n, np.uint8), rng_seed=3, rng_step=0)
    st["dof_pos"][:] = q
    st["dof_vel"][:] = (vel * rng.normal(0, 1.0, (n, 12))).astype(np.float32)
    st["root"][:, 2] += 1.0
    st["root"][:, 7:13] = (vel * rng.normal(0, 0.2, (n, 6))).astype(np.float32)
    st["episode_length"][:, 0] = 10
    g = native.Go1Native(c, DEV)
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    g.state.load(st.arrays)
    gr, gvec = CF.gravity_state([0.0, 0.0, 0.0])
    scales = np.zeros(c.n_terms, np.float32)
    a = np.zeros((n, 12), np.float32)
    g.step(_dev(a), gvec, gr, scales, rng_seed=5, rng_step=300)
    torch.cuda.synchronize()
    out = O.step(c, st, ter, a, gvec, gr, scales, rng_seed=5, rng_step=300, debug=False)
    cf = g.contact_forces.cpu().numpy()
    ref = out["contact_forces"]
    err = np.abs(cf - ref)
    print(f"vel {vel}: max err {err.max():.3e} p99 {np.percentile(err, 99):.3e} p99.9 {np.percentile(err, 99.9):.3e}")
    for b in range(17):
        e = err[:, b].max(axis=1)
        i = int(np.argmax(e))
        print(f"  body {b:2d}: max {e.max():.3e} at env {i}: gpu {cf[i, b]} ref {ref[i, b]}")
    g.close() if hasattr(g, "close") else None
