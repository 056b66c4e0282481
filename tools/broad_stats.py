"""CPU study: how loose the self-collision broad phase is on the bench workload (single_path, N(0, 1) actions).
Steps the f64 oracle, and after every control step compares, per env and per leg pair, the trunk-frame AABB
overlap of go1_device.h self_broad (thigh joint / knee / foot grown by the largest link radius, plus the hip
capsule) with exact sphere overlaps and with tighter candidate tests.  Prints rates per env and per 4-env wave."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_tracking_amd import config as CF, terrain as T, model as M, layout as L  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.self_geom import leg_spheres, pair_classes, spheres  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 150
cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=4, cols=8)
c = CF.build_abi_config(cfg)
td = T.build(cfg, n, np.random.RandomState(11))
ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
st = O.NpState(n, cfg=c)
O.reset_envs(c, st, ter, np.ones(n, np.uint8), rng_seed=1, rng_step=0)
rng = np.random.default_rng(0)
scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
gr, gvec = CF.gravity_state([0.0, 0.0, 0.0])
rmax = max(M.FOOT_RADIUS, M.THIGH_BOX_HALF_WIDTH, M.CALF_BOX_HALF_WIDTH)
LP = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
acc = {k: 0 for k in ("aabb_env", "aabb_wave", "exact_env", "exact_wave", "split_env", "split_wave", "n", "w")}
for t in range(steps):
    a = rng.normal(0, 1, (n, 12)).astype(np.float32)
    out = O.step(c, st, ter, a, gvec, gr, scales, rng_seed=3, rng_step=1 + t, debug=False)
    if t < 20:
        continue
    q = st["dof_pos"].astype(np.float64)
    P, r = spheres(q)
    flags, names = pair_classes(P, r)
    exact = flags[:, [i for i, nm in enumerate(names) if nm[0] == "cross"]].any(1)
    # the kernel's per-leg box: thigh joint, knee, foot grown by rmax; hip capsule ends grown by the hip radius
    lo, hi, slo, shi = [], [], [], []
    for l in range(4):
        o = [np.array(v) for v in M.joint_origins(L.LEGS[l])]
        Pl, rl = P[:, 8 * l:8 * l + 8], r[8 * l:8 * l + 8]
        # thigh joint / knee / foot from the spheres' chain (sphere 2 sits at the knee, 5 at the foot)
        from tests.self_geom import _rx  # noqa
        tj = o[0] + np.einsum("nij,j->ni", _rx(q[:, 3 * l]), o[1])
        pts = np.stack([tj, Pl[:, 2], Pl[:, 5]], 1)
        l0 = np.minimum(pts.min(1) - rmax, Pl[:, 6:8].min(1) - M.HIP_CAPSULE_RADIUS)
        h0 = np.maximum(pts.max(1) + rmax, Pl[:, 6:8].max(1) + M.HIP_CAPSULE_RADIUS)
        lo.append(l0); hi.append(h0)
        # split: upper (thigh spheres + hip ends) and lower (calf + foot) boxes from the spheres themselves
        up = [0, 1, 2, 6, 7]; dn = [2, 3, 4, 5]
        slo.append([(Pl[:, s] - rl[s][None, :, None]).min(1) for s in (up, dn)])
        shi.append([(Pl[:, s] + rl[s][None, :, None]).max(1) for s in (up, dn)])
    ab = np.zeros(n, bool); sp = np.zeros(n, bool)
    for la, lb in LP:
        ab |= ((lo[la] <= hi[lb]) & (lo[lb] <= hi[la])).all(1)
        for u in range(2):
            for v in range(2):
                sp |= ((slo[la][u] <= shi[lb][v]) & (slo[lb][v] <= shi[la][u])).all(1)
    acc["aabb_env"] += ab.sum(); acc["exact_env"] += exact.sum(); acc["split_env"] += sp.sum(); acc["n"] += n
    acc["aabb_wave"] += ab.reshape(-1, 4).any(1).sum(); acc["exact_wave"] += exact.reshape(-1, 4).any(1).sum()
    acc["split_wave"] += sp.reshape(-1, 4).any(1).sum(); acc["w"] += n // 4
    st = O.NpState(n, st.arrays, c) if False else st
print({k: (round(v / acc["n"], 4) if k.endswith("env") else round(v / acc["w"], 4)) for k, v in acc.items() if k not in ("n", "w")})
