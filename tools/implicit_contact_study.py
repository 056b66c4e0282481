"""Is one 5 ms integrator step per sim step stable?  (CPU, f64 oracle; the study behind n_internal = 1)

Round 1-2 ran two 2.5 ms semi-implicit Euler sub-steps per 5 ms sim step because explicit penalty
contacts (k = 2e4 N/m against ~0.1-0.3 kg links) go unstable at 5 ms.  The integrator now makes the
contact forces linearly implicit in the point velocity (added masses in the articulated inertias,
oracle sphere_contact_im / go1_step.hip sphere_contact_im) and takes one 5 ms step, as PhysX does
(substeps = 1).  go1o_set_implicit_contact(0) restores the explicit forces for this comparison.  The
tool drives the full oracle step on the README single_path workload under N(0, 1) actions:

  explicit 2 sub-steps (rounds 1-2)   explicit 1   implicit 1 (the product)   implicit 2

and reports joint speeds, base speeds, base heights (as -z) and divergence-guard resets
(profiles/r02/implicit_contact_study.json: 256 envs x 200 steps).

  python tools/implicit_contact_study.py [n_envs] [steps]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from legged_tracking_amd import config as CF, terrain as T  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(n, steps, n_internal, implicit, seed=5):
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=4, cols=4)
    c = CF.build_abi_config(cfg)
    c.n_internal = n_internal
    lib = O.lib("f64")
    lib.go1o_set_implicit_contact.argtypes = [C.c_int]
    lib.go1o_set_implicit_contact(int(implicit))
    td = T.build(cfg, n, np.random.RandomState(11))
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    rng = np.random.default_rng(seed)
    st = O.NpState(n, cfg=c)
    st["friction"][:, 0] = rng.uniform(0.1, 3.0, n)
    st["payload"][:, 0] = rng.uniform(-1.0, 3.0, n)
    O.reset_envs(c, st, ter, np.ones(n, np.uint8), rng_seed=seed, rng_step=0)
    st["episode_length"][:, 0] = rng.integers(0, 499, n)
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    grav, gvec = CF.gravity_state([0.0, 0.0, 0.0])
    qd_max, v_max, z_min, resets = [], [], [], 0
    for t in range(steps):
        a = rng.normal(0, 1, (n, 12)).astype(np.float32)
        out = O.step(c, st, ter, a, gvec, grav, scales, rng_seed=seed, rng_step=t, debug=False)
        rs = out["reset"].astype(bool)
        resets += int(rs.sum())
        live = ~rs
        qd_max.append(np.abs(st["dof_vel"][live]).max(axis=1))
        v_max.append(np.linalg.norm(st["root"][live, 7:10], axis=1))
        z_min.append(st["root"][live, 2])
    lib.go1o_set_implicit_contact(1)  # the oracle's default (the integrator's scheme)
    qd = np.concatenate(qd_max)
    v = np.concatenate(v_max)
    z = np.concatenate(z_min)
    pct = lambda x: {p: float(np.percentile(x, p)) for p in (50, 99, 99.9)} | {"max": float(x.max())}  # noqa: E731
    return {"n_internal": n_internal, "implicit": bool(implicit), "resets": resets,
            "max_joint_speed_rad_s": pct(qd), "base_speed_m_s": pct(v), "base_height_m": pct(-z)}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    res = [run(n, steps, 2, False), run(n, steps, 1, False), run(n, steps, 1, True), run(n, steps, 2, True)]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
