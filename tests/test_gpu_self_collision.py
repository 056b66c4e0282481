"""Self-collision and restitution on the GPU step against the f64 oracle (CPU invariants of the same
model in tests/test_self_collision.py).  One-step comparisons with the integrator bounds of
tests/test_gpu_parity.py (check_integrator_step) on states built to exercise the new terms:
  * test_self_contact_forces_of_colliding_states: states chosen (numpy kinematics, below) to be in self-contact
    at the step's only sim step (decimation 1), the base 1 m above the plane: every reported force is a
    self-contact force, per body against the oracle, with every class of primitive pair hit across the batch;
  * legs in random poses within the joint limits, some with the front feet crossed under the trunk, stepped
    through three control steps;
  * the robot dropped onto the plane at up to 2.5 m/s with restitution 0..1, through the rebound;
  * test_foot_overlapping_another_legs_link_meets_a_force: a foot overlapping another leg's thigh or calf capsule,
    all 24 (foot leg, link leg, link) combinations, most of them in a hole of the rounds-3..5 sphere chains: both
    bodies meet a force on the GPU.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from legged_tracking_amd import config as CF, layout as L, native, terrain as T  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_parity import DEV, _dev, _sim_setup, check_integrator_step  # noqa: E402
from tests.self_geom import capsules as _capsules, pair_classes as _pair_classes  # noqa: E402


def _run(c, td, ter, st, rng, steps, act_scale=1.0, grav=(0.0, 0.0, 0.0), act=None):
    g = native.Go1Native(c, DEV)
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    gr, gvec = CF.gravity_state(list(grav))
    scales = np.zeros(c.n_terms, np.float32)
    forces = []
    n = c.n_envs
    for t in range(steps):
        g.state.load(st.arrays)
        a = (act_scale * rng.normal(0, 1, (n, 12))).astype(np.float32) if act is None else act.astype(np.float32)
        g.step(_dev(a), gvec, gr, scales, rng_seed=5, rng_step=200 + t)
        torch.cuda.synchronize()
        s32 = st.copy()
        out = O.step(c, st, ter, a, gvec, gr, scales, rng_seed=5, rng_step=200 + t, debug=False)
        O.step(c, s32, ter, a, gvec, gr, scales, rng_seed=5, rng_step=200 + t, debug=False, precision="f32")
        gs = g.state.numpy()
        cf = g.contact_forces.cpu().numpy()
        check_integrator_step(gs, st, cf, out["contact_forces"], g.reset.cpu().numpy().astype(bool),
                              out["reset"].astype(bool), st32=s32)
        forces.append(cf)
        st = O.NpState(n, gs, c)
    return np.stack(forces)


def test_self_collision_step_vs_oracle():
    n = 256
    cfg, c, td, ter, st, rng = _sim_setup(n, "plane")
    c.camera_zero = 0
    assert c.self_stiffness > 0
    lim = np.array([L.JOINT_LIMITS[j % 3] for j in range(12)])
    q = rng.uniform(lim[:, 0], lim[:, 1], (n, 12)).astype(np.float32)
    # a quarter of the envs with the front feet crossing under the trunk (tests/test_self_collision.py)
    k = n // 4
    q[:k] = [0.1, 0.8, -1.5, -0.1, 0.8, -1.5, 0.1, 1.0, -1.5, -0.1, 1.0, -1.5]
    q[:k, 0] = -rng.uniform(0.30, 0.42, k)
    q[:k, 3] = rng.uniform(0.30, 0.42, k)
    st["dof_pos"][:] = q
    st["dof_vel"][:] = 0.0
    st["root"][:, 2] = st["root"][:, 2] + 1.0  # 1 m above the plane
    st["episode_length"][:, 0] = 10
    # actions that hold each pose (joint targets default + action_scale (x hip reduction) * action)
    scale = np.float32(c.action_scale) * np.array([c.hip_scale_reduction, 1.0, 1.0] * 4, np.float32)
    hold = (q - np.array(c.default_dof_pos, np.float32)) / scale
    forces = _run(c, td, ter, st, rng, 3, act=np.clip(hold, -9.0, 9.0))
    # every reported force is a self-contact force here: opposite pairs sum to zero per env
    np.testing.assert_allclose(forces.sum(axis=2), 0.0, atol=2e-3)
    # the springs push the crossed feet apart within a step (the actuator net does not hold the pose), so the
    # contacts of the reported (last) sim step are a minority, the same set on both sides (checked above)
    touching = (np.abs(forces).max(axis=(2, 3)) > 0)
    assert touching[0].sum() >= n // 64, touching.sum(axis=1)


def test_restitution_step_vs_oracle():
    n = 256
    cfg, c, td, ter, st, rng = _sim_setup(n, "plane")
    c.camera_zero = 0
    st["restitution"][:, 0] = rng.uniform(0.0, 1.0, n).astype(np.float32)
    st["root"][:, 2] = st["root"][:, 2] + rng.uniform(0.0, 0.05, n).astype(np.float32)
    st["root"][:, 9] = -rng.uniform(0.5, 2.5, n).astype(np.float32)  # falling
    st["episode_length"][:, 0] = 10
    forces = _run(c, td, ter, st, rng, 4, act_scale=0.5, grav=(0.0, 0.0, 0.0))
    assert (np.abs(forces).max(axis=(0, 2, 3)) > 0).mean() > 0.9


@pytest.mark.parametrize("pool_kind", ["within_limits", "folded"])
def test_self_contact_forces_of_colliding_states(pool_kind):
    """states in self-contact at the step's (only) sim step, GPU per-body contact forces against the
    f64 oracle.  within_limits: 60,000 poses drawn within the joint limits (half with the hips turned inward, which
    brings the knees and feet under the trunk); folded: poses up to 1.2 rad past the limits, where the same-leg
    pairs and the trunk box are reached (the kernel tests those only for a leg past its 0.1 rad band:
    tests/test_self_collision.py::test_fold_gate_is_sound).  The batch: for every pair class some pose hits, one
    pose that hits it, then poses in contact up to 3/4 of the batch, the rest free.  Requirements: >= 50 % of the
    envs in self-contact on the GPU, every kind of pair (within_limits: cross-leg thigh-thigh, with a hip capsule,
    calf / foot, each of the six leg pairs; folded: the same-leg pairs and the trunk box) hit, and the forces within
    1e-3 N + 1e-4 relative of the oracle."""
    n = 512
    cfg = CF.readme_config(n_envs=n, terrain="plane", rows=2, cols=4)
    cfg.control.decimation = 1  # the reported forces are those of the step's only sim step, at the given state
    c = CF.build_abi_config(cfg)
    c.camera_zero = 0
    assert c.self_stiffness > 0
    td = T.build(cfg, n, np.random.RandomState(11))
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    st = O.NpState(n, cfg=c)
    O.reset_envs(c, st, ter, np.ones(n, np.uint8), rng_seed=3, rng_step=0)
    rng = np.random.default_rng(21)
    lim = np.array([L.JOINT_LIMITS[j % 3] for j in range(12)])
    if pool_kind == "within_limits":
        pool = rng.uniform(lim[:, 0], lim[:, 1], (60000, 12))
        inward = rng.random(60000) < 0.5  # hips turned toward the body (FL / RL: q_hip < 0, FR / RR: > 0)
        sgn = np.array([-1.0, 1.0, -1.0, 1.0])
        for l in range(4):
            pool[inward, 3 * l] = sgn[l] * rng.uniform(0.2, 0.8, inward.sum())
    else:
        pool = rng.uniform(lim[:, 0] - 1.2, lim[:, 1] + 1.2, (60000, 12))
    P, r = _capsules(pool)
    flags, names = _pair_classes(P, r)
    anyc = flags.any(1)
    pick = []
    for j in range(flags.shape[1]):  # one pose per reachable class
        idx = np.nonzero(flags[:, j])[0]
        if len(idx) and not flags[pick, j].any():
            pick.append(int(idx[0]))
    assert len(pick) <= n // 2, len(pick)
    rest = [i for i in np.nonzero(anyc)[0] if i not in set(pick)]
    pick += rest[:3 * n // 4 - len(pick)]
    free = np.nonzero(~anyc)[0]
    pick += list(free[:n - len(pick)])
    q = pool[pick].astype(np.float32)
    reach = flags[pick].any(0)
    kinds = {}
    for j, nm in enumerate(names):
        key = nm[0] if nm[0] != "cross" else ("cross-hip" if nm[3] == 1 or nm[4] == 1 else
                                             ("cross-thigh" if nm[3] == 0 and nm[4] == 0 else "cross-calf-foot"))
        kinds.setdefault(key, []).append(reach[j])
    print("\npair classes hit per kind: " + ", ".join(f"{k} {sum(v)}/{len(v)}" for k, v in kinds.items()))
    if pool_kind == "within_limits":
        for key in ("cross-thigh", "cross-hip", "cross-calf-foot"):
            assert any(kinds[key]), key
        for lp in range(6):
            assert any(reach[j] for j, nm in enumerate(names) if nm[0] == "cross" and (nm[1], nm[2]) ==
                       [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)][lp]), lp
    else:
        for key in ("same", "box"):
            assert sum(kinds[key]) >= 4, (key, sum(kinds[key]))
    st["dof_pos"][:] = q
    st["dof_vel"][:] = rng.normal(0, 1.0, (n, 12)).astype(np.float32)
    st["root"][:, 2] = st["root"][:, 2] + 1.0  # 1 m above the plane: every reported force is a self-contact force
    # every env at the world origin (they do not interact): on the plane the integrator works in world coordinates,
    # and at the env origins' 10-60 m an f32 ulp (1-4 um) puts ~1e-5 m into each sphere centre, i.e. 0.02-0.04 N
    # of the 2000 N/m springs -- physically nothing, but it would hide the narrow phase's own arithmetic here
    st["root"][:, 0:2] = 0.0
    st["root"][:, 7:13] = rng.normal(0, 0.2, (n, 6)).astype(np.float32)
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
    touching = np.abs(cf).max(axis=(1, 2)) > 0
    print(f"envs in self-contact: GPU {touching.mean():.2f}, oracle {(np.abs(ref).max(axis=(1, 2)) > 0).mean():.2f}; "
          f"max |dF| {np.abs(cf - ref).max():.2e} N of max |F| {np.abs(ref).max():.2e} N")
    assert touching.mean() >= 0.5
    # f32 against f64 kinematics (the integrator's hardware sin / cos): ~1e-7 m in a closest point, 2e-4 N of a
    # spring; a deep overlap (centres ~1 mm apart, up to 100 N) turns its normal by ~1e-4 -- hence a looser bound on
    # the few worst elements and a tight one on almost all of them
    err = np.abs(cf - ref)
    print(f"force error p99 {np.percentile(err, 99):.2e} N, max {err.max():.2e} N")
    assert np.percentile(err, 99) <= 1e-3, np.percentile(err, 99)
    # round 6, capsules: a capsule's point nearest the trunk box comes from a bisection on its slope, and the f32 build
    # of the oracle itself lands 0.023 N (folded pool) / 0.042 N (within limits) from the f64 one at worst
    np.testing.assert_allclose(cf, ref, rtol=1e-3, atol=0.05)
    # internal forces: the per-env sum over the bodies vanishes
    np.testing.assert_allclose(cf.sum(axis=1), 0.0, atol=2e-3)


def test_foot_overlapping_another_legs_link_meets_a_force():
    """VERDICT r05 #4 / weak #7 on the GPU: the property the round-3..5 sphere chains failed.  Poses with the hips
    turned inward (feet and knees under the trunk) where a foot overlaps another leg's thigh or calf capsule by more
    than 1 mm -- every (foot leg, link leg, thigh / calf) combination the pool reaches, the poses whose overlap lies
    in a hole of the old sphere chain first.  One GPU step at decimation 1 (the reported forces are those of the
    given pose), the base 1 m above the plane: in every env both the foot and the link report a force, the per-env
    sum vanishes, and the forces match the f64 oracle's (bounds of test_self_contact_forces_of_colliding_states)."""
    from tests.self_geom import seg_dist
    from tests.test_capsules import _old_spheres
    n = 256
    cfg = CF.readme_config(n_envs=n, terrain="plane", rows=2, cols=4)
    cfg.control.decimation = 1
    c = CF.build_abi_config(cfg)
    c.camera_zero = 0
    assert c.self_stiffness > 0
    td = T.build(cfg, n, np.random.RandomState(11))
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    st = O.NpState(n, cfg=c)
    O.reset_envs(c, st, ter, np.ones(n, np.uint8), rng_seed=3, rng_step=0)
    rng = np.random.default_rng(17)
    lim = np.array([L.JOINT_LIMITS[j % 3] for j in range(12)])
    m = 40000
    pool = rng.uniform(lim[:, 0], lim[:, 1], (m, 12))
    sgn = np.array([-1.0, 1.0, -1.0, 1.0])
    for l in range(4):
        pool[:, 3 * l] = sgn[l] * rng.uniform(0.2, 0.8, m)
    P, r = _capsules(pool)
    S, rs = _old_spheres(pool)
    cases = []  # (pose, foot leg, link leg, kind, in a sphere-chain hole)
    per_combo = max(1, n // 24)
    for la in range(4):
        for lb in range(4):
            if la == lb:
                continue
            for kind in (0, 2):
                F, A = P[:, 4 * la + 3], P[:, 4 * lb + kind]
                depth = r[3] + r[kind] - seg_dist(F[:, 0], F[:, 1], A[:, 0], A[:, 1])
                chain = [S[:, la, 5] - S[:, lb, s] for s in ((0, 1, 2) if kind == 0 else (3, 4))]
                hit = np.any([np.linalg.norm(d, axis=1) < rs[5] + rs[3 if kind == 2 else 0] for d in chain], 0)
                idx = np.nonzero(depth > 1e-3)[0]
                idx = np.concatenate([idx[~hit[idx]], idx[hit[idx]]])[:per_combo]  # holes first
                cases += [(int(i), la, lb, kind, not bool(hit[i])) for i in idx]
    combos = {(la, lb, kind) for _, la, lb, kind, _ in cases}
    holes = sum(h for *_, h in cases)
    print(f"\nfoot-link overlaps: {len(cases)} poses over {len(combos)} (foot leg, link leg, link) combinations, "
          f"{holes} in a sphere-chain hole")
    assert len(combos) >= 12 and holes >= 5, (len(combos), holes)
    cases = cases[:n]
    k = len(cases)
    q = np.zeros((n, 12), np.float32)
    q[:k] = pool[[i for i, *_ in cases]]
    q[k:] = np.array([0.1, 0.8, -1.5, -0.1, 0.8, -1.5, 0.1, 1.0, -1.5, -0.1, 1.0, -1.5], np.float32)  # free stance
    st["dof_pos"][:] = q
    st["dof_vel"][:] = 0.0
    st["root"][:, 0:2] = 0.0  # at the world origin (see test_self_contact_forces_of_colliding_states)
    st["root"][:, 2] = st["root"][:, 2] + 1.0
    st["root"][:, 3:7] = [0.0, 0.0, 0.0, 1.0]
    st["root"][:, 7:13] = 0.0
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
    for e, (_, la, lb, kind, _) in enumerate(cases):
        foot, link = 1 + 4 * la + 3, 1 + 4 * lb + (1 if kind == 0 else 2)
        assert np.linalg.norm(cf[e, foot]) > 0.1, (e, la, lb, kind, cf[e, foot])
        assert np.linalg.norm(cf[e, link]) > 0.1, (e, la, lb, kind, cf[e, link])
    np.testing.assert_allclose(cf.sum(axis=1), 0.0, atol=2e-3)
    np.testing.assert_allclose(cf, out["contact_forces"], rtol=1e-3, atol=0.05)


def test_trunk_face_contacts_step_vs_oracle():
    """the trunk's top face against ceiling apexes and its bottom face against a floor ridge that
    lie between the box corners (go1_device.h face_scan / face_force against oracle/go1_oracle.c).  Every tile gets
    a flat floor and ceiling with three downward ceiling spikes and a raised floor ridge under the trunk; every
    env's trunk sits over them, level to within 0.1 rad and yawed up to 0.5 rad, at heights that put the spikes and
    the ridge 0-15 mm into its faces.  README configuration (decimation 4, the specialised kernel), three control
    steps, each against the f64 oracle from the same state within the integrator bounds of
    tests/test_gpu_parity.py; the trunk's reported contact force, which only the faces produce here, within
    1e-3 relative of the oracle's and present in most envs."""
    n = 256
    cfg, c, td, ter, st, rng = _sim_setup(n, "single_path")
    hs = float(c.horizontal_scale)
    tiles = td.tiles.copy()
    tiles[:, 1] = 0.0   # floor
    tiles[:, 0] = 0.5   # ceiling
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
    cy, sy, cp, sp, cr, sr = np.cos(yaw / 2), np.sin(yaw / 2), np.cos(pitch / 2), np.sin(pitch / 2), np.cos(roll / 2), np.sin(roll / 2)
    root[:, 3] = sr * cp * cy - cr * sp * sy
    root[:, 4] = cr * sp * cy + sr * cp * sy
    root[:, 5] = cr * cp * sy - sr * sp * cy
    root[:, 6] = cr * cp * cy + sr * sp * sy
    root[:, 7:13] = rng.normal(0, 0.1, (n, 6))
    st["episode_length"][:, 0] = 10
    g = native.Go1Native(c, DEV)
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    grav, gvec = CF.gravity_state([0.0, 0.0, 0.0])
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    hits = []
    for t in range(3):
        g.state.load(st.arrays)
        act = rng.normal(0, 0.3, (n, 12)).astype(np.float32)
        g.step(_dev(act), gvec, grav, scales, rng_seed=4, rng_step=400 + t)
        torch.cuda.synchronize()
        s32 = st.copy()
        out = O.step(c, st, ter, act, gvec, grav, scales, rng_seed=4, rng_step=400 + t, debug=False)
        O.step(c, s32, ter, act, gvec, grav, scales, rng_seed=4, rng_step=400 + t, debug=False, precision="f32")
        gs = g.state.numpy()
        cf = g.contact_forces.cpu().numpy()
        check_integrator_step(gs, st, cf, out["contact_forces"], g.reset.cpu().numpy().astype(bool),
                              out["reset"].astype(bool), st32=s32)
        base, base_ref = cf[:, 0], out["contact_forces"][:, 0]
        np.testing.assert_allclose(base, base_ref, rtol=1e-3, atol=2e-2)
        hits.append((np.linalg.norm(base_ref, axis=1) > 0).mean())
        st = O.NpState(n, gs, c)
    print(f"\nenvs with trunk-face forces per step: {hits}")
    assert hits[0] > 0.3
