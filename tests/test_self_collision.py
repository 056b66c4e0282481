"""Self-collision and restitution of the native contact model, in the f64 oracle (CPU) and the HIP step
against it (GPU).

Reference scene: asset.self_collisions = 0 enables PhysX self-collision (go1_gym/envs/go1/go1_crawling.py:44);
the per-env restitution goes to every rigid shape (legged_robot_trajectory_tracking.py:676), the terrain's from
cfg.terrain.restitution (:1421-1428), PhysX averages the two and bounces above bounce_threshold_velocity
(legged_robot_trajectory_tracking_config.py:369).  PhysX itself is absent here, so these are the model's own
invariants (parity with PhysX stays unpinned):
  * the self-contact forces are pairwise opposite: with no terrain contact, the reported contact forces of all
    17 bodies (trunk reaction included) sum to zero in every env, and some envs do collide;
  * no self-collision when asset.self_collisions = 1;
  * restitution 0 never gains energy, and restitution > 0 bounces higher;
  * the GPU step equals the f64 oracle within the integrator bounds on colliding and bouncing states.
"""
import numpy as np
import pytest

from legged_tracking_amd import config as CF, layout as L
from oracle import oracle as O

G = np.array([0.0, 0.0, -9.81])
DEFAULT_Q = np.array([0.1, 0.8, -1.5, -0.1, 0.8, -1.5, 0.1, 1.0, -1.5, -0.1, 1.0, -1.5])


def _cfg(**kw):
    cfg = CF.readme_config(n_envs=16, terrain="plane", rows=2, cols=4)
    cfg.env.camera_zero = False
    for k, v in kw.items():
        obj = cfg
        *path, last = k.split(".")
        for p in path:
            obj = getattr(obj, p)
        setattr(obj, last, v)
    return CF.build_abi_config(cfg)


def _body(z=2.0, q=DEFAULT_Q, vz=0.0):
    return dict(pos=[0.0, 0.0, z], quat=[0.0, 0.0, 0.0, 1.0], v=[0.0, 0.0, vz], w=[0.0, 0.0, 0.0],
                q=np.array(q, np.float64), qd=np.zeros(12))


def _random_poses(n, seed):
    """Joint angles uniform within the URDF limits (layout.JOINT_LIMITS, the native joint-limit model's)."""
    rng = np.random.default_rng(seed)
    lim = np.array([L.JOINT_LIMITS[j % 3] for j in range(12)])
    return rng.uniform(lim[:, 0], lim[:, 1], (n, 12))


def _inward_front_feet(a=0.36):
    """FL and FR abducted inward until their feet meet under the trunk (feet ~0.024 m apart at a = 0.36)."""
    q = DEFAULT_Q.copy()
    q[0], q[3] = -a, a
    return q


def test_front_feet_collide_with_opposite_forces():
    c = _cfg()
    b = _body(q=_inward_front_feet())
    cf = O.physics(c, b, np.zeros(12), 1, 0.005, G, 1.0, 0.0, 0.0)
    # bodies: 0 trunk, then per leg hip, thigh, calf, foot (1 + 4 l + j)
    f_fl, f_fr = cf[1 + 4 * 0 + 3], cf[1 + 4 * 1 + 3]
    assert np.linalg.norm(f_fl) > 1.0 and np.linalg.norm(f_fr) > 1.0
    np.testing.assert_allclose(f_fl, -f_fr, rtol=0, atol=1e-9)
    assert f_fl[1] > 0 > f_fr[1]  # pushed apart: FL (left, +y side) back to +y
    np.testing.assert_allclose(cf.sum(axis=0), 0.0, atol=1e-9)


def test_disabled_self_collision_has_no_forces():
    c = _cfg(**{"asset.self_collisions": 1})
    assert c.self_stiffness == 0.0
    cf = O.physics(c, _body(q=_inward_front_feet()), np.zeros(12), 1, 0.005, G, 1.0, 0.0, 0.0)
    np.testing.assert_array_equal(cf, 0.0)


def test_random_poses_forces_sum_to_zero():
    """Away from the terrain every reported force is a self-contact force or the trunk's reaction: they sum
    to zero per env (Newton's third law), and a good share of random poses do collide."""
    c = _cfg()
    hits = 0
    for q in _random_poses(200, 5):
        cf = O.physics(c, _body(q=q), np.zeros(12), 1, 0.005, G, 1.0, 0.0, 0.0)
        np.testing.assert_allclose(cf.sum(axis=0), 0.0, atol=1e-8)
        hits += np.abs(cf).max() > 0
    assert hits >= 5, hits  # 9 of these 200 poses (seed 5)


def test_trunk_box_contacts_oracle():
    """The calf / foot spheres cannot reach the Go1 trunk box within (or well beyond) the joint limits -- the
    thigh joints sit 0.08 m outboard of it (a search over hip angles up to 1.6 rad found none) -- so the
    sphere-box branch is exercised on an oracle model with the box widened to 0.3 m: the feet of a standing
    pose are then inside it, and every env's forces (the trunk's reported reaction included) still sum to
    zero while the trunk does report a reaction."""
    c = _cfg()
    k = 13 * 10 + 4 * 9 + 3 + 1  # model block: trunk half extents (model.py model_block)
    c.model[k + 1] = 0.15
    found = 0
    for q in _random_poses(400, 7):
        cf = O.physics(c, _body(q=q), np.zeros(12), 1, 0.005, G, 1.0, 0.0, 0.0)
        np.testing.assert_allclose(cf.sum(axis=0), 0.0, atol=1e-8)
        found += np.linalg.norm(cf[0]) > 0
    assert found >= 10, found


def _drop(c, restitution, steps=150, vz=-2.0, z=0.2):
    """The robot upside down (legs up, limp) dropped onto the plane on its trunk box corners."""
    b = _body(z=z, vz=vz)
    b["quat"] = [1.0, 0.0, 0.0, 0.0]  # 180 degrees about x
    e0 = O.energy(c, b, G, 0.0)
    energies, vzs = [], []
    for _ in range(steps):
        O.physics(c, b, np.zeros(12), 1, 0.005, G, 1.0, restitution, 0.0)
        energies.append(O.energy(c, b, G, 0.0))
        vzs.append(b["v"][2])
    return e0, np.array(energies), np.array(vzs)


@pytest.mark.parametrize("rest", [0.0, 0.5, 1.0])
def test_restitution_gains_no_energy(rest):
    """Mechanical energy never exceeds the start: the penalty springs return at most what they stored, the
    damping only removes energy, and restitution hands back at most all of the damping (e <= 1)."""
    c = _cfg()
    for vz in (-2.0, -1.0):
        e0, e, _ = _drop(c, rest, vz=vz)
        assert e.max() <= e0 + 1e-9, (rest, vz, e.max(), e0)
        assert e[-1] < e0 - 0.5  # the impact dissipated


def test_restitution_bounces_higher():
    """The rebound speed of the trunk grows with the restitution: 0.67 / 0.79 / 0.89 m/s from a 2 m/s drop
    at e = 0 / 0.5 / 1 (the model's own compliance bounces a little at e = 0, unlike PhysX's rigid contact)."""
    c = _cfg()
    v = [_drop(c, r)[2].max() for r in (0.0, 0.5, 1.0)]
    assert v[0] + 0.05 < v[1] < v[2] - 0.05, v


def test_restitution_below_threshold_changes_nothing():
    """The bounce threshold gates restitution: with cfg.sim.physx.bounce_threshold_velocity above every
    separating speed, e = 1 drops exactly as e = 0; with the reference's 0.5 m/s it does not."""
    c = _cfg(**{"sim.physx.bounce_threshold_velocity": 100.0})
    assert c.bounce_threshold == 100.0
    _, ea, va = _drop(c, 0.0)
    _, eb, vb = _drop(c, 1.0)
    np.testing.assert_array_equal(va, vb)
    np.testing.assert_array_equal(ea, eb)
    c = _cfg()
    assert c.bounce_threshold == np.float32(0.5)
    assert not np.array_equal(_drop(c, 0.0)[2], _drop(c, 1.0)[2])


def test_restitution_drop_apex_is_pinned():
    """the restitution model's rebound, pinned.  The trunk dropped upside down from 0.4 m (impact
    2.60 m/s) on its box corners: rebound / impact speed and the apex the trunk rises to after the first
    impact, for e = 0, 0.5, 1.  A penalty contact bounces a little by itself (its spring returns part of the
    stored energy) and e hands back part of the damping, so the rebound ratio goes from 0.28 to 0.35 -- where
    PhysX's rigid contact would give e itself above the 0.5 m/s threshold (a deliberate deviation,
    parity with PhysX unpinned).  Round 6: the limp legs' capsules (thigh and calf over their full length) meet
    the plane during the impact where the sphere chains did not, 0.257 / 0.302 / 0.345 before."""
    c = _cfg()
    want = {0.0: (0.2828, 0.03230), 0.5: (0.3124, 0.04134), 1.0: (0.3507, 0.05034)}
    for e, (ratio, rise) in want.items():
        b = _body(z=0.4)
        b["quat"] = [1.0, 0.0, 0.0, 0.0]
        zs, vs = [], []
        for _ in range(300):
            O.physics(c, b, np.zeros(12), 1, 0.005, G, 1.0, e, 0.0)
            zs.append(b["pos"][2])
            vs.append(b["v"][2])
        zs, vs = np.array(zs), np.array(vs)
        k = int(np.argmax(vs > 0))
        assert k > 0
        impact, rebound = -vs[:k].min(), vs[k:].max()
        assert abs(impact - 2.5996) < 1e-3, impact
        np.testing.assert_allclose(rebound / impact, ratio, rtol=0.01, err_msg=str(e))
        np.testing.assert_allclose(zs[k:].max() - zs[:k].min(), rise, rtol=0.02, err_msg=str(e))


def test_fold_gate_is_sound():
    """go1_device.h self_broad tests a leg's same-leg pairs and its primitives against the trunk box only while one of
    its joints is more than 0.1 rad past its URDF range (the oracle always tests them).  Sound if none of those
    pairs can touch inside the band: on a grid of step h the clearance stays above what a grid cell can close
    (per joint: the lever arm of the farthest collision point about its axis x h / 2).  The same-leg geometry does
    not depend on the hip joint (the hip capsule turns with the leg), so that grid is (thigh, knee).  Round 6: the
    capsules over the links' full length (tests/self_geom.py)."""
    from legged_tracking_amd import model as M
    from tests.self_geom import SAME, leg_capsules, seg_box_dist, seg_dist
    lim = np.array(L.JOINT_LIMITS)
    band = np.stack([lim[:, 0] - 0.1001, lim[:, 1] + 0.1001], 1)
    o = [np.linalg.norm(v) for v in M.joint_origins(L.LEGS[0])]
    calf = np.linalg.norm(M.FOOT_OFFSET)  # the knee axis to the farthest collision point (the foot)
    lever = np.array([o[1] + o[2] + calf, o[2] + calf, calf])  # hip, thigh, knee
    # same-leg pairs, (thigh, knee) grid
    h = 0.005
    qt, qk = [np.arange(band[j, 0], band[j, 1] + h, h) for j in (1, 2)]
    T2, K2 = (a.ravel() for a in np.meshgrid(qt, qk, indexing="ij"))
    P, r = leg_capsules(np.zeros_like(T2), T2, K2)
    clear = min(float((seg_dist(P[:, a, 0], P[:, a, 1], P[:, b, 0], P[:, b, 1]) - r[a] - r[b]).min())
                for a, b in SAME)
    bound = (lever[1] + lever[2]) * h / 2
    print(f"\nsame-leg clearance {clear * 1e3:.1f} mm > {bound * 1e3:.1f} mm")
    assert clear > bound, (clear, bound)
    # trunk box, (hip, thigh, knee) grid, one hip angle at a time
    h = 0.02
    th = np.array(M.TRUNK_BOX) / 2
    qt, qk = [np.arange(band[j, 0], band[j, 1] + h, h) for j in (1, 2)]
    T2, K2 = (a.ravel() for a in np.meshgrid(qt, qk, indexing="ij"))
    box = np.inf
    for qh in np.arange(band[0, 0], band[0, 1] + h, h):
        P, r = leg_capsules(np.full_like(T2, qh), T2, K2)
        for k in (0, 2, 3):
            box = min(box, float((seg_box_dist(P[:, k, 0], P[:, k, 1], th) - r[k]).min()))
    bound = lever.sum() * h / 2
    print(f"box clearance {box * 1e3:.1f} mm > {bound * 1e3:.1f} mm")
    assert box > bound, (box, bound)
