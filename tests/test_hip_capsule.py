"""Hip capsule contact (the reference's scene keeps the hip collision cylinders,
go1.urdf:106-111 / :229-234, as capsules, legged_robot_trajectory_tracking_config.py:214-215).

The native model carries each hip capsule as the two ends of its segment (model.py HIP_CAPSULE_*),
spheres of the capsule's radius on the hip link, in the f64 oracle (oracle/go1_oracle.c phys_substep
j == 0) and in the HIP integrator (csrc/go1_device.h hip_contact).  Scenario: the trunk rolled 34-46
degrees to the left with the legs folded up, lowered until the left hips' outer capsule ends press
2-10 mm into the plane, so the hips are the only bodies in contact.

Effects stated and tested:
  * the left hips (FL, RL) report an upward contact force, every other body (right hips, legs,
    trunk) none;
  * collision_count does not move: the reference penalises contacts on thighs and calves only
    (train.py:80 penalize_contacts_on) and terminates on the base, the hips are in neither;
  * the static stance is unchanged (test_physics_invariants.py): standing, the hips are 0.2 m above
    the plane and report no force;
  * the HIP kernel's hip forces and the resulting state match the f64 oracle's.
"""
import numpy as np
import pytest

from tests import physics_drive as D

N = 64
GZ = (0.0, 0.0, -9.81)
HIPS = [1, 5, 9, 13]  # FL, FR, RL, RR hip bodies in the 17-body contact_forces layout


def _rolled(n=N, seed=5):
    c, td, ter, st, scales = D.setup(n=n, seed=seed)
    rng = np.random.default_rng(seed)
    phi = rng.uniform(-0.8, -0.6, n)  # roll: left side down
    st["root"][:, 3:7] = np.stack([np.sin(phi / 2), 0 * phi, 0 * phi, np.cos(phi / 2)], 1)
    st["root"][:, 7:13] = 0.0
    st["dof_pos"][:] = np.tile([0.0, 3.0, -1.0], 4)  # thighs up, calves folded: the feet clear the plane
    st["dof_vel"][:] = 0.0
    depth = rng.uniform(0.002, 0.01, n)
    outer = 0.04675 + 0.065  # hip joint y + the capsule segment's outer end (model.py)
    st["root"][:, 2] = -outer * np.sin(phi) + 0.046 - depth
    return c, td, ter, st, scales


def _check_contacts(cf, st):
    cf = cf.reshape(st.n, 17, 3)
    left, right = cf[:, [1, 9]], cf[:, [5, 13]]
    assert (left[..., 2] > 1.0).all(), left[..., 2].min()  # every left hip pushed up
    others = np.delete(cf, [1, 9], axis=1)
    assert np.abs(others).max() == 0.0, np.abs(others).max()
    assert np.abs(right).max() == 0.0
    assert (st["collision_count"] == 0).all()


def test_oracle_hip_capsule_contact():
    c, td, ter, st, scales = _rolled()
    s, cf, reset = next(D.oracle_roll(c, ter, st, scales, 1, GZ))
    assert not reset.any()
    _check_contacts(cf, s)


@pytest.mark.gpu
def test_hip_capsule_contact_matches_oracle():
    c, td, ter, st, scales = _rolled()
    ref = _rolled()[3]
    steps = 3
    hip = list(D.hip_roll(c, td, st, scales, steps, GZ))
    orc = []
    for s, cf, reset in D.oracle_roll(c, ter, ref, scales, steps, GZ):
        orc.append((s["root"].copy(), s["dof_vel"].copy(), cf.copy(), reset.copy()))
    for t, ((hs, hcf, hreset), (oroot, odv, ocf, oreset)) in enumerate(zip(hip, orc)):
        assert not hreset.any() and not oreset.any()
        if t == 0:
            _check_contacts(hcf, hs)
        h = hcf.reshape(N, 17, 3)[:, HIPS]
        o = ocf.reshape(N, 17, 3)[:, HIPS]
        scale = np.abs(o).max()
        err = np.abs(h - o).max() / scale
        root_err = np.abs(hs["root"] - oroot).max()
        print(f"\nstep {t}: hip force max {scale:.1f} N, rel err {err:.2e}, root err {root_err:.2e}")
        assert err < 2e-2, err
        assert root_err < 5e-3, root_err
