"""The trunk box's faces against the heightfields: the deepest grid vertex of the ceiling
inside the top face's footprint and of the floor inside the bottom face's, chosen once per control step, carry a
penalty force every sim step (oracle/go1_oracle.c face_scan / face_force; go1_device.h the same on the GPU).

Reference scene: the trunk's collision box is 0.3762 x 0.0935 x 0.114 (resources/robots/go1/urdf/go1.urdf:53-58) and
PhysX collides it with the tunnel's trimesh (legged_robot_trajectory_tracking.py:1450-1480), whose ceiling is made
of downward pyramidal wedges (go1_gym/utils/tunnel_fn.py:99-163): an apex or ridge can enter the top face between
its corners, where the 8 corner contact points feel nothing.  PhysX parity stays unpinned (Isaac Gym is absent);
these are the model's own properties in the f64 oracle (CPU), and the GPU step against it (tests/
test_gpu_self_collision.py::test_trunk_face_contacts_step_vs_oracle).
"""
import numpy as np
import pytest

from legged_tracking_amd import config as CF
from oracle import oracle as O

G0 = np.zeros(3)
STAND = np.array([0.1, 0.8, -1.5, -0.1, 0.8, -1.5, 0.1, 1.0, -1.5, -0.1, 1.0, -1.5])
K_CONTACT = 2.0e4


def _cfg():
    cfg = CF.readme_config(n_envs=16, terrain="single_path", rows=2, cols=4)
    cfg.env.camera_zero = False
    return CF.build_abi_config(cfg)


def _tile(c, ceil=1.0, floor=-1.0):
    t = np.empty((2, c.hf_nx, c.hf_ny), np.float32)
    t[0] = ceil   # layer 0: ceiling
    t[1] = floor  # layer 1: floor
    return t


def _body(x, y, z, quat=(0.0, 0.0, 0.0, 1.0)):
    return dict(pos=[x, y, z], quat=list(quat), v=[0.0, 0.0, 0.0], w=[0.0, 0.0, 0.0], q=STAND.copy(),
                qd=np.zeros(12))


def _step(c, tile, body, n=1):
    return O.physics(c, body, np.zeros(12), n, 0.005, G0, 1.0, 0.0, 0.0, tile=tile)


def test_ceiling_apex_between_the_corners_pushes_the_trunk_down():
    c = _cfg()
    hs = float(c.horizontal_scale)
    i0, j0 = 40, 20
    x, y, z = i0 * hs + 0.012, j0 * hs + 0.01, 0.30
    top = z + 0.114 / 2
    # no apex: nothing touches the trunk (corners 0.64 m below the ceiling, legs above the floor)
    cf = _step(c, _tile(c), _body(x, y, z))
    assert np.abs(cf).max() == 0.0
    # a single ceiling vertex 17 mm inside the top face at the trunk's centre
    t = _tile(c)
    t[0, i0, j0] = top - 0.017
    b = _body(x, y, z)
    cf = _step(c, t, b)
    np.testing.assert_allclose(cf[0], [0.0, 0.0, -K_CONTACT * 0.017], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(np.abs(cf[1:]).max(), 0.0)
    assert b["v"][2] < 0.0
    # ahead of the centre, it pitches the nose down (rotation about +y)
    t = _tile(c)
    t[0, i0 + 3, j0] = top - 0.017
    b = _body(x, y, z)
    cf = _step(c, t, b)
    assert cf[0][2] < -300.0 and b["w"][1] > 0.0
    # outside the footprint (beside the trunk), nothing
    t = _tile(c)
    t[0, i0, j0 + 2] = top - 0.017
    assert np.abs(_step(c, t, _body(x, y, z))).max() == 0.0


def test_floor_ridge_under_the_bottom_face_and_the_deepest_vertex_wins():
    c = _cfg()
    hs = float(c.horizontal_scale)
    i0, j0 = 40, 20
    x, y, z = i0 * hs + 0.02, j0 * hs + 0.02, 0.30
    bottom = z - 0.114 / 2
    t = _tile(c)
    t[1, i0 - 2:i0 + 3, j0] = bottom + 0.004   # a ridge along the trunk, 4 mm into the bottom face
    t[1, i0 + 1, j0] = bottom + 0.009           # its highest vertex
    b = _body(x, y, z)
    cf = _step(c, t, b)
    np.testing.assert_allclose(cf[0], [0.0, 0.0, K_CONTACT * 0.009], rtol=1e-5)
    assert b["v"][2] > 0.0


def test_face_contacts_follow_a_yawed_trunk_and_conserve_energy_without_damping_gain():
    """A yawed and tilted trunk resting against a ceiling apex: the force stays on the face normal (the
    friction-free case: no lateral force at rest), and a trunk pushed up into the apex rebounds below its speed."""
    c = _cfg()
    hs = float(c.horizontal_scale)
    i0, j0 = 40, 20
    yaw = 0.7
    quat = (0.0, 0.0, np.sin(yaw / 2), np.cos(yaw / 2))
    x, y, z = i0 * hs + 0.013, j0 * hs - 0.004, 0.30
    t = _tile(c)
    t[0, i0 + 1, j0 + 1] = z + 0.057 - 0.01
    b = _body(x, y, z, quat)
    cf = _step(c, t, b)
    assert cf[0][2] < -150.0 and np.abs(cf[0][:2]).max() < 1e-9
    # moving up into it at 0.5 m/s: after 60 sim steps in zero gravity the trunk moves down, slower than it came
    b = _body(x, y, z - 0.02, quat)
    b["v"] = [0.0, 0.0, 0.5]
    _step(c, t, b, n=60)
    assert -0.5 < b["v"][2] < 0.0


def test_apex_entering_the_face_during_the_control_step_acts_at_once():
    """the scan at the control step's first sim step keeps the nearest vertex by signed depth, so an apex
    5 mm above the top face when the trunk starts moving up at 1 m/s (5 mm per sim step) pushes back on the sim step
    it enters, not a control step later."""
    c = _cfg()
    hs = float(c.horizontal_scale)
    i0, j0 = 40, 20
    x, y, z = i0 * hs + 0.012, j0 * hs + 0.01, 0.30
    t = _tile(c)
    t[0, i0, j0] = z + 0.057 + 0.005
    forces = []
    for n in (1, 2, 3, 4):  # n sim steps of one control step (the scan runs on the first)
        b = _body(x, y, z)
        b["v"] = [0.0, 0.0, 1.0]
        forces.append(_step(c, t, b, n=n)[0][2])
    assert forces[0] == 0.0
    assert min(forces[2:]) < -20.0, forces


def test_the_vertex_window_covers_a_face_end_at_45_degrees():
    """at a yaw near 45 degrees the footprint reaches 0.166 m along both axes; an apex 10 mm inside the top
    face near its end, 4 cells from the centre's cell on the short axis (outside a 10 x 8 window), is found."""
    c = _cfg()
    hs = float(c.horizontal_scale)
    i0, j0 = 40, 20
    yaw = 0.75
    quat = (0.0, 0.0, np.sin(yaw / 2), np.cos(yaw / 2))
    x, y, z = i0 * hs, (j0 + 0.9) * hs, 0.30
    t = _tile(c)
    t[0, i0 + 2, j0 + 4] = z + 0.057 - 0.010
    cf = _step(c, t, _body(x, y, z, quat))
    np.testing.assert_allclose(cf[0], [0.0, 0.0, -K_CONTACT * 0.010], rtol=1e-5, atol=1e-9)
