"""Go1 rigid-body model for the native articulated-dynamics step (data only).

Transcribed from resources/robots/go1/urdf/go1.urdf of the reference (line
numbers cited per constant; tests/test_model.py re-parses the URDF when the
reference tree is present and checks every value).  Bodies joined by fixed
joints are merged the way Isaac Gym's collapse_fixed_joints does
(go1_gym/envs/base/legged_robot_trajectory_tracking_config.py asset.collapse_fixed_joints):
trunk+imu_link -> base, calf+foot -> calf (the foot keeps its own contact
sphere and its own reported contact force).

Frames: every link frame sits at its joint origin with identity rotation at
q = 0 (all URDF joint rpy are 0).  Hip axis x, thigh and calf axis y.
"""
import numpy as np

from . import layout as L

# ---- raw URDF values --------------------------------------------------------
TRUNK = dict(mass=4.8, com=(0.011611, 0.004437, 0.000108),  # go1.urdf:60-62
             inertia=(0.016130741919, 0.000593180607, 7.324662e-06, 0.036507810812, 2.0969537e-05, 0.044693872053))
IMU = dict(mass=0.001, com=(-0.01592, -0.06659, -0.00617),  # go1.urdf:68-74
           inertia=(0.0001, 0.0, 0.0, 0.0001, 0.0, 0.0001))
# per leg: (sx, sy) sign of x (front +) and y (left +)
LEG_SIGNS = {"FL": (1, 1), "FR": (1, -1), "RL": (-1, 1), "RR": (-1, -1)}
HIP_OFFSET = (0.1881, 0.04675, 0.0)      # go1.urdf:91,214,337,460
THIGH_OFFSET_Y = 0.08                     # go1.urdf:133,256,379,502
CALF_OFFSET = (0.0, 0.0, -0.213)          # go1.urdf:161
FOOT_OFFSET = (0.0, 0.0, -0.213)          # go1.urdf:189
FOOT_RADIUS = 0.02                        # go1.urdf:202-204
# FR values; mirrored per leg below (go1.urdf:113-115, 155-157, 183-185, 208-209)
HIP_FR = dict(mass=0.510299, com=(-0.00541, 0.00074, 6e-06),
              inertia=(0.00030528937, 7.788013e-06, 2.2016e-07, 0.000590894859, 1.7175e-08, 0.000396594572))
THIGH_FR = dict(mass=0.898919, com=(-0.003468, 0.018947, -0.032736),
                inertia=(0.005395867678, -1.02809e-07, 0.000337529085, 0.005142451046, 5.816563e-06, 0.00102478732))
CALF = dict(mass=0.158015, com=(0.006286, 0.001307, -0.122269),
            inertia=(0.003607648222, 1.494971e-06, -0.000132778525, 0.003626771492, -2.8638535e-05, 3.5148003e-05))
FOOT = dict(mass=0.06, com=(0.0, 0.0, -0.213), inertia=(9.6e-06, 0.0, 0.0, 9.6e-06, 0.0, 9.6e-06))
TRUNK_BOX = (0.3762, 0.0935, 0.114)       # go1.urdf:54-56
THIGH_BOX_HALF_WIDTH = 0.0245 / 2         # go1.urdf:148-153 (0.213 x 0.0245 x 0.034)
CALF_BOX_HALF_WIDTH = 0.016 / 2           # go1.urdf:176-181
# hip collision cylinder, axis along the hip link's y, centred 0.045 m outboard of the hip joint
# (go1.urdf:106-111 FR at y = -0.045, :229-234 FL at +0.045); Isaac Gym's
# replace_cylinder_with_capsule (legged_robot_trajectory_tracking_config.py:214-215) makes it a capsule of
# the same radius whose segment is the cylinder's axis (half length 0.02).  A capsule's deepest point
# against a locally planar surface is an end of its segment, so the native model carries the two
# segment ends as spheres of the capsule's radius (FL values; y mirrors with the side).
HIP_CAPSULE_RADIUS = 0.046
HIP_CAPSULE_Y = (0.045 - 0.02, 0.045 + 0.02)


def _mirror(body, sx, sy):
    """Mirror an FR-frame body into leg (sx, sy): URDF mirrors y for left legs and
    x of the hip COM for rear legs; products of inertia flip with the mirrored axes."""
    m = body["mass"]
    cx, cy, cz = body["com"]
    ixx, ixy, ixz, iyy, iyz, izz = body["inertia"]
    fy = -1 if sy > 0 else 1  # FR is the reference (right)
    return dict(mass=m, com=(cx, cy * fy, cz), inertia=(ixx, ixy * fy, ixz, iyy, iyz * fy, izz))


def _hip(leg):
    sx, sy = LEG_SIGNS[leg]
    b = _mirror(HIP_FR, sx, sy)
    if sx < 0:  # rear hips mirror x as well (go1.urdf:359-361, 482-484)
        cx, cy, cz = b["com"]
        ixx, ixy, ixz, iyy, iyz, izz = b["inertia"]
        b = dict(mass=b["mass"], com=(-cx, cy, cz), inertia=(ixx, -ixy, -ixz, iyy, iyz, izz))
    return b


def _thigh(leg):
    sx, sy = LEG_SIGNS[leg]
    return _mirror(THIGH_FR, sx, sy)


def _sym(i6):
    ixx, ixy, ixz, iyy, iyz, izz = i6
    return np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]], dtype=np.float64)


def merge(bodies):
    """Merge rigid bodies given in one frame: mass, COM, inertia about the merged COM."""
    m = sum(b["mass"] for b in bodies)
    c = sum(b["mass"] * np.asarray(b["com"], np.float64) for b in bodies) / m
    inertia = np.zeros((3, 3))
    for b in bodies:
        d = np.asarray(b["com"], np.float64) - c
        inertia += _sym(b["inertia"]) + b["mass"] * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    return dict(mass=m, com=tuple(c), inertia=(inertia[0, 0], inertia[0, 1], inertia[0, 2], inertia[1, 1],
                                               inertia[1, 2], inertia[2, 2]))


BASE = merge([TRUNK, IMU])


def leg_bodies(leg):
    hip = _hip(leg)
    thigh = _thigh(leg)
    calf = merge([CALF, FOOT])
    return hip, thigh, calf


def joint_origins(leg):
    sx, sy = LEG_SIGNS[leg]
    hip = (sx * HIP_OFFSET[0], sy * HIP_OFFSET[1], 0.0)
    thigh = (0.0, sy * THIGH_OFFSET_Y, 0.0)
    return hip, thigh, CALF_OFFSET


# ---- flat parameter block consumed by the C-ABI (go1_model in include/go1_mi355x.h)
# Per body: mass, com[3], inertia about COM [xx, xy, xz, yy, yz, zz] (10 floats)
# Base first, then per leg (FL, FR, RL, RR): hip, thigh, calf   -> 13 bodies x 10
# Then per leg: hip origin[3], thigh origin[3], calf origin[3]  -> 4 x 9
# Then foot offset[3], foot radius, trunk half extents[3], thigh radius, calf radius,
# hip capsule radius, hip capsule segment ends y[2] (FL)
MODEL_FLOATS = 13 * 10 + 4 * 9 + 3 + 1 + 3 + 1 + 1 + 1 + 2  # 178


def model_block() -> np.ndarray:
    out = []

    def body(b):
        out.extend([b["mass"], *b["com"], *b["inertia"]])

    body(BASE)
    for leg in L.LEGS:
        for b in leg_bodies(leg):
            body(b)
    for leg in L.LEGS:
        for o in joint_origins(leg):
            out.extend(o)
    out.extend(FOOT_OFFSET)
    out.append(FOOT_RADIUS)
    out.extend([TRUNK_BOX[0] / 2, TRUNK_BOX[1] / 2, TRUNK_BOX[2] / 2])
    out.append(THIGH_BOX_HALF_WIDTH)
    out.append(CALF_BOX_HALF_WIDTH)
    out.append(HIP_CAPSULE_RADIUS)
    out.extend(HIP_CAPSULE_Y)
    a = np.asarray(out, dtype=np.float64)
    assert a.shape == (MODEL_FLOATS,), a.shape
    return a


def total_mass() -> float:
    m = BASE["mass"]
    for leg in L.LEGS:
        m += sum(b["mass"] for b in leg_bodies(leg))
    return m
