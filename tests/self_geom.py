"""Numpy kinematics of the 32 self-collision spheres in the trunk frame (shares nothing with the kernel or the
oracle): the self-collision tests' pose pools and the fold-gate soundness check (go1_device.h self_broad)."""
import numpy as np

from legged_tracking_amd import layout as L


def _rx(q):
    c, s_ = np.cos(q), np.sin(q)
    o, z = np.ones_like(q), np.zeros_like(q)
    return np.stack([np.stack([o, z, z], -1), np.stack([z, c, -s_], -1), np.stack([z, s_, c], -1)], -2)


def _ry(q):
    c, s_ = np.cos(q), np.sin(q)
    o, z = np.ones_like(q), np.zeros_like(q)
    return np.stack([np.stack([c, z, s_], -1), np.stack([z, o, z], -1), np.stack([-s_, z, c], -1)], -2)


def leg_spheres(qh, qt, qk, l=0):
    """(n, 8, 3) centres of leg l's spheres in the trunk frame, (8,) radii: s = thigh 0-2, calf 3-4, foot 5,
    hip-capsule ends 6-7 (go1_device.h self-collision; model.py for the geometry)."""
    from legged_tracking_amd import model as M
    leg = L.LEGS[l]
    n = qh.shape[0]
    P = np.zeros((n, 8, 3))
    o = [np.array(v, np.float64) for v in M.joint_origins(leg)]
    sy = M.LEG_SIGNS[leg][1]
    R0 = _rx(qh)
    p0 = np.broadcast_to(o[0], (n, 3))
    R1 = R0 @ _ry(qt)
    p1 = p0 + R0 @ o[1]
    R2 = R1 @ _ry(qk)
    p2 = p1 + R1 @ o[2]
    for k in range(3):
        P[:, k] = p1 + R1 @ np.array([0.0, 0.0, -0.071 * (k + 1)])
    for k in range(2):
        P[:, 3 + k] = p2 + R2 @ np.array([0.0, 0.0, -0.071 * (k + 1)])
    P[:, 5] = p2 + R2 @ np.array(M.FOOT_OFFSET)
    for k in range(2):
        P[:, 6 + k] = p0 + R0 @ np.array([0.0, sy * M.HIP_CAPSULE_Y[k], 0.0])
    r = np.array([M.THIGH_BOX_HALF_WIDTH] * 3 + [M.CALF_BOX_HALF_WIDTH] * 2 + [M.FOOT_RADIUS] +
                 [M.HIP_CAPSULE_RADIUS] * 2, np.float64)
    return P, r


def spheres(q):
    """(n, 32, 3) centres in the trunk frame, (32,) radii: leg l * 8 + s (leg_spheres)."""
    Ps, rs = zip(*(leg_spheres(q[:, 3 * l], q[:, 3 * l + 1], q[:, 3 * l + 2], l) for l in range(4)))
    return np.concatenate(Ps, 1), np.concatenate(rs)


SAME = [(6, 3), (6, 4), (6, 5), (7, 3), (7, 4), (7, 5), (0, 5), (1, 5), (2, 5)]


def pair_classes(P, r):
    """(n, n_classes) overlap flags and the class names: every cross-leg pair (la, lb, a, b), every same-leg pair
    (l, SAME[p]), every thigh / calf / foot sphere against the trunk box."""
    from legged_tracking_amd import model as M
    cols, names = [], []
    for la in range(4):
        for lb in range(la + 1, 4):
            for a in range(8):
                for b in range(8):
                    d = P[:, 8 * la + a] - P[:, 8 * lb + b]
                    cols.append((d * d).sum(-1) < (r[8 * la + a] + r[8 * lb + b]) ** 2)
                    names.append(("cross", la, lb, a, b))
    for l in range(4):
        for a, b in SAME:
            d = P[:, 8 * l + a] - P[:, 8 * l + b]
            cols.append((d * d).sum(-1) < (r[8 * l + a] + r[8 * l + b]) ** 2)
            names.append(("same", l, a, b))
    th = np.array(M.TRUNK_BOX) / 2
    for l in range(4):
        for s in range(6):
            c = P[:, 8 * l + s]
            d = c - np.clip(c, -th, th)
            cols.append((d * d).sum(-1) < r[8 * l + s] ** 2)
            names.append(("box", l, s))
    return np.stack(cols, 1), names
