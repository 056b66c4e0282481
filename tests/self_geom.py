"""Numpy kinematics of the 16 self-collision primitives in the trunk frame (shares nothing with the kernel or the
oracle): the self-collision tests' pose pools, the fold-gate soundness check (go1_device.h self_broad) and the
coverage properties of the capsule geometry (tests/test_self_collision.py).

Primitive 4 l + k of leg l (k: 0 thigh capsule, 1 hip capsule, 2 calf capsule, 3 foot sphere; model.py and
oracle/go1_oracle.c for the geometry): segment ends (.., 2, 3) and radius; the foot is a degenerate segment."""
import numpy as np

from legged_tracking_amd import layout as L

# names of the primitives, in order k
KINDS = ("thigh", "hip", "calf", "foot")
# the non-adjacent links of one leg (two joints apart): hip vs calf, hip vs foot, thigh vs foot
SAME = [(1, 2), (1, 3), (0, 3)]


def _rx(q):
    c, s_ = np.cos(q), np.sin(q)
    o, z = np.ones_like(q), np.zeros_like(q)
    return np.stack([np.stack([o, z, z], -1), np.stack([z, c, -s_], -1), np.stack([z, s_, c], -1)], -2)


def _ry(q):
    c, s_ = np.cos(q), np.sin(q)
    o, z = np.ones_like(q), np.zeros_like(q)
    return np.stack([np.stack([c, z, s_], -1), np.stack([z, o, z], -1), np.stack([-s_, z, c], -1)], -2)


def leg_capsules(qh, qt, qk, l=0):
    """(n, 4, 2, 3) segment ends of leg l's primitives in the trunk frame, (4,) radii."""
    from legged_tracking_amd import model as M
    leg = L.LEGS[l]
    n = qh.shape[0]
    P = np.zeros((n, 4, 2, 3))
    o = [np.array(v, np.float64) for v in M.joint_origins(leg)]
    sy = M.LEG_SIGNS[leg][1]
    R0 = _rx(qh)
    p0 = np.broadcast_to(o[0], (n, 3))
    R1 = R0 @ _ry(qt)
    p1 = p0 + R0 @ o[1]
    R2 = R1 @ _ry(qk)
    p2 = p1 + R1 @ o[2]
    foot = p2 + R2 @ np.array(M.FOOT_OFFSET)
    P[:, 0, 0], P[:, 0, 1] = p1, p2                                   # thigh: thigh joint .. knee
    for e in range(2):
        P[:, 1, e] = p0 + R0 @ np.array([0.0, sy * M.HIP_CAPSULE_Y[e], 0.0])  # hip capsule
    P[:, 2, 0], P[:, 2, 1] = p2, foot                                 # calf: knee .. foot
    P[:, 3, 0] = P[:, 3, 1] = foot                                    # foot sphere
    r = np.array([M.THIGH_BOX_HALF_WIDTH, M.HIP_CAPSULE_RADIUS, M.CALF_BOX_HALF_WIDTH, M.FOOT_RADIUS], np.float64)
    return P, r


def capsules(q):
    """(n, 16, 2, 3) segment ends in the trunk frame, (16,) radii: leg l * 4 + k (leg_capsules)."""
    Ps, rs = zip(*(leg_capsules(q[:, 3 * l], q[:, 3 * l + 1], q[:, 3 * l + 2], l) for l in range(4)))
    return np.concatenate(Ps, 1), np.concatenate(rs)


def seg_dist(A0, A1, B0, B1):
    """Distance between the segments A0 -> A1 and B0 -> B1 (batched over the leading axes; exact: the minimum of the
    convex distance over the parameter square, by the same clamped closest-point construction as the oracle)."""
    d1, d2, r = A1 - A0, B1 - B0, A0 - B0
    a = (d1 * d1).sum(-1)
    e = (d2 * d2).sum(-1)
    b = (d1 * d2).sum(-1)
    c = (d1 * r).sum(-1)
    f = (d2 * r).sum(-1)
    ea = np.maximum(a, 1e-30)
    ee = np.maximum(e, 1e-30)
    pa, pe = a > 1e-12, e > 1e-12
    den = a * e - b * b
    s = np.where(den > 1e-12 * ea * ee, np.clip((b * f - c * e) / np.where(den > 0, den, 1.0), 0, 1), 0.0)
    t = (b * s + f) / ee
    lo, hi = pa & pe & (t < 0), pa & pe & (t > 1)
    s = np.where(lo, np.clip(-c / ea, 0, 1), np.where(hi, np.clip((b - c) / ea, 0, 1), s))
    t = np.clip(t, 0, 1)
    # degenerate segments (points)
    s = np.where(pa & ~pe, np.clip(-c / ea, 0, 1), s)
    t = np.where(pa & ~pe, 0.0, t)
    s = np.where(~pa, 0.0, s)
    t = np.where(~pa & pe, np.clip(f / ee, 0, 1), t)
    t = np.where(~pa & ~pe, 0.0, t)
    d = (A0 + s[..., None] * d1) - (B0 + t[..., None] * d2)
    return np.sqrt((d * d).sum(-1))


def _box_sdf(P, th):
    q = np.abs(P) - th
    return np.sqrt((np.maximum(q, 0.0) ** 2).sum(-1)) + np.minimum(q.max(-1), 0.0)


def seg_box_dist(A0, A1, th, iters=48):
    """Signed distance of the segment A0 -> A1 to the box of half extents th about the origin (negative inside):
    the box's signed distance is convex, hence convex along the segment -- golden-section search (0.618^48 of the
    segment), batched over the leading axes."""
    g = (np.sqrt(5.0) - 1.0) / 2.0
    d = A1 - A0
    lo, hi = np.zeros(A0.shape[:-1]), np.ones(A0.shape[:-1])
    f = lambda t: _box_sdf(A0 + t[..., None] * d, th)  # noqa: E731
    x1, x2 = hi - g * (hi - lo), lo + g * (hi - lo)
    f1, f2 = f(x1), f(x2)
    for _ in range(iters):
        left = f1 <= f2  # the minimum lies in [lo, x2]
        hi = np.where(left, x2, hi)
        lo = np.where(left, lo, x1)
        nx1, nx2 = hi - g * (hi - lo), lo + g * (hi - lo)
        fn = f(np.where(left, nx1, nx2))
        x1, x2, f1, f2 = (np.where(left, nx1, x2), np.where(left, x1, nx2), np.where(left, fn, f2),
                          np.where(left, f1, fn))
    t = 0.5 * (lo + hi)
    return np.minimum(np.minimum(f(t), f(np.zeros_like(t))), f(np.ones_like(t)))


def pair_classes(P, r):
    """(n, n_classes) overlap flags and the class names: every cross-leg pair (la, lb, a, b), every same-leg pair
    (l, SAME[p]), the thigh / calf capsules and the foot against the trunk box (l, k)."""
    from legged_tracking_amd import model as M
    cols, names = [], []
    for la in range(4):
        for lb in range(la + 1, 4):
            for a in range(4):
                for b in range(4):
                    A, B = P[:, 4 * la + a], P[:, 4 * lb + b]
                    cols.append(seg_dist(A[:, 0], A[:, 1], B[:, 0], B[:, 1]) < r[4 * la + a] + r[4 * lb + b])
                    names.append(("cross", la, lb, a, b))
    for l in range(4):
        for a, b in SAME:
            A, B = P[:, 4 * l + a], P[:, 4 * l + b]
            cols.append(seg_dist(A[:, 0], A[:, 1], B[:, 0], B[:, 1]) < r[4 * l + a] + r[4 * l + b])
            names.append(("same", l, a, b))
    th = np.array(M.TRUNK_BOX) / 2
    for l in range(4):
        for k in (0, 2, 3):
            A = P[:, 4 * l + k]
            cols.append(seg_box_dist(A[:, 0], A[:, 1], th) < r[4 * l + k])
            names.append(("box", l, k))
    return np.stack(cols, 1), names
