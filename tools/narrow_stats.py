"""The narrow phase's candidate pairs in the bench workload's steady state (CPU study; input from
tools/dump_states.py on the GPU box): per env, the primitive pairs whose world-axis boxes overlap (what the
kernel's partner tests let through) against the pairs that touch, and the fold gate.
  python tools/narrow_stats.py gpurun_out/bench_states.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from legged_tracking_amd import layout as L  # noqa: E402
from tests.self_geom import SAME, capsules, seg_dist  # noqa: E402


def quat_R(q):
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
                     np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
                     np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)


def main():
    d = np.load(sys.argv[1])
    lim = np.array(L.JOINT_LIMITS)
    for key in sorted(k for k in d if k.startswith("root_")):
        step = key.split("_")[1]
        root, q = d[key].astype(np.float64), d["dof_pos_" + step].astype(np.float64)
        n = len(q)
        P, r = capsules(q)                                      # (n, 16, 2, 3) trunk frame
        R = quat_R(root[:, 3:7])
        W = np.einsum("nij,nkej->nkei", R, P) + root[:, None, None, 0:3]
        lo = W.min(2) - r[None, :, None]
        hi = W.max(2) + r[None, :, None]
        ov = np.all((lo[:, :, None] <= hi[:, None]) & (lo[:, None] <= hi[:, :, None]), -1)
        leg = np.arange(16) // 4
        qq = q.reshape(n, 4, 3)
        wild = ((qq < lim[None, :, 0] - 0.1) | (qq > lim[None, :, 1] + 0.1)).any(2)  # (n, 4)
        same = np.zeros((16, 16), bool)
        for l in range(4):
            for a, b in SAME:
                same[4 * l + a, 4 * l + b] = same[4 * l + b, 4 * l + a] = True
        allowed = (leg[:, None] != leg[None, :])[None] | (same[None] & wild[:, leg][:, :, None])
        cand = ov & allowed
        A, B = W[:, :, None], W[:, None]
        dist = seg_dist(np.broadcast_to(A[..., 0, :], (n, 16, 16, 3)), np.broadcast_to(A[..., 1, :], (n, 16, 16, 3)),
                        np.broadcast_to(B[..., 0, :], (n, 16, 16, 3)), np.broadcast_to(B[..., 1, :], (n, 16, 16, 3)))
        touch = cand & (dist < r[:, None] + r[None, :])
        per_lane = cand.sum(2).max(1)   # the pair loop's trips for the env (its busiest primitive)
        per_lane_touch = touch.sum(2).max(1)
        waves = per_lane.reshape(-1, 4).max(1)
        print(f"step {step}: envs with a candidate pair {np.mean(per_lane > 0):.3f}, touching {np.mean(per_lane_touch > 0):.3f};"
              f" legs past the fold band {wild.mean():.3f}")
        print("  busiest primitive's candidates per env (hist):", np.bincount(per_lane)[:10].tolist())
        print("  ... of which touching:", np.bincount(per_lane_touch)[:10].tolist())
        print("  pair-loop trips per wave (hist):", np.bincount(waves)[:12].tolist())
        cross = cand & (leg[:, None] != leg[None, :])[None]
        print(f"  candidate pairs: cross-leg {cross.sum() // 2}, same-leg {(cand & ~cross).sum() // 2}; touching "
              f"{touch.sum() // 2}")


if __name__ == "__main__":
    main()
