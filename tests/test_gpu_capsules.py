"""The capsule links against the triangle-mesh floor on the MI355X (round 6): the HIP step's deepest
point of a link segment (go1_device.h seg_deepest: ends, grid-line and diagonal crossings) against the f64 oracle, on
the case the round-3..5 sphere chains failed -- a single floor vertex raised under any point along the thigh or calf.

32 envs, one sub-terrain tile each (single_path layout, README configuration at decimation 1, so the reported
forces are those of the given state): every tile flat far below the robot except one vertex on a one-cell plateau,
4 mm into the capsule close under the link's axis at one of 16 positions from the joint to the link's end, for the
FL thigh held level (calf hanging) and the FL calf held level.  The link's reported contact force is upward and
above 10 N in every env, and every body's reported force equals the oracle's within 1e-3 relative (the point and
its triangle are chosen by quantised keys, so f32 and f64 pick the same one; the force then differs by rounding).  The oracle-only form of the
same property, with the sphere chains' misses counted, is tests/test_capsules.py."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from legged_tracking_amd import config as CF, native, terrain as T  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.self_geom import leg_capsules  # noqa: E402

DEV = "cuda:0"
STAND = np.array([0.1, 0.8, -1.5, -0.1, 0.8, -1.5, 0.1, 1.0, -1.5, -0.1, 1.0, -1.5], np.float32)


def test_link_over_a_raised_floor_vertex_step_vs_oracle():
    n = 32
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=4, cols=8)
    cfg.control.decimation = 1
    c = CF.build_abi_config(cfg)
    c.camera_zero = 0
    td = T.build(cfg, n, np.random.RandomState(11))
    assert td.tiles.shape[0] == n and (td.env_tile == np.arange(n)).all()
    hs = float(c.horizontal_scale)
    i0, j0 = 40, 20
    st = O.NpState(n, cfg=c)
    ter0 = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    O.reset_envs(c, st, ter0, np.ones(n, np.uint8), rng_seed=3, rng_step=0)
    tiles = np.empty_like(td.tiles)
    tiles[:, 0] = 3.0    # ceiling far above
    tiles[:, 1] = -1.0   # floor far below
    body_idx = []
    for e in range(n):
        kind = 0 if e < n // 2 else 2                 # FL thigh, then FL calf
        t = (e % (n // 2) + 0.5) / (n // 2)            # 16 positions along the link
        q = STAND.copy()
        q[0:3] = [0.0, np.pi / 2, -np.pi / 2] if kind == 0 else [0.0, 0.0, -np.pi / 2]
        P, r = leg_capsules(*(np.array([q[j]], np.float64) for j in range(3)), l=0)
        p = P[0, kind, 0] + t * (P[0, kind, 1] - P[0, kind, 0])
        org = td.env_terrain_origin[e].astype(np.float64)
        # the axis passes 1.3 mm / 0.7 mm off the vertex: exactly over it, the contact normal is any of its six
        # triangles', and f32 and f64 round a coordinate on a grid line to different sides
        local = np.array([i0 * hs - p[0] + 0.0013, j0 * hs - p[1] + 0.0007, 0.6])
        zc = local[2] + p[2]
        tiles[e, 1, i0 - 1:i0 + 2, j0 - 1:j0 + 2] = zc - r[kind] + 0.004 - 0.03  # one-cell plateau 3 cm lower
        tiles[e, 1, i0, j0] = zc - r[kind] + 0.004                               # the vertex, 4 mm into the capsule
        st["root"][e, 0:2] = (org[:2] + local[:2]).astype(np.float32)
        st["root"][e, 2] = np.float32(local[2])
        st["root"][e, 3:7] = [0.0, 0.0, 0.0, 1.0]
        st["root"][e, 7:13] = 0.0
        st["dof_pos"][e] = q
        st["dof_vel"][e] = 0.0
        body_idx.append(1 + (1 if kind == 0 else 2))  # FL thigh / calf in the 17-body layout
    st["episode_length"][:, 0] = 10
    td.tiles[:] = tiles
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    g = native.Go1Native(c, DEV)
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    g.state.load(st.arrays)
    gr, gvec = CF.gravity_state([0.0, 0.0, 0.0])
    scales = np.zeros(c.n_terms, np.float32)
    a = np.zeros((n, 12), np.float32)
    g.step(torch.from_numpy(a).to(DEV), gvec, gr, scales, rng_seed=5, rng_step=300)
    torch.cuda.synchronize()
    out = O.step(c, st, ter, a, gvec, gr, scales, rng_seed=5, rng_step=300, debug=False)
    cf = g.contact_forces.cpu().numpy()
    ref = out["contact_forces"]
    link = cf[np.arange(n), body_idx]
    link_ref = ref[np.arange(n), body_idx]
    print(f"\nlink forces z: GPU min {link[:, 2].min():.1f} N, oracle min {link_ref[:, 2].min():.1f} N; "
          f"max |dF| {np.abs(link - link_ref).max():.2e} N")
    assert (link[:, 2] > 10.0).all(), link[:, 2]
    assert (link_ref[:, 2] > 10.0).all(), link_ref[:, 2]
    # every body's reported force (the calf or foot hanging from a knee over the plateau touches it too)
    np.testing.assert_allclose(cf, ref, rtol=1e-3, atol=1e-3)
