"""Tunnel terrain tiles for the height scan and the contact model (host, init-time).

Restates the reference's terrain producer for the two terrains on this path:
  * single_path -- go1_gym/utils/tunnel_fn.py:99-163 (TerrainFunctions.single_path)
    placed by go1_gym/utils/tunnel.py:51-126, 189-217 (Terrain.__init__ /
    add_terrain_to_map), including the ceiling flip and 0.05 m clamp (:96-98),
    the 0.8 m ceiling / 0.5 m floor outside the tunnel (:80-81) and the global
    numpy RNG draw order, so a seeded run reproduces the reference's tiles
    bit for bit (tests/test_terrain.py vs the golden fixture);
  * plane -- no tiles (legged_robot_trajectory_tracking.py:1928-1932).

Output layout (HBM, one copy per unique sub-terrain; envs index it):
  tiles (n_rows*n_cols, 2, L, W) f32, layer 0 ceiling, layer 1 floor, metres;
  env_tile, env_terrain_origin, env_origins per env (legged_robot_trajectory_tracking.py:1816-1840).
"""
from dataclasses import dataclass

import numpy as np


@dataclass
class TerrainData:
    tiles: np.ndarray             # (S, 2, L, W) f32
    env_tile: np.ndarray          # (N,) int32
    env_terrain_origin: np.ndarray  # (N, 3) f32
    env_origins: np.ndarray       # (N, 3) f32
    kind: str


def _faces_height(wedges, xy):
    """Height of the union of pyramidal wedges at points xy (px, py, 2).

    A wedge is 4 triangular faces sharing an apex; each face is a plane
    z = d/c - a/c x - b/c y (normal (a, b, c) = (p3-p1) x (p3-p2)), clipped at 0;
    a wedge's height is the min over its faces, the union is the max over wedges."""
    px, py = xy.shape[:2]
    pts = xy.reshape(-1, 2)
    p1, p2, p3 = wedges[:, :, 0, :], wedges[:, :, 1, :], wedges[:, :, 2, :]
    n = np.cross(p3 - p1, p3 - p2)
    a, b, c = n[..., 0], n[..., 1], n[..., 2]
    d = np.sum(n * p3, axis=-1)
    assert np.all(c != 0)
    h = (d / c)[..., None] - (a / c)[..., None] * pts[:, 0] - (b / c)[..., None] * pts[:, 1]
    h = np.clip(h, 0, a_max=np.inf)
    return h.min(axis=1).max(axis=0).reshape(px, py)


def single_path_layer(shape, hs, vs, p_flat, p_double, top, rng=np.random):
    """One layer of one sub-terrain (tunnel_fn.py:99-163), integer height units."""
    pixel_x, pixel_y = shape
    l, w = pixel_x * hs, pixel_y * hs
    p1 = rng.uniform()
    p2 = rng.uniform()
    num_y = 2 if p2 < p_double else 1
    if top:
        off_y = rng.uniform(-0.6, 0.6, size=(num_y, 1))
        off_x = rng.uniform(-0.3, 0.3, size=(num_y, 1))
        hmax, hmin = (0.4, 0.7) if p1 < p_flat else (0.0, 0.0)
        lo, hi = 0.2, 0.4
    else:
        off_y = rng.uniform(-0.4, 0.4, size=(num_y, 1))
        off_x = rng.uniform(-0.2, 0.2, size=(num_y, 1))
        hmax, hmin = (0.15, 0.3) if p1 < p_flat else (0.0, 0.0)
        lo, hi = 0.1, 0.3
    cx = np.linspace(-w / 2, w / 2, 3)[1:-1]
    mx, my = np.meshgrid(cx, np.zeros(num_y))
    my = my + off_y
    mx = mx + off_x
    mz = rng.uniform(mx) * (hmax - hmin) + hmin  # numpy uniform(low=mx, high=1.0)
    centres = np.stack([mx.flatten(), my.flatten(), mz.flatten()], axis=1)
    pw, pl = rng.uniform(low=lo, high=hi, size=(2, centres.shape[0]))
    zero = np.zeros_like(pw)
    corners = [np.stack([sx * pw + centres[:, 0], sy * pl + centres[:, 1], zero], axis=1)
               for sx, sy in ((1, 1), (-1, 1), (-1, -1), (1, -1))]
    verts = np.stack(corners + [centres], axis=1)           # (k, 5, 3): 4 base corners + apex
    faces = verts[:, [[0, 1, 4], [1, 2, 4], [2, 3, 4], [3, 0, 4]], :]
    grid = np.stack(np.meshgrid(np.linspace(-w / 2, w / 2, pixel_y), np.linspace(-l / 2, l / 2, pixel_x)), axis=-1)
    h = _faces_height(faces, grid)
    if not top:
        h[0, :] = 0.5
        h[-1, :] = 0.5
        h[:, 0] = 0.5
        h[:, -1] = 0.5
    return (h / vs).astype(int)


@dataclass
class TunnelLayout:
    """The RNG-free part of the tunnel grid (tunnel.py:59-77, 189-217)."""
    tile_x: int                 # length_per_env_pixels
    tile_y: int                 # width_per_env_pixels
    sub_shape: tuple            # SubTerrain height_field_raw shape (pixel_x, pixel_y)
    extents: np.ndarray         # (rows * cols, 4) int32: start_x, end_x, start_y, end_y inside the tile
    env_origins: np.ndarray     # (rows, cols, 3)
    all_origins: np.ndarray     # (rows, cols, 3)


def tunnel_layout(cfg_terrain):
    t = cfg_terrain
    hs = t.horizontal_scale
    W = int(t.terrain_width / hs)
    Lp = int(t.terrain_length / hs)
    rows, cols = t.num_rows, t.num_cols
    ext = np.zeros((rows * cols, 4), np.int32)
    env_origins = np.zeros((rows, cols, 3))
    all_origins = np.zeros((rows, cols, 3))
    for k in range(rows * cols):
        i, j = np.unravel_index(k, (rows, cols))
        # add_terrain_to_map (:193-196), relative to the tile
        ext[k] = (int(round((i + 0.5 - t.terrain_ratio_x / 2.) * Lp, 4)) - i * Lp,
                  int(round((i + 0.5 + t.terrain_ratio_x / 2.) * Lp, 4)) - i * Lp,
                  int((j + 0.5 - t.terrain_ratio_y / 2.) * W) - j * W,
                  int((j + 0.5 + t.terrain_ratio_y / 2.) * W) - j * W)
        env_origins[i, j] = [(i + 0.5 - t.start_loc) * t.terrain_length, (j + 0.5) * t.terrain_width, 0.0]
        all_origins[i, j] = [i * t.terrain_length, j * t.terrain_width, 0.0]
    return TunnelLayout(Lp, W, (int(W * t.terrain_ratio_y), int(Lp * t.terrain_ratio_x)), ext, env_origins, all_origins)


def make_single_path(cfg_terrain, rng=np.random):
    """Tiles for a num_rows x num_cols tunnel grid (tunnel.py:51-126, 189-217), host numpy.

    The product env generates the same tiles on the GPU (go1_tunnel_tiles, native.tunnel_tiles);
    this host restatement is the checker the device generator is compared with bit for bit."""
    t = cfg_terrain
    hs, vs = t.horizontal_scale, t.vertical_scale
    lay = tunnel_layout(t)
    Lp, W = lay.tile_x, lay.tile_y
    rows, cols = t.num_rows, t.num_cols
    unit = int(1. / vs)
    tiles = np.empty((rows, cols, 2, Lp, W), np.float64)
    for k in range(rows * cols):
        i, j = np.unravel_index(k, (rows, cols))
        rng.uniform(0.0, 1.0)  # difficulty: drawn, unused by single_path (tunnel.py:90)
        top = single_path_layer(lay.sub_shape, hs, vs, t.p_flat, t.p_double, True, rng)
        bottom = single_path_layer(lay.sub_shape, hs, vs, t.p_flat, t.p_double, False, rng)
        top = t.ceiling_height / vs - top
        top = np.clip(top, a_max=None, a_min=0.05 / vs)
        sx, ex, sy, ey = (int(v) for v in lay.extents[k])
        tile = np.empty((2, Lp, W), np.float64)
        tile[0] = unit * t.ceiling_height
        tile[1] = 0.5 * unit
        tile[0, sx:ex, sy:ey] = top.T
        tile[1, sx:ex, sy:ey] = bottom.T
        tiles[i, j] = tile
    return (tiles * vs).astype(np.float32), lay.env_origins, lay.all_origins


def build(cfg, n_envs, rng=np.random, tiles_fn=None):
    """TerrainData for the envs (legged_robot_trajectory_tracking.py:1808-1858).

    tiles_fn(cfg.terrain, layout) -> tiles replaces the host tile generation (the env passes the
    device generator, native.tunnel_tiles, seeded like `rng`); env origins and tile indices are
    RNG-free and always built here."""
    t = cfg.terrain
    if t.mesh_type == "plane":
        # grid of robots (:1849-1858)
        num_cols = np.floor(np.sqrt(n_envs))
        num_rows = np.ceil(n_envs / num_cols)
        xx, yy = np.meshgrid(np.arange(num_rows), np.arange(num_cols), indexing="ij")
        eo = np.zeros((n_envs, 3), np.float32)
        eo[:, 0] = (cfg.env.env_spacing * xx.flatten()[:n_envs]).astype(np.float32)
        eo[:, 1] = (cfg.env.env_spacing * yy.flatten()[:n_envs]).astype(np.float32)
        return TerrainData(np.zeros((1, 2, 2, 2), np.float32), np.zeros(n_envs, np.int32),
                           np.zeros((n_envs, 3), np.float32), eo, "plane")
    if t.terrain_type != "single_path":
        raise ValueError(f"terrain_type {t.terrain_type!r}: only single_path is on this path "
                         "(multi_path is not implemented in the reference either, README.md:9)")
    if tiles_fn is None:
        tiles, env_origins, all_origins = make_single_path(t, rng)
    else:
        lay = tunnel_layout(t)
        tiles, env_origins, all_origins = tiles_fn(t, lay), lay.env_origins, lay.all_origins
    rows, cols = t.num_rows, t.num_cols
    S = rows * cols
    assert n_envs % S == 0, (n_envs, rows, cols)
    # env e -> sub-terrain (grid_r, grid_c) = divmod(e mod S, cols)  (:1816-1823)
    sub = np.arange(n_envs) % S
    gr, gc = sub // cols, sub % cols
    return TerrainData(tiles.reshape(S, *tiles.shape[2:]), sub.astype(np.int32),
                       all_origins[gr, gc].astype(np.float32), env_origins[gr, gc].astype(np.float32), "single_path")
