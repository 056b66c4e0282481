"""Terrain producer vs the reference's tiles (golden fixture generated with np.random.seed(11))."""
import numpy as np

from legged_tracking_amd import config as CF, terrain as T
from tests import golden_io as G


def test_single_path_tiles_bit_exact():
    d = G.load("step_single_path.npz")
    cfg = CF.readme_config(n_envs=64, terrain="single_path", rows=4, cols=4)
    rng = np.random.RandomState(11)
    td = T.build(cfg, 64, rng)
    ref = d["static/env_height_samples"]
    got = td.tiles[td.env_tile]
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(td.env_terrain_origin, d["static/env_terrain_origin"])
    np.testing.assert_array_equal(td.env_origins, d["static/env_origins"])


def test_tunnel_layout_properties():
    cfg = CF.readme_config(n_envs=256, terrain="single_path", rows=4, cols=8)
    td = T.build(cfg, 256, np.random.RandomState(3))
    assert td.tiles.shape == (32, 2, 80, 40)
    ceil, floor = td.tiles[:, 0], td.tiles[:, 1]
    # outside the 72 x 20 px tunnel: ceiling 0.8 m, floor 0.5 m (tunnel.py:80-81)
    assert np.all(ceil[:, :4] == np.float32(0.8)) and np.all(floor[:, :, :10] == np.float32(0.5))
    # tunnel side walls are 0.5 m floor pixels (tunnel_fn.py:155-159)
    assert np.all(floor[:, 4:76, 10] == np.float32(0.5)) and np.all(floor[:, 4:76, 29] == np.float32(0.5))
    # ceiling obstacles are clamped >= 0.05 m (tunnel.py:96-98)
    assert ceil.min() >= np.float32(0.05) - 1e-7
    assert np.all(td.env_tile == np.arange(256) % 32)


def test_plane_grid_origins():
    cfg = CF.readme_config(n_envs=10, terrain="plane")
    td = T.build(cfg, 10)
    assert td.kind == "plane"
    np.testing.assert_array_equal(td.env_origins[:4, :2], [[0, 0], [0, 3], [0, 6], [3, 0]])


def test_full_readme_grid_tiles_bit_exact():
    """The README grid at full size (32 x 32 sub-terrains, fixture step_full_grid.npz: the
    reference's Terrain built after np.random.seed(17), one env per sub-terrain)."""
    d = G.load("step_full_grid.npz")
    cfg = CF.readme_config(n_envs=1024, terrain="single_path", rows=32, cols=32)
    td = T.build(cfg, 1024, np.random.RandomState(17))
    np.testing.assert_array_equal(td.tiles[td.env_tile], d["static/env_height_samples"])
    np.testing.assert_array_equal(td.env_terrain_origin, d["static/env_terrain_origin"])
    np.testing.assert_array_equal(td.env_origins, d["static/env_origins"])


def test_device_generator_rejects_extents_that_do_not_fit_the_sub_terrain():
    """native.tunnel_tiles checks every tunnel extent against the SubTerrain shape before any device
    work: the reference's tile[0, sx:ex, sy:ey] = top.T (tunnel.py:193-196) raises on a mismatch,
    where the device rasteriser would extrapolate silently."""
    import pytest
    from legged_tracking_amd import native
    cfg = CF.readme_config(n_envs=64, terrain="single_path", rows=4, cols=4)
    lay = T.tunnel_layout(cfg.terrain)
    span = np.stack([lay.extents[:, 1] - lay.extents[:, 0], lay.extents[:, 3] - lay.extents[:, 2]], 1)
    assert (span == np.array([lay.sub_shape[1], lay.sub_shape[0]])).all()  # the README grid fits
    lay.extents = lay.extents.copy()
    lay.extents[5, 1] += 1
    with pytest.raises(ValueError, match="sub-terrain 5"):
        native.tunnel_tiles(cfg.terrain, lay, 11, "cpu")
