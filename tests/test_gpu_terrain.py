"""Tunnel terrain generated on the GPU (go1_tunnel_tiles) vs the host restatement.

terrain.make_single_path is pinned to the reference's own tiles by tests/test_terrain.py (fixture
made by importing the reference, np.random seed 11).  The device generator draws numpy's legacy
MT19937 stream itself and must give the same float32 tiles bit for bit, for the README grid
(32 x 32 sub-terrains) and for the variants train.py exposes (empty tunnel p_flat = 0, single /
double wedges p_double = 0 / 1), and through the env's own construction path.
"""
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from legged_tracking_amd import config as CF, native, terrain as T  # noqa: E402

DEV = "cuda:0"


def _device_tiles(cfg, seed):
    lay = T.tunnel_layout(cfg.terrain)
    return native.tunnel_tiles(cfg.terrain, lay, seed, torch.device(DEV)).cpu().numpy()


@pytest.mark.parametrize("rows,cols,seed", [(4, 4, 11), (32, 32, 11), (8, 16, 3), (32, 32, 4294967295)])
def test_device_tiles_bit_exact_vs_host(rows, cols, seed):
    cfg = CF.readme_config(n_envs=rows * cols, terrain="single_path", rows=rows, cols=cols)
    t0 = time.perf_counter()
    host, _, _ = T.make_single_path(cfg.terrain, np.random.RandomState(seed))
    t_host = time.perf_counter() - t0
    _device_tiles(cfg, seed)  # first call loads the library
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev = _device_tiles(cfg, seed)
    t_dev = time.perf_counter() - t0
    print(f"\ntunnel tiles {rows}x{cols} seed {seed}: host numpy {t_host * 1e3:.1f} ms, "
          f"GPU {t_dev * 1e3:.2f} ms (incl. D2H)")
    assert dev.shape == host.shape
    np.testing.assert_array_equal(dev.view(np.uint32), host.view(np.uint32))


@pytest.mark.parametrize("p_flat,p_double", [(0.0, 0.6), (0.9, 0.0), (0.9, 1.0)])
def test_device_tiles_variants(p_flat, p_double):
    cfg = CF.readme_config(n_envs=64, terrain="single_path", rows=8, cols=8)
    cfg.terrain.p_flat = p_flat
    cfg.terrain.p_double = p_double
    host, _, _ = T.make_single_path(cfg.terrain, np.random.RandomState(5))
    dev = _device_tiles(cfg, 5)
    np.testing.assert_array_equal(dev.view(np.uint32), host.view(np.uint32))
    if p_flat == 0.0:  # empty tunnel: no obstacles inside (ceiling 0.8 m, floor 0 with 0.5 m walls)
        assert np.all(dev[:, :, 0, 4:76, 11:29] == np.float32(0.8))


def test_env_builds_its_tiles_on_the_gpu():
    from legged_tracking_amd.env import TrajectoryTrackingEnv
    cfg = CF.readme_config(n_envs=256, terrain="single_path", rows=4, cols=8)
    env = TrajectoryTrackingEnv(sim_device=DEV, cfg=cfg, seed=5)
    assert isinstance(env.terrain.tiles, torch.Tensor) and env.terrain.tiles.is_cuda
    host = T.build(cfg, 256, np.random.RandomState(env.seed))
    np.testing.assert_array_equal(env.terrain.tiles.cpu().numpy(), host.tiles)
    np.testing.assert_array_equal(env.terrain.env_tile, host.env_tile)
    np.testing.assert_array_equal(env.terrain.env_origins, host.env_origins)


def test_device_tiles_match_reference_full_grid():
    """Against the reference's own tiles directly: the README grid (32 x 32 sub-terrains) the reference
    built after np.random.seed(17) (tests/golden/step_full_grid.npz, one env per sub-terrain)."""
    from tests import golden_io as G
    d = G.load("step_full_grid.npz")
    cfg = CF.readme_config(n_envs=1024, terrain="single_path", rows=32, cols=32)
    dev = _device_tiles(cfg, 17).reshape(1024, 2, 80, 40)
    env_tile = np.arange(1024) % 1024
    np.testing.assert_array_equal(dev[env_tile], d["static/env_height_samples"])
