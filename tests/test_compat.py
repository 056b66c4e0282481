"""The reference's unchanged scripts/train.py runs on this package (legged_tracking_amd.compat).

Container-only (marker `reference`: skipped where /root/reference is absent, e.g. on the
GPU box).  The step and the rollout kernels are replaced by their CPU test doubles so
the script's plumbing -- argument parsing, Cfg mutation, TrajectoryTrackingEnv /
HistoryWrapper / Runner construction, one learning iteration, checkpoint writing --
is exercised here; everything is written under the test's tmp directory.
"""
import os
import subprocess
import sys
import textwrap

import pytest

REF_TRAIN = "/root/reference/scripts/train.py"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = [pytest.mark.reference,
              pytest.mark.skipif(not os.path.exists(REF_TRAIN), reason="reference checkout not present")]


def test_reference_train_script_runs_through_compat(tmp_path):
    script = tmp_path / "run.py"
    script.write_text(textwrap.dedent(f"""
        import sys
        sys.dont_write_bytecode = True
        sys.path.insert(0, {REPO!r})
        from legged_tracking_amd import compat, env as E, rollout as R
        from tests.cpu_backend import OracleBackend
        from tests.rollout_ref import TorchRolloutKernels
        init = E.LeggedRobot.__init__
        def env_init(self, cfg, *a, **k):
            k["backend"] = OracleBackend
            return init(self, cfg, *a, **k)
        E.LeggedRobot.__init__ = env_init
        st_init = R.RolloutStorage.__init__
        def storage_init(self, *a, **k):
            k["kernels"] = TorchRolloutKernels()
            return st_init(self, *a, **k)
        R.RolloutStorage.__init__ = storage_init
        run_init = R.Runner.__init__
        def runner_init(self, env, device="cpu", *a, **k):
            return run_init(self, env, "cpu", *a, **k)
        R.Runner.__init__ = runner_init
        R.RunnerArgs.num_steps_per_env = 4
        R.PPO_Args.num_learning_epochs = 1
        compat.main([{REF_TRAIN!r}, "--headless", "--old_ppo", "--terrain", "single_path",
                     "--measure_front_half", "--camera_zero", "--penalty_scaler", "1.0", "--strategy", "e2e",
                     "--terminal_body_height", "0.0", "--device", "0", "--logdir", {str(tmp_path / "logs")!r}])
        import go1_gym.envs.go1.trajectory_tracking as tt
        print("RAN", R.RunnerArgs.save_video_interval)
    """))
    env = dict(os.environ, GO1_NUM_ENVS="1024", GO1_MAX_ITERATIONS="1", GO1_GYM_ROOT=str(tmp_path),
               PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg")
    r = subprocess.run([sys.executable, str(script)], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "RAN 500" in r.stdout  # train.py:243 mutated the RunnerArgs we exported
    ck = tmp_path / "last_run" / "checkpoints"
    for f in ("ac_weights.pt", "body_latest.jit", "adaptation_module_latest.jit"):
        assert (ck / f).exists(), f


REF_TRAIN_VEL = "/root/reference/scripts/train_velocity_tracking.py"


@pytest.mark.skipif(not os.path.exists(REF_TRAIN_VEL), reason="reference checkout not present")
def test_reference_velocity_train_script_reaches_the_velocity_env(tmp_path):
    """scripts/train_velocity_tracking.py (BASELINE configs[1]) through compat: the script's own Cfg edits
    land on the velocity Cfg mirror, and the env it constructs gets a configuration the HIP velocity step
    accepts and that equals velocity_config.train_velocity_config (on the plane).  The env constructor is
    intercepted after build_configs (no GPU here)."""
    script = tmp_path / "run_vel.py"
    script.write_text(textwrap.dedent(f"""
        import sys
        sys.dont_write_bytecode = True
        sys.path.insert(0, {REPO!r})
        import numpy as np
        from legged_tracking_amd import compat, velocity as VEL, velocity_config as V
        class Done(Exception):
            pass
        def env_init(self, sim_device="cuda:0", headless=True, num_envs=None, prone=False, deploy=False, cfg=None,
                     *a, **k):
            if num_envs is not None:  # as the env does (velocity_tracking/__init__.py:15-16)
                cfg.env.num_envs = num_envs
            c, v, grid, w0, names, sums = VEL.build_configs(cfg)
            c2, v2, grid2, w02, names2, sums2 = VEL.build_configs(V.train_velocity_config(n_envs=cfg.env.num_envs))
            assert bytes(v) == bytes(v2) and bytes(c) == bytes(c2) and names == names2
            assert np.array_equal(grid, grid2) and np.array_equal(w0, w02)
            print("VEL_ENV_OK", cfg.env.num_envs, cfg.terrain.mesh_type, len(names))
            raise Done()
        VEL.VelocityTrackingEasyEnv.__init__ = env_init
        try:
            compat.main([{REF_TRAIN_VEL!r}])
        except Done:
            pass
    """))
    env = dict(os.environ, GO1_NUM_ENVS="4096", GO1_GYM_ROOT=str(tmp_path), PYTHONDONTWRITEBYTECODE="1",
               MPLBACKEND="Agg")
    r = subprocess.run([sys.executable, str(script)], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "VEL_ENV_OK 4096 plane 19" in r.stdout, r.stdout[-2000:]
    # the rewrite of the script's trimesh terrain is announced, never silent
    assert "mesh_type 'trimesh' is replaced by 'plane'" in r.stderr, r.stderr[-2000:]
