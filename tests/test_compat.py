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
