"""Run the reference's unchanged scripts/train.py on the MI355X path.

`install()` registers module aliases so that the imports at scripts/train.py:3-26
resolve to this package:

  isaacgym                                            -> placeholder (nothing is called)
  params_proto (PrefixProto, ParamsProto)             -> legged_tracking_amd.config
  go1_gym (MINI_GYM_ROOT_DIR)                         -> $GO1_GYM_ROOT or the working directory
  go1_gym.envs.base.legged_robot_trajectory_tracking_config.Cfg -> config.make_cfg()
  go1_gym.envs.go1.go1_crawling.config_go1            -> config.config_go1
  go1_gym.envs.go1.trajectory_tracking.TrajectoryTrackingEnv -> env.TrajectoryTrackingEnv
  go1_gym.envs.wrappers.history_wrapper.HistoryWrapper -> env.HistoryWrapper
  go1_gym_learn.ppo_cse{,.actor_critic,.ppo}          -> rollout (Runner, RunnerArgs, AC_Args, PPO_Args)
  wandb                                               -> no-op stand-in when wandb is not installed
and, for scripts/train_velocity_tracking.py (BASELINE configs[1]):
  go1_gym.envs.base.legged_robot_velocity_tracking_config.Cfg -> velocity_config.make_vel_cfg()
  go1_gym.envs.go1.go1_config.config_go1              -> velocity_config.config_go1_vel
  go1_gym.envs.go1.velocity_tracking.VelocityTrackingEasyEnv -> velocity.VelocityTrackingEasyEnv
    (on the plane: configs[1] runs the velocity task on a plane, the script's own trimesh terrain is not on
    the accelerated path; GO1_VEL_MESH=trimesh keeps the script's value and raises)

Usage:
  python -m legged_tracking_amd.compat /path/to/legged_tracking/scripts/train.py --headless --old_ppo \\
      --terrain single_path --measure_front_half --camera_zero --penalty_scaler 1.0 --strategy e2e \\
      --terminal_body_height 0.0
GO1_NUM_ENVS overrides the num_envs that train.py:128 hard-codes (1024); GO1_MAX_ITERATIONS caps
the 10000 learning iterations of train.py:277 (smoke runs).
"""
import os
import runpy
import sys
import types
import warnings

from . import config as CF


def _module(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    m.__path__ = []  # importable as a package
    sys.modules[name] = m
    return m


def install(root_dir=None):
    from . import env as E, rollout as R

    class TrajectoryTrackingEnv(E.TrajectoryTrackingEnv):
        def __init__(self, sim_device, headless, num_envs=None, prone=False, deploy=False, cfg=None,
                     eval_cfg=None, initial_dynamics_dict=None, physics_engine="SIM_PHYSX"):
            if os.environ.get("GO1_NUM_ENVS"):
                num_envs = int(os.environ["GO1_NUM_ENVS"])
            super().__init__(sim_device, headless, num_envs, prone, deploy, cfg, eval_cfg, initial_dynamics_dict,
                             physics_engine)

    class Runner(R.Runner):
        def learn(self, num_learning_iterations, *a, **k):
            cap = os.environ.get("GO1_MAX_ITERATIONS")
            if cap:
                num_learning_iterations = min(num_learning_iterations, int(cap))
            return super().learn(num_learning_iterations, *a, **k)

    from . import velocity as VEL, velocity_config as VC

    class VelocityTrackingEasyEnv(VEL.VelocityTrackingEasyEnv):
        def __init__(self, sim_device, headless, num_envs=None, prone=False, deploy=False, cfg=None,
                     eval_cfg=None, initial_dynamics_dict=None, physics_engine="SIM_PHYSX"):
            if os.environ.get("GO1_NUM_ENVS"):
                num_envs = int(os.environ["GO1_NUM_ENVS"])
            if cfg is not None and os.environ.get("GO1_VEL_MESH", "plane") == "plane" and \
                    cfg.terrain.mesh_type != "plane":
                warnings.warn(f"legged_tracking_amd.compat: the velocity script's terrain mesh_type "
                              f"{cfg.terrain.mesh_type!r} is replaced by 'plane' (BASELINE configs[1]; the script's "
                              f"own terrain is not on the accelerated path). Set GO1_VEL_MESH=trimesh to keep it "
                              f"(the env then raises NotImplementedError).", RuntimeWarning, stacklevel=2)
                cfg.terrain.mesh_type = "plane"
            super().__init__(sim_device, headless, num_envs, prone, deploy, cfg, eval_cfg, initial_dynamics_dict,
                             physics_engine)

    Cfg = CF.make_cfg()
    VCfg = VC.make_vel_cfg()
    _module("isaacgym", gymapi=None, gymtorch=None, gymutil=None)
    _module("params_proto", PrefixProto=CF.PrefixProto, ParamsProto=CF.ParamsProto, Meta=type(CF.PrefixProto))
    root = root_dir or os.environ.get("GO1_GYM_ROOT", os.getcwd())
    _module("go1_gym", MINI_GYM_ROOT_DIR=root, MINI_GYM_ENVS_DIR=os.path.join(root, "go1_gym", "envs"))
    _module("go1_gym.envs")
    _module("go1_gym.envs.base")
    _module("go1_gym.envs.base.legged_robot_trajectory_tracking_config", Cfg=Cfg)
    _module("go1_gym.envs.base.legged_robot_trajectory_tracking", LeggedRobot=E.LeggedRobot, Cfg=Cfg)
    _module("go1_gym.envs.go1")
    _module("go1_gym.envs.go1.go1_crawling", config_go1=CF.config_go1)
    _module("go1_gym.envs.go1.trajectory_tracking", TrajectoryTrackingEnv=TrajectoryTrackingEnv,
            LeggedRobot=E.LeggedRobot, Cfg=Cfg)
    _module("go1_gym.envs.base.legged_robot_velocity_tracking_config", Cfg=VCfg)
    _module("go1_gym.envs.go1.go1_config", config_go1=VC.config_go1_vel)
    _module("go1_gym.envs.go1.velocity_tracking", VelocityTrackingEasyEnv=VelocityTrackingEasyEnv, Cfg=VCfg)
    _module("go1_gym.envs.wrappers")
    _module("go1_gym.envs.wrappers.history_wrapper", HistoryWrapper=E.HistoryWrapper)
    _module("go1_gym_learn")
    ppo = dict(Runner=Runner, RunnerArgs=R.RunnerArgs, ActorCritic=R.ActorCritic, AC_Args=R.AC_Args,
               PPO=R.PPO, PPO_Args=R.PPO_Args, RolloutStorage=R.RolloutStorage)
    _module("go1_gym_learn.ppo_cse", **ppo)
    _module("go1_gym_learn.ppo_cse.actor_critic", **ppo)
    _module("go1_gym_learn.ppo_cse.ppo", **ppo)
    _module("go1_gym_learn.ppo_cse.rollout_storage", **ppo)
    try:
        import wandb  # noqa: F401
    except ImportError:
        _module("wandb", init=lambda *a, **k: None, log=lambda *a, **k: None, save=lambda *a, **k: None,
                run=types.SimpleNamespace(dir="."), Video=lambda *a, **k: None)
    return Cfg


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        raise SystemExit(__doc__)
    script = os.path.abspath(argv[0])
    install()  # MINI_GYM_ROOT_DIR = $GO1_GYM_ROOT or the working directory (train.py logs under it)
    sys.argv = [script, *argv[1:]]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
