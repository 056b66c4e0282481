"""Generate golden fixtures by running the REFERENCE's own Python in this container.

Container-only test infrastructure: imports /root/reference (read-only, never
copied) behind offline stand-ins for Isaac Gym / params_proto / gym / wandb
(tests/golden/refstubs).  Never runs on the GPU box; the .npz files it writes
are committed under tests/golden/ and travel instead.

What runs is the reference's real code:
  * scripts/train.py:train_go1  -- builds Cfg exactly as the README command does
    (scripts/train.py:46-241); we intercept TrajectoryTrackingEnv construction to
    capture that Cfg, then shrink num_envs and the terrain grid;
  * go1_gym/envs/go1/trajectory_tracking/__init__.py TrajectoryTrackingEnv and
    go1_gym/envs/base/legged_robot_trajectory_tracking.py LeggedRobot -- step(),
    post_physics_step(), reset_idx(), compute_observations(), rewards, terrain.

Isaac Gym itself is absent (isaacgym==1.0rc4).  A fake gym hands out plain torch
tensors for root/dof/contact/rigid-body state; its simulate() writes a
synthetic post-physics state chosen by this harness (a seeded random walk), so
the fixtures pin everything AROUND the physics: actuator-net torques, height
scan, targets, rewards, terminations, resets, observations.  Every torch RNG
draw the reference makes is recorded and scattered into the canonical per-env
uniform layout the oracle and the HIP kernel consume (legged_tracking_amd/layout.py).

The actuator network is NOT loaded with torch.jit.load (that would execute code
from a file shipped in the reference); torch.jit.load is patched to return an
equivalent torch module built from weights extracted as raw data
(tests/golden/extract_actuator.py).

Usage: python tests/golden/make_golden.py  (writes tests/golden/*.npz)
"""
import argparse
import inspect
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.dont_write_bytecode = True  # the reference tree is read-only
os.environ.setdefault("MPLBACKEND", "Agg")
sys.path.insert(0, os.path.join(HERE, "refstubs"))
sys.path.insert(1, REF)
sys.path.insert(2, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from legged_tracking_amd import layout as L  # noqa: E402

# ---------------------------------------------------------------- actuator net
_W = np.load(os.path.join(REPO, "legged_tracking_amd", "data", "actuator_go1.npz"))


class _Softsign(torch.nn.Module):
    def forward(self, x):
        return torch.nn.functional.softsign(x)


def _actuator_module():
    m = torch.nn.Sequential(torch.nn.Linear(6, 32), _Softsign(), torch.nn.Linear(32, 32), _Softsign(),
                            torch.nn.Linear(32, 1))
    with torch.no_grad():
        m[0].weight.copy_(torch.from_numpy(_W["w1"]))
        m[0].bias.copy_(torch.from_numpy(_W["b1"]))
        m[2].weight.copy_(torch.from_numpy(_W["w2"]))
        m[2].bias.copy_(torch.from_numpy(_W["b2"]))
        m[4].weight.copy_(torch.from_numpy(_W["w3"]))
        m[4].bias.copy_(torch.from_numpy(_W["b3"]))
    m.requires_grad_(False)
    return m


def _jit_load(path, *a, **k):
    assert path.endswith("unitree_go1.pt"), path
    return _actuator_module()


torch.jit.load = _jit_load

# ---------------------------------------------------------------- robot asset
BODY_NAMES = L.BODY_NAMES
DOF_NAMES = L.DOF_NAMES


def _dof_props():
    dt = np.dtype([("lower", "f4"), ("upper", "f4"), ("velocity", "f4"), ("effort", "f4")])
    p = np.zeros(12, dtype=dt)
    for i in range(12):
        lo, hi = L.JOINT_LIMITS[i % 3]
        p[i] = (lo, hi, L.JOINT_VEL_LIMIT[i % 3], L.TORQUE_LIMIT)
    return p


class _Props:
    def __init__(self, **k):
        self.__dict__.update(k)


class FakeGym:
    """Hands the reference plain torch tensors; simulate() calls the harness hook."""

    hook = None

    def __init__(self):
        self.n_envs = 0
        self.tensors = {}
        self.gravity = None
        self.torque_log = []

    # --- sim / assets
    def create_sim(self, *a):
        return "sim"

    def load_asset(self, sim, root, fname, opts):
        return "robot" if fname.endswith("go1.urdf") else "arrow"

    def create_box(self, *a):
        return "box"

    def get_asset_dof_count(self, asset):
        return 12 if asset == "robot" else 0

    def get_asset_rigid_body_count(self, asset):
        return 17 if asset == "robot" else 1

    def get_asset_dof_properties(self, asset):
        return _dof_props()

    def get_asset_rigid_shape_properties(self, asset):
        return [_Props(friction=1.0, restitution=0.0) for _ in range(17)]

    def get_asset_rigid_body_names(self, asset):
        return list(BODY_NAMES)

    def get_asset_dof_names(self, asset):
        return list(DOF_NAMES)

    def create_env(self, *a):
        self.n_envs += 1
        return self.n_envs - 1

    def create_actor(self, env, asset, *a):
        return 0 if asset == "robot" else 1

    def get_actor_rigid_body_properties(self, env, actor):
        return [_Props(mass=L.BODY_MASS_PHYSX[i], com=None) for i in range(17)]

    def find_actor_rigid_body_handle(self, env, actor, name):
        return BODY_NAMES.index(name)

    def get_sim_params(self, sim):
        return _Props(gravity=None)

    def set_sim_params(self, sim, p):
        g = p.gravity
        self.gravity = (float(g.x), float(g.y), float(g.z))

    def prepare_sim(self, sim):
        n = self.n_envs
        self.tensors = {
            "root": torch.zeros(2 * n, 13),
            "dof": torch.zeros(12 * n, 2),
            "contact": torch.zeros(18 * n, 3),
            "rigid": torch.zeros(18 * n, 13),
        }

    def acquire_actor_root_state_tensor(self, sim):
        return self.tensors["root"]

    def acquire_dof_state_tensor(self, sim):
        return self.tensors["dof"]

    def acquire_net_contact_force_tensor(self, sim):
        return self.tensors["contact"]

    def acquire_rigid_body_state_tensor(self, sim):
        return self.tensors["rigid"]

    def set_dof_actuation_force_tensor(self, sim, t):
        self.torque_log.append(t.detach().clone())

    def simulate(self, sim):
        FakeGym.hook(self)

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return lambda *a, **k: None


from isaacgym import gymapi  # noqa: E402

gymapi._FACTORY = FakeGym

# ---------------------------------------------------------------- RNG recorder
_rand_log = []
_orig_rand, _orig_rand_like, _orig_randint = torch.rand, torch.rand_like, torch.randint


def _caller():
    for fr in inspect.stack()[2:8]:
        if fr.function in ("_randomize_dof_props", "_reset_dofs", "_reset_root_states", "compute_observations",
                           "_randomize_gravity", "_randomize_rigid_body_props", "_create_envs", "reset",
                           "_push_robots", "learn", "act", "mini_batch_generator", "_resample_trajectory"):
            return fr.function
    return "other"


def _rand(*a, **k):
    out = _orig_rand(*a, **k)
    _rand_log.append((_caller(), out.clone()))
    return out


def _rand_like(*a, **k):
    out = _orig_rand_like(*a, **k)
    _rand_log.append((_caller(), out.clone()))
    return out


def _randint(*a, **k):
    out = _orig_randint(*a, **k)
    _rand_log.append((_caller() + ":randint", out.clone()))
    return out


torch.rand, torch.rand_like, torch.randint = _rand, _rand_like, _randint


# ---------------------------------------------------------------- Cfg capture
class _Captured(Exception):
    pass


def capture_cfg(argv):
    """Run scripts/train.py:train_go1 up to env construction; return its Cfg."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_train", os.path.join(REF, "scripts", "train.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    import go1_gym.envs.go1.trajectory_tracking as tt
    real = tt.TrajectoryTrackingEnv
    captured = {}

    class _Intercept:
        def __init__(self, sim_device, headless, cfg=None, **k):
            captured["cfg"] = cfg
            raise _Captured()

    tt.TrajectoryTrackingEnv = _Intercept
    p = argparse.ArgumentParser()
    # flag set of scripts/train.py:287-338 (defaults are the reference's)
    for name, kw in [("--headless", dict(action="store_true")), ("--wandb", dict(action="store_true")),
                     ("--name", dict(type=str, default="velocity_tracking")), ("--resume", dict(type=str, default="")),
                     ("--freeze_model", dict(action="store_true")), ("--device", dict(default=0, type=int)),
                     ("--logdir", dict(type=str, default="/tmp/ref_logs")),
                     ("--strategy", dict(default="vel")), ("--old_ppo", dict(action="store_true")),
                     ("--gru", dict(action="store_true")), ("--cnn", dict(action="store_true")),
                     ("--learning_rate", dict(type=float, default=1e-3)), ("--gamma", dict(type=float, default=0.99)),
                     ("--exploration_steps", dict(type=int, default=2500)),
                     ("--normalize_obs", dict(action="store_true")),
                     ("--num_steps_per_env", dict(type=int, default=24)), ("--command_type", dict(default="xy")),
                     ("--timestep_in_obs", dict(action="store_true")), ("--num_history", dict(type=int, default=1)),
                     ("--measure_front_half", dict(action="store_true")),
                     ("--rotate_camera", dict(action="store_true")), ("--camera_zero", dict(action="store_true")),
                     ("--blind", dict(action="store_true")),
                     ("--terminal_body_height", dict(type=float, default=0.0)),
                     ("--terrain", dict(default="single_path")), ("--no_domain_rand", dict(action="store_true")),
                     ("--empty_tunnel", dict(action="store_true")), ("--random_target", dict(action="store_true")),
                     ("--terminate_after_reach", dict(action="store_true")),
                     ("--lin_vel_form", dict(default="exp")), ("--r_explore_lin", dict(type=float, default=1.0)),
                     ("--r_explore_yaw", dict(type=float, default=0.4)),
                     ("--penalty_scaler", dict(type=float, default=1.0)),
                     ("--only_positive", dict(action="store_true")),
                     ("--r_orientation", dict(type=float, default=0.0)),
                     ("--r_base_height", dict(type=float, default=20.0)),
                     ("--r_ang_vel", dict(type=float, default=0.001)), ("--t_reach", dict(type=int, default=0)),
                     ("--r_task", dict(type=float, default=1.0)), ("--r_collision", dict(type=float, default=5.0)),
                     ("--r_large_vel", dict(type=float, default=0.0))]:
        p.add_argument(name, **kw)
    mod.args = p.parse_args(argv)
    try:
        mod.train_go1(mod.args)
    except _Captured:
        pass
    tt.TrajectoryTrackingEnv = real
    return captured["cfg"], real


# ---------------------------------------------------------------- physics stand-in
class RandomWalkPhysics:
    """Seeded synthetic post-physics state (NOT dynamics): a bounded random walk."""

    def __init__(self, env, seed):
        self.env = env
        self.g = np.random.default_rng(seed)
        self.log = []  # per substep: dict of injected tensors

    def __call__(self, gym):
        T = gym.tensors
        n = gym.n_envs
        g = self.g
        dof = T["dof"].view(n, 12, 2)
        dof[..., 0] += torch.from_numpy(g.normal(0, 0.05, (n, 12)).astype(np.float32))
        dof[..., 1] = torch.from_numpy(g.normal(0, 1.5, (n, 12)).astype(np.float32))
        root = T["root"].view(n, 2, 13)[:, 0]
        root[:, 0:2] += torch.from_numpy(g.normal(0.01, 0.02, (n, 2)).astype(np.float32))
        root[:, 2] += torch.from_numpy(g.normal(-0.002, 0.03, (n,)).astype(np.float32))
        q = root[:, 3:7] + torch.from_numpy(g.normal(0, 0.05, (n, 4)).astype(np.float32))
        root[:, 3:7] = q / q.norm(dim=1, keepdim=True)
        root[:, 7:13] = torch.from_numpy(g.normal(0, 0.4, (n, 6)).astype(np.float32))
        cf = torch.from_numpy(g.normal(0, 2.0, (n, 18, 3)).astype(np.float32))
        cf *= torch.from_numpy((g.random((n, 18, 1)) < 0.3).astype(np.float32))
        cf[:, 17] = 0
        T["contact"].view(n, 18, 3)[:] = cf
        rb = T["rigid"].view(n, 18, 13)
        rb[:, :17, 0:3] = root[:, None, 0:3] + torch.from_numpy(g.normal(0, 0.15, (n, 17, 3)).astype(np.float32))
        self.log.append({"dof": T["dof"].clone(), "root": T["root"].view(n, 2, 13)[:, 0].clone(),
                         "contact": T["contact"].view(n, 18, 3)[:, :17].clone(),
                         "feet": rb[:, [4, 8, 12, 16], 0:3].clone()})


# ---------------------------------------------------------------- state extraction
def env_state(env):
    """Canonical per-env state (legged_tracking_amd/layout.py) read off the reference env."""
    n = env.num_envs
    rs = env.root_states[::env.num_actor]
    s = {
        "root": rs[:, 0:13].clone(),
        "dof_pos": env.dof_pos.clone(),
        "dof_vel": env.dof_vel.clone(),
        "last_actions": env.last_actions.clone(),
        "last_dof_vel": env.last_dof_vel.clone(),
        "lag": torch.stack([b.clone() for b in env.lag_buffer], 1),  # (n, 7, 12), slot 0 oldest
        "pos_err_hist": torch.stack([env.joint_pos_err_last, env.joint_pos_err_last_last], 1),
        "vel_hist": torch.stack([env.joint_vel_last, env.joint_vel_last_last], 1),
        "motor_strength": env.motor_strengths.clone(),
        "motor_offset": env.motor_offsets.clone(),
        "friction": env.friction_coeffs[:, 0].clone(),
        "restitution": env.restitutions[:, 0].clone(),
        "payload": env.payloads.clone(),
        "episode_length": env.episode_length_buf.clone(),
        "curr_pose_index": env.curr_pose_index.clone(),
        "trajectory": env.trajectories.reshape(n, -1).clone(),
        "base_rotation": env.base_rotation.clone(),
        "collision_count": env.collision_count.clone(),
        "episode_sums": torch.stack([env.episode_sums[k] for k in sum_keys(env)], 1),
        "joint_pos_target": env.joint_pos_target.clone(),
        "feet_air_time": env.feet_air_time.clone(),
        "last_contacts": env.last_contacts.float().clone(),
    }
    return {k: v.detach().cpu().numpy() for k, v in s.items()}


def sum_keys(env):
    return list(env.reward_scales.keys()) + ["total", "total_pos", "total_neg"]


def scatter_draws(env, log):
    """Map the recorded torch draws of ONE step onto the canonical per-env layout: slots 0..46
    reset / DR draws, 47 + i the obs noise of column i, then the trajectory function's draws
    (legged_tracking_amd/layout.py, include/go1_mi355x.h GO1_U_NOISE)."""
    n = env.num_envs
    n_obs = env.num_obs
    u_traj = L.U_NOISE + n_obs
    fn = env.cfg.commands.traj_function
    n_traj = 6 * (env.cfg.commands.traj_length // env.cfg.commands.num_interpolation + 1) \
        if fn == "random_target" else (3 if fn == "random_goal" else 0)
    u = np.full((n, u_traj + n_traj), np.nan, dtype=np.float32)
    ug = np.full((3,), np.nan, dtype=np.float32)
    ids = scatter_draws.ids  # env ids per call, pushed by the patched reset/dr hooks
    it = iter(ids)
    for tag, t in log:
        a = t.detach().cpu().numpy().astype(np.float32)
        if tag == "compute_observations":
            u[:, L.U_NOISE:L.U_NOISE + a.shape[1]] = a
        elif tag == "_randomize_gravity":
            ug[:] = a
        elif tag == "_randomize_dof_props":
            kind, e = next(it)
            base = L.U_RESET_STRENGTH if kind == "reset" else L.U_DR_STRENGTH
            if a.ndim == 1:
                u[e, base] = a
            else:
                u[e, base + 1:base + 13] = a
        elif tag == "_reset_dofs":
            kind, e = next(it)
            u[e, L.U_RESET_DOF:L.U_RESET_DOF + 12] = a
        elif tag == "_resample_trajectory":
            kind, e = next(it)
            ch = scatter_draws.traj_k
            scatter_draws.traj_k = ch + 1
            nt = a.shape[1]
            u[e, u_traj + ch * nt:u_traj + (ch + 1) * nt] = a
        elif tag == "_reset_root_states":
            kind, e = next(it)
            j = scatter_draws.root_k
            if a.shape[1] == 6:
                u[e, L.U_RESET_VEL:L.U_RESET_VEL + 6] = a
            else:
                u[e, L.U_RESET_XY + j] = a[:, 0]
            scatter_draws.root_k = j + 1
        else:
            raise RuntimeError(f"unexpected RNG draw in step from {tag}")
    return u, ug


def install_id_tracking(env):
    """Wrap the reference's own DR/reset helpers to learn which env ids each draw covers."""
    cls = type(env)
    orig_dr, orig_dofs, orig_root = cls._randomize_dof_props, cls._reset_dofs, cls._reset_root_states
    state = {"in_reset": False}
    orig_reset_idx = cls.reset_idx

    def reset_idx(self, env_ids):
        state["in_reset"] = True
        try:
            return orig_reset_idx(self, env_ids)
        finally:
            state["in_reset"] = False

    def dr(self, env_ids, cfg):
        e = env_ids.cpu().numpy()
        kind = "reset" if state["in_reset"] else "dr"
        if len(e):
            scatter_draws.ids.extend([(kind, e), (kind, e)])
        return orig_dr(self, env_ids, cfg)

    def dofs(self, env_ids, cfg):
        scatter_draws.ids.append(("reset", env_ids.cpu().numpy()))
        return orig_dofs(self, env_ids, cfg)

    orig_traj = cls._resample_trajectory

    def traj(self, env_ids):
        e = env_ids.cpu().numpy()
        fn = self.cfg.commands.traj_function
        k = 6 if fn == "random_target" else (3 if fn == "random_goal" else 0)
        scatter_draws.ids.extend([("reset", e)] * k)
        scatter_draws.traj_k = 0
        return orig_traj(self, env_ids)

    cls._resample_trajectory = traj

    def root(self, env_ids, cfg):
        e = env_ids.cpu().numpy()
        k = 4 if self.custom_origins else 2
        scatter_draws.ids.extend([("reset", e)] * k)
        if not self.custom_origins:
            scatter_draws.root_k = 2
        return orig_root(self, env_ids, cfg)

    cls.reset_idx, cls._randomize_dof_props, cls._reset_dofs, cls._reset_root_states = reset_idx, dr, dofs, root


scatter_draws.ids = []
scatter_draws.root_k = 0
scatter_draws.traj_k = 0


def readme_argv(terrain, extra_argv=(), front_half=True):
    argv = ["--terrain", terrain, "--penalty_scaler", "1.0", "--strategy", "e2e", "--terminal_body_height", "0.0"]
    if front_half:
        argv.append("--measure_front_half")
    if terrain != "plane":
        argv.append("--camera_zero")
    return argv + list(extra_argv)


def build_env(terrain, n_envs, rows, seed, extra_argv=(), cfg_overrides=None, front_half=True):
    argv = readme_argv(terrain, extra_argv, front_half)
    cfg, Env = capture_cfg(["--old_ppo"] + argv)
    cfg.env.num_envs = n_envs
    cfg.terrain.num_rows = rows
    cfg.terrain.num_cols = rows
    for path, v in (cfg_overrides or {}).items():  # Cfg edits after train.py (e.g. another reward container)
        obj = cfg
        parts = path.split(".")
        for part in parts[:-1]:
            obj = getattr(obj, part)
        setattr(obj, parts[-1], v)
    # seeding as scripts/train.py:33-40 does
    np.random.seed(seed)
    torch.manual_seed(seed)
    env = Env(sim_device="cpu", headless=True, cfg=cfg)
    return env, cfg


def run(terrain, n_envs, rows, n_steps, seed, out, extra_argv=(), actions_scale=1.0, counter_start=None,
        events=False, cfg_overrides=None, front_half=True):
    env, cfg = build_env(terrain, n_envs, rows, seed, extra_argv, cfg_overrides, front_half)
    install_id_tracking(env)
    term_log = {}

    def _wrap(name, fn):
        def w():
            out = fn()
            term_log[name] = out.detach().clone()
            return out
        return w

    env.reward_functions = [_wrap(nm, fn) for nm, fn in zip(env.reward_names, env.reward_functions)]
    # measured_heights is later modified in place by the camera_zero branch of
    # compute_observations (:399-403); record _get_heights' own output
    orig_gh = env._get_heights

    def _gh(env_ids):
        out = orig_gh(env_ids)
        term_log["heights"] = out.detach().clone()
        return out

    env._get_heights = _gh
    gym = env.gym
    phys = RandomWalkPhysics(env, seed + 1)
    FakeGym.hook = phys
    n = env.num_envs
    rec = {"static": {}, "steps": []}
    st = rec["static"]
    st["env_height_samples"] = (env.env_height_samples.numpy() if terrain != "plane"
                                else np.zeros((n, 2, 1, 1), np.float32))
    st["env_terrain_origin"] = (env.env_terrain_origin.numpy() if terrain != "plane" else np.zeros((n, 3), np.float32))
    st["env_origins"] = env.env_origins.numpy()
    st["default_dof_pos"] = env.default_dof_pos.numpy()[0]
    st["dof_pos_limits"] = env.dof_pos_limits.numpy()
    st["torque_limits"] = env.torque_limits.numpy()
    st["max_episode_length"] = np.float64(env.max_episode_length)
    keys = list(env.reward_scales.keys())
    st["reward_scales"] = np.array([env.reward_scales[k] for k in keys], np.float64)
    st["reward_keys"] = np.array(list(env.reward_scales.keys()))
    st["gravities"] = env.gravities.numpy()[0]

    # reset() as the reference's TrajectoryTrackingEnv.reset (trajectory_tracking/__init__.py:46-55)
    _rand_log.clear()
    scatter_draws.ids.clear()
    env.reset()
    rec["after_reset"] = env_state(env)
    rec["after_reset_obs"] = env.obs_buf.numpy().copy()
    if counter_start is not None:
        env.common_step_counter = counter_start
    if events:
        # drive rarely-hit branches: DR at episode_length % rand_interval == 0
        # (:822-824), waypoint switch/reached (:836-844), timeouts (:203)
        env.episode_length_buf[:8] = int(env.cfg.domain_rand.rand_interval) - 2
        env.episode_length_buf[8:12] = int(env.max_episode_length) - 1
        rs = env.root_states[::env.num_actor]
        T = env.cfg.commands.traj_length
        env.trajectories[12:28, :, 0:2] = rs[12:28, None, 0:2] + torch.linspace(-0.3, 0.3, 16)[:, None, None]
        if T > 1:  # waypoints: some envs one switch away from the last one
            env.curr_pose_index[20:28] = T - 2
    g = np.random.default_rng(seed + 2)
    for t in range(n_steps):
        pre = env_state(env)
        pre_counter = env.common_step_counter
        pre_scales = np.array([env.reward_scales[k] for k in keys], np.float64)
        pre_grav = env.gravities.numpy()[0].copy()
        pre_gvec = env.gravity_vec.numpy()[0].copy()
        pre_simg = np.array(gym.gravity, np.float32)
        actions = torch.from_numpy((g.normal(0, 1.0, (n, 12)) * actions_scale).astype(np.float32))
        if t % 7 == 3:  # exercise the +/-10 action clip (scripts/train.py:241)
            actions[:4] *= 20.0
        _rand_log.clear()
        scatter_draws.ids.clear()
        scatter_draws.root_k = 0
        phys.log.clear()
        gym.torque_log.clear()
        ep_before = {k: len(v) for k, v in env.extras["train/episode"].items() if hasattr(v, "__len__")}
        to_before = len(env.extras["timeouts"])
        obs, rew, reset, extras = env.step(actions)
        u, ug = scatter_draws(env, list(_rand_log))
        ep_new = {}
        for k, v in extras["train/episode"].items():
            if hasattr(v, "__len__"):
                ep_new["episode/" + k] = np.asarray(list(v)[ep_before.get(k, 0):], np.float64)
            else:
                ep_new["episode_scalar/" + k] = np.float64(v)
        step = {
            "pre": pre, "post": env_state(env), "actions": actions.numpy(),
            "common_step_counter": np.int64(pre_counter), "reward_scales": pre_scales, "gravity": pre_grav,
            "gravity_after": env.gravities.numpy()[0].copy(),
            "gravity_vec": pre_gvec, "sim_gravity": pre_simg,
            "uniforms": u, "uniforms_gravity": ug,
            "inj_dof": np.stack([p["dof"].view(n, 12, 2).numpy() for p in phys.log]),  # (4, n, 12, 2)
            "inj_root": phys.log[-1]["root"].numpy(), "inj_contact": phys.log[-1]["contact"].numpy(),
            "inj_feet": phys.log[-1]["feet"].numpy(),
            "torques": np.stack([x.view(n, 12).numpy() for x in gym.torque_log]),  # (4, n, 12)
            "obs": obs.numpy().copy(), "priv": extras["privileged_obs"].numpy().copy(),
            "rew": rew.numpy().copy(), "reset": reset.numpy().copy(),
            "time_out": env.time_out_buf.numpy().copy(),
            "extras_time_outs": (extras["time_outs"].numpy().copy() if "time_outs" in extras
                                 else np.zeros(0, bool)),
            "measured_heights": (term_log["heights"].numpy().copy() if "heights" in term_log  # blind: no scan
                                 else np.zeros((n, 2, 21, 11), np.float32)),
            "rew_terms": np.stack([term_log[k].float().numpy() if k in term_log else np.zeros(n, np.float32)
                                   for k in keys], 1),
            "arrow_root": env.root_states[1::2, 0:7].numpy().copy(),
            "reached": env.reached_buf.numpy().copy(),
            "commands": env.commands.numpy().copy(),
            "x_body_linear_vel": np.asarray(extras["body_linear_vel"]).copy(),
            "x_body_angular_vel": np.asarray(extras["body_angular_vel"]).copy(),
            "x_body_linear_vel_cmd": np.asarray(extras["body_linear_vel_cmd"]).copy(),
            "x_torques": np.asarray(extras["torques"]).copy(),
            "x_timeouts_new": np.array([bool(x) for x in list(extras["timeouts"])[to_before:]], bool),
            **ep_new,
        }
        rec["steps"].append(step)
    flat = {}
    for k, v in rec["static"].items():
        flat["static/" + k] = v
    for k, v in rec["after_reset"].items():
        flat["after_reset/" + k] = v
    flat["after_reset_obs"] = rec["after_reset_obs"]
    for t, s in enumerate(rec["steps"]):
        for k, v in s.items():
            if isinstance(v, dict):
                for kk, vv in v.items():
                    flat[f"s{t}/{k}/{kk}"] = vv
            else:
                flat[f"s{t}/{k}"] = v
    flat["meta/n_steps"] = np.int64(n_steps)
    flat["meta/terrain"] = np.array(terrain)
    flat["meta/rows"] = np.int64(rows)
    flat["meta/argv"] = np.array(readme_argv(terrain, extra_argv, front_half))
    import json
    flat["meta/cfg_overrides"] = np.array(json.dumps(cfg_overrides or {}))
    np.savez_compressed(out, **flat)
    print("wrote", out, len(flat), "arrays")


# Variant fixtures (train.py flags / Cfg edits beyond the README command), 32 envs x 4 steps each.
# TrajectoryTrackingRewards: the container the env selects with Cfg.rewards.reward_container_name
# (:1373-1377); its scales are set after train.py as a user would.
_TT_A = {"rewards.reward_container_name": "TrajectoryTrackingRewards", "rewards.large_dist_threshold": 0.5,
         "reward_scales.dof_vel": -1e-4, "reward_scales.dof_pos": -0.05, "reward_scales.survive": 0.1,
         "reward_scales.feet_air_time": 0.5, "reward_scales.exploration": 0.3, "reward_scales.stalling": 0.2,
         "reward_scales.task": 0.7, "reward_scales.reach_goal": 2.0, "reward_scales.linear_vel": -0.1,
         "reward_scales.lin_vel_z": -0.5}
_TT_B = {"rewards.reward_container_name": "TrajectoryTrackingRewards", "reward_scales.task_old": 0.4,
         "reward_scales.reach_goal_t": 0.01, "reward_scales.reach_goal_T": 1.5,
         "reward_scales.reaching_linear_vel": 0.6, "reward_scales.reaching_yaw": 0.3,
         "reward_scales.reaching_yaw_abs": -0.2, "reward_scales.reaching_z": -0.3}
VARIANTS = {
    "only_positive_l1": dict(extra_argv=["--only_positive", "--lin_vel_form", "l1", "--r_orientation", "0.5",
                                         "--r_large_vel", "0.3"]),
    "ji22_l2": dict(extra_argv=["--lin_vel_form", "l2"], cfg_overrides={"rewards.only_positive_rewards_ji22_style": True}),
    "prod_ji22": dict(extra_argv=["--lin_vel_form", "prod"],
                      cfg_overrides={"rewards.only_positive_rewards_ji22_style": True}),
    "terminate_rotate_timestep": dict(extra_argv=["--terminate_after_reach", "--rotate_camera", "--timestep_in_obs",
                                                  "--t_reach", "2"]),
    "random_target": dict(extra_argv=["--random_target"]),
    "full_scan_blind_plane": dict(terrain="plane", extra_argv=["--blind", "--timestep_in_obs"], front_half=False),
    "full_scan": dict(front_half=False, extra_argv=["--strategy", "vel", "--t_reach", "3"]),
    "tt_container_a": dict(extra_argv=["--strategy", "vel", "--r_base_height", "0", "--r_explore_lin", "0",
                                       "--r_explore_yaw", "0"], cfg_overrides=_TT_A),
    "tt_container_b": dict(extra_argv=["--t_reach", "3", "--r_orientation", "0.2", "--r_explore_lin", "0",
                                       "--r_explore_yaw", "0"], cfg_overrides=_TT_B),
}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--which", default="all")
    a = ap.parse_args()
    if a.which == "all":
        # one fresh process per fixture: the reference mutates its module-level Cfg
        import subprocess
        for w in ("single_path", "plane", "events", "full_grid", *VARIANTS):
            subprocess.run([sys.executable, __file__, "--steps", str(a.steps), "--which", w], check=True)
    elif a.which == "single_path":
        # gravity zeroing at counter 396 and resampling at 400 fall inside the window
        run("single_path", 64, 4, a.steps, 11, os.path.join(HERE, "step_single_path.npz"), counter_start=393)
    elif a.which == "events":
        run("single_path", 64, 4, 5, 13, os.path.join(HERE, "step_single_path_events.npz"), counter_start=398,
            events=True)
    elif a.which == "plane":
        # plane (no camera_zero: the reference raises with it, :402); exploration decay after 2500
        run("plane", 64, 4, a.steps, 12, os.path.join(HERE, "step_plane.npz"), counter_start=2497)
    elif a.which == "full_grid":
        # the README grid at full size: 32 x 32 sub-terrains, one env on each (1024 envs), 2 steps
        run("single_path", 1024, 32, 2, 17, os.path.join(HERE, "step_full_grid.npz"), counter_start=120)
    elif a.which in VARIANTS:
        kw = dict(VARIANTS[a.which])
        terrain = kw.pop("terrain", "single_path")
        run(terrain, 32, 4, kw.pop("steps", 4), kw.pop("seed", 21), os.path.join(HERE, f"step_v_{a.which}.npz"),
            counter_start=398, events=True, **kw)
