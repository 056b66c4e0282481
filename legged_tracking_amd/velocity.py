"""Drop-in host side of the velocity-tracking env (BASELINE configs[1]) over the HIP step.

Mirrors, for scripts/train_velocity_tracking.py's configuration on a plane:

  VelocityTrackingEasyEnv <- go1_gym/envs/go1/velocity_tracking/__init__.py:11-55
                             on go1_gym/envs/base/legged_robot_velocity_tracking.py (bare :N below)
  HistoryWrapper          <- go1_gym/envs/wrappers/history_wrapper.py:6-41 (legged_tracking_amd.env)

Everything per env runs in libgo1_velocity.so (legged_tracking_amd/csrc/go1_velocity.hip) through the C
ABI of include/go1_velocity.h; this module keeps what the reference keeps on the host or globally: the
configuration, common_step_counter with the global gravity schedule (:719-723, _randomize_gravity
:564-579), and the extras (lazy: "train/episode" means are built from the kernel's compact episode log
when read).  No CPU fallback: without the HIP library or a GPU the constructor raises.

Differences from the reference: physics is the native integrator (plane terrain, the
contact model of go1_device.h), random draws are Philox keyed by (seed, global env, slot, step) instead
of torch's global generator and the curricula's RandomState, output tensors rotate through OUT_RING
buffers, and the interval resample of a step runs ahead in the previous step's curriculum launch.
"""
import ctypes as C
import math
import os
from collections import deque

import numpy as np
import torch

from . import abi, config as CF, layout as L, vel_abi as VA, vel_layout as VL, velocity_config as V

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GO1_VEL_LIB_OVERRIDE") or os.path.join(HERE, "_build", "libgo1_velocity.so")
OUT_RING = 4
# obs_history windows per wide buffer: the history lives in rows of width W + 70 x HIST_WINDOW, and each step
# returns the next W-wide window of the row (go1_vel_step's sliding-window form, no shift); the rows are
# rewound -- the last W - 70 columns shifted into the other buffer -- once every HIST_WINDOW steps
HIST_WINDOW = 32
_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load the HIP velocity library (fails loudly; build with __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"HIP extension missing: {LIB_PATH} (run python -c 'import __graft_entry__ as g; g.build()')")
    l = C.CDLL(LIB_PATH)
    l.go1_vel_abi_version.restype = C.c_int
    l.go1_vel_last_error.restype = C.c_char_p
    l.go1_vel_abi_sizes.argtypes = [C.POINTER(C.c_int64)]
    l.go1_vel_create.argtypes = [C.POINTER(abi.Go1Config), C.POINTER(VA.Go1VelConfig), C.c_void_p,
                                 C.POINTER(C.c_void_p)]
    l.go1_vel_bind.argtypes = [C.c_void_p, C.POINTER(VA.Go1VelState), C.POINTER(abi.Go1Plane)]
    l.go1_vel_set_origins.argtypes = [C.c_void_p, C.c_void_p]
    l.go1_vel_step.argtypes = [C.c_void_p, C.POINTER(VA.Go1VelStepArgs), C.c_void_p]
    l.go1_vel_reset_idx.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_uint64,
                                    C.c_uint64, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
    l.go1_vel_resample.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                   C.c_void_p]
    l.go1_vel_destroy.argtypes = [C.c_void_p]
    if l.go1_vel_abi_version() != VA.GO1_VEL_ABI_VERSION:
        raise NativeError("velocity ABI version mismatch")
    _lib = l
    return l


def _check(rc):
    if rc != 0:
        raise NativeError(lib().go1_vel_last_error().decode())


# ---------------------------------------------------------------------------- configuration
PHYSICS = dict(CF.PHYSICS)


def unsupported(cfg):
    """Cfg values of the velocity env the HIP step does not implement (each raises NotImplementedError
    at construction instead of training on something else)."""
    bad = []
    e, t, c, r, dr, ctl = cfg.env, cfg.terrain, cfg.commands, cfg.rewards, cfg.domain_rand, cfg.control
    if t.mesh_type != "plane":
        bad.append(f"terrain.mesh_type={t.mesh_type!r} (the velocity step runs on the plane, BASELINE configs[1])")
    want = dict(observe_command=True, observe_two_prev_actions=True, observe_clock_inputs=True, observe_vel=False,
                observe_only_ang_vel=False, observe_only_lin_vel=False, observe_yaw=False,
                observe_contact_states=False, observe_timing_parameter=False)
    for k, v in want.items():
        if bool(getattr(e, k)) != v:
            bad.append(f"env.{k}={getattr(e, k)!r}")
    # the privileged observations compute_observations implements (:401-506); other priv_observe_* flags
    # (joint_friction, Kp / Kd factors, ...) have no code path in the reference and are ignored there too
    known = ("friction", "ground_friction", "restitution", "base_mass", "com_displacement", "motor_strength",
             "motor_offset", "body_height", "body_velocity", "gravity", "clock_inputs", "desired_contact_states")
    priv = [f"priv_observe_{k}" for k in known if getattr(e, f"priv_observe_{k}", False)]
    if sorted(priv) != ["priv_observe_friction", "priv_observe_restitution"]:
        bad.append(f"privileged observations {sorted(priv)} (friction and restitution only)")
    if int(e.num_observations) != VL.NUM_OBS or int(e.num_privileged_obs) != VL.NUM_PRIV:
        bad.append("num_observations / num_privileged_obs")
    if int(c.num_commands) != VL.NUM_COMMANDS:
        bad.append(f"commands.num_commands={c.num_commands}")
    if c.curriculum_type != "RewardThresholdCurriculum":
        bad.append(f"commands.curriculum_type={c.curriculum_type!r}")
    if not c.gaitwise_curricula and (c.exclusive_phase_offset or c.balance_gait_distribution):
        bad.append("exclusive_phase_offset / balance_gait_distribution without gaitwise_curricula")
    if c.pacing_offset:
        bad.append("commands.pacing_offset")
    if ctl.control_type != "actuator_net":
        bad.append(f"control.control_type={ctl.control_type!r}")
    if not dr.randomize_lag_timesteps or int(dr.lag_timesteps) != L.LAG_SLOTS - 1:
        bad.append("domain_rand lag (randomize_lag_timesteps with lag_timesteps 6)")
    for k in ("push_robots", "randomize_rigids_after_start", "randomize_com_displacement", "randomize_Kp_factor",
              "randomize_Kd_factor", "randomize_friction_indep"):
        if getattr(dr, k, False):
            bad.append(f"domain_rand.{k}")
    if t.teleport_robots:
        bad.append("terrain.teleport_robots")
    if r.reward_container_name != "CoRLRewards":
        bad.append(f"rewards.reward_container_name={r.reward_container_name!r}")
    for k, v in vars(cfg.reward_scales).items():
        if v != 0 and k not in VA.VTERM_IDS:
            bad.append(f"reward_scales.{k} (a CoRLRewards term the HIP step does not evaluate)")
    if getattr(r, "use_terminal_foot_height", False):
        bad.append("rewards.use_terminal_foot_height")
    return bad


def build_configs(cfg, n_envs=None, physics=None, env_id_offset=0, history_len=None):
    """(go1_config for the integrator / actuator, go1_vel_config, curriculum grid (15, n_bins) f64, initial
    weights (n_bins,) f64) for a velocity Cfg; raises NotImplementedError for unsupported values."""
    bad = unsupported(cfg)
    if bad:
        raise NotImplementedError("velocity step: unsupported configuration: " + "; ".join(bad))
    physics = dict(PHYSICS, **(physics or {}))
    d = V.vel_derived(cfg)
    n = int(n_envs if n_envs is not None else cfg.env.num_envs)
    f32 = CF.f32
    # ---- physics / actuator block (go1_config; trajectory-only fields stay zero)
    c = abi.Go1Config()
    c.n_envs = n
    c.terrain_kind = 0
    c.decimation = int(cfg.control.decimation)
    c.n_internal = int(physics["n_internal"])
    c.rand_interval = int(d["rand_interval"])
    c.env_id_offset = int(env_id_offset)
    c.sim_dt = f32(cfg.sim.dt)
    c.dt = f32(d["dt"])
    c.action_scale = f32(cfg.control.action_scale)
    c.hip_scale_reduction = f32(cfg.control.hip_scale_reduction)
    c.clip_actions = f32(cfg.normalization.clip_actions)
    c.clip_obs = f32(cfg.normalization.clip_observations)
    c.max_episode_length = f32(d["max_episode_length"])
    for i, nme in enumerate(L.DOF_NAMES):
        c.default_dof_pos[i] = f32(cfg.init_state.default_joint_angles[nme])
    soft = CF.soft_dof_limits(getattr(cfg.rewards, "soft_dof_pos_limit", 1.0))
    for i in range(12):
        c.dof_pos_limits[2 * i], c.dof_pos_limits[2 * i + 1] = float(soft[i, 0]), float(soft[i, 1])
        c.torque_limits[i] = f32(L.TORQUE_LIMIT)
        lo, hi = L.JOINT_LIMITS[i % 3]
        c.hard_limits[2 * i], c.hard_limits[2 * i + 1] = f32(lo), f32(hi)
    CF.set_contact_fields(c, cfg, physics)
    from . import model as M
    for i, x in enumerate(M.model_block()):
        c.model[i] = float(x)
    for i, x in enumerate(CF.load_actuator()):
        c.actuator[i] = float(x)
    # ---- velocity block (go1_vel_config)
    v = VA.Go1VelConfig()
    v.n_envs = n
    scales = d["reward_scales"]
    names = [k for k in scales if k != "termination"]
    if "termination" in scales:
        raise NotImplementedError("reward_scales.termination (the post-clip termination reward, :308-312)")
    if len(names) > VA.GO1_VEL_MAX_TERMS:
        raise NotImplementedError(f"{len(names)} reward terms > {VA.GO1_VEL_MAX_TERMS}")
    v.n_terms = len(names)
    nonpos = 0
    for k, name in enumerate(names):
        v.term_ids[k] = VA.VTERM_IDS[name]
        if VA.VTERM_SIGN[name] * scales[name] < 0:
            nonpos |= 1 << k
    v.nonpos_slots = nonpos
    rw = cfg.rewards
    v.reward_mode = 1 if rw.only_positive_rewards else (2 if rw.only_positive_rewards_ji22_style else 0)
    v.resample_interval = int(d["resample_interval"])
    v.rand_interval = int(d["rand_interval"])
    v.add_noise = int(bool(cfg.noise.add_noise))
    v.use_terminal_body_height = int(bool(rw.use_terminal_body_height))
    v.history_len = int(history_len if history_len is not None else cfg.env.num_observation_history)
    grid, bin_sizes, w0 = V.curriculum_grid(cfg)
    v.n_bins = grid.shape[1]
    if v.n_bins > VA.GO1_VEL_MAX_BINS:
        raise NotImplementedError(f"{v.n_bins} curriculum bins > {VA.GO1_VEL_MAX_BINS}")
    v.gaitwise_curricula = int(bool(cfg.commands.gaitwise_curricula))
    v.binary_phases = int(bool(cfg.commands.binary_phases))
    sum_keys = names + ["lin_vel_raw", "ang_vel_raw", "lin_vel_residual", "ang_vel_residual", "ep_timesteps"]
    task = [k for k in V.TASK_KEYS if k in scales]
    v.n_task = len(task)
    for i, k in enumerate(task):
        v.task_slot[i] = sum_keys.index(k)
        v.task_threshold[i] = f32(getattr(cfg.curriculum_thresholds, k) * scales[k])
    v.curriculum_ep_len = f32(d["curriculum_ep_len"])
    v.max_episode_length = f32(d["max_episode_length"])
    v.dt = f32(d["dt"])
    v.clip_obs = f32(cfg.normalization.clip_observations)
    for i, s in enumerate(V.commands_scale(cfg)):
        v.cmd_scale[i] = float(s)
    F = np.float32
    lvl, ns, os_ = cfg.noise.noise_level, cfg.noise_scales, cfg.obs_scales
    nv = np.zeros(VL.NUM_OBS, np.float32)  # _get_noise_scale_vec (:1071-1139)
    nv[0:3] = F(F(1.0) * F(ns.gravity)) * F(lvl)
    nv[18:30] = F(F(F(1.0) * F(ns.dof_pos)) * F(lvl)) * F(os_.dof_pos)
    nv[30:42] = F(F(F(1.0) * F(ns.dof_vel)) * F(lvl)) * F(os_.dof_vel)
    for i in range(VL.NUM_OBS):
        v.noise_vec[i] = float(nv[i])
    v.obs_scale_dof_pos, v.obs_scale_dof_vel = f32(os_.dof_pos), f32(os_.dof_vel)
    fs, fsh = V.get_scale_shift(cfg.normalization.friction_range)
    rs, rsh = V.get_scale_shift(cfg.normalization.restitution_range)
    v.priv_friction_shift, v.priv_friction_scale = f32(fsh), f32(fs)
    v.priv_rest_shift, v.priv_rest_scale = f32(rsh), f32(rs)
    dr = cfg.domain_rand
    lo, hi = dr.motor_strength_range
    v.strength_range, v.strength_lo = (f32(hi - lo), f32(lo)) if dr.randomize_motor_strength else (0.0, 1.0)
    lo, hi = dr.motor_offset_range
    v.offset_range, v.offset_lo = (f32(hi - lo), f32(lo)) if dr.randomize_motor_offset else (0.0, 0.0)
    v.reset_dof_range, v.reset_dof_lo = f32(1.5 - 0.5), f32(0.5)
    v.reset_vel_range, v.reset_vel_lo = f32(0.5 - (-0.5)), f32(-0.5)
    yr = cfg.terrain.yaw_init_range
    v.yaw_range, v.yaw_lo = f32(yr - (-yr)), f32(-yr)
    init = list(cfg.init_state.pos) + list(cfg.init_state.rot) + list(cfg.init_state.lin_vel) + \
        list(cfg.init_state.ang_vel)
    for i, x in enumerate(init):
        v.base_init_state[i] = f32(x)
    for i in range(12):
        v.default_dof_pos[i] = c.default_dof_pos[i]
    for i in range(24):
        v.dof_pos_limits[i] = c.dof_pos_limits[i]
    v.tracking_sigma, v.tracking_sigma_yaw = f32(rw.tracking_sigma), f32(rw.tracking_sigma_yaw)
    v.gait_force_sigma, v.gait_vel_sigma = f32(rw.gait_force_sigma), f32(rw.gait_vel_sigma)
    v.kappa_gait_probs = f32(rw.kappa_gait_probs)
    v.base_height_target, v.sigma_rew_neg = f32(rw.base_height_target), f32(rw.sigma_rew_neg)
    v.terminal_body_height = f32(rw.terminal_body_height)
    for i in range(VA.GO1_VEL_N_KEYS):
        v.local_range[i] = float(V.LOCAL_RANGE[i])
        v.bin_sizes[i] = float(bin_sizes[i])
    return c, v, np.ascontiguousarray(grid, np.float64), w0.astype(np.float64), names, sum_keys


def plane_env_origins(n_local, cfg, n_global=None, first=0):
    """_get_env_origins (:1693-1733) for the plane: a num_rows x num_cols grid spaced env_spacing, env i at
    (spacing xx_i, spacing yy_i, 0) with torch.meshgrid's 'ij' order; `first` = global id of local env 0."""
    n = int(n_global if n_global is not None else n_local)
    num_cols = np.floor(np.sqrt(n))
    num_rows = np.ceil(n / num_cols)
    xx, yy = np.meshgrid(np.arange(num_rows, dtype=np.int64), np.arange(num_cols, dtype=np.int64), indexing="ij")
    sp = np.float32(cfg.env.env_spacing)
    o = np.zeros((n, 3), np.float32)
    o[:, 0] = sp * xx.reshape(-1)[:n].astype(np.float32)
    o[:, 1] = sp * yy.reshape(-1)[:n].astype(np.float32)
    return o[first:first + n_local]


# ---------------------------------------------------------------------------- native handle
class VelNative:
    """Owns one go1_vel_handle, the state planes and the device buffers the C ABI writes."""

    def __init__(self, phys, vel, grid, w0, device="cuda:0"):
        if not torch.cuda.is_available():
            raise NativeError("no GPU visible: the MI355X velocity step has no CPU fallback")
        self.device = torch.device(device)
        self.phys, self.vel = phys, vel
        self.n = n = phys.n_envs
        self.h = C.c_void_p()
        g = np.ascontiguousarray(grid, np.float64)
        with torch.cuda.device(self.device):
            _check(lib().go1_vel_create(C.byref(phys), C.byref(vel), g.ctypes.data_as(C.c_void_p), C.byref(self.h)))
            self.state = {}
            for name, rows, w, dt in VA.vel_state_spec(vel.n_terms, vel.n_bins):
                dtype = {"f32": torch.float32, "i32": torch.int32, "f64": torch.float64}[dt]
                self.state[name] = torch.zeros((rows or n, w), dtype=dtype, device=self.device)
            self.state["curriculum_weights"].copy_(torch.as_tensor(np.broadcast_to(w0, (4, len(w0))).copy()))
            self.bind(self.state)
            dev = self.device
            self.extras_time_outs = torch.zeros(n, dtype=torch.bool, device=dev)
            self.contact_forces = torch.zeros((n, 17, 3), device=dev)
            self.aux = torch.zeros((n, VA.GO1_VEL_AUX), device=dev)
        self._origins = None
        self._lib_step = lib().go1_vel_step
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()

    def bind(self, state):
        s = VA.Go1VelState(**{k: state[k].data_ptr() for k, _ in VA.Go1VelState._fields_})
        arr = (abi.Go1Plane * VA.GO1_VEL_STATE_PLANES)()
        for i, (name, _) in enumerate(VA.Go1VelState._fields_):
            t = state[name]
            shape = tuple(t.shape) + (1,) * (2 - t.dim())
            stride = tuple(t.stride()) + (1,) * (2 - t.dim())
            dt = {torch.int32: abi.GO1_DTYPE_I32, torch.float64: VA.GO1_DTYPE_F64}.get(t.dtype, abi.GO1_DTYPE_F32)
            arr[i] = abi.Go1Plane(rows=shape[0], cols=shape[1], row_stride=stride[0], col_stride=stride[1], dtype=dt)
        _check(lib().go1_vel_bind(self.h, C.byref(s), arr))

    def set_origins(self, origins):
        t = torch.as_tensor(np.ascontiguousarray(origins, np.float32)).to(self.device)
        self._origins = t
        _check(lib().go1_vel_set_origins(self.h, C.c_void_p(t.data_ptr())))

    def args(self):
        a = VA.Go1VelStepArgs()
        a.extras_time_outs = self.extras_time_outs.data_ptr()
        a.contact_forces = self.contact_forces.data_ptr()
        a.aux = self.aux.data_ptr()
        a.resample_next = 1
        return a

    def step(self, a, stream=None):
        rc = self._lib_step(self.h, C.byref(a), stream if stream is not None else
                            torch._C._cuda_getCurrentRawStream(self._dev_index))
        if rc:
            _check(rc)

    def resample(self, mask=None, uniforms=None, uniforms_f64=None, rng_seed=0, rng_step=0):
        m = None if mask is None else mask.to(torch.uint8).contiguous()
        _check(lib().go1_vel_resample(self.h, None if m is None else m.data_ptr(),
                                      None if uniforms is None else uniforms.data_ptr(),
                                      None if uniforms_f64 is None else uniforms_f64.data_ptr(), int(rng_seed),
                                      int(rng_step), C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        return m

    def reset_idx(self, env_ids, uniforms=None, uniforms_f64=None, rng_seed=0, rng_step=0, log=None, log_count=None,
                  log_tag=0):
        ids = torch.as_tensor(env_ids, device=self.device).to(torch.int32).flatten().contiguous()
        _check(lib().go1_vel_reset_idx(self.h, ids.data_ptr(), int(ids.numel()),
                                       None if uniforms is None else uniforms.data_ptr(),
                                       None if uniforms_f64 is None else uniforms_f64.data_ptr(), int(rng_seed),
                                       int(rng_step), None if log is None else log.data_ptr(),
                                       None if log_count is None else log_count.data_ptr(),
                                       0 if log is None else int(log.shape[0]), int(log_tag),
                                       C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        return ids

    def close(self):
        if self.h:
            lib().go1_vel_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------------------- the env
class VelocityTrackingEasyEnv:
    """VelocityTrackingEasyEnv (velocity_tracking/__init__.py:11-55) for scripts/train_velocity_tracking.py's
    configuration on a plane (BASELINE configs[1]), backed by the HIP step."""

    def __init__(self, sim_device="cuda:0", headless=True, num_envs=None, prone=False, deploy=False, cfg=None,
                 eval_cfg=None, initial_dynamics_dict=None, physics_engine="SIM_PHYSX", *, seed=1, rank=None,
                 world_size=None, physics=None):
        if eval_cfg is not None:
            raise NotImplementedError("eval envs (eval_cfg) are not on the accelerated path")
        if cfg is None:
            cfg = V.train_velocity_config(n_envs=num_envs or 4096)
        if num_envs is not None:
            cfg.env.num_envs = num_envs
        if rank is None or world_size is None:
            from .env import _dist_info
            r, w = _dist_info()
            rank = r if rank is None else rank
            world_size = w if world_size is None else world_size
        self.rank, self.world_size = rank, world_size
        self.cfg = cfg
        self.eval_cfg = None
        self.sim_device = sim_device
        self.headless = headless
        self.num_obs = int(cfg.env.num_observations)
        self.num_privileged_obs = int(cfg.env.num_privileged_obs)
        self.num_actions = int(cfg.env.num_actions)
        self.num_envs = self.num_train_envs = n = int(cfg.env.num_envs)
        self.num_eval_envs = 0
        self.seed = int(seed)
        d = V.vel_derived(cfg)
        self.dt = d["dt"]
        self.max_episode_length = d["max_episode_length"]
        self._gravity_interval = d["gravity_rand_interval"]
        self._gravity_duration = d["gravity_rand_duration"]
        self._phys, self._vcfg, grid, w0, self.reward_names, self.command_sum_keys = build_configs(
            cfg, n_envs=n, physics=physics, env_id_offset=rank * n)
        self.reward_scales = dict(d["reward_scales"])
        self.episode_keys = list(self.reward_names) + ["total"]
        self.curriculum_grid = grid
        self.category_names = list(V.CATEGORIES) if cfg.commands.gaitwise_curricula else ["nominal"]
        self._sim = VelNative(self._phys, self._vcfg, grid, w0, sim_device)
        self.device = dev = self._sim.device
        self._n_global = n * world_size
        self.env_origins = torch.as_tensor(plane_env_origins(n, cfg, self._n_global, rank * n), device=dev)
        self._sim.set_origins(self.env_origins.cpu().numpy())
        st = self._sim.state
        # _init_buffers / _randomize_rigid_body_props at creation: per-env DR keyed by GLOBAL env id
        dr = cfg.domain_rand
        st["friction"].copy_(self._global_uniform(1, *dr.friction_range) if dr.randomize_friction else
                             torch.ones((n, 1), device=dev))
        if dr.randomize_restitution:
            st["restitution"].copy_(self._global_uniform(2, *dr.restitution_range))
        if dr.randomize_base_mass:
            st["payload"].copy_(self._global_uniform(3, *dr.added_mass_range))
        st["motor_strength"].fill_(1.0)
        st["root"][:, 6] = 1.0
        st["root"][:, :3] = self.env_origins + torch.as_tensor(list(cfg.init_state.pos), device=dev)
        for i, nme in enumerate(L.DOF_NAMES):
            st["dof_pos"][:, i] = float(cfg.init_state.default_joint_angles[nme])
        # outputs
        self._obs = torch.zeros((OUT_RING, n, self.num_obs), device=dev)
        self._priv = torch.zeros((OUT_RING, n, self.num_privileged_obs), device=dev)
        self._rew = torch.zeros((OUT_RING, n), device=dev)
        self._reset = torch.zeros((OUT_RING, n), dtype=torch.bool, device=dev)
        self._time_out = torch.zeros((OUT_RING, n), dtype=torch.bool, device=dev)
        self._slot = 0
        self._hist = None  # 2 wide (n, 70 x (history + HIST_WINDOW)) buffers when a HistoryWrapper attaches
        self._hist_buf, self._hist_off = 0, 0  # buffer and window (in observations) of the last returned history
        self._last_hist = None
        # compact episode log: one row per reset env (n_terms + 1 sums, tag, env)
        self._log_cap = max(4 * n, 1024)
        self._log = torch.zeros((self._log_cap, len(self.episode_keys) + 2), device=dev)
        self._log_count = torch.zeros(1, dtype=torch.int32, device=dev)
        self._log_tag = 0
        # gravity: Cfg.sim.gravity until the first scheduled draw (:719-723); projection vector -z (:1186)
        self.common_step_counter = 0
        self.gravities = np.zeros(3, np.float32)
        self._sim_gravity = np.asarray(cfg.sim.gravity, np.float32)
        self._gravity_vec = np.array([0.0, 0.0, -1.0], np.float32)
        self._host_rng = np.random.default_rng(self.seed)
        self._rng_step = 0
        self._args = [None] * OUT_RING
        self._args_grav = [None] * OUT_RING  # per output slot: the gravity versions / reward scales its args hold
        self._args_rs = [None] * OUT_RING
        self._grav_version = 0
        self._gravity_interval_i = int(self._gravity_interval)
        self.extras = self._make_extras()
        self.kernel_events = deque()
        # the first step's interval resample (none unless episode lengths were set)
        self._sim.resample(None, rng_seed=self.seed, rng_step=self._rng_step)

    # ---------------------------------------------------------------- host state
    def _global_uniform(self, tag, lo, hi):
        u = np.random.Generator(np.random.Philox(key=[self.seed, tag])).random(self._n_global).astype(np.float32)
        u = u[self.rank * self.num_envs:(self.rank + 1) * self.num_envs, None]
        return torch.from_numpy(u * np.float32(hi - lo) + np.float32(lo)).to(self.device)

    def _randomize_gravity(self, external_force=None):
        """_randomize_gravity (:564-579): one global draw shared by every env (and rank)."""
        if external_force is not None:
            self.gravities[:] = np.asarray(external_force, np.float32)
        elif self.cfg.domain_rand.randomize_gravity:
            lo, hi = self.cfg.domain_rand.gravity_range
            u = self._host_rng.random(3).astype(np.float32)
            self.gravities[:] = u * np.float32(hi - lo) + np.float32(lo)
        self._sim_gravity, self._gravity_vec = CF.gravity_state(self.gravities)
        self._grav_version += 1

    @property
    def state(self):
        return self._sim.state

    @property
    def obs_buf(self):
        return self._obs[(self._slot - 1) % OUT_RING]

    @property
    def privileged_obs_buf(self):
        return self._priv[(self._slot - 1) % OUT_RING]

    @property
    def rew_buf(self):
        return self._rew[(self._slot - 1) % OUT_RING]

    @property
    def reset_buf(self):
        return self._reset[(self._slot - 1) % OUT_RING]

    @property
    def time_out_buf(self):
        return self._time_out[(self._slot - 1) % OUT_RING]

    @property
    def episode_length_buf(self):
        return self._sim.state["episode_length"][:, 0]

    @property
    def commands(self):
        return self._sim.state["commands"]

    @property
    def root_states(self):
        return self._sim.state["root"]

    @property
    def dof_pos(self):
        return self._sim.state["dof_pos"]

    @property
    def dof_vel(self):
        return self._sim.state["dof_vel"]

    @property
    def base_lin_vel(self):
        return self._sim.aux[:, 0:3]

    @property
    def base_ang_vel(self):
        return self._sim.aux[:, 3:6]

    @property
    def foot_positions(self):
        return self._sim.aux[:, 6:18].view(-1, 4, 3)

    @property
    def torques(self):
        return self._sim.aux[:, 18:30]

    @property
    def joint_pos_target(self):
        return self._sim.aux[:, 30:42]

    @property
    def contact_forces(self):
        return self._sim.contact_forces

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    # ---------------------------------------------------------------- history (HistoryWrapper fusion)
    def attach_history(self, length):
        """Fuse HistoryWrapper.step's shift-and-append into the step.  The env keeps two buffers of rows
        70 x (length + HIST_WINDOW) wide; the history a step returns is a (n, 70 x length) window of one of
        them (row stride 70 x (length + HIST_WINDOW), inner stride 1): the next step's window starts one
        observation further, so cat(obs_history[:, 70:], obs) is only the new observation written past the
        window's end (history_wrapper.py:22 without moving 33 MB per step at 4096 envs x 30).  Every
        HIST_WINDOW steps, or when the caller hands in a history that is not the last window, the step
        shifts it into the start of the other buffer.  A returned window keeps its values for HIST_WINDOW
        further steps; the wrapper's in-place zeroing (reset / reset_idx) writes through to the following
        windows, as it would to the reference's tensor."""
        if length != self._vcfg.history_len:
            return False
        if self._hist is None:
            self._hist = torch.zeros((2, self.num_envs, (length + HIST_WINDOW) * self.num_obs), device=self.device)
        return True

    def _history_windows(self, history_in):
        """-> (in, in_ld, out view) of this step's history (see attach_history)."""
        no, W = self.num_obs, self._vcfg.history_len * self.num_obs
        last = self._last_hist
        if (last is not None and history_in.data_ptr() == last.data_ptr() and history_in.stride() == last.stride()
                and self._hist_off < HIST_WINDOW):
            self._hist_off += 1
            o = self._hist_off * no
            return history_in, history_in.stride(0), self._hist[self._hist_buf][:, o:o + W]
        if history_in.shape != (self.num_envs, W) or history_in.stride(1) != 1:
            history_in = history_in.contiguous()
        if history_in.untyped_storage().data_ptr() == self._hist.untyped_storage().data_ptr() and \
                (last is None or history_in.data_ptr() != last.data_ptr()):
            history_in = history_in.clone()  # an older window: it may lie where the rewind writes
        self._hist_buf ^= 1
        self._hist_off = 0
        return history_in, history_in.stride(0), self._hist[self._hist_buf][:, :W]

    # ---------------------------------------------------------------- step
    def step(self, actions, history_in=None):
        """VelocityTrackingEasyEnv.step (__init__.py:22-44): obs, rew, reset, extras."""
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(actions)
        if a.device != self.device or a.dtype != torch.float32:
            a = a.to(self.device, torch.float32)
        if a.requires_grad:
            a = a.detach()
        if not a.is_contiguous():
            a = a.contiguous()
        if a.shape != (self.num_envs, self.num_actions):
            raise ValueError(f"actions must be ({self.num_envs}, {self.num_actions}), got {tuple(a.shape)}")
        s = self._slot
        args = self._args[s]
        if args is None:
            args = self._args[s] = self._sim.args()
            args.obs, args.priv, args.rew = self._obs[s].data_ptr(), self._priv[s].data_ptr(), self._rew[s].data_ptr()
            args.reset, args.time_out = self._reset[s].data_ptr(), self._time_out[s].data_ptr()
            args.episode_log, args.episode_log_count = self._log.data_ptr(), self._log_count.data_ptr()
            args.episode_log_cap = self._log_cap
        # post_physics bookkeeping order (:120-121, :719-723): the step's gravity projection uses the vector
        # before this step's schedule, orientation_control the one after, the physics the sim gravity before
        # (_randomize_gravity replaces the arrays, so these references keep the values before it)
        gvec, sgrav, vb = self._gravity_vec, self._sim_gravity, self._grav_version
        self.common_step_counter += 1
        c = self.common_step_counter
        gi = self._gravity_interval_i
        if c % gi == 0:
            self._randomize_gravity()
        if int(c - self._gravity_duration) % gi == 0:
            self._randomize_gravity(np.zeros(3, np.float32))
        args.actions = a.data_ptr()
        # the args of an output slot are rewritten only where they changed since that slot's last step
        gkey = (vb, self._grav_version)
        if self._args_grav[s] != gkey:
            args.gravity_vec[:] = [float(x) for x in gvec]
            args.gravity_vec_after[:] = [float(x) for x in self._gravity_vec]
            args.sim_gravity[:] = [float(x) for x in sgrav]
            self._args_grav[s] = gkey
        rs = tuple(self.reward_scales[k] for k in self.reward_names)
        if self._args_rs[s] != rs:
            args.reward_scales[:] = [float(np.float32(x)) for x in rs] + [0.0] * (VA.GO1_VEL_MAX_TERMS - len(rs))
            self._args_rs[s] = rs
        args.rng_seed, args.rng_step = self.seed, self._rng_step
        self._log_tag += 1
        args.episode_log_tag = self._log_tag
        hist = None
        if history_in is not None and self._hist is not None:
            hin, ld_in, hist = self._history_windows(history_in)
            args.obs_history_in, args.obs_history_out = hin.data_ptr(), hist.data_ptr()
            args.obs_history_in_ld, args.obs_history_out_ld = ld_in, hist.stride(0)
            self._hist_in_keep = hin  # alive until the launch is enqueued
        else:
            args.obs_history_in = args.obs_history_out = None
        events = self.kernel_events.popleft() if self.kernel_events else None
        args.ev_begin, args.ev_end = events if events is not None else (None, None)
        self._sim.step(args)
        self._last_hist = hist
        self._rng_step += 1
        self._slot = (s + 1) % OUT_RING
        self._last_actions_t = a
        dict.__setitem__(self.extras, "privileged_obs", self._priv[s])
        return self._obs[s], self._rew[s], self._reset[s], self.extras

    def _make_extras(self):
        """The env's extras dict, built once: the VelocityTrackingEasyEnv.step numpy extras (:25-41) and
        reset_idx's "train/episode" are computed when read (no device->host copy per step)."""
        from .env import StepExtras
        ex = StepExtras(self)
        ex.set_lazy("time_outs", lambda: self._sim.extras_time_outs[: self.num_train_envs])
        ex.set_lazy("train/episode", self._episode_extras)
        ex.set_lazy("joint_pos", lambda: self.dof_pos.cpu().numpy())
        ex.set_lazy("joint_vel", lambda: self.dof_vel.cpu().numpy())
        ex.set_lazy("joint_pos_target", lambda: self.joint_pos_target.cpu().numpy())
        dict.__setitem__(ex, "joint_vel_target", torch.zeros(12))
        ex.set_lazy("body_linear_vel", lambda: self.base_lin_vel.cpu().numpy())
        ex.set_lazy("body_angular_vel", lambda: self.base_ang_vel.cpu().numpy())
        ex.set_lazy("body_linear_vel_cmd", lambda: self.commands.cpu().numpy()[:, 0:2])
        ex.set_lazy("body_angular_vel_cmd", lambda: self.commands.cpu().numpy()[:, 2:])
        ex.set_lazy("contact_states",
                    lambda: (self.contact_forces[:, list(L.FEET_INDICES), 2] > 1.0).cpu().numpy().copy())
        ex.set_lazy("foot_positions", lambda: self.foot_positions.cpu().numpy().copy())
        ex.set_lazy("body_pos", lambda: self.root_states[:, 0:3].cpu().numpy())
        ex.set_lazy("torques", lambda: self.torques.cpu().numpy())
        return ex

    def _flush_episode_log(self):
        pass

    def _deferred_time_outs(self):
        """extras["time_outs"] for the PPO record kernel: the curriculum launch of go1_vel_step already applied
        the step's rebinding in stream order, so nothing is pending."""
        return self._sim.extras_time_outs[: self.num_train_envs], None

    def _episode_extras(self):
        """extras["train/episode"] of the last step's reset_idx (:199-249): means of the episode sums over the
        envs reset by that step, the command range statistics and the curricula's areas."""
        cnt = min(int(self._log_count.item()), self._log_cap)
        rows = self._log[:cnt].cpu().numpy()
        ne = len(self.episode_keys)
        if cnt:  # the latest reset's rows (the reference rebuilds the dict at each reset_idx, :199-205)
            tags = np.ascontiguousarray(rows[:, ne]).view(np.int32)  # the kernels store the tag's int32 bits
            rows = rows[tags == tags.max()]
        out = {}
        if rows.shape[0]:
            rows = rows[np.argsort(rows[:, ne + 1], kind="stable")]
            for i, k in enumerate(self.episode_keys):
                out["rew_" + k] = np.float32(rows[:, i].astype(np.float32).mean(dtype=np.float32))
        cmd = self.commands.cpu().numpy()
        for name, col in (("duration", 8), ("bound", 7), ("offset", 6), ("phase", 5), ("freq", 4), ("x_vel", 0),
                          ("y_vel", 1), ("yaw_vel", 2), ("swing_height", 9)):
            out[f"min_command_{name}"] = cmd[:, col].min()
            out[f"max_command_{name}"] = cmd[:, col].max()
        w = self._sim.state["curriculum_weights"].cpu().numpy()
        for i, cat in enumerate(self.category_names):
            out[f"command_area_{cat}"] = np.sum(w[i]) / w.shape[1]
        act = getattr(self, "_last_actions_t", None)
        if act is not None:
            out["min_action"] = float(act.min())
            out["max_action"] = float(act.max())
        return out

    def reset_idx(self, env_ids):
        """reset_idx (:168-257) for explicit ids (the step resets its own envs in the kernel)."""
        env_ids = torch.as_tensor(env_ids, device=self.device).long().flatten()
        if env_ids.numel() == 0:
            return
        if int(env_ids.min()) < -self.num_envs or int(env_ids.max()) >= self.num_envs:
            raise IndexError(f"env id out of range for {self.num_envs} envs")
        env_ids = torch.remainder(env_ids, self.num_envs)
        self._log_tag += 1
        self._sim.reset_idx(env_ids, rng_seed=self.seed, rng_step=(1 << 62) + self._rng_step, log=self._log,
                            log_count=self._log_count, log_tag=self._log_tag)
        self._rng_step += 1
        self._sim.extras_time_outs.copy_(self.time_out_buf)  # extras["time_outs"] rebinding (:251-252)

    def reset(self):
        """VelocityTrackingEasyEnv.reset (__init__.py:46-49): reset_idx(all), then a zero-action step."""
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        obs, _, _, _ = self.step(torch.zeros(self.num_envs, self.num_actions, device=self.device))
        return obs

    # ---------------------------------------------------------------- misc API
    def start_recording(self):
        pass

    def pause_recording(self):
        pass

    def start_recording_eval(self):
        pass

    def pause_recording_eval(self):
        pass

    def get_complete_frames(self):
        return []

    def get_complete_frames_eval(self):
        return []

    def render(self, mode="rgb_array"):
        return None

    def close(self):
        self._sim.close()


del math
