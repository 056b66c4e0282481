"""Drop-in host side of the trajectory-tracking env over the HIP step.

Mirrors the reference's env API for the hot path:

  LeggedRobot            <- go1_gym/envs/base/legged_robot_trajectory_tracking.py:24-362
  TrajectoryTrackingEnv  <- go1_gym/envs/go1/trajectory_tracking/__init__.py:11-55
  HistoryWrapper         <- go1_gym/envs/wrappers/history_wrapper.py:6-41

Everything per-env runs in the fused HIP kernel (legged_tracking_amd/csrc/go1_step.hip)
through the C ABI (include/go1_mi355x.h); this module keeps only what the
reference keeps on the host or as global state:

  * common_step_counter, the global gravity schedule (_randomize_gravity :645-660,
    resampled every gravity_rand_interval steps and zeroed gravity_rand_duration
    later, :826-830) and the init quirk that projected_gravity uses [0, 0, -1]
    until the first resample (:1221 runs after create_sim's draw at :1574);
  * the exploration-scale decay of update_curriculum (:171-182), in float64 like
    the reference's Python floats;
  * extras: "train/episode" / "timeouts" are filled from the kernel's episode
    log lazily (one device->host copy when read, or every EPISODE_RING steps);
    the TrajectoryTrackingEnv.step numpy extras (:25-41) are computed on read.

Output tensors (obs, priv, rew, reset, time_out) rotate through OUT_RING buffers
so that a tensor returned by step() stays valid for OUT_RING-1 further steps
(the reference rebinds them every step; Runner / PPO hold the previous step's
observations across one env.step).

Differences from the reference, all documented in DESIGN.md:
  * root_states is (num_envs, 13) (the reference's also interleaves the arrow
    actors, num_actor = 2); the arrow actor is visual only;
  * extras["time_outs"] exists from the first step (all False until the first
    reset), which is numerically identical for PPO's bootstrapping (adds 0);
  * eval envs (eval_cfg), curriculum (cl_fix_target), push_robots and
    randomize_rigids_after_start are not on this path and raise.
"""
import math
from collections import defaultdict, deque

import numpy as np
import torch

from . import abi, config as CF, layout as L, terrain as T

OUT_RING = 4
EPISODE_RING = 64  # steps per half of the episode-log ring (fewer for very large n_envs)
_LAZY = object()


def _dist_info():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except Exception:
        pass
    return 0, 1


class StepExtras(dict):
    """The env's `extras` dict: device-backed entries are materialised on read."""

    def __init__(self, env):
        super().__init__()
        self._env = env
        self._lazy = {}

    def set_lazy(self, key, fn):
        self._lazy[key] = fn
        dict.__setitem__(self, key, _LAZY)

    def __getitem__(self, key):
        if key in ("train/episode", "eval/episode", "timeouts"):
            self._env._flush_episode_log()
        v = dict.__getitem__(self, key)
        return self._lazy[key]() if v is _LAZY else v

    def get(self, key, default=None):
        return self[key] if key in self else default

    def deferred_time_outs(self):
        """extras["time_outs"] with its pending rebinding left to the consumer: returns
        (tensor, (flag, pending, dst) device pointers or None).  The PPO record kernel resolves
        it (rollout.py PPO.process_env_step), saving the sync launch a plain read costs."""
        return self._env._deferred_time_outs()

    def items(self):
        return [(k, self[k]) for k in list(self.keys())]

    def values(self):
        return [self[k] for k in list(self.keys())]


class EpisodeLogRing:
    """Device ring of the kernel's per-step episode log (go1_step_args.episode_log) and its
    asynchronous trip to the host.

    Two halves of R steps.  When a half fills, a side stream copies it to pinned host
    memory while the next half is written; one half later (long finished, no wait) the
    copy's rows are set aside on the host (compact log), and they become deque entries only
    when extras["train/episode"] / ["timeouts"] is read -- building ~14 deques of 4000
    numpy scalars costs milliseconds, which the rollout loop used to pay every R steps.
    Reading those extras drains everything synchronously.
    Deques keep their last 4000 entries (deque(maxlen=4000), as the reference), so only
    the newest 4000 values per key are materialised.

    On the HIP backend the log is compact (go1_step_args.episode_log_count): only envs
    reset in a step append a row (+ step tag, env index), so a half's host trip and its
    processing scale with the resets, not with n_envs x R.  The async copy takes a prefix of
    `prefix` rows; a half with more rows fetches the rest when it is processed."""

    def __init__(self, env, n, device, compact=False):
        self.env = env
        self.dev = device
        self.n = n
        # steps per half: R x n_envs <= 4 M (dense layout: R x n x W floats per half, e.g. 64 x 4096 x 16 x 4 B
        # = 16 MB at the README size; at 256 k envs R = 16)
        self.R = R = int(min(EPISODE_RING, max(4, (1 << 22) // max(n, 1))))
        self.W = W = abi.episode_log_width(len(env.reward_names))
        self.cuda = device.type == "cuda"
        self.compact = compact and self.cuda
        self.dropped = 0  # compact rows the device had no room for (counted, never silently lost)
        if self.compact:
            # Rows of one half: the resets of R steps.  Every env resetting on every step would need
            # R x n rows (300 MB of (W + 2)-float rows per half at 256 k envs); the cap allows a quarter
            # of the envs resetting on EVERY step of the half (timeouts alone are n / 500 per step) and
            # at least 256 k rows.  The kernel counts every row it appends, kept or not (its atomic runs
            # before the cap test), so an overflow shows up as count > cap on the host.
            self.cap = min(R * n, max(4 * n, 1 << 18))
            self.prefix = min(self.cap, max(4 * n, 1024))
            self.buf = torch.zeros((2, self.cap, W + 2), device=device)
            self.count = torch.zeros((2, 1), dtype=torch.int32, device=device)
        else:
            self.buf = torch.zeros((2, R, n, W), device=device)
        self.half, self.slot, self.done = 0, 0, 0  # write position; slots (compact: rows) already drained
        if self.cuda:
            hshape = (2, self.prefix, W + 2) if self.compact else (2, R, n, W)
            self.host = torch.zeros(hshape, pin_memory=True)
            self.host_count = torch.zeros((2, 1), dtype=torch.int32, pin_memory=True)
            self.side = torch.cuda.Stream(device)
            self.copied = [None, None]  # event per half: host copy finished
            # the first device->pinned copy on the side stream costs ~6 ms of one-time setup
            # (measured by tools/rollout_jitter.py at the first hand-off): pay it here, not in
            # the rollout loop
            with torch.cuda.stream(self.side):
                for h in range(2):
                    if self.compact:
                        self.host_count[h].copy_(self.count[h], non_blocking=True)
                        self.host[h].copy_(self.buf[h, :self.prefix], non_blocking=True)
                    else:
                        self.host[h].copy_(self.buf[h], non_blocking=True)
            self.side.synchronize()
        self.inflight = None  # (half, first slot / row) copied to host, not yet turned into deque entries
        self.pending, self.pending_rows = [], 0  # compact rows on the host, oldest first, not yet in the deques

    def next_slot(self):
        """Buffer the kernel writes this step's log into (compact: the half's row buffer)."""
        if self.slot == 0 and self.cuda and self.copied[self.half] is not None:
            torch.cuda.current_stream(self.dev).wait_event(self.copied[self.half])  # half free again
        return self.buf[self.half] if self.compact else self.buf[self.half, self.slot]

    def advance(self):
        self.slot += 1
        if self.slot == self.R:
            h, first = self.half, self.done
            self.half, self.slot, self.done = h ^ 1, 0, 0
            if self.cuda:
                self._drain_inflight()
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.dev))
                self.side.wait_event(ev)
                with torch.cuda.stream(self.side):
                    if self.compact:
                        self.host_count[h].copy_(self.count[h], non_blocking=True)
                        self.host[h].copy_(self.buf[h, :self.prefix], non_blocking=True)
                    else:
                        self.host[h].copy_(self.buf[h], non_blocking=True)
                    done = torch.cuda.Event()
                    done.record(self.side)
                self.copied[h] = done
                self.inflight = (h, first)
            else:
                self._process(self.buf[h, first:].numpy())

    def _half_rows(self, h, first, cnt, host):
        """Rows [first, cnt) of compact half h (host prefix + a synchronous fetch beyond it)."""
        if cnt > self.cap:
            import warnings
            self.dropped += cnt - max(self.cap, first)
            warnings.warn(f"episode log: {cnt - self.cap} rows beyond the ring's capacity {self.cap} were dropped "
                          "(extras['episode_log_dropped'])")
            cnt = self.cap
        p = min(cnt, self.prefix) if host else first
        parts = [self.host[h, first:p].numpy()] if host and p > first else []
        if cnt > max(p, first):
            parts.append(self.buf[h, max(p, first):cnt].cpu().numpy())
        return np.concatenate(parts) if parts else np.zeros((0, self.W + 2), np.float32)

    def _drain_inflight(self):
        if self.inflight is not None:
            h, first = self.inflight
            self.inflight = None
            self.copied[h].synchronize()
            if self.compact:
                rows = self._half_rows(h, first, int(self.host_count[h, 0]), host=True)
                with torch.cuda.stream(self.side):  # after the copy (same stream): the half starts empty
                    self.count[h].zero_()
                done = torch.cuda.Event()
                done.record(self.side)
                self.copied[h] = done
                self._defer(rows)
            else:
                self._process(self.host[h, first:].numpy())

    PENDING_MAX = 1 << 17  # rows set aside before they are turned into deque entries anyway

    def _defer(self, rows):
        if rows.shape[0]:
            self.pending.append(rows)
            self.pending_rows += rows.shape[0]
            if self.pending_rows > self.PENDING_MAX:
                self._flush_pending()

    def _flush_pending(self):
        """Rows set aside, oldest chunk first.  A row's tag is its step's slot in its half, so
        chunk i's tags are shifted by i R to make them increase across chunks; a step's rows
        never straddle two chunks, so one pass equals processing the chunks one by one."""
        if self.pending:
            for i, r in enumerate(self.pending):
                if i:
                    r[:, self.W] += np.float32(i * self.R)
            rows = np.concatenate(self.pending) if len(self.pending) > 1 else self.pending[0]
            self.pending, self.pending_rows = [], 0
            self._process_rows(rows)

    def drain(self):
        """Everything logged so far, synchronously (extras read)."""
        if self.cuda:
            self._drain_inflight()
        self._flush_pending()
        if self.compact:
            cnt = int(self.count[self.half, 0].item())
            if cnt > self.done:
                self._process_rows(self._half_rows(self.half, self.done, cnt, host=False))
                self.done = cnt
        elif self.slot > self.done:
            self._process(self.buf[self.half, self.done:self.slot].cpu().numpy())
            self.done = self.slot

    def _process_rows(self, rows):
        """Compact rows (m, W + 2) -> the dense (steps, envs, W) processing of _process, without
        building the dense array: order by (step tag, env) as the reference logs them (:256-271)."""
        env = self.env
        ntr = env.num_train_envs
        ns = len(env.sum_keys)
        W = self.W
        if rows.shape[0] == 0:
            return
        tag, eid = rows[:, W].astype(np.int64), rows[:, W + 1].astype(np.int64)
        keep = (eid < ntr) & (rows[:, ns] > 0)
        rows, tag, eid = rows[keep], tag[keep], eid[keep]
        if rows.shape[0] == 0:
            return
        order = np.lexsort((eid, tag))
        rows, tag, eid = rows[order], tag[order], eid[order]
        # timeouts: for each step with a reset, time_out of every train env (False unless reset
        # with episode length > max_episode_length), newest 4000 values
        steps = np.unique(tag)
        need = min(len(steps), 4000 // max(ntr, 1) + 1)
        tail = steps[len(steps) - need:]
        to = np.zeros((need, ntr), bool)
        sel = tag >= tail[0]
        pos = np.searchsorted(tail, tag[sel])
        to[pos, eid[sel]] = rows[sel, ns] > np.float32(env.max_episode_length)
        env._timeouts.extend(to.reshape(-1)[-4000:])
        self._extend(rows[-4000:])

    def _extend(self, rows):
        env = self.env
        ns = len(env.sum_keys)
        for i, key in enumerate(env.sum_keys):
            env._train_ep["rew_" + key].extend(rows[:, i])
        env._train_ep["episode_length"].extend(rows[:, ns])
        env._train_ep["reached"].extend(rows[:, ns + 1] > 0)
        env._train_ep["goal_distance"].extend(rows[:, ns + 2])

    def _process(self, logs):
        env = self.env
        ntr = env.num_train_envs
        ns = len(env.sum_keys)
        col = logs[:, :ntr, ns]                              # episode length, 0 = no reset
        steps, envs = np.nonzero(col > 0)                    # by step, then env
        if steps.size == 0:
            return
        rows = logs[steps, envs][-4000:]
        reset_steps = np.unique(steps)
        timeouts = (col[reset_steps] > np.float32(env.max_episode_length)).reshape(-1)[-4000:]
        env._timeouts.extend(timeouts)
        self._extend(rows)


def _episode_dicts():
    return defaultdict(lambda: deque([], 4000)), defaultdict(lambda: deque([], 4000)), deque([], 4000)


class LeggedRobot:
    """LeggedRobot (:24-362) for the README configuration, backed by the HIP step."""

    def __init__(self, cfg, sim_params=None, physics_engine="SIM_PHYSX", sim_device="cuda:0", headless=True,
                 eval_cfg=None, initial_dynamics_dict=None, *, seed=11, rank=None, world_size=None, backend=None,
                 physics=None):
        if eval_cfg is not None:
            raise NotImplementedError("eval envs (eval_cfg) are not on the accelerated path")
        if cfg.curriculum_thresholds.cl_fix_target:
            raise NotImplementedError("cl_fix_target curriculum is not on the accelerated path")
        dr = cfg.domain_rand
        if getattr(dr, "push_robots", False) or getattr(dr, "randomize_rigids_after_start", False):
            raise NotImplementedError("push_robots / randomize_rigids_after_start are not on the accelerated path")
        self.cfg = cfg
        self.eval_cfg = None
        self.sim_device = sim_device
        self.headless = headless
        if rank is None or world_size is None:
            r, w = _dist_info()
            rank = r if rank is None else rank
            world_size = w if world_size is None else world_size
        self.rank, self.world_size = rank, world_size
        self.num_obs = cfg.env.num_observations
        self.num_privileged_obs = cfg.env.num_privileged_obs
        self.num_actions = cfg.env.num_actions
        self.num_envs = self.num_train_envs = cfg.env.num_envs
        self.num_eval_envs = 0
        self.seed = int(seed)
        d = CF.derived(cfg)
        self.dt = d["dt"]
        self.max_episode_length_s = cfg.env.episode_length_s
        self.max_episode_length = d["max_episode_length"]
        self.reward_scales = dict(d["reward_scales"])
        # reward slots in Cfg.reward_scales order (the C ABI's term table; unknown terms raise in
        # build_abi_config, terms the container lacks keep a zero sum as in the reference :1390-1395)
        self.reward_names = list(self.reward_scales)
        self.sum_keys = tuple(self.reward_names) + ("total", "total_pos", "total_neg")
        self._gravity_interval = d["gravity_rand_interval"]
        self._gravity_duration = d["gravity_rand_duration"]
        n, n_global = self.num_envs, self.num_envs * world_size
        self._abi_cfg = CF.build_abi_config(cfg, n_envs=n, physics=physics)
        self._abi_cfg.env_id_offset = rank * n
        # terrain: the global grid is built identically on every rank (same seed), each
        # rank binds the slice of global env ids it owns (_get_env_origins :1808-1847)
        # the tunnel tiles come from the GPU generator (go1_tunnel_tiles) with the native backend,
        # bit-identical to the host restatement T.make_single_path that injected test backends use
        tiles_fn = None
        if backend is None:  # the HIP library (no CPU fallback); tests inject a factory
            from . import native
            backend = lambda c: native.Go1Native(c, sim_device)  # noqa: E731
            tiles_fn = lambda t, lay: native.tunnel_tiles(t, lay, self.seed, self._sim.device)  # noqa: E731
        self._sim = backend(self._abi_cfg)
        self.device = self._sim.device
        td = T.build(cfg, n_global, np.random.RandomState(self.seed), tiles_fn=tiles_fn)
        sl = slice(rank * n, (rank + 1) * n)
        self.terrain = td
        self._sim.set_terrain(td.tiles, td.env_tile[sl], td.env_terrain_origin[sl], td.env_origins[sl])
        self.env_origins = torch.as_tensor(td.env_origins[sl], device=self.device)
        dev = self.device
        # output rings
        self._obs = torch.zeros((OUT_RING, n, self.num_obs), device=dev)
        self._obs_hist = None  # ring of kernel-written obs copies, allocated by _history_tap()
        self._last_hist = None
        self._priv = torch.zeros((OUT_RING, n, self.num_privileged_obs), device=dev)
        self._rew = torch.zeros((OUT_RING, n), device=dev)
        self._reset = torch.zeros((OUT_RING, n), dtype=torch.bool, device=dev)
        self._time_out = torch.zeros((OUT_RING, n), dtype=torch.bool, device=dev)
        self._slot = 0
        # the compact episode log needs the HIP backend's prepared-args path, and rows that the
        # global pos/neg bucket pass (indefinite reward slots) does not rewrite by env index
        self._fast = hasattr(self._sim, "prepare")
        self._elog = EpisodeLogRing(self, n, dev, compact=self._fast and not self._abi_cfg.indefinite_slots)
        self._prepared = {}
        self._aux = torch.zeros((n, abi.GO1_AUX), device=dev)
        # which per-step outputs the kernel stores beyond obs / rewards / resets (set_output_demand)
        self._demand = (True, True)
        # envs the native integrator's divergence guard reset, cumulative (extras["diverged"])
        self._diverged = torch.zeros(1, dtype=torch.int64, device=dev)
        # host RNG for the global gravity draws: identical on every rank
        self._host_rng = np.random.default_rng(self.seed)
        self._n_global = n_global
        self._reset_draws = 0
        # _init_custom_buffers__ / _randomize_rigid_body_props (:1329-1350, :710-733): per-env draws
        # keyed by GLOBAL env id (every rank draws the global vector and keeps its slice), so an
        # N-rank run starts from exactly the state one rank with N x the envs does
        st = self._sim.state
        if dr.randomize_friction:
            lo, hi = dr.friction_range
            st["friction"].copy_(self._global_uniform(1, lo, hi))
        else:
            st["friction"].fill_(1.0)
        if dr.randomize_restitution:
            lo, hi = dr.restitution_range
            st["restitution"].copy_(self._global_uniform(2, lo, hi))
        if dr.randomize_base_mass:
            lo, hi = dr.added_mass_range
            st["payload"].copy_(self._global_uniform(3, lo, hi))
        st["motor_strength"].fill_(1.0)
        # gravity (:1574 then :1221): sim gravity drawn, projection vector reset to -z
        self.common_step_counter = 0
        self.gravities = np.zeros(3, np.float32)
        self._randomize_gravity()
        self._gravity_vec = np.array([0.0, 0.0, -1.0], np.float32)
        self.extras = StepExtras(self)
        self._train_ep, self._eval_ep, self._timeouts = _episode_dicts()
        self._install_extras()
        self._rng_step = 0
        # measurement hook (bench.py): hipEvent_t pairs to record around the next steps' kernel
        self.kernel_events = deque()

    # ------------------------------------------------------------------ host state
    def _global_rng(self, tag):
        """numpy Philox stream of (seed, tag): the same on every rank, indexed by global env id."""
        return np.random.Generator(np.random.Philox(key=[self.seed, tag]))

    def _global_uniform(self, tag, lo, hi):
        """(n, 1) f32 U(lo, hi) for this rank's envs, element i = global env rank * n + i."""
        u = self._global_rng(tag).random(self._n_global).astype(np.float32)
        u = u[self.rank * self.num_envs:(self.rank + 1) * self.num_envs, None]
        return torch.from_numpy(u * np.float32(hi - lo) + np.float32(lo)).to(self.device)

    def _randomize_gravity(self, external_force=None):
        """_randomize_gravity (:645-660): one global draw shared by every env (and rank)."""
        if external_force is not None:
            self.gravities[:] = np.asarray(external_force, np.float32)
        elif self.cfg.domain_rand.randomize_gravity:
            lo, hi = self.cfg.domain_rand.gravity_range
            u = self._host_rng.random(3).astype(np.float32)
            self.gravities[:] = u * np.float32(hi - lo) + np.float32(lo)
        self._sim_gravity, self._gravity_vec = CF.gravity_state(self.gravities)

    @property
    def gravity_vec(self):
        return torch.as_tensor(self._gravity_vec, device=self.device).repeat(self.num_envs, 1)

    def _scale_vector(self):
        return CF.reward_scale_vector(self.reward_scales, self.reward_names)

    def _step_consts(self):
        """(key, gravity_vec, sim_gravity, reward_scales) of the next step; the key changes
        only when one of them does (gravity schedule, exploration decay)."""
        key = (self._gravity_vec.tobytes(), self._sim_gravity.tobytes(),
               tuple(self.reward_scales[k] for k in self.reward_names))
        c = getattr(self, "_consts_cache", None)
        if c is None or c[0] != key:
            c = self._consts_cache = (key, self._gravity_vec, self._sim_gravity, self._scale_vector())
        return c

    def _install_extras(self):
        ex = self.extras
        dict.__setitem__(ex, "train/episode", self._train_ep)
        dict.__setitem__(ex, "eval/episode", self._eval_ep)
        dict.__setitem__(ex, "timeouts", self._timeouts)
        # the rebinding of the last step is applied on read (go1_sync_time_outs)
        ex.set_lazy("time_outs", lambda: self._sim.sync_time_outs()[: self.num_train_envs])
        # native-integrator health (no reference counterpart): envs reset by the divergence guard so far
        ex.set_lazy("diverged", lambda: int(self._diverged.item()))
        # compact episode-log rows that overflowed the device ring (0 unless a quarter of the envs reset
        # on every step of a half)
        ex.set_lazy("episode_log_dropped", lambda: (self._elog.drain(), self._elog.dropped)[1])

    def _deferred_time_outs(self):
        sim = self._sim
        p = sim.time_outs_pending() if hasattr(sim, "time_outs_pending") else None
        if p is None and hasattr(sim, "time_outs_pending"):
            return sim.extras_time_outs[: self.num_train_envs], None
        if p is None:  # a backend without the deferred protocol: plain (synchronising) read
            return self.extras["time_outs"], None
        return sim.extras_time_outs[: self.num_train_envs], p

    # ------------------------------------------------------------------ views
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

    @episode_length_buf.setter
    def episode_length_buf(self, v):
        self._sim.state["episode_length"][:, 0].copy_(torch.as_tensor(v, device=self.device))

    @property
    def root_states(self):
        return self._sim.state["root"]

    @property
    def base_pos(self):
        return self._sim.state["root"][:, 0:3]

    @property
    def base_quat(self):
        return self._sim.state["root"][:, 3:7]

    @property
    def dof_pos(self):
        return self._sim.state["dof_pos"]

    @property
    def dof_vel(self):
        return self._sim.state["dof_vel"]

    @property
    def last_actions(self):
        return self._sim.state["last_actions"]

    @property
    def joint_pos_target(self):
        return self._sim.state["joint_pos_target"]

    def set_output_demand(self, contact_forces=True, aux=True):
        """Whether each step stores the contact forces (n, 17, 3) and the aux block (base velocities, commands,
        foot positions, torques) -- 204 + 128 B per env-step of HBM writes.  Both default on: the reference
        refreshes them every step (legged_robot_trajectory_tracking.py:64-112, gym.refresh_net_contact_force_tensor)
        and the extras read them.  Runner.learn switches both off while it collects rollouts, which read neither
        (ppo_cse/__init__.py:164-214), and restores them; reading one while it is off raises instead of returning
        a stale step."""
        self._demand = (bool(contact_forces), bool(aux))

    def _aux_view(self, a, b):
        if not self._demand[1]:
            raise RuntimeError("the aux outputs are not stored while set_output_demand(aux=False) is in effect")
        return self._aux[:, a:b]

    @property
    def contact_forces(self):
        if not self._demand[0]:
            raise RuntimeError("contact_forces are not stored while set_output_demand(contact_forces=False) is in "
                               "effect")
        return self._sim.contact_forces

    @property
    def torques(self):
        return self._aux_view(20, 32)

    @property
    def base_lin_vel(self):
        return self._aux_view(0, 3)

    @property
    def base_ang_vel(self):
        return self._aux_view(3, 6)

    @property
    def commands(self):
        return self._aux_view(6, 8)

    @property
    def foot_positions(self):
        return self._aux_view(8, 20).view(-1, 4, 3)

    @property
    def episode_sums(self):
        s = self._sim.state["episode_sums"]
        return {k: s[:, i] for i, k in enumerate(self.sum_keys)}

    def get_observations(self):
        return self.obs_buf

    def _history_tap(self):
        """Have the step kernel also write each step's obs into a ring of its own: the
        HistoryWrapper's obs_history for a history length of 1 (a fresh copy of obs every
        step, history_wrapper.py:18-24) without a separate copy launch."""
        if self._obs_hist is None:
            self._obs_hist = torch.zeros_like(self._obs)
        return True

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    # ------------------------------------------------------------------ step
    def step(self, actions):
        """LeggedRobot.step (:64-112): returns obs, privileged_obs, rew, reset, extras."""
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
        events = self.kernel_events.popleft() if self.kernel_events else None
        if self._fast:
            el = self._elog
            log = el.next_slot()
            key = (s, el.half if el.compact else el.slot + el.R * el.half, self._obs_hist is not None, self._demand)
            p = self._prepared.get(key)
            if p is None:
                p = self._prepared[key] = self._prepare_slot(s, log)
            args, out, hist = p
            ck, gvec, sgrav, scales = self._step_consts()
            self._sim.step_prepared(args, a, gvec, sgrav, scales, ck, self.seed, self._rng_step, events=events,
                                    log_tag=el.slot)
        else:
            out = dict(obs=self._obs[s], priv=self._priv[s], rew=self._rew[s], reset=self._reset[s],
                       time_out=self._time_out[s])
            hist = self._obs_hist[s] if self._obs_hist is not None else None
            cf = {} if self._demand[0] else {"contact_forces": False}
            self._sim.step(a, self._gravity_vec, self._sim_gravity, self._scale_vector(), rng_seed=self.seed,
                           rng_step=self._rng_step, out=out, episode_log=self._elog.next_slot(),
                           aux=self._aux if self._demand[1] else None, obs_history=hist, events=events,
                           diverged_count=self._diverged, **cf)
        self._last_hist = hist
        self._rng_step += 1
        self._elog.advance()
        self._slot = (s + 1) % OUT_RING
        # post-physics host bookkeeping (:126, :826-830, :171-182)
        self.common_step_counter += 1
        c = self.common_step_counter
        if c % int(self._gravity_interval) == 0:
            self._randomize_gravity()
        if int(c - self._gravity_duration) % int(self._gravity_interval) == 0:
            self._randomize_gravity(np.zeros(3, np.float32))
        self.update_curriculum()
        return out["obs"], out["priv"], out["rew"], out["reset"], self.extras

    def _prepare_slot(self, s, log):
        """Validated go1_step_args for output-ring slot s and this episode-log buffer."""
        out = dict(obs=self._obs[s], priv=self._priv[s], rew=self._rew[s], reset=self._reset[s],
                   time_out=self._time_out[s])
        hist = self._obs_hist[s] if self._obs_hist is not None else None
        el = self._elog
        args = self._sim.prepare(out, aux=self._aux if self._demand[1] else None, obs_history=hist,
                                 diverged_count=self._diverged, episode_log=log,
                                 log_count=el.count[el.half] if el.compact else None,
                                 contact_forces=self._demand[0])
        return args, out, hist

    def update_curriculum(self):
        """update_curriculum (:171-182): exploration scales decay after exploration_steps."""
        rw = self.cfg.rewards
        for key in ("exploration_lin", "exploration_yaw"):
            if key in self.reward_scales:
                if self.common_step_counter > rw.exploration_steps:
                    self.reward_scales[key] -= getattr(self.cfg.reward_scales, key) * self.dt / rw.exploration_steps
                    self.reward_scales[key] = max(self.reward_scales[key], 0)
                self._train_ep[key] = self.reward_scales[key]

    def reset_idx(self, env_ids):
        """reset_idx (:218-296) for explicit ids (the step resets its own envs in the kernel)."""
        env_ids = torch.as_tensor(env_ids, device=self.device).long().flatten()
        if env_ids.numel() == 0:
            return
        if int(env_ids.min()) < -self.num_envs or int(env_ids.max()) >= self.num_envs:
            raise IndexError(f"env id out of range for {self.num_envs} envs")  # as the reference's indexing
        env_ids = torch.remainder(env_ids, self.num_envs)
        self._flush_episode_log()
        st = self._sim.state
        sums = st["episode_sums"][env_ids].cpu().numpy()
        ep = st["episode_length"][env_ids, 0].float().cpu().numpy()
        for i, key in enumerate(self.sum_keys):
            self._train_ep["rew_" + key].extend(sums[:, i])
        self._train_ep["episode_length"].extend(ep)
        self._sim.reset_idx(env_ids, rng_seed=self.seed, rng_step=(1 << 62) + self._rng_step)
        self._rng_step += 1
        tb = self.time_out_buf[: self.num_train_envs]
        self._timeouts.extend(tb.cpu().numpy())
        self._sim.extras_time_outs.copy_(tb)  # extras["time_outs"] rebinding (:289-291)

    def reset(self):
        """BaseTask.reset (base_task.py:93-99)."""
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        obs, privileged_obs, _, _, _ = self.step(torch.zeros(self.num_envs, self.num_actions, device=self.device))
        return obs, privileged_obs

    # ------------------------------------------------------------------ episode log
    def _flush_episode_log(self):
        self._elog.drain()

    # ------------------------------------------------------------------ misc API
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


class TrajectoryTrackingEnv(LeggedRobot):
    """TrajectoryTrackingEnv (trajectory_tracking/__init__.py:11-55)."""

    def __init__(self, sim_device="cuda:0", headless=True, num_envs=None, prone=False, deploy=False, cfg=None,
                 eval_cfg=None, initial_dynamics_dict=None, physics_engine="SIM_PHYSX", **kw):
        if cfg is None:
            cfg = CF.readme_config(n_envs=num_envs or 4096)
        if num_envs is not None:
            cfg.env.num_envs = num_envs
        super().__init__(cfg, None, physics_engine, sim_device, headless, eval_cfg, initial_dynamics_dict, **kw)
        n = self.num_envs
        ex = self.extras
        ex.set_lazy("joint_pos", lambda: self.dof_pos.cpu().numpy())
        ex.set_lazy("joint_vel", lambda: self.dof_vel.cpu().numpy())
        ex.set_lazy("joint_pos_target", lambda: self.joint_pos_target.cpu().numpy())
        dict.__setitem__(ex, "joint_vel_target", torch.zeros(12))
        ex.set_lazy("body_linear_vel", lambda: self.base_lin_vel.cpu().numpy())
        ex.set_lazy("body_angular_vel", lambda: self.base_ang_vel.cpu().numpy())
        ex.set_lazy("body_linear_vel_cmd", lambda: self.commands.cpu().numpy())
        ex.set_lazy("body_angular_vel_cmd", lambda: np.zeros((n, 0), np.float32))
        ex.set_lazy("contact_states",
                    lambda: (self.contact_forces[:, list(L.FEET_INDICES), 2] > 1.0).cpu().numpy().copy())
        ex.set_lazy("foot_positions", lambda: self.foot_positions.cpu().numpy().copy())
        ex.set_lazy("body_pos", lambda: self.base_pos.cpu().numpy())
        ex.set_lazy("torques", lambda: self.torques.cpu().numpy())

    def step(self, actions):
        obs, priv, rew, reset, extras = super().step(actions)
        dict.__setitem__(extras, "privileged_obs", priv)
        return obs, rew, reset, extras

    def reset(self):
        # reset_idx logs every finished episode into the current dicts (it drains the episode log
        # first); the reference then swaps in empty extras (trajectory_tracking/__init__.py:46-55),
        # so nothing logged before this reset reaches the new dicts
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        # torch.randint(max_episode_length, (num_envs,)) (:49), keyed by global env id like the DR draws
        self._reset_draws += 1
        el = self._global_rng(1000 + self._reset_draws).integers(0, int(self.max_episode_length), self._n_global)
        el = el[self.rank * self.num_envs:(self.rank + 1) * self.num_envs].astype(np.int32)
        self.episode_length_buf = torch.from_numpy(el).to(self.device)
        self._elog.drain()  # into the old dicts (empty: reset_idx drained), never into the new ones
        self._train_ep, self._eval_ep, self._timeouts = _episode_dicts()
        self._install_extras()
        obs, _, _, _ = self.step(torch.zeros(self.num_envs, self.num_actions, device=self.device))
        return obs


class HistoryWrapper:
    """HistoryWrapper (history_wrapper.py:6-41): dict observations with an obs history.

    History length 1 (the README configuration): the reference rebuilds obs_history every step as
    cat(obs_history[:, num_obs:], obs) = a fresh copy of obs.  Here obs_history IS the step's obs
    tensor (no copy: 1,044 B per env-step less HBM traffic); the wrapper's own in-place writes
    (reset_idx zeroing rows, reset zeroing it) go to a separate buffer, so obs is never touched.
    Only a caller that mutates obs_history in place would see obs change -- the Runner never does;
    copy_history=True restores a distinct tensor per step (the step kernel writes the second copy)."""

    def __init__(self, env, copy_history=False):
        self.env = env
        self.obs_history_length = self.env.cfg.env.num_observation_history
        self.num_obs_history = self.obs_history_length * self.env.num_obs
        self.obs_history = torch.zeros(self.env.num_envs, self.num_obs_history, dtype=torch.float,
                                       device=self.env.device)
        self.num_privileged_obs = self.env.num_privileged_obs
        self._alias = self.obs_history_length == 1 and not copy_history
        # history length 1 with a distinct tensor: the step kernel writes obs_history (a copy of obs) itself
        self._tap = (self.obs_history_length == 1 and copy_history and hasattr(self.env, "_history_tap") and
                     self.env._history_tap())
        # longer histories on an env that fuses the shift into its step (velocity.py: the step reads this
        # wrapper's obs_history and writes cat(obs_history[:, num_obs:], obs) into a buffer of its own)
        self._fused = (self.obs_history_length > 1 and hasattr(self.env, "attach_history") and
                       self.env.attach_history(self.obs_history_length))

    def __getattr__(self, name):
        return getattr(self.env, name)

    def _push(self, obs):
        if self.obs_history_length == 1:
            self.obs_history = obs if self._alias else obs.clone()
        else:
            self.obs_history = torch.cat((self.obs_history[:, self.env.num_obs:], obs), dim=-1)

    def step(self, action):
        if self._fused:
            obs, rew, done, info = self.env.step(action, history_in=self.obs_history)
            self.obs_history = self.env._last_hist
            return {"obs": obs, "privileged_obs": info["privileged_obs"], "obs_history": self.obs_history}, rew, \
                done, info
        obs, rew, done, info = self.env.step(action)
        privileged_obs = info["privileged_obs"]
        if self._tap:
            self.obs_history = self.env._last_hist
        else:
            self._push(obs)
        return {"obs": obs, "privileged_obs": privileged_obs, "obs_history": self.obs_history}, rew, done, info

    def get_observations(self):
        obs = self.env.get_observations()
        privileged_obs = self.env.get_privileged_observations()
        self._push(obs)
        return {"obs": obs, "privileged_obs": privileged_obs, "obs_history": self.obs_history}

    def reset_idx(self, env_ids):
        ret = self.env.reset_idx(env_ids)
        # never zero rows of the env's obs / its output ring in place; a fused window shares columns with the
        # windows returned before it (velocity.py), so it is cloned too: the next step then takes the rewind path
        if self._alias or self._tap or self._fused:
            self.obs_history = self.obs_history.clone()
        self.obs_history[env_ids, :] = 0
        return ret

    def reset(self):
        ret = self.env.reset()
        privileged_obs = self.env.get_privileged_observations()
        if self._alias or self._tap or self._fused:
            self.obs_history = torch.zeros_like(self.obs_history)
        else:
            self.obs_history[:, :] = 0
        return {"obs": ret, "privileged_obs": privileged_obs, "obs_history": self.obs_history}
