"""Thin host binding of the HIP C ABI (include/go1_mi355x.h) over PyTorch-ROCm tensors.

torch provides device memory and the stream; every computation of the step runs
in the HIP library legged_tracking_amd/_build/libgo1_mi355x.so.  If that library
is missing or the GPU is absent this module raises -- there is no CPU fallback.
"""
import ctypes as C
import os

import numpy as np
import torch

from . import abi, layout as L

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GO1_LIB_OVERRIDE") or os.path.join(HERE, "_build", "libgo1_mi355x.so")
_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load the HIP library (fails loudly; build with __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"HIP extension missing: {LIB_PATH} (run python -c 'import __graft_entry__ as g; g.build()')")
    l = C.CDLL(LIB_PATH)
    l.go1_abi_version.restype = C.c_int
    l.go1_last_error.restype = C.c_char_p
    l.go1_create.argtypes = [C.POINTER(abi.Go1Config), C.POINTER(C.c_void_p)]
    l.go1_bind.argtypes = [C.c_void_p, C.POINTER(abi.Go1State), C.POINTER(abi.Go1Plane)]
    l.go1_set_terrain.argtypes = [C.c_void_p, C.POINTER(abi.Go1Terrain)]
    l.go1_step.argtypes = [C.c_void_p, C.POINTER(abi.Go1StepArgs), C.c_void_p]
    l.go1_reset_envs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p]
    l.go1_reset_idx.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p]
    l.go1_sync_time_outs.argtypes = [C.c_void_p, C.c_void_p]
    l.go1_time_outs_pending.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    l.go1_actuator_net.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    l.go1_destroy.argtypes = [C.c_void_p]
    l.go1_specialize.argtypes = [C.c_void_p, C.c_int]
    l.go1_is_specialized.argtypes = [C.c_void_p]
    l.go1_tunnel_tiles.argtypes = [C.POINTER(abi.Go1TunnelParams), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    if l.go1_abi_version() != abi.GO1_ABI_VERSION:
        raise NativeError("ABI version mismatch")
    _lib = l
    return l


def _check(rc):
    if rc != 0:
        raise NativeError(lib().go1_last_error().decode())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def tunnel_tiles(cfg_terrain, layout, seed, device):
    """single_path tiles generated on the GPU (go1_tunnel_tiles): the tiles the reference's
    Terrain(cfg) builds after np.random.seed(seed), as a (rows, cols, 2, tile_x, tile_y) f32
    tensor on `device` (tunnel.py:51-217, tunnel_fn.py:99-163)."""
    t = cfg_terrain
    rows, cols = int(t.num_rows), int(t.num_cols)
    if not 0 <= int(seed) < 2 ** 32:
        raise ValueError("seed must be in [0, 2**32) (numpy RandomState)")
    p = abi.Go1TunnelParams(num_rows=rows, num_cols=cols, tile_x=layout.tile_x, tile_y=layout.tile_y,
                            sub_x=layout.sub_shape[0], sub_y=layout.sub_shape[1], seed=int(seed),
                            horizontal_scale=float(t.horizontal_scale), vertical_scale=float(t.vertical_scale),
                            ceiling_height=float(t.ceiling_height), p_flat=float(t.p_flat),
                            p_double=float(t.p_double))
    ex = np.ascontiguousarray(layout.extents, np.int32)
    span = np.stack([ex[:, 1] - ex[:, 0], ex[:, 3] - ex[:, 2]], 1)
    bad = np.nonzero((span != np.array([layout.sub_shape[1], layout.sub_shape[0]])).any(1))[0]
    if bad.size:  # the reference's tile[0, sx:ex, sy:ey] = top.T raises on this mismatch (tunnel.py:193-196)
        k = int(bad[0])
        raise ValueError(f"sub-terrain {k}: tunnel extent {tuple(span[k])} does not match the sub-terrain shape "
                         f"{(layout.sub_shape[1], layout.sub_shape[0])} (could not broadcast)")
    ext = torch.as_tensor(ex).to(device)
    rec = torch.empty((rows * cols, abi.GO1_TUNNEL_REC), dtype=torch.float64, device=device)
    tiles = torch.empty((rows, cols, 2, layout.tile_x, layout.tile_y), dtype=torch.float32, device=device)
    with torch.cuda.device(device):
        _check(lib().go1_tunnel_tiles(C.byref(p), ext.data_ptr(), rec.data_ptr(), tiles.data_ptr(), _stream()))
    torch.cuda.current_stream(device).synchronize()  # ext / rec are freed on return
    return tiles


class StateTensors:
    """go1_state planes as torch tensors on the device (SoA, row-major (n, width))."""

    def __init__(self, n, device, cfg):
        self.n = n
        self.t = {}
        for name, w, dt in abi.state_spec(cfg):
            self.t[name] = torch.zeros((n, w), dtype=torch.float32 if dt == "f32" else torch.int32, device=device)

    def struct(self):
        return abi.Go1State(**{k: v.data_ptr() for k, v in self.t.items()})

    def __getitem__(self, k):
        return self.t[k]

    def load(self, arrays: dict):
        for k, v in arrays.items():
            if k in self.t:
                self.t[k].copy_(torch.as_tensor(np.asarray(v)).reshape(self.t[k].shape).to(self.t[k].dtype))

    def numpy(self):
        return {k: v.cpu().numpy() for k, v in self.t.items()}


class Go1Native:
    """Owns one go1_handle and the device buffers the C ABI writes."""

    def __init__(self, cfg: abi.Go1Config, device="cuda:0"):
        if not torch.cuda.is_available():
            raise NativeError("no GPU visible: the MI355X step has no CPU fallback")
        self.device = torch.device(device)
        self.cfg = cfg
        self.n = n = cfg.n_envs
        self.h = C.c_void_p()
        with torch.cuda.device(self.device):
            _check(lib().go1_create(C.byref(cfg), C.byref(self.h)))
            self.state = StateTensors(n, self.device, cfg)
            self.bind(self.state)
            dev = self.device
            self.obs = torch.zeros((n, cfg.num_obs), device=dev)
            self.priv = torch.zeros((n, abi.GO1_NUM_PRIV), device=dev)
            self.rew = torch.zeros(n, device=dev)
            self.reset = torch.zeros(n, dtype=torch.bool, device=dev)
            self.time_out = torch.zeros(n, dtype=torch.bool, device=dev)
            self.extras_time_outs = torch.zeros(n, dtype=torch.bool, device=dev)
            self.contact_forces = torch.zeros((n, 17, 3), device=dev)
        self._terrain_keep = None
        self._args = None
        self._consts = None
        self._lib_step = lib().go1_step
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()

    def bind(self, state):
        """go1_bind the planes of `state` (StateTensors or {name: tensor}); the library checks their
        shapes, dtypes and strides and raises NativeError for anything but dense (n_envs, width)."""
        t = state.t if hasattr(state, "t") else state
        s = abi.Go1State(**{k: t[k].data_ptr() for k, _ in abi.Go1State._fields_})
        _check(lib().go1_bind(self.h, C.byref(s), abi.plane_descs(t)))

    def set_terrain(self, tiles, env_tile, env_terrain_origin, env_origins):
        d = self.device
        if isinstance(tiles, torch.Tensor):  # device-generated tiles (tunnel_tiles)
            tiles = tiles.to(d, torch.float32).contiguous()
        else:
            tiles = torch.as_tensor(np.ascontiguousarray(tiles, np.float32)).to(d)
        t = [tiles,
             torch.as_tensor(np.ascontiguousarray(env_tile, np.int32)).to(d),
             torch.as_tensor(np.ascontiguousarray(env_terrain_origin, np.float32)).to(d),
             torch.as_tensor(np.ascontiguousarray(env_origins, np.float32)).to(d)]
        self._terrain_keep = t
        s = abi.Go1Terrain(tiles=t[0].data_ptr(), env_tile=t[1].data_ptr(), env_terrain_origin=t[2].data_ptr(),
                           env_origins=t[3].data_ptr(), n_tiles=int(t[0].shape[0]))
        _check(lib().go1_set_terrain(self.h, C.byref(s)))

    def step(self, actions, gravity_vec, sim_gravity, reward_scales, rng_seed=0, rng_step=0, uniforms=None,
             inj=None, debug=None, events=None, episode_log=None, aux=None, out=None, obs_history=None,
             diverged_count=None, contact_forces=True):
        """One fused LeggedRobot.step on the current stream.  `debug` is an optional dict
        of preallocated tensors (torques, heights, terms, commands, reached); `out` may
        replace the default output buffers (obs, priv, rew, reset, time_out); contact_forces=False
        skips the (n, 17, 3) contact-force store (the kernel writes nothing there).

        The go1_step_args struct is kept between calls (the rollout calls this every
        few hundred microseconds); only the fields that change are rewritten."""
        a = self._args
        if a is None:
            a = self._args = abi.Go1StepArgs()
            a.extras_time_outs = self.extras_time_outs.data_ptr()
        a.contact_forces = self.contact_forces.data_ptr() if contact_forces else None
        if actions.dtype != torch.float32 or actions.shape != (self.n, 12) or not actions.is_contiguous() or \
                actions.device != self.device:
            raise NativeError("actions must be a contiguous (n_envs, 12) float32 tensor on the env's device")
        a.actions = actions.data_ptr()
        key = (tuple(gravity_vec), tuple(sim_gravity), tuple(reward_scales))
        if key != self._consts:
            self._consts = key
            a.gravity_vec[:] = [float(x) for x in gravity_vec]
            a.sim_gravity[:] = [float(x) for x in sim_gravity]
            rs = np.zeros(abi.GO1_MAX_TERMS, np.float32)
            rs[:len(reward_scales)] = np.asarray(reward_scales, np.float32)
            a.reward_scales[:] = [float(x) for x in rs]
        a.rng_seed, a.rng_step = int(rng_seed), int(rng_step)
        a.uniforms = None
        if uniforms is not None:
            assert uniforms.is_contiguous() and uniforms.shape == (self.n, self.cfg.u_per_env)
            a.uniforms = uniforms.data_ptr()
        if inj is not None:
            a.inj_dof, a.inj_root, a.inj_contact = (inj[k].data_ptr() for k in ("dof", "root", "contact"))
        else:
            a.inj_dof = a.inj_root = a.inj_contact = None
        if out:
            for k in ("obs", "priv", "rew", "reset", "time_out"):
                v = out.get(k)
                if v is None:
                    v = getattr(self, k)
                elif v.device != self.device or not v.is_contiguous() or v.shape != getattr(self, k).shape or \
                        v.dtype != getattr(self, k).dtype:
                    raise NativeError(f"output buffer {k!r} does not match the expected shape / dtype / device")
                setattr(a, k, v.data_ptr())
        else:
            a.obs, a.priv, a.rew = self.obs.data_ptr(), self.priv.data_ptr(), self.rew.data_ptr()
            a.reset, a.time_out = self.reset.data_ptr(), self.time_out.data_ptr()
        for k, fld in (("torques", "dbg_torques"), ("heights", "dbg_heights"), ("terms", "dbg_terms"),
                       ("commands", "dbg_commands"), ("reached", "dbg_reached")):
            setattr(a, fld, debug[k].data_ptr() if debug and k in debug else None)
        if episode_log is not None:
            assert episode_log.is_contiguous() and episode_log.shape == (self.n, abi.episode_log_width(self.cfg.n_terms))
        a.episode_log = episode_log.data_ptr() if episode_log is not None else None
        if aux is not None:
            assert aux.is_contiguous() and aux.shape == (self.n, abi.GO1_AUX)
        a.aux = aux.data_ptr() if aux is not None else None
        a.ev_begin, a.ev_end = events if events is not None else (None, None)  # hipEvent_t pair as ints
        if obs_history is not None:
            assert obs_history.is_contiguous() and obs_history.shape == (self.n, self.cfg.num_obs)
        a.obs_history = obs_history.data_ptr() if obs_history is not None else None
        if diverged_count is not None:
            assert diverged_count.dtype == torch.int64 and diverged_count.numel() == 1 and \
                diverged_count.device == self.device
        a.diverged_count = diverged_count.data_ptr() if diverged_count is not None else None
        _check(self._lib_step(self.h, C.byref(a), C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))

    # ------------------------------------------------------------------ per-step fast path
    def prepare(self, out, aux=None, obs_history=None, diverged_count=None, episode_log=None, log_count=None,
                contact_forces=True):
        """A validated go1_step_args for step_prepared: the env builds one per (output-ring slot,
        episode-log half) once, so the per-step host work is a handful of field writes and the
        ctypes call (the loop is otherwise host-bound at ~60 us per step).  `episode_log` with
        `log_count` selects the compact log (go1_step_args.episode_log_count); contact_forces=False
        leaves the contact-force store out."""
        a = abi.Go1StepArgs()
        a.contact_forces = self.contact_forces.data_ptr() if contact_forces else None
        a.extras_time_outs = self.extras_time_outs.data_ptr()
        for k in ("obs", "priv", "rew", "reset", "time_out"):
            v, ref = out[k], getattr(self, k)
            if v.device != self.device or not v.is_contiguous() or v.shape != ref.shape or v.dtype != ref.dtype:
                raise NativeError(f"output buffer {k!r} does not match the expected shape / dtype / device")
            setattr(a, k, v.data_ptr())
        if aux is not None:
            if not aux.is_contiguous() or aux.shape != (self.n, abi.GO1_AUX) or aux.device != self.device:
                raise NativeError("aux must be a contiguous (n_envs, GO1_AUX) float32 tensor on the env's device")
            a.aux = aux.data_ptr()
        if obs_history is not None:
            if not obs_history.is_contiguous() or obs_history.shape != (self.n, self.cfg.num_obs):
                raise NativeError("obs_history must be a contiguous (n_envs, num_obs) tensor")
            a.obs_history = obs_history.data_ptr()
        if diverged_count is not None:
            if diverged_count.dtype != torch.int64 or diverged_count.numel() != 1 or \
                    diverged_count.device != self.device:
                raise NativeError("diverged_count must be one int64 on the env's device")
            a.diverged_count = diverged_count.data_ptr()
        if episode_log is not None:
            w = abi.episode_log_width(self.cfg.n_terms)
            if log_count is None:
                if episode_log.shape != (self.n, w) or not episode_log.is_contiguous():
                    raise NativeError("episode_log must be a contiguous (n_envs, n_terms + 6) tensor")
            else:
                if episode_log.dim() != 2 or episode_log.shape[1] != w + 2 or not episode_log.is_contiguous() or \
                        log_count.dtype != torch.int32 or log_count.device != self.device:
                    raise NativeError("a compact episode log is a contiguous (cap, n_terms + 8) tensor + an int32 count")
                a.episode_log_count = log_count.data_ptr()
                a.episode_log_cap = int(episode_log.shape[0])
            a.episode_log = episode_log.data_ptr()
        a._consts = None
        return a

    def step_prepared(self, a, actions, gravity_vec, sim_gravity, reward_scales, consts_key, rng_seed, rng_step,
                      events=None, log_tag=0):
        """go1_step with a prepare()d argument block.  `consts_key` identifies (gravity_vec,
        sim_gravity, reward_scales): they are re-copied into the block only when it changes."""
        if actions.dtype != torch.float32 or actions.shape != (self.n, 12) or not actions.is_contiguous() or \
                actions.device != self.device:
            raise NativeError("actions must be a contiguous (n_envs, 12) float32 tensor on the env's device")
        a.actions = actions.data_ptr()
        if a._consts != consts_key:
            a._consts = consts_key
            a.gravity_vec[:] = [float(x) for x in gravity_vec]
            a.sim_gravity[:] = [float(x) for x in sim_gravity]
            rs = np.zeros(abi.GO1_MAX_TERMS, np.float32)
            rs[:len(reward_scales)] = np.asarray(reward_scales, np.float32)
            a.reward_scales[:] = [float(x) for x in rs]
        a.rng_seed, a.rng_step, a.episode_log_tag = rng_seed, rng_step, log_tag
        a.ev_begin, a.ev_end = events if events is not None else (None, None)
        rc = self._lib_step(self.h, C.byref(a), torch._C._cuda_getCurrentRawStream(self._dev_index))
        if rc:
            _check(rc)

    def specialize(self, enable):
        """Force the generic step kernel (False) or the README-config specialisation (True; raises
        if this config differs from it).  go1_create picks the specialisation when it applies."""
        _check(lib().go1_specialize(self.h, int(bool(enable))))

    @property
    def specialized(self):
        return bool(lib().go1_is_specialized(self.h))

    def sync_time_outs(self):
        """Make extras_time_outs current for the last step (the rebinding of step k is
        otherwise applied by the kernel of step k+1)."""
        _check(lib().go1_sync_time_outs(self.h, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        return self.extras_time_outs

    def time_outs_pending(self):
        """(flag, pending, extras) device pointers of the last step's deferred extras["time_outs"]
        rebinding (None before the first step); see go1_time_outs_pending."""
        out = (C.c_int64 * 3)()
        _check(lib().go1_time_outs_pending(self.h, out))
        return tuple(int(x) for x in out) if out[0] else None

    def reset_idx(self, env_ids, uniforms=None, rng_seed=0, rng_step=0):
        """go1_reset_idx for local env ids (any integer tensor; converted to int32 on the device)."""
        ids = torch.as_tensor(env_ids, device=self.device).to(torch.int32).flatten().contiguous()
        _check(lib().go1_reset_idx(self.h, ids.data_ptr(), int(ids.numel()),
                                   None if uniforms is None else uniforms.data_ptr(), int(rng_seed), int(rng_step),
                                   _stream()))
        return ids  # keep alive until the stream passes it

    def reset_envs(self, mask, uniforms=None, rng_seed=0, rng_step=0):
        m = mask.to(torch.uint8).contiguous()
        _check(lib().go1_reset_envs(self.h, m.data_ptr(), None if uniforms is None else uniforms.data_ptr(),
                                    int(rng_seed), int(rng_step), _stream()))
        return m  # keep alive until the stream passes it

    def actuator(self, x):
        x = x.contiguous()
        out = torch.empty(x.shape[0], device=x.device)
        _check(lib().go1_actuator_net(self.h, x.data_ptr(), out.data_ptr(), x.shape[0], _stream()))
        return out

    def close(self):
        if self.h:
            lib().go1_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def debug_buffers(n, decimation, device):
    return dict(torques=torch.zeros((decimation, n, 12), device=device),
                heights=torch.zeros((n, 2, 21, 11), device=device),
                terms=torch.zeros((n, abi.GO1_MAX_TERMS), device=device), commands=torch.zeros((n, 2), device=device),
                reached=torch.zeros(n, dtype=torch.uint8, device=device))
