"""ctypes front-end of the CPU oracle (oracle/_build/libgo1_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker -- never by the product path.
"""
import ctypes as C
import os

import numpy as np

from legged_tracking_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libgo1_oracle.so")
# same source with an f32 integrator: bench.py's like-for-like CPU baseline (never the checker)
LIB_PATH_F32 = os.path.join(HERE, "_build", "libgo1_oracle_f32.so")
_lib = None
_libs = {}


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(precision="f64"):
    """The oracle library: "f64" integrator (the checker) or "f32" (CPU timing baseline)."""
    path = {"f64": LIB_PATH, "f32": LIB_PATH_F32}[precision]
    _lib = _libs.get(path)
    if _lib is None:
        if not os.path.exists(path):
            build()
        _lib = _libs[path] = C.CDLL(path)
        _lib.go1o_step.argtypes = [C.POINTER(abi.Go1Config), C.POINTER(abi.Go1State), C.POINTER(abi.Go1Terrain),
                                   C.POINTER(abi.Go1StepArgs)]
        _lib.go1o_reset_envs.argtypes = [C.POINTER(abi.Go1Config), C.POINTER(abi.Go1State),
                                         C.POINTER(abi.Go1Terrain), C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64]
        _lib.go1o_actuator_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _lib.go1o_uniform.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32]
        _lib.go1o_uniform.restype = C.c_float
        _lib.go1o_physics.argtypes = [C.POINTER(abi.Go1Config)] + [C.c_void_p] * 7 + [
            C.c_int, C.c_double, C.c_void_p, C.c_double, C.c_double, C.c_double, C.c_void_p, C.c_double,
            C.c_double, C.c_void_p]
        _lib.go1o_energy.argtypes = [C.POINTER(abi.Go1Config)] + [C.c_void_p] * 7 + [C.c_double]
        _lib.go1o_energy.restype = C.c_double
    return _lib


def _d(x, n):
    return np.ascontiguousarray(np.asarray(x, np.float64).reshape(n))


def physics(cfg, body, tau, n_sub, h, g, friction, restitution, payload, tile=None, origin=(0.0, 0.0)):
    """n_sub integrator steps of length h on one env's state given as a dict of f64 arrays (pos 3, quat 4 xyzw,
    v 3, w 3 world; q 12, qd 12), updated in place; returns the last step's reported contact forces (17, 3).
    tile: one (2, hf_nx, hf_ny) heightfield at `origin`, or None for the plane."""
    b = {k: _d(body[k], n) for k, n in (("pos", 3), ("quat", 4), ("v", 3), ("w", 3), ("q", 12), ("qd", 12))}
    t, gg = _d(tau, 12), _d(g, 3)
    cf = np.zeros(17 * 3, np.float64)
    tl = None if tile is None else np.ascontiguousarray(tile, np.float32)
    lib().go1o_physics(C.byref(cfg), *(b[k].ctypes.data for k in ("pos", "quat", "v", "w", "q", "qd")),
                       t.ctypes.data, int(n_sub), float(h), gg.ctypes.data, float(friction), float(restitution),
                       float(payload), None if tl is None else tl.ctypes.data, float(origin[0]), float(origin[1]),
                       cf.ctypes.data)
    body.update(b)
    return cf.reshape(17, 3)


def seg_deepest(tile, hs, A, B, r):
    """t in [0, 1] of the deepest point of the segment A -> B (a capsule of radius r) against one (2, nx, ny) tile
    at the origin (go1_oracle.c seg_deepest)."""
    tl = np.ascontiguousarray(tile, np.float32)
    a, b = _d(A, 3), _d(B, 3)
    f = lib().go1o_seg_deepest
    f.restype = C.c_double
    f.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p, C.c_double]
    return f(tl.ctypes.data, int(tl.shape[1]), int(tl.shape[2]), hs, a.ctypes.data, b.ctypes.data, r)


def set_rescan_every_step(faces=False, segments=False):
    """Test knob (tests/test_held_contacts.py): choose the trunk faces' vertices / the capsules' deepest points every
    sim step instead of once per control step (the kernel's and the oracle's default)."""
    f = lib().go1o_set_rescan_every_step
    f.argtypes = [C.c_int]
    f(int(bool(faces)) | 2 * int(bool(segments)))


def seg_closest(P0, P1, Q0, Q1):
    """(s, t): parameters of the closest points of the segments P0 -> P1 and Q0 -> Q1 (go1_oracle.c)."""
    st = np.zeros(2)
    args = [_d(x, 3) for x in (P0, P1, Q0, Q1)]
    f = lib().go1o_seg_closest
    f.argtypes = [C.c_void_p] * 5
    f(*(x.ctypes.data for x in args), st.ctypes.data)
    return float(st[0]), float(st[1])


def energy(cfg, body, g, payload):
    """Kinetic + potential energy of one env's state (dict as `physics`) in the gravity field g."""
    b = {k: _d(body[k], n) for k, n in (("pos", 3), ("quat", 4), ("v", 3), ("w", 3), ("q", 12), ("qd", 12))}
    gg = _d(g, 3)
    return lib().go1o_energy(C.byref(cfg), *(b[k].ctypes.data for k in ("pos", "quat", "v", "w", "q", "qd")),
                             gg.ctypes.data, float(payload))


class _Readme:
    """Plane widths of the README configuration (10 reward terms, one waypoint, decimation 4)."""
    n_terms = 10
    traj_length = 1
    decimation = 4


class NpState:
    """Numpy SoA state matching go1_state (plane widths from `cfg`: a go1_config)."""

    def __init__(self, n, init=None, cfg=None):
        self.n = n
        self.cfg = cfg if cfg is not None else _Readme
        self.arrays = {}
        for name, w, dt in abi.state_spec(self.cfg):
            a = np.zeros((n, w), np.float32 if dt == "f32" else np.int32)
            if init is not None and name in init:
                src = np.asarray(init[name])
                a[...] = src.reshape(n, w).astype(a.dtype)
            self.arrays[name] = np.ascontiguousarray(a)

    def struct(self):
        return abi.Go1State(**{k: abi.ptr(v) for k, v in self.arrays.items()})

    def __getitem__(self, k):
        return self.arrays[k]

    def copy(self):
        s = NpState(self.n, cfg=self.cfg)
        for k, v in self.arrays.items():
            s.arrays[k] = v.copy()
        return s


class NpTerrain:
    def __init__(self, tiles, env_tile, env_terrain_origin, env_origins):
        self.tiles = np.ascontiguousarray(tiles, np.float32)
        self.env_tile = np.ascontiguousarray(env_tile, np.int32)
        self.eto = np.ascontiguousarray(env_terrain_origin, np.float32)
        self.eo = np.ascontiguousarray(env_origins, np.float32)

    def struct(self):
        return abi.Go1Terrain(tiles=abi.ptr(self.tiles), env_tile=abi.ptr(self.env_tile),
                              env_terrain_origin=abi.ptr(self.eto), env_origins=abi.ptr(self.eo),
                              n_tiles=int(self.tiles.shape[0]))


def step(cfg, state, terrain, actions, gravity_vec, sim_gravity, reward_scales, uniforms=None, rng_seed=0,
         rng_step=0, inj=None, debug=True, precision="f64"):
    """One oracle step; mutates `state`; returns a dict of outputs.  precision="f32" runs the
    f32-integrator build (CPU timing baseline only)."""
    n = cfg.n_envs
    out = dict(obs=np.zeros((n, cfg.num_obs), np.float32), priv=np.zeros((n, 2), np.float32),
               rew=np.zeros(n, np.float32), reset=np.zeros(n, np.uint8), time_out=np.zeros(n, np.uint8),
               contact_forces=np.zeros((n, 17, 3), np.float32))
    if debug:
        out.update(torques=np.zeros((cfg.decimation, n, 12), np.float32),
                   heights=np.zeros((n, 2, 21, 11), np.float32),
                   terms=np.zeros((n, abi.GO1_MAX_TERMS), np.float32),
                   commands=np.zeros((n, 2), np.float32), reached=np.zeros(n, np.uint8),
                   episode_log=np.full((n, abi.episode_log_width(cfg.n_terms)), np.nan, np.float32),
                   aux=np.zeros((n, abi.GO1_AUX), np.float32))
    actions = np.ascontiguousarray(actions, np.float32)
    keep = [actions]
    a = abi.Go1StepArgs()
    a.actions = abi.ptr(actions)
    for i in range(3):
        a.gravity_vec[i] = float(gravity_vec[i])
        a.sim_gravity[i] = float(sim_gravity[i])
    rs = np.zeros(abi.GO1_MAX_TERMS, np.float32)
    rs[:len(reward_scales)] = np.asarray(reward_scales, np.float32)
    for i in range(abi.GO1_MAX_TERMS):
        a.reward_scales[i] = float(rs[i])
    a.rng_seed, a.rng_step = rng_seed, rng_step
    if uniforms is not None:
        u = np.ascontiguousarray(uniforms, np.float32)
        assert u.shape == (n, cfg.u_per_env), (u.shape, cfg.u_per_env)
        keep.append(u)
        a.uniforms = abi.ptr(u)
    if inj is not None:
        d, r, c = (np.ascontiguousarray(inj[k], np.float32) for k in ("dof", "root", "contact"))
        keep += [d, r, c]
        a.inj_dof, a.inj_root, a.inj_contact = abi.ptr(d), abi.ptr(r), abi.ptr(c)
    for k, fld in (("obs", "obs"), ("priv", "priv"), ("rew", "rew"), ("reset", "reset"), ("time_out", "time_out"),
                   ("contact_forces", "contact_forces")):
        setattr(a, fld, abi.ptr(out[k]))
    if debug:
        a.dbg_torques, a.dbg_heights, a.dbg_terms = abi.ptr(out["torques"]), abi.ptr(out["heights"]), abi.ptr(
            out["terms"])
        a.dbg_commands, a.dbg_reached = abi.ptr(out["commands"]), abi.ptr(out["reached"])
        a.episode_log, a.aux = abi.ptr(out["episode_log"]), abi.ptr(out["aux"])
    st = state.struct()
    ts = terrain.struct()
    rc = lib(precision).go1o_step(C.byref(cfg), C.byref(st), C.byref(ts), C.byref(a))
    assert rc == 0
    return out


def reset_envs(cfg, state, terrain, mask, uniforms=None, rng_seed=0, rng_step=0):
    mask = np.ascontiguousarray(mask, np.uint8)
    u = None if uniforms is None else np.ascontiguousarray(uniforms, np.float32)
    st = state.struct()
    ts = terrain.struct()
    lib().go1o_reset_envs(C.byref(cfg), C.byref(st), C.byref(ts), abi.ptr(mask), abi.ptr(u), rng_seed, rng_step)


def actuator(weights, x):
    x = np.ascontiguousarray(x, np.float32)
    w = np.ascontiguousarray(weights, np.float32)
    out = np.zeros(x.shape[0], np.float32)
    lib().go1o_actuator_batch(abi.ptr(w), abi.ptr(x), abi.ptr(out), x.shape[0])
    return out


def uniform(seed, step, env, slot):
    return lib().go1o_uniform(seed, step, env, slot)
