"""Benchmark of the MI355X Go1 trajectory-tracking env step (BASELINE.json metric).

One "step" = one VecEnv.step of HistoryWrapper(TrajectoryTrackingEnv) -- the call
scripts/train.py's Runner makes ("wall time of the VecEnv.step loop"):
the fused HIP LeggedRobot.step (4 sim sub-steps of actuator net + native articulated-
body integrator, then the whole post-physics: height scan, targets, rewards,
terminations, resets, observations) plus the env's host bookkeeping (gravity schedule,
output ring, episode-log ring, HistoryWrapper).  4096 envs per GPU on the single_path
tunnel (BASELINE configs[2]).  Inputs are synthetic and already resident in HBM when
the timed region starts: a ring of N(0,1) action batches (the actor's init_noise_std
= 1.0, ppo_cse/actor_critic.py:11) generated on the device.

Multi-GPU: one process per GPU.  `--gpus N` (N > 1) launches the N ranks itself
(children started before anything touches the GPU, rendezvous on 127.0.0.1), or runs
as one rank of an external `torch.distributed.run` (RANK / WORLD_SIZE in the env; the
world size must equal --gpus).  Envs are sharded by global env id (rank r owns
[r*N, (r+1)*N)); the step has no collective -> "scaling": "weak";
value = sum over ranks of envs x steps / max-over-ranks time.

Also reported: the raw fused-kernel loop (Go1Native.step alone), the roofline of the
fused step kernel (HIP events around that kernel, on its launch stream, over the timed
region), the PPO rollout rate (act + step + record) and the CPU oracle timed on a
bounded sample on rank 0's host cores (N = 1 only).
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "env-steps/sec (whole node) at 4096 Go1/GPU, 1/2/4/8 MI355X; %HBM roofline"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA

# Algorithmic HBM bytes per env-step, SURVEY.md 8(d) (the roofline's unit of work, fixed by the survey):
#   reads 1,764 B = actions 48 + q 76 + qd 72 + actuator history 192 + 4 consumed lag slots 192 +
#   last_actions 48 + last_dof_vel 48 + DR params 108 + episode/target state 48 + 13 episode sums 52 +
#   220 height gathers 880; writes 1,758 B = q, qd 148 + history 192 + lag 192 + last_* 96 + obs 1,044 +
#   priv 8 + rew/reset/timeout 6 + episode state 20 + sums 52.
SURVEY_BYTES_PER_ENV_STEP = 3522
# What the measured VecEnv.step path actually moves per env-step (its own item list),
# reported beside it as bytes_written_by_path:
#   reads 1,696 B = actions 48, root 52, dof pos/vel 96, stored lag 96 (2 steps of scaled actions),
#     err/vel history 192, motor strength/offset 96, last actions/dof vel 96, friction/restitution/payload
#     12, episode length/pose index/collisions 12, trajectory 24, base rotation 12, episode sums 52,
#     terrain index + origins 28, 110 height samples x 2 layers x 4 B = 880
#   writes 2,047 B = obs 1,044, priv 8, rew 4, reset/time-out/extras 3, contact forces 204, aux 128,
#     root 52, dof pos/vel 96, stored lag 96, err/vel history 192, last actions/dof vel 96, joint
#     targets 48, base rotation 12, episode sums 52, counters 12 (motor strength/offset and the
#     trajectory are written only on reset / DR steps: < 1 B per env-step)
PATH_BYTES_PER_ENV_STEP = 1696 + 2047
PREWARM_S = 0.25
# Algorithmic FLOPs per env-step, SURVEY.md 8(d): actuator MLP 132,144 (exact) + ABA / contact /
# integration ~40,000 (estimate) + post-physics ~6,000 -> ~1.8e5.  The measured count (PMC VALU / MFMA
# FLOP counters of the step kernel, profiles/r05/step_counters.json) is reported beside it.
SURVEY_FLOPS_PER_ENV_STEP = 1.8e5

# PMC-measured HBM bytes per launch of the step kernel (tools/profile.sh + tools/prof_summary.py;
# FETCH_SIZE + WRITE_SIZE, separate --pmc passes).  Re-collected whenever the kernel changes.
TRAFFIC_FILES = [os.path.join(REPO, "profiles", r, "step_counters.json") for r in ("r06", "r05", "r04", "r03", "r02", "r01")]
# the same kernel with the rollout's stores only (no contact forces, no aux block: Runner.learn's output demand)
ROLLOUT_TRAFFIC_FILE = os.path.join(REPO, "profiles", "r06", "step_rollout_counters.json")


def pmc_counters(n_envs):
    """From the newest committed PMC summary of the step kernel at this env count: HBM bytes per
    launch (raw FETCH + WRITE, and with FETCH doubled), written bytes, counted FP32 FLOPs per launch
    (None if that pass is absent), VALU issue fraction, source file."""
    for path in TRAFFIC_FILES:
        try:
            with open(path) as f:
                d = json.load(f)
            if int(d["resources"]["Grid_Size"]) != 16 * n_envs:  # 16 lanes per env
                continue
            pw = d.get("per_wave", {})
            valu = pw["SQ_ACTIVE_INST_VALU"] / pw["SQ_WAVE_CYCLES"] if "SQ_ACTIVE_INST_VALU" in pw else None
            h = d["hbm_bytes_per_launch"]
            return dict(traffic=h["traffic"], traffic_x2=h.get("traffic_upper_fetch_doubled"),
                        written=h.get("write"), flops=d.get("flops_per_launch"), valu=valu,
                        src=os.path.relpath(path, REPO))
        except (OSError, KeyError, ValueError, ZeroDivisionError):
            continue
    return dict(traffic=None, traffic_x2=None, written=None, flops=None, valu=None, src=None)


def rollout_traffic(n_envs):
    """HBM bytes per launch of the step kernel with the rollout's stores only (profiles/r06, tools/profile.sh)."""
    try:
        with open(ROLLOUT_TRAFFIC_FILE) as f:
            d = json.load(f)
        if int(d["resources"]["Grid_Size"]) != 16 * n_envs:
            return None
        h = d["hbm_bytes_per_launch"]
        return {"traffic": h["traffic"], "written": h["write"], "over_algorithmic": h["traffic"] / (3522 * n_envs),
                "written_per_env_step": h["write"] / n_envs, "source": os.path.relpath(ROLLOUT_TRAFFIC_FILE, REPO),
                "what": "bench.py --kernel-only --rollout-outputs: the rollout's stores (Runner.learn switches the "
                        "contact-force and aux stores off, LeggedRobot.set_output_demand)"}
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None


def hip():
    h = C.CDLL("libamdhip64.so")
    h.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    h.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    h.hipEventSynchronize.argtypes = [C.c_void_p]
    h.hipEventDestroy.argtypes = [C.c_void_p]
    return h


class EventPairs:
    """hipEvent_t pairs recorded by the library around the fused kernel (on its launch stream)."""

    def __init__(self, n):
        self.hp = hip()
        self.ev = []
        for _ in range(2 * n):
            e = C.c_void_p()
            assert self.hp.hipEventCreate(C.byref(e)) == 0
            self.ev.append(e)

    def pair(self, k):
        return self.ev[2 * k].value, self.ev[2 * k + 1].value

    def ms(self, k):
        m = C.c_float()
        assert self.hp.hipEventElapsedTime(C.byref(m), self.ev[2 * k], self.ev[2 * k + 1]) == 0
        return m.value

    def close(self):
        for e in self.ev:
            self.hp.hipEventDestroy(e)


def cpu_threads():
    """Threads for the CPU baseline: the process's CPU share.  The GPU box sets OMP_NUM_THREADS to
    its per-GPU share (16) and asks jobs to stay within it; otherwise every core in the affinity mask."""
    cores = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    return (min(int(share), cores) if share and share.isdigit() and int(share) > 0 else cores), cores


def cpu_baseline(n_envs, budget_s=12.0, max_steps=400):
    """Time the CPU oracle's f32-integrator build (a C restatement, OpenMP over envs) on the same
    workload (checker code timed as a baseline only; never the measured product)."""
    from legged_tracking_amd import config as CF, terrain as T
    from oracle import oracle as O
    threads, cores = cpu_threads()
    os.environ["OMP_NUM_THREADS"] = str(threads)
    cfg = CF.readme_config(n_envs=n_envs, terrain="single_path", rows=32, cols=32)
    c = CF.build_abi_config(cfg)
    td = T.build(cfg, n_envs, np.random.RandomState(11))
    ter = O.NpTerrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    st = O.NpState(n_envs)
    rng = np.random.default_rng(1)
    st["friction"][:, 0] = rng.uniform(0.1, 3.0, n_envs)
    O.reset_envs(c, st, ter, np.ones(n_envs, np.uint8), rng_seed=1, rng_step=0)
    st["episode_length"][:, 0] = rng.integers(0, 500, n_envs)
    grav, gvec = CF.gravity_state(rng.uniform(-1, 1, 3))
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    acts = [rng.normal(0, 1, (n_envs, 12)).astype(np.float32) for _ in range(8)]
    O.step(c, st, ter, acts[0], gvec, grav, scales, rng_seed=1, rng_step=1, debug=False, precision="f32")  # warm
    t0 = time.perf_counter()
    k = 0
    while k < max_steps and time.perf_counter() - t0 < budget_s:
        O.step(c, st, ter, acts[k % 8], gvec, grav, scales, rng_seed=1, rng_step=2 + k, debug=False, precision="f32")
        k += 1
    dt = time.perf_counter() - t0
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": n_envs * k / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{k} steps x {n_envs} envs of the C oracle (f32 integrator, same single_path workload), "
                      f"{dt:.1f} s on {threads} OpenMP threads (this process's CPU share; {cores} cores in its "
                      f"affinity mask, {model})"}


def make_env(n, rank, world, dev):
    from legged_tracking_amd import config as CF, env as E
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=32, cols=32)
    return E.HistoryWrapper(E.TrajectoryTrackingEnv(sim_device=str(dev), cfg=cfg, seed=11, rank=rank,
                                                    world_size=world))


def kernel_loop(env, ring, steps, warmup, every=4, contact_forces=True):
    """The fused kernel alone (Go1Native.step, no env host code) on the env's own handle; no aux block, and
    contact_forces=False leaves the contact-force store out as well (the rollout's outputs)."""
    import torch
    base = env.env
    sim = base._sim
    grav, gvec = base._sim_gravity, base._gravity_vec
    scales = base._scale_vector()
    ev = EventPairs((steps + every - 1) // every)
    for k in range(warmup):
        sim.step(ring[k % len(ring)], gvec, grav, scales, rng_seed=7, rng_step=(1 << 40) + k,
                 contact_forces=contact_forces)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        e = ev.pair(k // every) if k % every == 0 else None
        sim.step(ring[k % len(ring)], gvec, grav, scales, rng_seed=7, rng_step=(1 << 40) + warmup + k, events=e,
                 contact_forces=contact_forces)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kt = [ev.ms(i) for i in range((steps + every - 1) // every)]
    ev.close()
    kernel_loop.last = kt
    return dt, float(np.mean(kt))


def env_sweep(n, dev, steps=100, warmup=10):
    """Env-only VecEnv.step throughput at n envs on this GPU (4k ... 256k envs/GPU sweep)."""
    import torch
    env = make_env(n, 0, 1, dev)
    env.reset()
    ring = torch.randn((8, n, 12), device=dev)
    for k in range(warmup):
        env.step(ring[k % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        env.step(ring[k % 8])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kdt, kms = kernel_loop(env, ring, steps, warmup)
    env.close()
    return {"envs_per_gpu": n, "value": n * steps / dt, "ms_per_step": dt / steps * 1e3,
            "kernel_ms": kms, "kernel_loop_env_steps_per_s": n * steps / kdt}


def _max_over_ranks(x, world):
    """The slowest rank's value (the whole job's time) at world > 1 (RCCL all-reduce MAX)."""
    if world == 1:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def _barrier(world):
    if world > 1:
        import torch
        torch.distributed.barrier()
        torch.cuda.synchronize()


def rollout_rate(n, dev, steps, warmup, rank=0, world=1):
    """Secondary line (SURVEY 8(d) "report both env-only and rollout (act + step) rates"): the
    Runner's rollout loop -- fused PPO.act kernel, env.step through TrajectoryTrackingEnv /
    HistoryWrapper, transition record kernel -- at n envs per rank (every rank runs it at world > 1)."""
    import torch
    from legged_tracking_amd import rollout as R
    env = make_env(n, rank, world, dev)
    ac = R.ActorCritic(env.num_obs, env.num_privileged_obs, env.num_obs_history, env.num_actions).to(dev)
    alg = R.PPO(ac, device=dev)
    T = 24
    alg.init_storage(n, T, [env.num_obs], [env.num_privileged_obs], [env.num_obs_history], [env.num_actions])
    env.reset()
    od = env.get_observations()
    obs, priv, hist = od["obs"], od["privileged_obs"], od["obs_history"]

    def one():
        nonlocal obs, priv, hist
        if alg.storage.step == T:
            alg.storage.clear()
        a = alg.act(obs, priv, hist)
        od, rew, done, info = env.step(a)
        obs, priv, hist = od["obs"], od["privileged_obs"], od["obs_history"]
        alg.process_env_step(rew, done, info)

    with torch.inference_mode():
        for _ in range(warmup):
            one()
        torch.cuda.synchronize()
        _barrier(world)
        t0 = time.perf_counter()
        for _ in range(steps):
            one()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    env.close()
    dt = _max_over_ranks(dt, world)
    return {"value": n * world * steps / dt, "unit": "env-steps/s", "ms_per_step": dt / steps * 1e3, "steps": steps,
            "what": "PPO.act (fused MFMA adaptation+actor+critic kernel, Normal sample) + TrajectoryTrackingEnv.step "
                    f"+ HistoryWrapper + process_env_step record kernel, {world} GPU(s), slowest rank's time",
            "fused_policy": alg.fused is not None}


def velocity_rate(n, dev, steps, warmup):
    """BASELINE configs[1] (4096 Go1, plane, velocity_tracking reward): VecEnv.step of
    HistoryWrapper(VelocityTrackingEasyEnv) -- the fused HIP velocity step (native integrator, CoRL rewards,
    gait clock), the curriculum / history-shift launch (30-deep obs_history), the env's host bookkeeping --
    with N(0,1) actions resident on the device; HIP events around the step kernel."""
    import torch
    from legged_tracking_amd import env as E, velocity as VEL
    env = E.HistoryWrapper(VEL.VelocityTrackingEasyEnv(sim_device=str(dev), num_envs=n, seed=11))
    env.reset()
    env.get_observations()
    ring = torch.randn((64, n, 12), device=dev, generator=torch.Generator(device=dev).manual_seed(7))
    for k in range(warmup):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    every = 4
    ev = EventPairs((steps + every - 1) // every)
    env.env.kernel_events.extend(ev.pair(k // every) if k % every == 0 else None for k in range(steps))
    t0 = time.perf_counter()
    for k in range(steps):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    env.env.kernel_events.clear()
    kms = float(np.mean([ev.ms(i) for i in range((steps + every - 1) // every)]))
    ev.close()
    assert torch.isfinite(env.env.obs_buf).all(), "non-finite observations"
    resets = int(env.env.state["episode_length"].eq(0).sum())
    env.env.close()
    return {"value": n * steps / dt, "unit": "env-steps/s", "ms_per_step": dt / steps * 1e3, "steps": steps,
            "kernel_ms": kms, "envs_per_gpu": n, "dtype": "f32",
            "what": "BASELINE configs[1]: VecEnv.step of HistoryWrapper(VelocityTrackingEasyEnv) on the plane, "
                    "scripts/train_velocity_tracking.py config (CoRL rewards, gait commands, curriculum, 30-deep "
                    "obs history); kernel_ms = go1_vel_step_kernel alone (HIP events on its dispatch)",
            "envs_at_episode_start": resets}


def learn_rate(n, dev, iters=6, warmup=2, velocity=False, rank=0, world=1):
    """The whole training loop, as the reference's wandb train/fps measures it (ppo_cse/__init__.py:184:
    (it + 1) x num_envs x num_steps_per_env / elapsed): Runner iterations of rollout (24 x [PPO.act +
    VecEnv.step + record]), compute_returns (GAE) and PPO.update (5 epochs x 4 mini-batches, Adam, the
    adaptation-module step), each phase bracketed by a device sync to split the time.  Checkpoint
    writes (every 400 iterations in the reference) are outside the timed iterations."""
    import torch
    from legged_tracking_amd import rollout as R
    if velocity:  # configs[1]: scripts/train_velocity_tracking.py's env (30-deep history: torch policy path)
        from legged_tracking_amd import env as E, velocity as VEL
        env = E.HistoryWrapper(VEL.VelocityTrackingEasyEnv(sim_device=str(dev), num_envs=n, seed=11))
        env.close = env.env.close
    else:
        env = make_env(n, rank, world, dev)
    runner = R.Runner(env, device=dev, save_dir=None)
    alg, T = runner.alg, runner.num_steps_per_env
    od = env.get_observations()
    obs, priv, hist = od["obs"], od["privileged_obs"], od["obs_history"]
    runner.alg.actor_critic.train()
    split = {"rollout": 0.0, "gae": 0.0, "update": 0.0}
    for it in range(warmup + iters):
        torch.cuda.synchronize()
        if it == warmup:
            _barrier(world)
        t0 = time.perf_counter()
        with torch.inference_mode():
            obs, priv, hist, _ = runner.rollout(obs, priv, hist)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            alg.compute_returns(hist, priv)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        alg.update()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if it >= warmup:
            split["rollout"] += t1 - t0
            split["gae"] += t2 - t1
            split["update"] += t3 - t2
    env.close()
    # at world > 1 the ranks meet in the gradient / KL / advantage all-reduces; the job runs at the slowest rank
    it_s = _max_over_ranks(sum(split.values()), world) / iters
    split = {k: _max_over_ranks(v, world) for k, v in split.items()}
    return {"value": n * world * T / it_s, "unit": "env-steps/s", "ms_per_iteration": it_s * 1e3, "iterations": iters,
            "world": world, "update": getattr(alg, "_engine", None) is not None and "hip-engine" or "torch",
            "split_ms_per_iteration": {k: v / iters * 1e3 for k, v in split.items()},
            "env": "VelocityTrackingEasyEnv (configs[1])" if velocity else "TrajectoryTrackingEnv (configs[2])",
            "fused_policy": runner.alg.fused is not None,
            "what": f"Runner iteration at {n} envs: {T} rollout steps + GAE + PPO.update "
                    "(5 epochs x 4 mini-batches), env-steps/s as ppo_cse/__init__.py:184 computes train/fps; "
                    "BASELINE.md derives ~8,960 (A100) and ~27,300 (A40) whole-loop env-steps/s from the "
                    "reference's wandb runs (other configs)"}


# ---------------------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n, argv):
    """Start n ranks of this script (one per GPU) and wait for them.  Runs before anything in this
    process touches the GPU (no torch import), so the children are ordinary fresh processes."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        for p in procs:
            r = p.wait()
            rc = rc or r
            if r != 0:  # one rank failed: the others would wait at a barrier forever
                for q in procs:
                    if q.poll() is None:
                        q.terminate()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def selftest_rank(args, rank, world):
    """--selftest: the launcher and the cross-rank reduction on CPU (gloo), no GPU and no env:
    each rank 'steps' a tiny numpy workload; rank 0 prints the line the real run would."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world
    x = np.zeros(1024, np.float32)
    t0 = time.perf_counter()
    for k in range(args.steps):
        x += np.float32(k)
    elapsed = time.perf_counter() - t0 + 1e-3 * (rank + 1)
    t = torch.tensor([elapsed, float(rank)], dtype=torch.float64)
    per = [torch.zeros_like(t) for _ in range(world)]
    if world > 1:
        dist.all_gather(per, t)
    else:
        per = [t]
    if rank == 0:
        el = max(float(p[0]) for p in per)
        n = args.envs_per_gpu
        print(json.dumps({"metric": METRIC, "value": n * world * args.steps / el, "n_gpus": world,
                          "world_size_seen": world, "ranks": [int(p[1]) for p in per], "selftest": True,
                          "config": {"global_envs": n * world, "parallelism": f"env-shard x{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


# ---------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs-per-gpu", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-rollout", action="store_true")
    ap.add_argument("--no-learn", action="store_true", help="skip the whole-training-loop leg")
    ap.add_argument("--no-velocity", action="store_true", help="skip the configs[1] velocity-tracking leg")
    ap.add_argument("--velocity-only", action="store_true", help="profile helper: time only the velocity env")
    ap.add_argument("--learn-only", action="store_true", help="profile helper: time only Runner iterations")
    ap.add_argument("--velocity-learn", action="store_true",
                    help="profile helper: time Runner iterations over the configs[1] velocity env")
    ap.add_argument("--rollout-only", action="store_true", help="profile helper: time only the rollout loop")
    ap.add_argument("--event-every", type=int, default=4,
                    help="record the HIP event pair around every k-th step kernel of the timed loop")
    ap.add_argument("--sweep", default="", help="comma-separated envs/GPU for an extra size sweep (e.g. 16384,65536)")
    ap.add_argument("--selftest", action="store_true", help="CPU-only launcher test (gloo, no GPU work)")
    ap.add_argument("--kernel-only", action="store_true", help="A/B helper: time only the fused kernel")
    ap.add_argument("--rollout-outputs", action="store_true",
                    help="with --kernel-only: the rollout's stores only (no contact forces, no aux block)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the line would misreport n_gpus")
    if args.selftest:
        sys.exit(selftest_rank(args, rank, world))

    import torch
    dev = torch.device("cuda", local)
    if args.kernel_only:  # A/B helper: the fused kernel alone, HIP-event statistics
        torch.cuda.set_device(dev)
        env = make_env(args.envs_per_gpu, 0, 1, dev)
        env.reset()
        ring = torch.randn((64, args.envs_per_gpu, 12), device=dev)
        kdt, kms = kernel_loop(env, ring, args.steps, args.warmup, every=1, contact_forces=not args.rollout_outputs)
        kt = np.array(kernel_loop.last)
        print(json.dumps({"kernel_ms_mean": kms, "kernel_ms_median": float(np.median(kt)),
                          "kernel_ms_p10": float(np.percentile(kt, 10)), "loop_ms_per_step": kdt / args.steps * 1e3}))
        return
    if args.rollout_only:
        torch.cuda.set_device(dev)
        print(json.dumps(rollout_rate(args.envs_per_gpu, dev, args.steps, args.warmup)))
        return
    if args.velocity_only:
        torch.cuda.set_device(dev)
        print(json.dumps(velocity_rate(args.envs_per_gpu, dev, args.steps, args.warmup)))
        return
    if args.learn_only or args.velocity_learn:
        torch.cuda.set_device(dev)
        print(json.dumps(learn_rate(args.envs_per_gpu, dev, velocity=args.velocity_learn)))
        return
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != world:
            raise SystemExit("world size mismatch")
    torch.cuda.set_device(dev)

    n = args.envs_per_gpu
    n_global = n * world
    env = make_env(n, rank, world, dev)
    env.reset()
    ring = torch.randn((64, n, 12), device=dev, generator=torch.Generator(device=dev).manual_seed(100 + rank))
    torch.cuda.synchronize()

    every = max(1, args.event_every)
    n_ev = (args.steps + every - 1) // every
    ev = EventPairs(n_ev)
    base = env.env
    # clock pre-warm: the GPU ramps its clocks over the first ~10-20 ms of sustained load (a 500-step
    # loop right after 50 warmup steps measured 68.5 us/step, after 200 warmup steps 57.7), so the
    # env is stepped for PREWARM_S seconds (untimed, reported as "prewarm_steps") before the W
    # warmup steps the caller asked for
    prewarm = 0
    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < PREWARM_S:
        for _ in range(16):
            env.step(ring[prewarm % 64])
            prewarm += 1
        torch.cuda.synchronize()
    for k in range(args.warmup):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    base.kernel_events.extend(ev.pair(k // every) if k % every == 0 else None for k in range(args.steps))
    t0 = time.perf_counter()
    for k in range(args.steps):
        env.step(ring[k % 64])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    base.kernel_events.clear()
    kernel_ms = float(np.mean([ev.ms(i) for i in range(n_ev)]))
    ev.close()
    if not os.environ.get("GO1_BENCH_ALLOW_NONFINITE"):
        assert torch.isfinite(base.obs_buf).all(), "non-finite observations"
    # the fused kernel alone on the same handle (no env host code)
    kdt, kms_raw = kernel_loop(env, ring, min(args.steps, 200), min(args.warmup, 10))
    mine = torch.tensor([elapsed, kernel_ms, kdt, kms_raw], device=dev, dtype=torch.float64)
    per_rank = [mine]
    if dist:
        per_rank = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
    per_rank = [p.tolist() for p in per_rank]
    elapsed = max(p[0] for p in per_rank)
    kernel_ms = max(p[1] for p in per_rank)
    kdt = max(p[2] for p in per_rank)
    # the rollout loop and the whole training loop run on every rank (RCCL all-reduces inside the timed
    # learn iterations at world > 1); rank 0 reports the slowest rank's time
    legs = {}
    if not args.no_rollout:
        legs["rollout"] = rollout_rate(n, dev, steps=min(args.steps, 240), warmup=min(args.warmup, 24), rank=rank,
                                       world=world)
    if not args.no_learn:
        legs["learn"] = learn_rate(n, dev, rank=rank, world=world)

    if rank == 0:
        value = n_global * args.steps / elapsed
        ks = kernel_ms * 1e-3
        alg = SURVEY_BYTES_PER_ENV_STEP * n
        achieved_gbs = alg / ks / 1e9
        pmc = pmc_counters(n)
        traffic = pmc["traffic"]
        ratio = lambda t, b: None if t is None else t / b  # noqa: E731
        fp32 = {"bound_note": "SURVEY 8(d): FP32 compute binds first (~50 flop/B)",
                "survey_flops_per_env_step": SURVEY_FLOPS_PER_ENV_STEP,
                "achieved_tflops_survey_flops": SURVEY_FLOPS_PER_ENV_STEP * n / ks / 1e12,
                "frac_survey_flops": SURVEY_FLOPS_PER_ENV_STEP * n / ks / 1e12 / FP32_PEAK_TFLOPS,
                "peak_tflops": FP32_PEAK_TFLOPS}
        if pmc["flops"]:
            fp32.update(counted_flops_per_launch=pmc["flops"], counted_flops_per_env_step=pmc["flops"] / n,
                        achieved_tflops_counted=pmc["flops"] / ks / 1e12,
                        frac_counted=pmc["flops"] / ks / 1e12 / FP32_PEAK_TFLOPS)
        ksteps = min(args.steps, 200)
        line = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "prewarm_steps": prewarm, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "BASELINE configs[2]: VecEnv.step of HistoryWrapper(TrajectoryTrackingEnv), Go1 "
                                   "single_path tunnel (32x32 sub-terrains), 2x10x11 front height scan, actuator "
                                   "net, e2e rewards, DR; N(0,1) actions",
                       "envs_per_gpu": n, "global_envs": n_global, "decimation": base._abi_cfg.decimation,
                       "integrator_substeps": base._abi_cfg.n_internal, "parallelism": f"env-shard x{world}",
                       "world_size_seen": world},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_fetch_doubled": pmc["traffic_x2"],
                         "traffic_over_algorithmic": ratio(traffic, alg),
                         "traffic_over_algorithmic_fetch_doubled": ratio(pmc["traffic_x2"], alg),
                         "write_traffic_over_algorithmic_writes": ratio(pmc["written"], 1758 * n),
                         "traffic_source": pmc["src"],
                         "traffic_rollout_outputs": rollout_traffic(n),
                         "algorithmic_bytes_per_launch": alg, "bytes_per_env_step": SURVEY_BYTES_PER_ENV_STEP,
                         "bytes_source": "SURVEY.md 8(d): 3,522 B per env-step",
                         "bytes_written_by_path": {"bytes_per_env_step": PATH_BYTES_PER_ENV_STEP,
                                                   "achieved_gbs": PATH_BYTES_PER_ENV_STEP * n / ks / 1e9},
                         "kernel": "go1_step_kernel<false, 7, true> (README-config specialisation)",
                         "kernel_ms": kernel_ms,
                         "kernel_ms_method": "hipExtLaunchKernelGGL start/stop events on the kernel's dispatch, "
                                             "every k-th step of the timed loop, on the launch stream",
                         "fp32": fp32,
                         "valu_issue_frac_pmc": pmc["valu"],
                         "note": "latency/VALU-issue bound, not HBM bound: see DESIGN.md section 5"},
            "kernel_loop": {"value": n_global * ksteps / kdt, "unit": "env-steps/s", "ms_per_step": kdt / ksteps * 1e3,
                            "kernel_ms": max(p[3] for p in per_rank),
                            "what": "Go1Native.step alone (the fused kernel launch, no env host code)"},
            "per_rank": [{"rank": r, "elapsed_s": p[0], "kernel_ms": p[1]} for r, p in enumerate(per_rank)],
        }
        if args.sweep:
            line["sweep"] = [env_sweep(int(x), dev) for x in args.sweep.split(",")]
        for k, v in legs.items():
            line[k] = v
        if not args.no_velocity and world == 1:
            # at least two full 32-step history windows (velocity.py HIST_WINDOW), whatever --steps is
            line["velocity"] = velocity_rate(n, dev, steps=max(2 * 32, min(args.steps, 300)),
                                             warmup=min(args.warmup, 30))
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(n, budget_s=args.cpu_budget)
        print(json.dumps(line), flush=True)
    env.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
