"""Benchmark of the fused MI355X Go1 step (BASELINE.json metric).

One "step" = one LeggedRobot.step() (4 sim sub-steps of actuator net + native
articulated-body integrator, then the full post-physics: height scan, targets,
rewards, terminations, resets, observations) over 4096 envs per GPU on the
single_path tunnel (BASELINE configs[2]; configs[1] is the velocity-tracking env,
which is not on this path).  Inputs are synthetic and already resident in HBM
when the timed region starts: a ring of N(0,1) action batches (the actor's
init_noise_std = 1.0, ppo_cse/actor_critic.py:11) generated on the device.

Multi-GPU: one process per GPU (torch.distributed.run), envs sharded by global
env id (rank r owns [r*N, (r+1)*N)), no collective inside the step ->
"scaling": "weak".  value = sum over ranks of envs x steps / max-over-ranks time.

Also reported: roofline of the fused step kernel (HIP events around that kernel
alone on the launch stream) and the CPU oracle (oracle/, "port") timed on a
bounded sample on the host cores of rank 0.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "env-steps/sec (whole node) at 4096 Go1/GPU, 1/2/4/8 MI355X; %HBM roofline"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA

# Algorithmic HBM bytes per env-step of the fused kernel (DESIGN.md "Roofline accounting"):
#   reads : actions 48, root 52, dof pos/vel 96, lag 336, err/vel history 192, motor strength/offset 96,
#           last actions/dof vel 96, friction/restitution/payload 12, episode length/pose index/collisions 12,
#           trajectory 24, base rotation 12, episode sums 52, terrain index+origins 28,
#           110 height samples x 2 layers x 4 B = 880                                  -> 1,936 B
#   writes: obs 1044, priv 8, rew 4, reset/time-out/extras 3, contact forces 204, root 52, dof pos/vel 96,
#           lag 336, err/vel history 192, last actions/dof vel 96, joint targets 48, strength/offset 96,
#           trajectory 24, base rotation 12, episode sums 52, counters 12               -> 2,279 B
BYTES_PER_ENV_STEP = 1936 + 2279
# Algorithmic FLOPs per env-step: actuator net 12 joints x 4 sub-steps x 2,688 (exact: 1,248 FMA + 64
# softsign x 3 flops + 32 ...); the integrator and post-physics are not counted here.
FLOPS_PER_ENV_STEP = 12 * 4 * 2688


# PMC-measured HBM bytes per launch of the step kernel (tools/profile.sh + tools/prof_summary.py;
# FETCH_SIZE + WRITE_SIZE, separate --pmc passes).  Re-collected whenever the kernel changes.
TRAFFIC_FILE = os.path.join(REPO, "profiles", "r01", "step_counters.json")


def pmc_traffic(n_envs):
    """(HBM bytes per launch, VALU issue fraction, source) from the committed PMC summary."""
    try:
        with open(TRAFFIC_FILE) as f:
            d = json.load(f)
        if int(d["resources"]["Grid_Size"]) != 16 * n_envs:  # 16 lanes per env
            return None, None, None
        pw = d.get("per_wave", {})
        valu = pw["SQ_ACTIVE_INST_VALU"] / pw["SQ_WAVE_CYCLES"] if "SQ_ACTIVE_INST_VALU" in pw else None
        return d["hbm_bytes_per_launch"]["traffic"], valu, os.path.relpath(TRAFFIC_FILE, REPO)
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None, None, None


def hip():
    h = C.CDLL("libamdhip64.so")
    h.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    h.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    h.hipEventSynchronize.argtypes = [C.c_void_p]
    h.hipEventDestroy.argtypes = [C.c_void_p]
    return h


def cpu_baseline(n_envs, budget_s=12.0, max_steps=400):
    """Time the CPU oracle (a C restatement, OpenMP over envs) on the same workload."""
    from legged_tracking_amd import config as CF, terrain as T
    from oracle import oracle as O
    cores = len(os.sched_getaffinity(0))
    threads = min(cores, 16)
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
    O.step(c, st, ter, acts[0], gvec, grav, scales, rng_seed=1, rng_step=1, debug=False)  # warm
    t0 = time.perf_counter()
    k = 0
    while k < max_steps and time.perf_counter() - t0 < budget_s:
        O.step(c, st, ter, acts[k % 8], gvec, grav, scales, rng_seed=1, rng_step=2 + k, debug=False)
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
            "sample": f"{k} steps x {n_envs} envs of the C oracle (f64 integrator, same single_path workload), "
                      f"{dt:.1f} s on {threads} threads of {cores} visible ({model})"}


def env_sweep(n, dev, steps=100, warmup=10):
    """Env-only throughput at n envs on this GPU (4k ... 256k envs/GPU sweep)."""
    import torch
    from legged_tracking_amd import config as CF, native, terrain as T
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=32, cols=32)
    c = CF.build_abi_config(cfg, n_envs=n)
    td = T.build(cfg, n, np.random.RandomState(11))
    g = native.Go1Native(c, str(dev))
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    rng = np.random.default_rng(5)
    g.state["friction"].copy_(torch.from_numpy(rng.uniform(0.1, 3.0, (n, 1)).astype(np.float32)))
    g.reset_envs(torch.ones(n, dtype=torch.bool, device=dev), rng_seed=5, rng_step=0)
    g.state["episode_length"].copy_(torch.from_numpy(rng.integers(0, 500, (n, 1)).astype(np.int32)))
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    grav, gvec = CF.gravity_state([0.1, -0.2, 0.3])
    ring = torch.randn((8, n, 12), device=dev)
    for k in range(warmup):
        g.step(ring[k % 8], gvec, grav, scales, rng_seed=5, rng_step=1 + k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        g.step(ring[k % 8], gvec, grav, scales, rng_seed=5, rng_step=1 + warmup + k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    g.close()
    return {"envs_per_gpu": n, "value": n * steps / dt, "ms_per_step": dt / steps * 1e3}


def rollout_rate(n, dev, steps, warmup, prof=None):
    """Secondary line (SURVEY 8(d) "report both env-only and rollout (act + step) rates"):
    the Runner's rollout loop -- ActorCritic.act + value (hipBLASLt GEMMs), env.step
    through TrajectoryTrackingEnv/HistoryWrapper, transition record kernel -- at n envs."""
    import torch
    from legged_tracking_amd import config as CF, env as E, rollout as R
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=32, cols=32)
    env = E.HistoryWrapper(E.TrajectoryTrackingEnv(sim_device=str(dev), cfg=cfg, seed=11, rank=0, world_size=1))
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
        if prof is not None:
            prof.enable()
        t0 = time.perf_counter()
        for _ in range(steps):
            one()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if prof is not None:
            prof.disable()
    return {"value": n * steps / dt, "unit": "env-steps/s", "ms_per_step": dt / steps * 1e3, "steps": steps,
            "what": "PPO.act (fused MFMA adaptation+actor+critic kernel, Normal sample) + TrajectoryTrackingEnv.step "
                    "+ HistoryWrapper + process_env_step record kernel, 1 GPU",
            "fused_policy": alg.fused is not None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs-per-gpu", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-rollout", action="store_true")
    ap.add_argument("--rollout-only", action="store_true", help="profile helper: time only the rollout loop")
    ap.add_argument("--event-every", type=int, default=4,
                    help="record the HIP event pair around every k-th step kernel of the timed loop")
    ap.add_argument("--sweep", default="", help="comma-separated envs/GPU for an extra size sweep (e.g. 16384,65536)")
    args = ap.parse_args()

    import torch
    if args.rollout_only:
        print(json.dumps(rollout_rate(args.envs_per_gpu, torch.device("cuda", 0), args.steps, args.warmup)))
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from legged_tracking_amd import config as CF, native, terrain as T
    n = args.envs_per_gpu
    n_global = n * world
    cfg = CF.readme_config(n_envs=n_global, terrain="single_path", rows=32, cols=32)
    c = CF.build_abi_config(cfg, n_envs=n)
    c.env_id_offset = rank * n  # global env ids key the Philox streams, as in TrajectoryTrackingEnv
    d = CF.derived(cfg)
    # terrain: 32 x 32 tunnels replicated on every rank; env (global id) -> tile (id mod 1024)
    td = T.build(cfg, n_global, np.random.RandomState(11))
    sl = slice(rank * n, (rank + 1) * n)
    g = native.Go1Native(c, str(dev))
    g.set_terrain(td.tiles, td.env_tile[sl], td.env_terrain_origin[sl], td.env_origins[sl])
    rng = np.random.default_rng(100 + rank)
    g.state["friction"].copy_(torch.from_numpy(rng.uniform(0.1, 3.0, (n, 1)).astype(np.float32)))
    g.state["restitution"].copy_(torch.from_numpy(rng.uniform(0.0, 0.4, (n, 1)).astype(np.float32)))
    g.state["payload"].copy_(torch.from_numpy(rng.uniform(-1.0, 3.0, (n, 1)).astype(np.float32)))
    keep = g.reset_envs(torch.ones(n, dtype=torch.bool, device=dev), rng_seed=11, rng_step=rank)
    g.state["episode_length"].copy_(torch.from_numpy(rng.integers(0, 500, (n, 1)).astype(np.int32)))
    scales = CF.reward_scale_vector(d["reward_scales"])
    grav, gvec = CF.gravity_state(rng.uniform(-1, 1, 3))
    ring = torch.randn((64, n, 12), device=dev)
    torch.cuda.synchronize()
    del keep

    hp = hip()
    n_ev = args.steps
    evs = []
    for _ in range(2 * n_ev):
        e = C.c_void_p()
        assert hp.hipEventCreate(C.byref(e)) == 0
        evs.append(e)

    seed = 20240101
    for k in range(args.warmup):
        g.step(ring[k % 64], gvec, grav, scales, rng_seed=seed, rng_step=k)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    every = max(1, args.event_every)
    for k in range(args.steps):
        ev = (evs[2 * k].value, evs[2 * k + 1].value) if k % every == 0 else None
        g.step(ring[k % 64], gvec, grav, scales, rng_seed=seed, rng_step=args.warmup + k, events=ev)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kt = []
    for k in range(0, args.steps, every):
        ms = C.c_float()
        hp.hipEventElapsedTime(C.byref(ms), evs[2 * k], evs[2 * k + 1])
        kt.append(ms.value)
    kernel_ms = float(np.mean(kt))
    if not os.environ.get("GO1_BENCH_ALLOW_NONFINITE"):
        assert torch.isfinite(g.obs).all(), "non-finite observations"
    if dist:
        t = torch.tensor([elapsed, kernel_ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])

    if rank == 0:
        value = n_global * args.steps / elapsed
        achieved_gbs = BYTES_PER_ENV_STEP * n / (kernel_ms * 1e-3) / 1e9
        achieved_tf = FLOPS_PER_ENV_STEP * n / (kernel_ms * 1e-3) / 1e12
        traffic, valu_frac, traffic_src = pmc_traffic(n)
        line = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "BASELINE configs[2]: Go1 single_path tunnel (32x32 sub-terrains), 2x10x11 front "
                                   "height scan, actuator net, e2e rewards, DR; N(0,1) actions",
                       "envs_per_gpu": n, "global_envs": n_global, "decimation": c.decimation,
                       "integrator_substeps": c.n_internal, "parallelism": f"env-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src, "algorithmic_bytes_per_launch": BYTES_PER_ENV_STEP * n,
                         "kernel": "go1_step_kernel<false>", "kernel_ms": kernel_ms,
                         "bytes_per_env_step": BYTES_PER_ENV_STEP,
                         "fp32_tflops_actuator_only": achieved_tf, "fp32_frac_actuator_only": achieved_tf / FP32_PEAK_TFLOPS,
                         "valu_issue_frac_pmc": valu_frac,
                         "note": "latency/VALU-issue bound, not HBM bound: see DESIGN.md section 5"},
        }
        if args.sweep:
            line["sweep"] = [env_sweep(int(x), dev) for x in args.sweep.split(",")]
        if not args.no_rollout:
            line["rollout"] = rollout_rate(n, dev, steps=min(args.steps, 240), warmup=min(args.warmup, 24))
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(n, budget_s=args.cpu_budget)
        print(json.dumps(line), flush=True)
    for e in evs:
        hp.hipEventDestroy(e)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
