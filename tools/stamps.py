"""Where one step-kernel launch spends its time, per source section (diagnostic build).

The stamp buffer is zeroed before each of the GO1_STAMPS_MEASURE launches read (after
GO1_STAMPS_STEPS warm-up launches); every statistic is over (launch, wave) records.

  local:  bash tools/variants.sh build stamps "-DGO1_STAMPS"
  gpurun: python tools/stamps.py [n_envs]

Runs the bench workload on the stamps build (every MARK() records (line, s_memtime)),
then prints, per section (the code after a marker, up to the next executed marker), the
mean cycles per wave summed over all its executions in the launch and its share of the
wave's lifetime.  Read the SHARES: the stamps' waits forbid overlaps the real kernel has.
"""
import ctypes as C
import collections
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GO1_LIB_OVERRIDE"] = os.path.join(ROOT, "legged_tracking_amd", "_build", "libgo1_var_%s.so" % os.environ.get("GO1_STAMPS_VARIANT", "stamps"))
WAVES, SLOTS = 4096, int(os.environ.get("GO1_STAMPS_SLOTS", "320"))


def main():
    import torch
    from legged_tracking_amd import config as CF, native, terrain as T
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda", 0)
    cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=32, cols=32)
    c = CF.build_abi_config(cfg, n_envs=n)
    td = T.build(cfg, n, np.random.RandomState(11))
    g = native.Go1Native(c, str(dev))
    g.set_terrain(td.tiles, td.env_tile, td.env_terrain_origin, td.env_origins)
    rng = np.random.default_rng(100)
    g.state["friction"].copy_(torch.from_numpy(rng.uniform(0.1, 3.0, (n, 1)).astype(np.float32)))
    g.reset_envs(torch.ones(n, dtype=torch.bool, device=dev), rng_seed=11, rng_step=0)
    g.state["episode_length"].copy_(torch.from_numpy(rng.integers(0, 500, (n, 1)).astype(np.int32)))
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    grav, gvec = CF.gravity_state(rng.uniform(-1, 1, 3))
    ring = torch.randn((8, n, 12), device=dev)
    warm = int(os.environ.get('GO1_STAMPS_STEPS', '30'))
    meas = int(os.environ.get('GO1_STAMPS_MEASURE', '8'))
    lib = native.lib()
    bufs = []
    for k in range(warm + meas):
        if k >= warm:  # every measured launch starts from a zeroed buffer (stale slots of an earlier launch
            torch.cuda.synchronize()  # with more markers would otherwise be read as this launch's)
            assert lib.go1_debug_stamps_clear() == 0
        g.step(ring[k % 8], gvec, grav, scales, rng_seed=11, rng_step=1 + k)
        if k >= warm:
            torch.cuda.synchronize()
            buf = np.zeros(WAVES * SLOTS, np.uint64)
            assert lib.go1_debug_stamps(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
            bufs.append(buf)
    g.close()

    name = {}
    for f in ("go1_step.hip", "go1_device.h"):  # (a line number marked in both files names both)
        src = open(os.path.join(ROOT, "legged_tracking_amd", "csrc", f)).read().splitlines()
        for i, l in enumerate(src):
            m = re.search(r"MARK\((\w+)\)", l)
            if m:
                name[i + 1] = name[i + 1] + "|" + m.group(1) if i + 1 in name else m.group(1)
    nw = min(WAVES, n // 4)
    b = np.concatenate([x[: nw * SLOTS].reshape(nw, SLOTS) for x in bufs])  # (launches x waves, slots)
    line = (b >> np.uint64(48)).astype(np.int64)
    t = (b & np.uint64((1 << 48) - 1)).astype(np.int64)
    nrec = np.count_nonzero(line, 1)
    # a record is written in slot order: the count of non-zero slots is the number of markers executed
    assert all(np.count_nonzero(line[w, : nrec[w]]) == nrec[w] for w in range(len(line)))
    tot = collections.Counter()
    cnt = collections.Counter()
    life = []
    per_wave = []  # per (launch, wave): section -> cycles (the tail analysis below)
    keep = []
    for w in range(len(line)):
        k = int(nrec[w])
        if k < 2:
            continue
        keep.append(w)
        life.append(t[w, k - 1] - t[w, 0])
        pw = collections.Counter()
        for i in range(k - 1):
            nm = name.get(int(line[w, i]), str(line[w, i]))
            tot[nm] += int(t[w, i + 1] - t[w, i])
            pw[nm] += int(t[w, i + 1] - t[w, i])
            cnt[nm] += 1
        per_wave.append(pw)
    assert min(life) > 0, "negative wave lifetime: stale stamps"
    L = float(np.mean(life))
    lf = np.array(life, np.float64)
    print(f"wave lifetime cycles: p50 {np.percentile(lf, 50):.0f}  p90 {np.percentile(lf, 90):.0f}  "
          f"p99 {np.percentile(lf, 99):.0f}  max {lf.max():.0f}  min {lf.min():.0f}")
    print(f"wave records {len(life)} ({len(bufs)} launches x {nw} waves); mean wave lifetime {L:.0f} cycles "
          f"(s_memtime, per-wave differences only: the counters of different XCDs are not aligned); "
          f"stamps per wave {np.mean(nrec):.0f}")
    print(f"{'section (after marker)':28s} {'cycles/wave':>12s} {'share':>7s} {'execs':>6s}")
    for nm, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{nm:28s} {v / len(life):12.0f} {v / len(life) / L:7.1%} {cnt[nm] / len(life):6.1f}")
    # the launch lasts as long as its slowest waves: where do the slowest 5 % spend their extra cycles?
    order = np.argsort(lf)
    slow = order[-max(1, len(lf) // 20):]
    mid = order[len(lf) // 4: 3 * len(lf) // 4]
    print(f"\nslowest 5 % of waves ({len(slow)}): mean lifetime {lf[slow].mean():.0f} vs the middle half "
          f"{lf[mid].mean():.0f} cycles; extra cycles per section:")
    secs = sorted(tot)
    extra = {nm: np.mean([per_wave[i][nm] for i in slow]) - np.mean([per_wave[i][nm] for i in mid]) for nm in secs}
    for nm, v in sorted(extra.items(), key=lambda x: -x[1])[:12]:
        print(f"{nm:28s} {v:+12.0f}")
    # per-execution cost of the sections in the slowest waves (execs there vs the middle half)
    cw = []
    for w in keep:
        k = int(nrec[w])
        c = collections.Counter(name.get(int(line[w, i]), str(line[w, i])) for i in range(max(0, k - 1)))
        cw.append(c)
    print(f"\n{'section':28s} {'execs slow':>10s} {'execs mid':>10s} {'cyc/exec slow':>14s} {'cyc/exec mid':>13s}")
    for nm in sorted(secs, key=lambda x: -extra[x])[:14]:
        es = np.mean([cw[i][nm] for i in slow]); em = np.mean([cw[i][nm] for i in mid])
        ts = np.mean([per_wave[i][nm] for i in slow]); tm = np.mean([per_wave[i][nm] for i in mid])
        print(f"{nm:28s} {es:10.2f} {em:10.2f} {ts / max(es, 1e-9):14.0f} {tm / max(em, 1e-9):13.0f}")
    # the very slowest waves one by one (the launch time is the slowest wave's): their largest extra sections
    mid_mean = {nm: np.mean([per_wave[i][nm] for i in mid]) for nm in secs}
    print("\nthe 6 slowest waves: lifetime, then the sections with the most extra cycles over the middle half")
    for i in order[-6:][::-1]:
        ex = sorted(((per_wave[i][nm] - mid_mean[nm], nm) for nm in secs), reverse=True)[:5]
        print(f"  {lf[i]:8.0f}  " + "  ".join(f"{nm} {v:+.0f} ({cw[i][nm]}x)" for v, nm in ex))


if __name__ == "__main__":
    main()
