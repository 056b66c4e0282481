"""Build the HIP C-ABI libraries for gfx950 in-tree (legged_tracking_amd/_build)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
INC = os.path.join(HERE, "..", "include")
BUILD = os.path.join(HERE, "_build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off"]

# The step kernel is VALU-issue bound.  One wave issues a v_pk_fma_f32 (two FMAs) as fast
# as a v_fma_f32 (tools/probes/pk_rate.hip), so the kernel packs by hand where the data
# pair up naturally (f2 types); the SLP auto-vectoriser stays off: its packing of scalar
# code adds register-pair moves that cost more than they save (measured -3 %).
STEP_FLAGS = ["-fno-slp-vectorize"]

# name -> (sources, extra dependencies, extra flags)
LIBS = {
    "libgo1_mi355x.so": (["go1_step.hip", "go1_terrain.hip"],
                         ["pmath.h", "go1_device.h", "go1_model_consts.h", "go1_spec.h", os.path.join(INC, "go1_mi355x.h")], STEP_FLAGS),
    "libgo1_rollout.so": (["rollout.hip"], [os.path.join(INC, "go1_rollout.h")], []),
    "libgo1_ppo.so": (["ppo_update.hip"], [os.path.join(INC, "go1_ppo.h")], []),
    # kernel-argument preloading: the curriculum launch's leading scalar arguments arrive in SGPRs with the wave
    # (11.75-11.78 against 12.02-12.10 us average per launch, alternating runs of one session)
    "libgo1_velocity.so": (["go1_velocity.hip"],
                           ["pmath.h", "go1_device.h", "go1_model_consts.h", os.path.join(INC, "go1_mi355x.h"),
                            os.path.join(INC, "go1_velocity.h")],
                           STEP_FLAGS + ["-mllvm", "-amdgpu-kernarg-preload-count=16"]),
}
OUT = os.path.join(BUILD, "libgo1_mi355x.so")  # the step library (kept for callers of build())


def _paths(name):
    srcs, deps, _ = LIBS[name]
    srcs = [os.path.join(HERE, "csrc", s) for s in srcs]
    return srcs, srcs + [d if os.path.isabs(d) else os.path.join(HERE, "csrc", d) for d in deps]


def needs_build(name):
    out = os.path.join(BUILD, name)
    if not os.path.exists(out):
        return True
    return any(os.path.getmtime(d) > os.path.getmtime(out) for d in _paths(name)[1])


def build(force=False, verbose=False, names=None):
    os.makedirs(BUILD, exist_ok=True)
    for name in names or LIBS:
        if not force and not needs_build(name):
            continue
        srcs, _ = _paths(name)
        cmd = [HIPCC, *FLAGS, *LIBS[name][2], "-o", os.path.join(BUILD, name), *srcs]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        # the device-only feature flag is also seen (and ignored) by the host pass
        err = "\n".join(l for l in r.stderr.splitlines() if "not a recognized feature" not in l)
        if err.strip():
            print(err, file=sys.stderr)
        if r.returncode != 0:
            raise subprocess.CalledProcessError(r.returncode, cmd)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
