"""Phase timing of the policy kernel (diagnostic build with -DGO1_POLICY_STAMPS).

  local:  hipcc ... -DGO1_POLICY_STAMPS -o legged_tracking_amd/_build/libgo1_rollout_stamps.so rollout.hip
  gpurun: python tools/policy_stamps.py [--variant 1]   (default: variant 0, policy_kernel_split)

Phases end at the kernel's barriers: 1 input staging, 2 adaptation L1, 3 adaptation L2,
4 adaptation L3 (latent), 5 actor/critic L1, 6 L2, 7 L3, 8 output layer + sampling.
Prints per phase the mean over workgroups of (max over waves of the phase end) minus the
previous phase end, in s_memtime cycles, and the share of the workgroup lifetime."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GO1_ROLLOUT_LIB_OVERRIDE"] = os.path.join(ROOT, "legged_tracking_amd", "_build",
                                                      "libgo1_rollout_stamps.so")
NAMES = ["staging", "adapt L1 256", "adapt L2 128", "adapt L3 2", "A/C L1 512", "A/C L2 256", "A/C L3 128",
         "out + sample"]


def main():
    import torch
    from legged_tracking_amd import rollout as R
    n = 4096
    dev = torch.device("cuda", 0)
    ac = R.ActorCritic(261, 2, 261, 12).to(dev)
    alg = R.PPO(ac, device=dev)
    alg.init_storage(n, 24, [261], [2], [261], [12])
    assert alg.fused is not None
    obs = torch.randn(n, 261, device=dev)
    priv = torch.randn(n, 2, device=dev)
    with torch.inference_mode():
        for _ in range(5):
            alg.act(obs, priv, obs)
    torch.cuda.synchronize()
    variant = int(sys.argv[sys.argv.index("--variant") + 1]) if "--variant" in sys.argv else 0
    alg.fused.variant = variant
    with torch.inference_mode():
        for _ in range(5):
            alg.act(obs, priv, obs)
    torch.cuda.synchronize()
    lib = alg.fused.lib
    buf = np.zeros(512 * 16 * 12, np.uint64)
    assert lib.go1_policy_stamps(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
    t_full = buf.reshape(512, 16, 12).astype(np.int64)[:256]
    t_all = t_full[:, :, :9]
    used = t_all[:, 0, 0] != 0  # workgroups of the launch (the stamp buffer holds 256)
    na = -(-n // (16 * int(os.environ.get("GO1_SPLIT_ET_A", "2"))))
    groups = [("all", t_all[used])] if variant else [("actor workgroups", t_all[:na][used[:na]]),
                                                     ("critic workgroups", t_all[na:][used[na:]])]
    for label, t in groups:
        t = t - t[:, :, :1].min(axis=1, keepdims=True)
        print(f"{label}: wave start spread within a workgroup: mean {t[:, :, 0].max(axis=1).mean():.0f} cycles")
        ends = t.max(axis=1)  # (wg, 9): phase end = last wave through the barrier
        d = np.diff(ends, axis=1).mean(axis=0)
        life = ends[:, 8].mean()
        print(f"{label}: {t.shape[0]}; mean lifetime {life:.0f} cycles")
        for nm, v in zip(NAMES, d):
            print(f"  {nm:14s} {v:9.0f} {v / life:7.1%}")
    # inside the staging: 9 = the f32 copy stored (the input loads landed), 10 = past the barrier after it
    tf = t_full[used]
    t0 = tf[:, :, :1].min(axis=1)
    for k, nm in ((9, "inputs landed"), (10, "copy barrier")):
        if (tf[:, :, k] != 0).all():
            print(f"  staging: {nm:14s} at {(tf[:, :, k].max(axis=1) - t0[:, 0]).mean():9.0f} cycles (last wave)")
    print(f"  wave start -> first stamp of wave: mean spread {(tf[:, :, 0] - t0).mean():.0f}")
    # spread of the workgroups' start times (launch ramp) and end times
    st = t_all[used][:, :, 0].min(axis=1)
    en = t_all[used][:, :, 8].max(axis=1)
    print(f"start spread {np.ptp(st)} cycles, end spread {np.ptp(en)}, first start -> last end {en.max() - st.min()}")


if __name__ == "__main__":
    main()
