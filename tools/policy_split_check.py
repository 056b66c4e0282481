"""policy_kernel_split against policy_kernel: identical outputs on the same weights and inputs.

  python tools/policy_split_check.py dump OUT.npz      (GO1_ROLLOUT_LIB_OVERRIDE selects the library)
  python tools/policy_split_check.py compare A.npz B.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(out, n=4096 + 48):
    import torch
    from legged_tracking_amd import rollout as R
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    hist_dim, n_priv, n_obs = 261, 2, 87
    ac = R.ActorCritic(n_obs, n_priv, hist_dim, 12).to(dev)
    alg = R.PPO(ac, device=dev)
    alg.init_storage(n, 4, [n_obs], [n_priv], [hist_dim], [12])
    g = torch.Generator(device=dev).manual_seed(1)
    hist = torch.randn((n, hist_dim), device=dev, generator=g)
    priv = torch.randn((n, n_priv), device=dev, generator=g)
    with torch.inference_mode():
        mean, value, latent, actions, sigma, logp = alg.fused.forward(hist, priv, sample=(7, 3, 0))
    torch.cuda.synchronize()
    np.savez(out, mean=mean.cpu().numpy(), value=value.cpu().numpy(), latent=latent.cpu().numpy(),
             actions=actions.cpu().numpy(), sigma=sigma.cpu().numpy(), logp=logp.cpu().numpy())
    print("dumped", out, {k: v.shape for k, v in np.load(out).items()})


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A if not np.array_equal(A[k], B[k])]
    for k in bad:
        print(k, "max abs diff", np.abs(A[k] - B[k]).max())
    print("identical" if not bad else f"DIFFER: {bad}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    dump(sys.argv[2]) if sys.argv[1] == "dump" else compare(sys.argv[2], sys.argv[3])
