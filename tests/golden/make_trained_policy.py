"""Fixture of the reference's trained policy (container-only test infrastructure).

Reads runs/trajectory_tracking/run-20230904_112307-rhi1my71/checkpoints/ac_weights.pt from the reference
with torch.load(weights_only=True) -- data only, nothing executed -- and records its state dict (6
privileged obs: the adaptation module's latent is 6 wide, the actor / critic inputs 267), a batch of
inputs (observation rows of tests/golden/ppo_rollout.npz, which the reference's own env produced, plus
random rows and privileged values) and the ActorCritic outputs computed on the CPU in f64 (latent, action
mean, value): the reference point of tests/test_rollout.py's fused-kernel test on trained weights.

Usage: python tests/golden/make_trained_policy.py   (writes tests/golden/trained_policy.npz)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from legged_tracking_amd import rollout as R  # noqa: E402

CKPT = "/root/reference/runs/trajectory_tracking/run-20230904_112307-rhi1my71/checkpoints/ac_weights.pt"


def main():
    sd = torch.load(CKPT, weights_only=True, map_location="cpu")
    npriv = sd["adaptation_module.4.weight"].shape[0]
    ac = R.ActorCritic(261, npriv, 261, 12)
    ac.load_state_dict(sd)
    ppo = np.load(os.path.join(HERE, "ppo_rollout.npz"))
    rng = np.random.default_rng(5)
    real = ppo["in/hist"][:48].astype(np.float32)
    hist = np.concatenate([real, rng.normal(0, 1, (16, 261)).astype(np.float32)])
    priv = rng.uniform(-1, 1, (len(hist), npriv)).astype(np.float32)
    ac64 = ac.double()
    with torch.no_grad():
        h, p = torch.from_numpy(hist).double(), torch.from_numpy(priv).double()
        lat = ac64.adaptation_module(h)
        mean = ac64.actor_body(torch.cat((h, lat), -1))
        val = ac64.critic_body(torch.cat((h, p), -1))
    out = {f"sd/{k}": v.float().numpy() for k, v in sd.items()}
    out.update({"in/hist": hist, "in/priv": priv, "out/latent": lat.numpy(), "out/mean": mean.numpy(),
                "out/value": val.numpy()})
    np.savez_compressed(os.path.join(HERE, "trained_policy.npz"), **out)
    print("wrote trained_policy.npz", {k: v.shape for k, v in out.items() if not k.startswith("sd/")})


if __name__ == "__main__":
    main()
