"""Test double for the HIP step: the CPU oracle behind Go1Native's interface.

TEST INFRASTRUCTURE ONLY.  Lets the host-side env logic (legged_tracking_amd/env.py,
the PPO rollout and the multi-rank sharding) run in `-m "not gpu"` tests; the
product env always binds legged_tracking_amd.native.Go1Native.
"""
import numpy as np
import torch

from legged_tracking_amd import abi
from oracle import oracle as O


class _State:
    def __init__(self, n, cfg):
        self.np = O.NpState(n, cfg=cfg)
        self.t = {k: torch.from_numpy(v) for k, v in self.np.arrays.items()}

    def __getitem__(self, k):
        return self.t[k]

    def load(self, arrays):
        for k, v in arrays.items():
            if k in self.t:
                self.t[k].copy_(torch.as_tensor(np.asarray(v)).reshape(self.t[k].shape).to(self.t[k].dtype))

    def numpy(self):
        return {k: v.numpy().copy() for k, v in self.t.items()}


class OracleBackend:
    def __init__(self, cfg):
        self.cfg = cfg
        self.n = n = cfg.n_envs
        self.device = torch.device("cpu")
        self.state = _State(n, cfg)
        self.contact_forces = torch.zeros((n, 17, 3))
        self.extras_time_outs = torch.zeros(n, dtype=torch.bool)
        self.ter = None
        self.calls = []

    def set_terrain(self, tiles, env_tile, env_terrain_origin, env_origins):
        self.ter = O.NpTerrain(tiles, env_tile, env_terrain_origin, env_origins)

    def step(self, actions, gravity_vec, sim_gravity, reward_scales, rng_seed=0, rng_step=0, out=None,
             episode_log=None, aux=None, **kw):
        self.calls.append(dict(gravity_vec=np.array(gravity_vec), sim_gravity=np.array(sim_gravity),
                               reward_scales=np.array(reward_scales), rng_step=rng_step))
        o = O.step(self.cfg, self.state.np, self.ter, actions.numpy(), gravity_vec, sim_gravity, reward_scales,
                   rng_seed=rng_seed, rng_step=rng_step, debug=True)
        out["obs"].copy_(torch.from_numpy(o["obs"]))
        if kw.get("obs_history") is not None:  # the kernel's optional second copy of obs
            kw["obs_history"].copy_(out["obs"])
        out["priv"].copy_(torch.from_numpy(o["priv"]))
        out["rew"].copy_(torch.from_numpy(o["rew"]))
        out["reset"].copy_(torch.from_numpy(o["reset"].astype(bool)))
        out["time_out"].copy_(torch.from_numpy(o["time_out"].astype(bool)))
        if kw.get("contact_forces", True):
            self.contact_forces.copy_(torch.from_numpy(o["contact_forces"]))
        if o["reset"].any():
            self.extras_time_outs.copy_(torch.from_numpy(o["time_out"].astype(bool)))
        if episode_log is not None:
            el = o["episode_log"]
            rs = o["reset"].astype(bool)
            episode_log[~torch.from_numpy(rs), self.cfg.n_terms + 3] = 0.0
            episode_log[torch.from_numpy(rs)] = torch.from_numpy(el[rs])
        if aux is not None:
            aux.copy_(torch.from_numpy(o["aux"]))
        return o

    def sync_time_outs(self):
        return self.extras_time_outs

    def reset_idx(self, env_ids, uniforms=None, rng_seed=0, rng_step=0):
        mask = torch.zeros(self.n, dtype=torch.uint8)
        mask[torch.as_tensor(env_ids).long().cpu()] = 1
        return self.reset_envs(mask, uniforms, rng_seed, rng_step)

    def reset_envs(self, mask, uniforms=None, rng_seed=0, rng_step=0):
        O.reset_envs(self.cfg, self.state.np, self.ter, mask.numpy().astype(np.uint8), rng_seed=rng_seed,
                     rng_step=rng_step)
        return mask

    def close(self):
        pass
