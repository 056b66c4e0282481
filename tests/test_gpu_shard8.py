"""BASELINE configs[3] on one GPU: 32,768 Go1 (4096 x 8) on the 32 x 32 single_path grid, env-sharded over
eight ranks.  The multi-GPU path has no collective in the env step and the fused policy's sampling is keyed by the
global env id, so what rank r of an 8-GPU run computes is fully determined by its shard: here eight handles of
4096 envs with env_id_offset = r * 4096 run side by side on one MI355X next to one 32,768-env handle, and every
step's sampled actions (fused policy kernel, Philox keyed by the global env), observations, rewards, resets and
the final state must be bit-identical.  The only cross-rank coupling of the rollout, the global advantage
normalisation (rollout_storage.py:88-90: the (sum, sum of squares) statistics all-reduced over ranks), is
checked by summing the eight shards' statistics as the RCCL all-reduce does.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from legged_tracking_amd import config as CF, native, rollout as R, terrain as T  # noqa: E402

DEV = "cuda:0"
RANKS = 8
NR = 4096
N = RANKS * NR


def _handle(cfg, td, dr, ep, lo, hi):
    c = CF.build_abi_config(cfg, n_envs=hi - lo)
    c.env_id_offset = lo
    g = native.Go1Native(c, DEV)
    sl = slice(lo, hi)
    g.set_terrain(td.tiles, td.env_tile[sl], td.env_terrain_origin[sl], td.env_origins[sl])
    for k, v in dr.items():
        g.state[k].copy_(torch.from_numpy(v[sl].astype(np.float32)))
    keep = g.reset_envs(torch.ones(hi - lo, dtype=torch.bool, device=DEV), rng_seed=21, rng_step=0)
    g.state["episode_length"].copy_(torch.from_numpy(ep[sl]))
    return g, keep


def test_configs3_eight_shards_bit_identical_to_one_32768_env_handle():
    cfg = CF.readme_config(n_envs=N, terrain="single_path", rows=32, cols=32)
    td = T.build(cfg, N, np.random.RandomState(17))
    rng = np.random.default_rng(23)
    dr = {"friction": rng.uniform(0.1, 3.0, (N, 1)), "restitution": rng.uniform(0.0, 0.4, (N, 1)),
          "payload": rng.uniform(-1.0, 3.0, (N, 1))}
    ep = rng.integers(0, 500, (N, 1)).astype(np.int32)
    whole, kw = _handle(cfg, td, dr, ep, 0, N)
    shards, ks = zip(*[_handle(cfg, td, dr, ep, r * NR, (r + 1) * NR) for r in range(RANKS)])
    torch.manual_seed(29)
    ac = R.ActorCritic(261, 2, 261, 12).to(DEV)
    pol = R.HipRolloutKernels().policy(ac)
    assert pol is not None
    scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
    grav, gvec = CF.gravity_state([0.2, -0.1, 0.05])
    torch.cuda.synchronize()
    del kw, ks
    T_STEPS = 12
    kern = R.HipRolloutKernels()
    st_whole = R.RolloutStorage(N, T_STEPS, [261], [2], [261], [12], device=DEV, kernels=kern)
    st_shard = [R.RolloutStorage(NR, T_STEPS, [261], [2], [261], [12], device=DEV, kernels=kern)
                for _ in range(RANKS)]
    n_reset = 0
    for t in range(T_STEPS):
        # PPO.act through the fused policy kernel: rank r samples with env_id_offset r * 4096
        ow = pol.forward(whole.obs, whole.priv, sample=(0x5EED, t + 1, 0))
        os_ = [pol.forward(g.obs, g.priv, sample=(0x5EED, t + 1, r * NR)) for r, g in enumerate(shards)]
        for i, name in enumerate(("mean", "value", "latent", "actions", "sigma", "log_prob")):
            got = torch.cat([o[i] for o in os_])
            assert torch.equal(ow[i], got), f"step {t}: policy {name}"
        whole.step(ow[3], gvec, grav, scales, rng_seed=5, rng_step=t)
        for r, g in enumerate(shards):
            g.step(os_[r][3], gvec, grav, scales, rng_seed=5, rng_step=t)
        # record the transitions as the Runner does (rewards bootstrapped with the time-outs)
        for st, o, g in [(st_whole, ow, whole)] + [(st_shard[r], os_[r], shards[r]) for r in range(RANKS)]:
            tr = R.RolloutStorage.Transition()
            tr.observations = tr.observation_histories = g.obs
            tr.privileged_observations = g.priv
            tr.action_mean, tr.values, tr.actions, tr.action_sigma, tr.actions_log_prob = o[0], o[1], o[3], o[4], o[5]
            tr.rewards, tr.dones, tr.time_outs = g.rew, g.reset, g.time_out
            st.add_transitions(tr, 0.99)
        torch.cuda.synchronize()
        for name in ("obs", "priv", "rew", "reset", "time_out", "contact_forces"):
            got = torch.cat([getattr(g, name) for g in shards])
            assert torch.equal(getattr(whole, name), got), f"step {t}: {name}"
        n_reset += int(whole.reset.sum())
    assert n_reset > 0
    sw = whole.state.numpy()
    ss = [g.state.numpy() for g in shards]
    for k in sw:
        np.testing.assert_array_equal(sw[k], np.concatenate([s[k] for s in ss]), err_msg=k)
    for name in ("observations", "actions", "rewards", "dones", "values", "actions_log_prob"):
        got = torch.cat([getattr(s, name) for s in st_shard], dim=1)
        assert torch.equal(getattr(st_whole, name), got), name
    # GAE per shard, then the global normalisation with the all-reduced statistics (what RolloutStorage.
    # compute_returns does at world size 8) against the single storage
    last = pol.forward(whole.obs, whole.priv)[1]
    kern.gae(st_whole, last, 0.99, 0.95)
    kern.normalize(st_whole, float(st_whole.advantages.numel()))
    stats = torch.zeros(2, dtype=torch.float64, device=DEV)
    for r, s in enumerate(st_shard):
        kern.gae(s, last[r * NR:(r + 1) * NR], 0.99, 0.95)
        stats += s.adv_stats
    for s in st_shard:
        raw_returns = s.returns.clone()
        s.adv_stats.copy_(stats)
        kern.normalize(s, float(s.advantages.numel() * RANKS))
        assert torch.equal(s.returns, raw_returns)
    torch.cuda.synchronize()
    assert torch.equal(st_whole.returns, torch.cat([s.returns for s in st_shard], dim=1))
    got = torch.cat([s.advantages for s in st_shard], dim=1)
    # the f64 statistics are summed in another order (8 partial sums): the normalised advantages agree to
    # the f32 rounding of mean and std
    torch.testing.assert_close(got, st_whole.advantages, rtol=1e-6, atol=1e-6)
