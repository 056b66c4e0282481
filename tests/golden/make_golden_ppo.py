"""Golden fixtures for the PPO rollout half of the path, from the REFERENCE's own code.

Container-only test infrastructure (see make_golden.py for the stub setup): imports
go1_gym_learn.ppo_cse (ActorCritic, RolloutStorage, PPO) from /root/reference and
records, on seeded synthetic inputs:
  * ActorCritic (actor_critic.py:21-156): state dict, adaptation latent, action mean,
    value, log-prob and entropy for given actions;
  * PPO.process_env_step time-out bootstrap (ppo.py:79-92);
  * RolloutStorage.compute_returns GAE + normalisation (rollout_storage.py:76-90);
  * one PPO.update (ppo.py:98-206): minibatch permutation, losses, adaptive learning rate,
    updated weights.
Writes tests/golden/ppo_rollout.npz.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "refstubs"))
sys.path.insert(1, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from go1_gym_learn.ppo_cse.actor_critic import ActorCritic
    from go1_gym_learn.ppo_cse.rollout_storage import RolloutStorage
    from go1_gym_learn.ppo_cse.ppo import PPO, PPO_Args

    torch.manual_seed(3)
    n, T, n_obs, n_priv, n_act = 64, 24, 261, 2, 12
    ac = ActorCritic(n_obs, n_priv, n_obs, n_act)
    with torch.no_grad():
        ac.std.mul_(0.7)  # a non-trivial std
    g = np.random.default_rng(5)
    hist = torch.from_numpy(g.normal(0, 1, (n, n_obs)).astype(np.float32))
    priv = torch.from_numpy(g.normal(0, 1, (n, n_priv)).astype(np.float32))
    acts = torch.from_numpy(g.normal(0, 1, (n, n_act)).astype(np.float32))
    out = {}
    for k, v in ac.state_dict().items():
        out["sd/" + k] = v.numpy().copy()
    with torch.no_grad():
        ac.update_distribution(hist)
        out["ac/latent"] = ac.adaptation_module(hist).numpy()
        out["ac/mean"] = ac.action_mean.numpy()
        out["ac/std"] = ac.action_std.numpy()
        out["ac/log_prob"] = ac.get_actions_log_prob(acts).numpy()
        out["ac/entropy"] = ac.entropy.numpy()
        out["ac/value"] = ac.evaluate(hist, priv).numpy()
        out["ac/teacher_mean"] = ac.act_teacher(hist, priv).numpy()
    out["in/hist"], out["in/priv"], out["in/actions"] = hist.numpy(), priv.numpy(), acts.numpy()

    # process_env_step bootstrap + add_transitions, then compute_returns
    alg = PPO(ac, device="cpu")
    alg.init_storage(n, T, [n_obs], [n_priv], [n_obs], [n_act])
    rewards_in, dones_in, touts_in, values_in = [], [], [], []
    for t in range(T):
        o = torch.from_numpy(g.normal(0, 1, (n, n_obs)).astype(np.float32))
        p = torch.from_numpy(g.normal(0, 1, (n, n_priv)).astype(np.float32))
        with torch.no_grad():
            alg.act(o, p, o)
        # overwrite the values with wide-range synthetic ones so the GAE is exercised
        v = torch.from_numpy(g.normal(0, 3, (n, 1)).astype(np.float32))
        alg.transition.values = v
        r = torch.from_numpy(g.normal(0, 1, n).astype(np.float32))
        d = torch.from_numpy(g.random(n) < 0.1)
        to = torch.from_numpy(g.random(n) < 0.5) & d
        alg.process_env_step(r, d, {"time_outs": to})
        rewards_in.append(r.numpy()); dones_in.append(d.numpy()); touts_in.append(to.numpy()); values_in.append(v.numpy())
    st = alg.storage
    out["gae/rewards_in"] = np.stack(rewards_in)
    out["gae/dones"] = np.stack(dones_in)
    out["gae/time_outs"] = np.stack(touts_in)
    out["gae/values"] = np.stack(values_in)[..., 0]
    out["gae/rewards_boot"] = st.rewards.numpy()[..., 0].copy()
    last_v = torch.from_numpy(g.normal(0, 3, (n, 1)).astype(np.float32))
    st.compute_returns(last_v, PPO_Args.gamma, PPO_Args.lam)
    out["gae/last_values"] = last_v.numpy()[:, 0]
    out["gae/returns"] = st.returns.numpy()[..., 0]
    out["gae/advantages"] = st.advantages.numpy()[..., 0]
    out["gae/raw_advantages"] = (st.returns - st.values).numpy()[..., 0]
    out["gae/gamma"] = np.float64(PPO_Args.gamma)
    out["gae/lam"] = np.float64(PPO_Args.lam)

    # one PPO.update (ppo.py:98-206) on this storage: the minibatch permutation it draws, its
    # returned losses, the adaptive learning rate after the KL steps and the updated weights
    for k in ("observations", "privileged_observations", "observation_histories", "actions", "values", "returns",
              "actions_log_prob", "advantages", "mu", "sigma", "rewards", "dones"):
        out["upd/storage/" + k] = getattr(st, k).numpy().copy()
    for k, v in ac.state_dict().items():
        out["upd/sd_before/" + k] = v.numpy().copy()
    out["upd/lr_before"] = np.float64(alg.learning_rate)
    perms = []
    real_randperm = torch.randperm

    def randperm(*a, **k):
        r = real_randperm(*a, **k)
        perms.append(r.numpy().copy())
        return r

    torch.manual_seed(17)
    torch.randperm = randperm
    try:
        losses = alg.update()
    finally:
        torch.randperm = real_randperm
    assert len(perms) == 1
    out["upd/perm"] = perms[0]
    out["upd/losses"] = np.array(losses, np.float64)
    out["upd/lr_after"] = np.float64(alg.learning_rate)
    for k, v in ac.state_dict().items():
        out["upd/sd_after/" + k] = v.numpy().copy()
    for k in ("num_learning_epochs", "num_mini_batches", "clip_param", "learning_rate", "max_grad_norm",
              "value_loss_coef", "entropy_coef", "desired_kl", "num_adaptation_module_substeps"):
        out["upd/args/" + k] = np.float64(getattr(PPO_Args, k))
    path = os.path.join(HERE, "ppo_rollout.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out))


if __name__ == "__main__":
    main()
