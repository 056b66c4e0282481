"""PPO rollout half of the path against the reference's own outputs
(tests/golden/ppo_rollout.npz from tests/golden/make_golden_ppo.py).

CPU tests drive the host logic with the torch restatement of the rollout kernels
(tests/rollout_ref.py); the HIP kernels are checked in the gpu-marked tests:
returns / raw advantages / bootstrapped rewards bit-exact (same f32 op order),
normalised advantages within 2e-6 (f64 statistics vs torch's f32 reductions).
"""
import os

import numpy as np
import pytest
import torch

from legged_tracking_amd import rollout as R
from tests import golden_io as G
from tests.rollout_ref import TorchRolloutKernels


def _fixture():
    return G.load("ppo_rollout.npz")


def _ac(d, device="cpu"):
    ac = R.ActorCritic(261, 2, 261, 12)
    sd = {k[3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("sd/")}
    ac.load_state_dict(sd)  # the reference's parameter names load unchanged
    return ac.to(device)


def test_actor_critic_matches_reference():
    d = _fixture()
    ac = _ac(d)
    hist, priv, acts = (torch.from_numpy(d[k]) for k in ("in/hist", "in/priv", "in/actions"))
    with torch.no_grad():
        ac.update_distribution(hist)
        np.testing.assert_allclose(ac.adaptation_module(hist).numpy(), d["ac/latent"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(ac.action_mean.numpy(), d["ac/mean"], rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(ac.action_std.numpy(), d["ac/std"])
        np.testing.assert_allclose(ac.get_actions_log_prob(acts).numpy(), d["ac/log_prob"], rtol=1e-6, atol=1e-5)
        np.testing.assert_allclose(ac.entropy.numpy(), d["ac/entropy"], rtol=1e-6)
        np.testing.assert_allclose(ac.evaluate(hist, priv).numpy(), d["ac/value"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(ac.act_teacher(hist, priv).numpy(), d["ac/teacher_mean"], rtol=1e-6, atol=1e-6)


def _storage_from_fixture(d, kernels, device="cpu"):
    T, n = d["gae/rewards_in"].shape
    st = R.RolloutStorage(n, T, [261], [2], [261], [12], device, kernels=kernels)
    tr = R.RolloutStorage.Transition()
    for t in range(T):
        tr.observations = torch.zeros(n, 261, device=device)
        tr.privileged_observations = torch.zeros(n, 2, device=device)
        tr.observation_histories = torch.zeros(n, 261, device=device)
        tr.actions = torch.zeros(n, 12, device=device)
        tr.action_mean = torch.zeros(n, 12, device=device)
        tr.action_sigma = torch.ones(n, 12, device=device)
        tr.actions_log_prob = torch.zeros(n, device=device)
        tr.values = torch.from_numpy(d["gae/values"][t][:, None]).to(device)
        tr.rewards = torch.from_numpy(d["gae/rewards_in"][t]).to(device)
        tr.dones = torch.from_numpy(d["gae/dones"][t]).to(device)
        tr.time_outs = torch.from_numpy(d["gae/time_outs"][t]).to(device)
        st.add_transitions(tr, gamma=float(d["gae/gamma"]))
    return st


def _check_gae(d, st):
    np.testing.assert_array_equal(st.rewards.cpu().numpy()[..., 0], d["gae/rewards_boot"])
    last_v = torch.from_numpy(d["gae/last_values"][:, None]).to(st.device)
    st.compute_returns(last_v, float(d["gae/gamma"]), float(d["gae/lam"]))
    np.testing.assert_array_equal(st.returns.cpu().numpy()[..., 0], d["gae/returns"])
    np.testing.assert_allclose(st.advantages.cpu().numpy()[..., 0], d["gae/advantages"], rtol=2e-6, atol=2e-6)


def test_gae_restatement_matches_reference():
    d = _fixture()
    _check_gae(d, _storage_from_fixture(d, TorchRolloutKernels()))


@pytest.mark.gpu
def test_hip_rollout_kernels_match_reference():
    d = _fixture()
    st = _storage_from_fixture(d, R.HipRolloutKernels(), device="cuda:0")
    # raw advantages before normalisation are bit-exact too
    k = st.kernels
    last_v = torch.from_numpy(d["gae/last_values"][:, None]).cuda()
    k.gae(st, last_v, float(d["gae/gamma"]), float(d["gae/lam"]))
    np.testing.assert_array_equal(st.advantages.cpu().numpy()[..., 0], d["gae/raw_advantages"])
    _check_gae(d, st)


def _runner(tmp_path, n=16, steps=4, kernels=None):
    from legged_tracking_amd import env as E
    from tests.test_env_host import make_env
    R.RunnerArgs.num_steps_per_env = steps
    R.PPO_Args.num_learning_epochs = 1
    R.PPO_Args.num_mini_batches = 2
    env = E.HistoryWrapper(make_env(n=n))
    return R.Runner(env, device="cpu", kernels=kernels or TorchRolloutKernels(),
                    save_dir=str(tmp_path / "checkpoints"))


def test_runner_learns_and_writes_reference_checkpoints(tmp_path):
    torch.manual_seed(0)
    try:
        runner = _runner(tmp_path)
        before = {k: v.clone() for k, v in runner.alg.actor_critic.state_dict().items()}
        # the rollout steps with the contact-force and aux stores off (it reads neither), restored afterwards
        inner, demand = runner.env.env, []
        step = inner.step
        inner.step = lambda a: (demand.append(inner._demand), step(a))[1]
        runner.learn(2, init_at_random_ep_len=True)
    finally:
        R.RunnerArgs.num_steps_per_env, R.PPO_Args.num_learning_epochs, R.PPO_Args.num_mini_batches = 24, 5, 4
    assert len(demand) > 0
    assert set(demand) == {(False, False)} and inner._demand == (True, True)
    after = runner.alg.actor_critic.state_dict()
    assert any(not torch.equal(before[k], after[k]) for k in before)
    ck = tmp_path / "checkpoints"
    sd = torch.load(ck / "ac_weights.pt", weights_only=True)
    assert set(sd) == set(after)
    body = torch.jit.load(str(ck / "body_latest.jit"))
    adapt = torch.jit.load(str(ck / "adaptation_module_latest.jit"))
    x = torch.randn(3, 261)
    with torch.no_grad():
        lat = adapt(x)
        np.testing.assert_allclose(body(torch.cat([x, lat], 1)).numpy(),
                                   runner.alg.actor_critic.act_student(x).numpy(), rtol=1e-5, atol=1e-6)


def _ddp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = _fixture()
        T, n = d["gae/rewards_in"].shape
        half = n // world
        # global advantage normalisation: each rank holds half of the envs
        sl = slice(rank * half, (rank + 1) * half)
        st = R.RolloutStorage(half, T, [261], [2], [261], [12], "cpu", kernels=TorchRolloutKernels())
        st.rewards[..., 0] = torch.from_numpy(d["gae/rewards_boot"][:, sl])
        st.dones[..., 0] = torch.from_numpy(d["gae/dones"][:, sl].astype(np.uint8))
        st.values[..., 0] = torch.from_numpy(d["gae/values"][:, sl])
        st.compute_returns(torch.from_numpy(d["gae/last_values"][sl, None]), float(d["gae/gamma"]),
                           float(d["gae/lam"]))
        ok_adv = np.allclose(st.advantages.numpy()[..., 0], d["gae/advantages"][:, sl], rtol=2e-6, atol=2e-6)
        # gradient all-reduce: ranks with different data end with identical weights
        torch.manual_seed(123)  # same init on both ranks is not required: PPO broadcasts rank 0's
        if rank == 1:
            torch.manual_seed(999)
        ac = R.ActorCritic(261, 2, 261, 12)
        alg = R.PPO(ac, "cpu", kernels=TorchRolloutKernels())
        alg.storage = st
        g = np.random.default_rng(rank)
        for name in ("observations", "privileged_observations", "observation_histories", "actions", "mu"):
            getattr(st, name).copy_(torch.from_numpy(g.normal(0, 1, getattr(st, name).shape).astype(np.float32)))
        st.sigma.fill_(1.0)
        st.actions_log_prob.copy_(torch.from_numpy(g.normal(-15, 1, st.actions_log_prob.shape).astype(np.float32)))
        R.PPO_Args.num_learning_epochs, R.PPO_Args.num_mini_batches = 1, 2
        alg.update()
        flat = torch.cat([p.detach().reshape(-1) for p in ac.parameters()])
        other = flat.clone()
        dist.broadcast(other, 0)
        lr = torch.tensor([alg.learning_rate])
        lr0 = lr.clone()
        dist.broadcast(lr0, 0)
        q.put((rank, bool(ok_adv), bool(torch.equal(flat, other)), bool(torch.equal(lr, lr0))))
    finally:
        dist.destroy_process_group()


def test_ddp_normalisation_and_gradients_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs)
    res = sorted(q.get(timeout=5) for _ in range(2))
    for rank, ok_adv, same_w, same_lr in res:
        assert ok_adv and same_w and same_lr, res


@pytest.mark.gpu
def test_fused_policy_kernel_matches_reference_actor_critic():
    """One MFMA kernel for adaptation module + actor + critic (f32; summation order
    differs from hipBLASLt / the reference's CPU GEMMs: rtol 2e-5)."""
    d = _fixture()
    ac = _ac(d, "cuda:0")
    k = R.HipRolloutKernels()
    pol = k.policy(ac)
    assert pol is not None
    hist, priv = (torch.from_numpy(d[x]).cuda() for x in ("in/hist", "in/priv"))
    mean, value, latent = pol.forward(hist, priv)
    torch.cuda.synchronize()
    np.testing.assert_allclose(latent.cpu().numpy(), d["ac/latent"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(mean.cpu().numpy(), d["ac/mean"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(value.cpu().numpy(), d["ac/value"], rtol=2e-5, atol=2e-5)
    # ragged batch (not a multiple of the 16-env tile) and a larger one
    for n in (37, 4096):
        g = torch.Generator(device="cuda").manual_seed(n)
        h = torch.randn(n, 261, device="cuda", generator=g)
        p = torch.randn(n, 2, device="cuda", generator=g)
        m2, v2, l2 = pol.forward(h, p)
        with torch.no_grad():
            lt = ac.adaptation_module(h)
            mt = ac.actor_body(torch.cat((h, lt), -1))
            vt = ac.critic_body(torch.cat((h, p), -1))
        torch.cuda.synchronize()
        np.testing.assert_allclose(l2.cpu().numpy(), lt.cpu().numpy(), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(m2.cpu().numpy(), mt.cpu().numpy(), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(v2.cpu().numpy(), vt.cpu().numpy(), rtol=1e-4, atol=1e-4)


def _trained():
    """The reference's trained checkpoint (6 privileged obs), tests/golden/make_trained_policy.py."""
    d = G.load("trained_policy.npz")
    npriv = d["in/priv"].shape[1]
    ac = R.ActorCritic(261, npriv, 261, 12)
    ac.load_state_dict({k[3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("sd/")})
    return d, ac


def test_trained_checkpoint_fixture_matches_the_torch_restatement():
    d, ac = _trained()
    h, p = torch.from_numpy(d["in/hist"]), torch.from_numpy(d["in/priv"])
    with torch.no_grad():  # f32 CPU against the f64 record: tolerance relative to each output's scale
        lat = ac.adaptation_module(h)
        for got, k in ((lat, "latent"), (ac.actor_body(torch.cat((h, lat), -1)), "mean"),
                       (ac.critic_body(torch.cat((h, p), -1)), "value")):
            want = d["out/" + k]
            np.testing.assert_allclose(got.numpy(), want, rtol=1e-5, atol=1e-5 * np.abs(want).max())


@pytest.mark.gpu
def test_fused_policy_kernel_runs_the_reference_trained_checkpoint():
    """The fused 3xF16 kernel on the reference's only trained weights (6-wide latent, 267 actor / critic
    inputs), both kernel variants, against the f64 forward of the checkpoint: the split keeps f32 accuracy
    on trained (not just freshly initialised) weights."""
    d, ac = _trained()
    ac = ac.to("cuda:0")
    pol = R.HipRolloutKernels().policy(ac)
    assert pol is not None
    h, p = (torch.from_numpy(d[x]).cuda() for x in ("in/hist", "in/priv"))
    for variant in (0, 1):
        pol.variant = variant
        mean, value, latent = pol.forward(h, p)
        torch.cuda.synchronize()
        for got, k in ((latent, "latent"), (mean, "mean"), (value, "value")):
            want = d["out/" + k]  # f64 record; f32 accuracy relative to the output's scale
            np.testing.assert_allclose(got.cpu().numpy(), want, rtol=2e-5, atol=2e-5 * np.abs(want).max())
    assert int(pol.overflow.item()) == 0


def _split_values_max(ac, h, p):
    """The largest |value| the fused kernel splits into f16 (hi, lo): inputs, the latent and every hidden
    layer's output (the output layers' values are written unsplit)."""
    vals = [h.abs().max(), p.abs().max()]
    with torch.no_grad():
        def run(seq, x):
            for m in list(seq)[:-1]:
                x = m(x)
                if not isinstance(m, torch.nn.Linear):
                    vals.append(x.abs().max())
            return seq[-1](x)
        lat = run(ac.adaptation_module, h)
        vals.append(lat.abs().max())
        run(ac.actor_body, torch.cat((h, lat), -1))
        run(ac.critic_body, torch.cat((h, p), -1))
    return max(float(v) for v in vals)


@pytest.mark.gpu
def test_fused_policy_range_guard():
    """Split values near and beyond the f16 range of the 3xF16 split.  The first layers' weights are scaled
    so that the largest value the kernel splits is 5e4 (inside f16's range: the split stays exact to f32,
    no fallback) and 2e5 (beyond it: f16(x) would be inf; the workgroup's guard recomputes its envs in f32
    from the unsplit weights).  Both match torch f32 (sampling included); only the second touches the
    fallback counter."""
    d = _fixture()
    n = 64 + 7
    g = torch.Generator(device="cuda").manual_seed(3)
    h = torch.rand(n, 261, device="cuda", generator=g) + 0.5
    p = torch.rand(n, 2, device="cuda", generator=g)
    for target, expect_fallback in ((5.0e4, False), (2.0e5, True)):
        base = _ac(d, "cuda:0")
        with torch.no_grad():
            for body in (base.actor_body, base.critic_body, base.adaptation_module):
                body[0].weight.copy_(body[0].weight.abs())
                body[0].bias.zero_()
        lo, hi = 1.0, 1.0e4
        for _ in range(60):  # bisect the layer-1 scale for the target maximum (monotone in the scale)
            mid = (lo * hi) ** 0.5
            ac = _ac(d, "cuda:0")
            ac.load_state_dict(base.state_dict())
            with torch.no_grad():
                for body in (ac.actor_body, ac.critic_body, ac.adaptation_module):
                    body[0].weight.mul_(mid)
            lo, hi = (mid, hi) if _split_values_max(ac, h, p) < target else (lo, mid)
        mx = _split_values_max(ac, h, p)
        assert 0.95 * target < mx < 1.05 * target, mx
        with torch.no_grad():
            lt = ac.adaptation_module(h)
            mt = ac.actor_body(torch.cat((h, lt), -1))
            vt = ac.critic_body(torch.cat((h, p), -1))
        pol = R.HipRolloutKernels().policy(ac)
        for variant in (0, 1):
            pol.variant = variant
            pol.overflow.zero_()
            mean, value, latent, actions, sigma, logp = pol.forward(h, p, sample=(5, 1, 0))
            torch.cuda.synchronize()
            for got, want in ((latent, lt), (mean, mt), (value, vt)):
                scale = want.abs().max().item()
                np.testing.assert_allclose(got.cpu().numpy(), want.cpu().numpy(), rtol=1e-4, atol=1e-5 * scale)
            assert torch.isfinite(actions).all() and torch.isfinite(logp).all()
            assert (int(pol.overflow.item()) > 0) == expect_fallback, (target, variant, int(pol.overflow.item()))


@pytest.mark.gpu
def test_split_policy_kernel_is_bit_identical_to_single_workgroup_kernel():
    """policy_kernel_split (a workgroup per net for 32 envs, weight fragments shared by two env
    tiles; the default) against policy_kernel (16 envs, all three nets per workgroup): same K
    order, tile split and partial-sum order, so every output is bit-identical, sampling included,
    on a ragged batch (the last split workgroup holds 16 + 9 envs)."""
    d = _fixture()
    ac = _ac(d, "cuda:0")
    k = R.HipRolloutKernels()
    pol = k.policy(ac)
    n = 4096 + 25
    g = torch.Generator(device="cuda").manual_seed(11)
    h = torch.randn(n, 261, device="cuda", generator=g)
    p = torch.randn(n, 2, device="cuda", generator=g)
    outs = []
    for variant in (0, 1):  # per call (go1_policy_args.variant)
        pol.variant = variant
        outs.append([t.cpu().numpy() for t in pol.forward(h, p, sample=(123, 7, 0))])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_fused_policy_sampling_is_normal_with_matching_log_prob():
    d = _fixture()
    ac = _ac(d, "cuda:0")
    pol = R.HipRolloutKernels().policy(ac)
    n = 8192
    g = torch.Generator(device="cuda").manual_seed(1)
    h = torch.randn(n, 261, device="cuda", generator=g)
    p = torch.randn(n, 2, device="cuda", generator=g)
    mean, value, latent, act, sigma, logp = pol.forward(h, p, sample=(123, 7, 0))
    torch.cuda.synchronize()
    z = ((act - mean) / sigma).cpu().numpy()
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    np.testing.assert_array_equal(sigma.cpu().numpy(), np.broadcast_to(d["ac/std"][0], sigma.shape))
    ref = torch.distributions.Normal(mean, sigma).log_prob(act).sum(-1)
    np.testing.assert_allclose(logp.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5, atol=1e-4)
    # same counter -> same draws; next counter -> different draws
    act2 = pol.forward(h, p, sample=(123, 7, 0))[3]
    act3 = pol.forward(h, p, sample=(123, 8, 0))[3]
    assert torch.equal(act, act2) and not torch.equal(act, act3)


def _ppo_update_from_fixture(d, device, kernels):
    """One rollout.PPO.update on the storage the reference's PPO.update saw (ppo.py:98-206), with
    the reference's minibatch permutation."""
    ac = R.ActorCritic(261, 2, 261, 12)
    ac.load_state_dict({k[len("upd/sd_before/"):]: torch.from_numpy(d[k]) for k in d.files
                        if k.startswith("upd/sd_before/")})
    for k in ("num_learning_epochs", "num_mini_batches", "clip_param", "learning_rate", "max_grad_norm",
              "value_loss_coef", "entropy_coef", "desired_kl", "num_adaptation_module_substeps"):
        assert float(getattr(R.PPO_Args, k)) == float(d["upd/args/" + k]), k
    alg = R.PPO(ac, device=device, kernels=kernels)
    T, n = d["gae/rewards_in"].shape
    alg.init_storage(n, T, [261], [2], [261], [12])
    st = alg.storage
    for k in ("observations", "privileged_observations", "observation_histories", "actions", "values", "returns",
              "actions_log_prob", "advantages", "mu", "sigma", "rewards"):
        getattr(st, k).copy_(torch.from_numpy(d["upd/storage/" + k]))
    st.step = T
    perm = torch.from_numpy(d["upd/perm"])
    real = torch.randperm
    torch.randperm = lambda *a, **k: perm.to(k.get("device") or "cpu")
    try:
        losses = alg.update()
    finally:
        torch.randperm = real
    return alg, losses


def _check_update(d, alg, losses, rtol_loss, atol_w, atol_max=None):
    """Losses, the adaptive learning rate and every updated weight.  `atol_w` bounds 99.99 % of the
    weights; `atol_max` (default atol_w) every weight."""
    want = d["upd/losses"]
    np.testing.assert_allclose(np.array(losses, np.float64), want, rtol=rtol_loss, atol=1e-7)
    assert alg.learning_rate == float(d["upd/lr_after"])  # adaptive-KL schedule: same decisions
    sd = alg.actor_critic.state_dict()
    diffs = []
    for k in d.files:
        if k.startswith("upd/sd_after/"):
            got = sd[k[len("upd/sd_after/"):]].detach().cpu().numpy()
            before = d["upd/sd_before/" + k[len("upd/sd_after/"):]]
            diff = np.abs(got - d[k]).ravel()
            assert diff.max() <= (atol_max or atol_w), (k, diff.max())
            diffs.append(diff)
            assert not np.array_equal(d[k], before) or k.endswith("std")  # the update moved the weights
    diffs = np.concatenate(diffs)
    assert np.percentile(diffs, 99.99) <= atol_w, np.percentile(diffs, 99.99)
    return float(diffs.max())


def test_ppo_update_matches_reference_on_cpu():
    """CPU: the same torch ops in the same order as ppo.py -> losses within 1e-5, weights within 1e-6
    after 20 Adam steps (5 epochs x 4 minibatches) with the adaptive-KL learning rate."""
    d = _fixture()
    alg, losses = _ppo_update_from_fixture(d, "cpu", TorchRolloutKernels())
    _check_update(d, alg, losses, rtol_loss=1e-5, atol_w=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["1", "0"])
def test_ppo_update_matches_reference_on_gpu(engine, monkeypatch):
    """MI355X: the update's GEMMs run on hipBLASLt with another reduction order than the CPU's.  Adam
    normalises each gradient component, so a component whose gradient is near zero can step by up
    to the learning rate in either direction on either side: the weights may differ by at most the
    schedule's total step, sum_t lr_t < 1e-3 / (1 - 1 / 1.5) = 3e-3 (the adaptive KL rule divides lr
    by 1.5 per minibatch here); 99.99 % of the 700k weights agree within 1e-4, the losses within
    1e-3 relative, and the KL schedule takes the same decisions."""
    monkeypatch.setenv("GO1_PPO_ENGINE", engine)  # 1: the HIP update engine (default), 0: torch autograd
    d = _fixture()
    alg, losses = _ppo_update_from_fixture(d, "cuda:0", R.HipRolloutKernels())
    assert (getattr(alg, "_engine", None) is not None) == (engine == "1")
    w = _check_update(d, alg, losses, rtol_loss=1e-3, atol_w=1e-4, atol_max=3e-3)
    print(f"\nPPO.update on the GPU ({'engine' if engine == '1' else 'torch'}) vs the reference (CPU): max |dw| {w:.2e}")


@pytest.mark.gpu
def test_runner_learn_on_gpu_through_hip_env_and_rollout_kernels(tmp_path):
    """Runner.learn(2) end to end on the MI355X: HIP env step, fused policy / record / GAE kernels,
    PPO.update on the GPU, checkpoints in the reference's three formats."""
    from legged_tracking_amd import config as CF, env as E
    n = 256
    R.RunnerArgs.num_steps_per_env = 8
    R.PPO_Args.num_learning_epochs, R.PPO_Args.num_mini_batches = 2, 2
    try:
        cfg = CF.readme_config(n_envs=n, terrain="single_path", rows=4, cols=4)
        env = E.HistoryWrapper(E.TrajectoryTrackingEnv(sim_device="cuda:0", cfg=cfg, seed=4, rank=0, world_size=1))
        assert env.env._sim.__class__.__name__ == "Go1Native"
        runner = R.Runner(env, device="cuda:0", save_dir=str(tmp_path / "checkpoints"))
        assert runner.alg.fused is not None  # the fused MFMA policy kernel drives the rollout
        before = {k: v.clone() for k, v in runner.alg.actor_critic.state_dict().items()}
        runner.learn(2, init_at_random_ep_len=True)
        torch.cuda.synchronize()
    finally:
        R.RunnerArgs.num_steps_per_env, R.PPO_Args.num_learning_epochs, R.PPO_Args.num_mini_batches = 24, 5, 4
    after = runner.alg.actor_critic.state_dict()
    assert any(not torch.equal(before[k], after[k]) for k in before)
    assert all(torch.isfinite(v).all() for v in after.values())
    sd = torch.load(tmp_path / "checkpoints" / "ac_weights.pt", weights_only=True, map_location="cpu")
    assert set(sd) == set(after)
    assert env.extras["diverged"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("hist,npriv", [(2100, 2), (1020, 6), (70, 2)])
def test_fused_policy_kernel_streams_long_histories(hist, npriv):
    """The default launch streams the first layers' inputs in chunks of 288 (the velocity task's 30-deep
    history: 2,100 inputs, BASELINE configs[1]; a 1,020-wide history whose 6-wide latent straddles two
    32-input groups; a short one): against an f64 forward of the same weights, a ragged batch, and the
    single-workgroup variant refusing what it cannot stage."""
    torch.manual_seed(3)
    ac = R.ActorCritic(70, npriv, hist, 12).to("cuda:0")
    pol = R.HipRolloutKernels().policy(ac)
    assert pol is not None
    n = 1000 + 25
    g = torch.Generator(device="cuda").manual_seed(5)
    h = torch.randn(n, hist, device="cuda", generator=g)
    p = torch.randn(n, npriv, device="cuda", generator=g)
    mean, value, latent = pol.forward(h, p)
    torch.cuda.synchronize()
    ac64 = R.ActorCritic(70, npriv, hist, 12).double()
    ac64.load_state_dict({k: v.double().cpu() for k, v in ac.state_dict().items()})
    with torch.no_grad():
        h64, p64 = h.double().cpu(), p.double().cpu()
        lt = ac64.adaptation_module(h64)
        mt = ac64.actor_body(torch.cat((h64, lt), -1))
        vt = ac64.critic_body(torch.cat((h64, p64), -1))
    for got, want in ((latent, lt), (mean, mt), (value, vt)):
        want = want.numpy()
        np.testing.assert_allclose(got.cpu().numpy(), want, rtol=2e-5, atol=2e-5 * np.abs(want).max())
    assert int(pol.overflow.item()) == 0
    if hist + npriv > 288:
        pol.variant = 1
        with pytest.raises(RuntimeError, match="variant 1"):
            pol.forward(h, p)


@pytest.mark.gpu
def test_ppo_update_graph_replays_the_eager_update(monkeypatch):
    """The HIP-graph mini-batch step (PPO._graphed_minibatches: 3 eager warm-up mini-batches, one capture,
    replays) computes the eager update: two consecutive updates from the reference fixture's storage, with
    the graph captured in the first and replayed through the second, against GO1_PPO_GRAPH=0."""
    import warnings
    monkeypatch.setenv("GO1_PPO_ENGINE", "0")  # the torch autograd update's graph (the engine: test_ppo_engine.py)
    d = _fixture()
    runs = {}
    clip0 = R.PPO_Args.clip_param
    for flag in ("0", "1"):
        monkeypatch.setenv("GO1_PPO_GRAPH", flag)
        with warnings.catch_warnings(record=True) as wrec:
            warnings.simplefilter("always")
            alg, losses = _ppo_update_from_fixture(d, "cuda:0", R.HipRolloutKernels())
            assert (alg._graph is not None) == (flag == "1")
            st = alg.storage
            out = [losses]
            for upd in range(2):
                for k in ("observations", "privileged_observations", "observation_histories", "actions", "values",
                          "returns", "actions_log_prob", "advantages", "mu", "sigma", "rewards"):
                    getattr(st, k).copy_(torch.from_numpy(d["upd/storage/" + k]))
                st.step = st.num_transitions_per_env
                torch.manual_seed(5 + upd)
                g_before = alg._graph
                if upd == 1:  # a PPO_Args change between updates: the captured step must not replay stale values
                    R.PPO_Args.clip_param = 0.15
                try:
                    out.append(alg.update())
                finally:
                    R.PPO_Args.clip_param = clip0
                if flag == "1":
                    assert (alg._graph is g_before) == (upd == 0), "replayed across updates, recaptured on a change"
        assert not [w for w in wrec if "AccumulateGrad" in str(w.message)], [str(w.message) for w in wrec]
        runs[flag] = (out, alg.learning_rate,
                      {k: v.detach().cpu().numpy() for k, v in alg.actor_critic.state_dict().items()})
    e, g = runs["0"], runs["1"]
    np.testing.assert_allclose(np.array(sum(g[0], ())), np.array(sum(e[0], ())), rtol=1e-5, atol=1e-7)
    assert g[1] == e[1]
    dmax = max(float(np.abs(g[2][k] - e[2][k]).max()) for k in e[2])
    print(f"\ngraph vs eager after three updates (PPO_Args changed before the third): max |dw| {dmax:.2e}")
    assert dmax <= 1e-5, dmax


@pytest.mark.gpu
def test_colsum_kernel_matches_f64_sums_and_is_deterministic():
    """go1_colsum (the bias gradients of PPO.update's backward) against f64 column sums, ragged shapes included;
    two calls agree bit for bit (fixed partition and order)."""
    g = torch.Generator(device="cuda").manual_seed(3)
    for rows, cols in ((24576, 512), (24576, 12), (24577, 1), (1000, 70), (64, 3), (4096, 2100)):
        x = torch.randn(rows, cols, device="cuda", generator=g)
        got = R._colsum(x)
        ref = x.double().sum(0)
        scale = x.double().abs().sum(0)
        assert ((got.double() - ref).abs() <= 1e-6 * scale + 1e-6).all(), (rows, cols)
        assert torch.equal(got, R._colsum(x))


@pytest.mark.gpu
def test_policy_and_record_read_row_strided_history_windows():
    """The velocity env returns obs_history as a window of wider rows (row stride > width, velocity.py
    attach_history): the fused policy kernel (both launches) and the record kernel read it in place and
    give exactly what they give for the same history made contiguous."""
    torch.manual_seed(4)
    n, hist, npriv, wide = 777, 2100, 2, 2100 + 70 * 5
    ac = R.ActorCritic(70, npriv, hist, 12).to("cuda:0")
    kern = R.HipRolloutKernels()
    pol = kern.policy(ac)
    g = torch.Generator(device="cuda").manual_seed(9)
    buf = torch.randn(n, wide, device="cuda", generator=g)
    for off in (0, 70, 350):  # 16-byte aligned and 8-byte aligned window starts
        win = buf[:, off:off + hist]
        assert not win.is_contiguous() and win.stride() == (wide, 1)
        p = torch.randn(n, npriv, device="cuda", generator=g)
        got = pol.forward(win, p)
        want = pol.forward(win.contiguous(), p)
        for a, b in zip(got, want):
            assert torch.equal(a, b)
    # the single-workgroup variant (one 288-input chunk: the strided-block staging path); it walks exactly
    # nine packed K groups, so a narrower history is refused at the boundary before any launch
    narrow = kern.policy(R.ActorCritic(70, npriv, 210, 12).to("cuda:0"))
    narrow.variant = 1
    with pytest.raises(RuntimeError, match="variant 1"):
        narrow.forward(buf[:, 70:280], torch.randn(n, npriv, device="cuda", generator=g))
    ac2 = R.ActorCritic(70, npriv, 265, 12).to("cuda:0")
    pol2 = kern.policy(ac2)
    pol2.variant = 1
    win2 = buf[:, 70:335]
    p = torch.randn(n, npriv, device="cuda", generator=g)
    for a, b in zip(pol2.forward(win2, p), pol2.forward(win2.contiguous(), p)):
        assert torch.equal(a, b)
    pol2.variant = 0
    for a, b in zip(pol2.forward(win2, p), pol2.forward(win2.contiguous(), p)):
        assert torch.equal(a, b)
    # record: the storage row equals the window
    st = R.RolloutStorage(n, 2, [70], [npriv], [hist], [12], device="cuda:0", kernels=kern)
    for step, off in enumerate((70, 140)):
        t = R.RolloutStorage.Transition()
        t.observations = torch.randn(n, 70, device="cuda", generator=g)
        t.privileged_observations = torch.randn(n, npriv, device="cuda", generator=g)
        t.observation_histories = buf[:, off:off + hist]
        t.actions = t.action_mean = t.action_sigma = torch.randn(n, 12, device="cuda", generator=g)
        t.actions_log_prob = t.values = t.rewards = torch.randn(n, device="cuda", generator=g)
        t.dones = torch.zeros(n, dtype=torch.bool, device="cuda")
        st.add_transitions(t, 0.99)
        torch.cuda.synchronize()
        assert torch.equal(st.observation_histories[step], buf[:, off:off + hist])


@pytest.mark.gpu
@pytest.mark.parametrize("n,alias", [(4096, False), (4096, True), (777, False), (16, True)])
def test_record_flat_kernel_equals_segment_kernel(n, alias, monkeypatch):
    """process_env_step's record (rollout_storage.py:76-90 add_transitions + the time-out bootstrap ppo.py:85-87):
    the flat kernel (one 16-byte chunk per thread, a segment per workgroup; the default when every buffer is
    16-byte aligned) writes exactly what the segment-walking kernel (GO1_RECORD_FLAT=0) writes -- with obs and
    obs_history one tensor (the README configuration: history depth 1) or two, ragged sizes, time-outs."""
    kern = R.HipRolloutKernels()
    nh = 261
    g = torch.Generator(device="cuda").manual_seed(n + alias)
    outs = {}
    data = []
    for step in range(3):
        t = R.RolloutStorage.Transition()
        t.observations = torch.randn(n, nh, device="cuda", generator=g)
        t.observation_histories = t.observations if alias else torch.randn(n, nh, device="cuda", generator=g)
        t.privileged_observations = torch.randn(n, 2, device="cuda", generator=g)
        t.actions = torch.randn(n, 12, device="cuda", generator=g)
        t.action_mean = torch.randn(n, 12, device="cuda", generator=g)
        t.action_sigma = torch.rand(n, 12, device="cuda", generator=g)
        t.actions_log_prob = torch.randn(n, device="cuda", generator=g)
        t.values = torch.randn(n, 1, device="cuda", generator=g)
        t.rewards = torch.randn(n, device="cuda", generator=g)
        t.dones = torch.rand(n, device="cuda", generator=g) < 0.1
        t.time_outs = torch.rand(n, device="cuda", generator=g) < 0.5
        data.append(t)
    for flat in ("1", "0"):
        monkeypatch.setenv("GO1_RECORD_FLAT", flat)
        st = R.RolloutStorage(n, 3, [nh], [2], [nh], [12], device="cuda:0", kernels=kern)
        for t in data:
            st.add_transitions(t, 0.99)
        torch.cuda.synchronize()
        outs[flat] = {k: getattr(st, k).clone() for k in ("observations", "privileged_observations",
                                                          "observation_histories", "actions", "mu", "sigma",
                                                          "actions_log_prob", "values", "rewards", "dones")}
    for k, v in outs["0"].items():
        assert torch.equal(outs["1"][k], v), k
    assert torch.equal(outs["1"]["observations"][1], data[1].observations)
