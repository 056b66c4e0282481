"""The hand-written HIP PPO update (csrc/ppo_update.hip, C ABI include/go1_ppo.h, host legged_tracking_amd/ppo_engine.py)
against float64 references and the reference's PPO.update fixture (ppo.py:98-206).

CPU tests: the library loads and exports every go1_ppo.h entry point, the flat parameter layout matches the module,
argument errors are reported.  GPU tests: each GEMM kernel against an f64 product (ragged rows, the first layers'
K = 261 / 263, the velocity task's 2,102, operands down to 1e-7 to exercise the per-tensor scaling), the whole
update against the reference fixture and against the torch autograd update, graph replay = eager, the world-size
split into graph segments = one graph, and determinism.
"""
import ctypes as C
import os
import re
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from legged_tracking_amd import ppo_engine as PE, rollout as R  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "go1_ppo.h")
DEV = "cuda:0"


def test_library_exports_every_go1_ppo_symbol_and_layout_matches_module():
    lib = PE.load_library()
    names = sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(go1_\w+)\s*\(", open(HEADER).read(), re.M)))
    assert len(names) >= 8
    for n in names:
        assert hasattr(lib, n), n
    for hist, priv, na in ((261, 2, 12), (2100, 2, 12), (1020, 6, 12), (70, 8, 16)):
        ac = R.ActorCritic(70, priv, hist, na)
        assert PE.supported(ac)
        d = PE._Dims(hist=hist, priv=priv, actions=na, mb=384, rows=1536)
        tot, ad = C.c_int64(), C.c_int64()
        assert lib.go1_ppo_param_count(C.byref(d), C.byref(tot), C.byref(ad)) == 0
        sd = dict(ac.named_parameters())
        assert tot.value == sum(sd[k].numel() for k in PE.PARAM_NAMES) == sum(p.numel() for p in ac.parameters())
        assert ad.value == sum(p.numel() for p in ac.adaptation_module.parameters())
        nb = C.c_int64()
        assert lib.go1_ppo_workspace_bytes(C.byref(d), C.byref(nb)) == 0 and nb.value > 0
    bad = PE._Dims(hist=261, priv=9, actions=12, mb=384, rows=1536)
    assert lib.go1_ppo_param_count(C.byref(bad), None, None) == -1
    assert b"priv 1..8" in lib.go1_ppo_last_error()
    # a module the engine does not implement (another activation) falls back to the torch update
    R.AC_Args.activation = "tanh"
    try:
        assert not PE.supported(R.ActorCritic(70, 2, 261, 12))
    finally:
        R.AC_Args.activation = "elu"


def _work(nbytes):
    w = torch.zeros(nbytes + 512, dtype=torch.uint8, device=DEV)
    base = (w.data_ptr() + 255) // 256 * 256
    return w, base, nbytes


@pytest.mark.gpu
@pytest.mark.parametrize("rows,k,n,elu,scale", [(384, 261, 256, 1, 1.0), (1000, 263, 512, 1, 1e-3),
                                                 (24576, 512, 256, 1, 1.0), (777, 128, 128, 0, 1e-7),
                                                 (4100, 2102, 512, 1, 3.0)])
def test_linear_kernel_against_f64(rows, k, n, elu, scale):
    lib = PE.load_library()
    g = torch.Generator(device=DEV).manual_seed(rows + k)
    x = (torch.randn(rows, k, device=DEV, generator=g) * scale).contiguous()
    x[:, ::7] *= 1e-4  # a wide dynamic range inside one tensor
    w = torch.randn(n, k, device=DEV, generator=g) / k ** 0.5
    b = torch.randn(n, device=DEV, generator=g) * 0.1
    y = torch.empty(rows, n, device=DEV)
    hold, base, nb = _work(1024 + (-(-k // 32)) * 32 * n * 4 + rows * (-(-k // 4)) * 16)
    rc = lib.go1_ppo_test_linear(x.data_ptr(), rows, k, w.data_ptr(), b.data_ptr(), n, elu, y.data_ptr(), base, nb, 1,
                                 C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, lib.go1_ppo_last_error()
    torch.cuda.synchronize()
    z = x.double() @ w.double().t() + b.double()
    ref = torch.where(z > 0, z, torch.expm1(z)) if elu else z
    # error budget of the 3xF16 products (~2^-21 relative per product) on f32 accumulation: 3e-6 of the scale of
    # sum |w x| per output
    mag = x.double().abs() @ w.double().abs().t() + b.double().abs()
    err = (y.double() - ref).abs()
    assert (err <= 3e-6 * mag + 1e-30).all(), float((err / (mag + 1e-30)).max())


@pytest.mark.gpu
@pytest.mark.parametrize("rows,k,n,xs,ds", [(384, 263, 512, 1.0, 1e-6), (24576, 512, 256, 1.0, 1e-5),
                                             (1000, 261, 256, 10.0, 1e-8), (24576, 128, 128, 0.3, 1.0),
                                             (4133, 2102, 512, 1.0, 1e-6)])
def test_wgrad_kernel_against_f64(rows, k, n, xs, ds):
    lib = PE.load_library()
    g = torch.Generator(device=DEV).manual_seed(rows * 3 + k)
    x = torch.randn(rows, k, device=DEV, generator=g) * xs
    d = torch.randn(rows, n, device=DEV, generator=g) * ds
    d[::5] = 0.0  # rows whose gradient is zero (clipped ratios)
    dw = torch.empty(n, k, device=DEV)
    kpad = -(-k // 128) * 128
    hold, base, nb = _work(1024 + 16 * n * kpad * 4 + rows * (-(-k // 4)) * 16)
    rc = lib.go1_ppo_test_wgrad(x.data_ptr(), d.data_ptr(), rows, k, n, dw.data_ptr(), base, nb, 1,
                                C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, lib.go1_ppo_last_error()
    torch.cuda.synchronize()
    ref = d.double().t() @ x.double()
    mag = d.double().abs().t() @ x.double().abs()
    err = (dw.double() - ref).abs()
    assert (err <= 3e-6 * mag + 1e-30).all(), float((err / (mag + 1e-30)).max())


def _fixture():
    return np.load(os.path.join(REPO, "tests", "golden", "ppo_rollout.npz"))


def _storage_update(d, device, env=None, monkeypatch=None, updates=1, seed=5):
    from tests.test_rollout import _ppo_update_from_fixture
    if env:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
    alg, losses = _ppo_update_from_fixture(d, device, R.HipRolloutKernels() if device != "cpu" else None)
    out = [losses]
    st = alg.storage
    for u in range(updates - 1):
        for k in ("observations", "privileged_observations", "observation_histories", "actions", "values",
                  "returns", "actions_log_prob", "advantages", "mu", "sigma", "rewards"):
            getattr(st, k).copy_(torch.from_numpy(d["upd/storage/" + k]))
        st.step = st.num_transitions_per_env
        torch.manual_seed(seed + u)
        out.append(alg.update())
    sd = {k: v.detach().cpu().numpy().copy() for k, v in alg.actor_critic.state_dict().items()}
    return alg, out, sd


@pytest.mark.gpu
def test_engine_update_matches_reference_fixture(monkeypatch):
    """The reference's PPO.update (5 epochs x 4 mini-batches of 384 rows, adaptive KL rate, clip, both Adam
    steps) against the engine: losses, the learning-rate decisions and every weight, at the tolerances of the
    hipBLASLt path (tests/test_rollout.py::test_ppo_update_matches_reference_on_gpu)."""
    from tests.test_rollout import _check_update
    monkeypatch.setenv("GO1_PPO_ENGINE", "1")
    d = _fixture()
    alg, out, sd = _storage_update(d, DEV)
    assert getattr(alg, "_engine", None) is not None, "the engine did not run"
    w = _check_update(d, alg, out[0], rtol_loss=1e-3, atol_w=1e-4, atol_max=1e-3)  # measured 2.7e-4
    print(f"\nengine PPO.update vs the reference (CPU): max |dw| {w:.2e}")


@pytest.mark.gpu
def test_engine_graph_split_and_eager_agree_bitwise(monkeypatch):
    """Three updates from the fixture storage: eager launches, one HIP graph per mini-batch, and the
    world-size split (three graph segments around identity all-reduces) give bit-identical weights, losses and
    learning rates; a PPO_Args change between updates reaches the replayed graph (device-side hyper-parameters)."""
    d = _fixture()
    runs = {}
    clip0 = R.PPO_Args.clip_param
    for name, env in (("eager", {"GO1_PPO_GRAPH": "0"}), ("graph", {"GO1_PPO_GRAPH": "1"}),
                      ("split", {"GO1_PPO_GRAPH": "1", "GO1_PPO_SPLIT": "1"})):
        monkeypatch.setenv("GO1_PPO_SPLIT", "0")
        R.PPO_Args.clip_param = clip0
        orig_update = R.PPO.update

        def update(self, _orig=orig_update):
            self._n_upd = getattr(self, "_n_upd", 0) + 1
            if self._n_upd == 3:
                R.PPO_Args.clip_param = 0.15
            return _orig(self)
        monkeypatch.setattr(R.PPO, "update", update)
        try:
            alg, out, sd = _storage_update(d, DEV, env=env, monkeypatch=monkeypatch, updates=3)
        finally:
            R.PPO_Args.clip_param = clip0
            monkeypatch.setattr(R.PPO, "update", orig_update)
        eng = alg._engine
        assert (eng.graphs is not None) == (name != "eager")
        runs[name] = (out, alg.learning_rate, sd)
    for name in ("graph", "split"):
        assert runs[name][0] == runs["eager"][0], name
        assert runs[name][1] == runs["eager"][1], name
        for k, v in runs["eager"][2].items():
            assert np.array_equal(runs[name][2][k], v), (name, k)
    # the PPO_Args change took effect: the third update differs from a run without it
    monkeypatch.setenv("GO1_PPO_GRAPH", "1")
    alg, out, sd = _storage_update(d, DEV, updates=3)
    assert out[2] != runs["graph"][0][2]


@pytest.mark.gpu
def test_engine_matches_torch_update_at_full_size(monkeypatch):
    """BASELINE configs[2]'s update: 4096 envs x 24 steps, 4 mini-batches of 24,576 rows, 5 epochs, random
    storage with realistic scales: the engine against the torch autograd update (GO1_PPO_ENGINE=0, hipBLASLt
    GEMMs) from the same weights and permutation; both against each other within the update test's budget."""
    torch.manual_seed(11)
    n, T = 4096, 24
    sds, losses = [], []
    base = R.ActorCritic(261, 2, 261, 12)
    g = torch.Generator().manual_seed(3)
    data = {"observation_histories": torch.randn(T, n, 261, generator=g),
            "privileged_observations": torch.randn(T, n, 2, generator=g) * 0.5,
            "actions": torch.randn(T, n, 12, generator=g), "values": torch.randn(T, n, 1, generator=g),
            "returns": torch.randn(T, n, 1, generator=g), "advantages": torch.randn(T, n, 1, generator=g),
            "mu": torch.randn(T, n, 12, generator=g) * 0.3, "sigma": torch.ones(T, n, 12)}
    with torch.no_grad():
        h = data["observation_histories"].reshape(-1, 261)
        base_mu = base.actor_body(torch.cat((h, base.adaptation_module(h)), -1)).reshape(T, n, 12)
        data["mu"] = base_mu + 0.01 * data["mu"]
        data["actions"] = data["mu"] + data["actions"]
        lp = -(data["actions"] - base_mu) ** 2 / 2 - 0.9189385332046727
        data["actions_log_prob"] = lp.sum(-1, keepdim=True)
    perm = torch.randperm(n * T, generator=g)
    for flag in ("0", "1"):
        monkeypatch.setenv("GO1_PPO_ENGINE", flag)
        ac = R.ActorCritic(261, 2, 261, 12)
        ac.load_state_dict(base.state_dict())
        alg = R.PPO(ac, device=DEV, kernels=R.HipRolloutKernels())
        alg.init_storage(n, T, [261], [2], [261], [12])
        for k, v in data.items():
            getattr(alg.storage, k).copy_(v)
        alg.storage.step = T
        real = torch.randperm
        torch.randperm = lambda *a, **k: perm.to(k.get("device") or "cpu")
        try:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            losses.append(alg.update())
            torch.cuda.synchronize()
            print(f"\nupdate ({'engine' if flag == '1' else 'torch'}, first call incl. capture): "
                  f"{(time.perf_counter() - t0) * 1e3:.1f} ms")
        finally:
            torch.randperm = real
        assert (getattr(alg, "_engine", None) is not None) == (flag == "1")
        sds.append({k: v.detach().cpu().numpy() for k, v in alg.actor_critic.state_dict().items()})
        lr = alg.learning_rate
        if flag == "0":
            lr0 = lr
    # the adaptive rate takes the same decisions; torch's device division by a scalar multiplies by the
    # reciprocal (an ulp off the Python float division of ppo.py:128 that the engine reproduces)
    assert abs(lr - lr0) <= 1e-14 * lr0, (lr, lr0)
    np.testing.assert_allclose(np.array(losses[1]), np.array(losses[0]), rtol=1e-3, atol=1e-7)
    diffs = np.concatenate([np.abs(sds[1][k] - sds[0][k]).ravel() for k in sds[0]])
    print(f"\nengine vs torch update at 4096 envs: max |dw| {diffs.max():.2e}, p99.99 {np.percentile(diffs, 99.99):.2e}")
    assert np.percentile(diffs, 99.99) <= 5e-5 and diffs.max() <= 4e-4  # measured 9e-6 / 3.7e-5


def _storage_data(n, T, seed, base):
    """Random rollout storage of realistic scales for the ActorCritic `base` (as the full-size test)."""
    g = torch.Generator().manual_seed(seed)
    data = {"observation_histories": torch.randn(T, n, 261, generator=g),
            "privileged_observations": torch.randn(T, n, 2, generator=g) * 0.5,
            "actions": torch.randn(T, n, 12, generator=g), "values": torch.randn(T, n, 1, generator=g),
            "returns": torch.randn(T, n, 1, generator=g), "advantages": torch.randn(T, n, 1, generator=g),
            "mu": torch.randn(T, n, 12, generator=g) * 0.3, "sigma": torch.ones(T, n, 12)}
    data = {k: v.to(DEV) for k, v in data.items()}
    with torch.no_grad():
        b = R.ActorCritic(261, 2, 261, 12).to(DEV)
        b.load_state_dict(base.state_dict())
        h = data["observation_histories"].reshape(-1, 261)
        base_mu = b.actor_body(torch.cat((h, b.adaptation_module(h)), -1)).reshape(T, n, 12)
        data["mu"] = base_mu + 0.01 * data["mu"]
        data["actions"] = data["mu"] + data["actions"]
        lp = -(data["actions"] - base_mu) ** 2 / 2 - 0.9189385332046727
        data["actions_log_prob"] = lp.sum(-1, keepdim=True)
    return data


def _engine_for(base, data, n, T):
    ac = R.ActorCritic(261, 2, 261, 12)
    ac.load_state_dict(base.state_dict())
    alg = R.PPO(ac, device=DEV, kernels=R.HipRolloutKernels())
    alg.init_storage(n, T, [261], [2], [261], [12])
    for k, v in data.items():
        getattr(alg.storage, k).copy_(v.to(DEV))
    alg.storage.step = T
    return alg, PE.PPOEngine(alg)


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_loc", [(2, 2048), (8, 4096)])
def test_engine_world_n_arithmetic_equals_one_engine_over_the_union(world, n_loc):
    """The world > 1 arithmetic of the update (finalize_kernel's / world on the KL mean, the gradient norm, the loss
    sums and the Adam gradient scale, ppo_update.hip; ppo.py:119-133, 155-159, 188-190) executed on the GPU: `world`
    engines in one process, each bound to its shard of the rollout rows with hyper.world = world, the gradient
    all-reduce replaced by an in-process device sum of their [aux | grads] slices between the three segments
    (PPOEngine._segments, the order RCCL runs them in).  Against one engine over the union of the shards (every
    mini-batch = the union of the ranks' mini-batches, train rows first as each rank's num_train split of ppo.py:174
    gives them):
      * the same learning-rate decisions, after the first mini-batch and after the whole update (5 epochs x 4
        mini-batches); after the first mini-batch the loss sums within rtol 1e-6 (a wrong / world is off by the
        factor world in the loss sums and the KL mean) and the weights p99.99 within 1e-5;
      * losses and weights as close to the union's as one engine over the same union with the rows of every
        mini-batch in another order (the floor: the 3xF16 operand scaling is per tensor, so any regrouping of the
        rows rounds differently -- Adam's first step is lr g / (|g| + eps), which turns that into weight
        differences where |g| ~ eps -- and 20 steps compound it), within 4x that floor.
    T = 20 rollout steps keeps each rank's mini-batch a multiple of 5, so the ranks' num_train = data_size // 5 * 4
    splits add up to the union's (with 24 steps the union would train on 4 more rows)."""
    T, nmb, epochs = 20, 4, 5
    A = R.PPO_Args
    assert A.num_adaptation_module_substeps == 1
    torch.manual_seed(7)
    base = R.ActorCritic(261, 2, 261, 12)
    n = world * n_loc
    data = _storage_data(n, T, 17, base)
    mb_loc = n_loc * T // nmb
    ntr = mb_loc // 5 * 4
    g = torch.Generator().manual_seed(23)
    perms = [torch.randperm(nmb * mb_loc, generator=g) for _ in range(world)]
    order = [(ep, i) for ep in range(epochs) for i in range(nmb)]

    def snap(alg, eng):
        torch.cuda.synchronize()
        return (eng.losses.cpu().tolist(), float(eng.lr.item()),
                {k: v.detach().cpu().numpy().copy() for k, v in alg.actor_critic.state_dict().items()})

    # ---- world engines, one per shard of the envs
    ranks = []
    for r in range(world):
        shard = {k: v[:, r * n_loc:(r + 1) * n_loc].contiguous() for k, v in data.items()}
        alg, eng = _engine_for(base, shard, n_loc, T)
        eng._bind(alg.storage, mb_loc)
        eng._write_hyper(A, world)
        eng.pack()
        eng.losses.zero_()
        ranks.append((alg, eng))
    del shard
    segs = [eng._segments(world, True) for _, eng in ranks]
    snaps_w = []
    for step, (ep, i) in enumerate(order):
        for r, (_, eng) in enumerate(ranks):
            eng.idx.copy_(perms[r][i * mb_loc:(i + 1) * mb_loc].to(DEV))
        for j, (kind, _) in enumerate(segs[0]):
            if kind == "ar":  # all-reduce (sum) of the first NAUX + n gradient entries, as RCCL's
                m = PE.NAUX + (ranks[0][1].n_total if j == 1 else ranks[0][1].n_adapt)
                tot = torch.stack([eng.grads[:m] for _, eng in ranks]).sum(0)
                for _, eng in ranks:
                    eng.grads[:m].copy_(tot)
            else:
                for r in range(world):
                    segs[r][j][1]()
        if step in (0, len(order) - 1):
            sn = [snap(a, e) for a, e in ranks]
            for r in range(1, world):  # every rank applied the same update
                assert sn[r][0] == sn[0][0] and sn[r][1] == sn[0][1]
                for k in sn[0][2]:
                    assert np.array_equal(sn[r][2][k], sn[0][2][k]), (r, k)
            snaps_w.append(sn[0])
    del ranks, segs, sn
    torch.cuda.empty_cache()

    # ---- one engine over the union: row (t, r * n_loc + e) of the flat storage is rank r's row (t, e)
    def glob(r, loc):
        return (loc // n_loc) * n + r * n_loc + loc % n_loc

    def single(reorder):
        alg1, eng1 = _engine_for(base, data, n, T)
        eng1._bind(alg1.storage, world * mb_loc)
        eng1._write_hyper(A, 1)
        eng1.pack()
        eng1.losses.zero_()
        out = []
        for step, (ep, i) in enumerate(order):
            parts = [glob(r, perms[r][i * mb_loc:(i + 1) * mb_loc]) for r in range(world)]
            tr, te = torch.cat([p[:ntr] for p in parts]), torch.cat([p[ntr:] for p in parts])
            if reorder:  # the same train / test sets, each in another order
                tr, te = tr.flip(0), te.flip(0)
            eng1.idx.copy_(torch.cat([tr, te]).to(DEV))
            for _, fn in eng1._segments(1, False):
                fn()
            if step in (0, len(order) - 1):
                out.append(snap(alg1, eng1))
        del alg1, eng1
        torch.cuda.empty_cache()
        return out

    snaps_1 = single(False)
    snaps_f = single(True)
    base_sd = {k: v.numpy() for k, v in base.state_dict().items()}

    def dw(a, b):
        return np.concatenate([np.abs(a[k] - b[k]).ravel() for k in b])

    for when, k, loss_rtol in (("first mini-batch", 0, 1e-6), ("whole update", 1, None)):
        (lw, rw, sw), (l1, r1, s1), (lf, rf, sf) = snaps_w[k], snaps_1[k], snaps_f[k]
        assert rw == r1 == rf, (when, rw, r1, rf)  # the same learning-rate decisions
        dl_w = np.abs(np.array(lw) - np.array(l1)) / np.abs(np.array(l1))
        dl_f = np.abs(np.array(lf) - np.array(l1)) / np.abs(np.array(l1))
        d_w, d_f = dw(sw, s1), dw(sf, s1)
        print(f"\nworld {world} x {n_loc} envs vs one engine over {n}, {when}: losses rel {dl_w.max():.2e} "
              f"(reorder floor {dl_f.max():.2e}); weights max {d_w.max():.2e} p99.99 {np.percentile(d_w, 99.99):.2e} "
              f"(floor {d_f.max():.2e} / {np.percentile(d_f, 99.99):.2e}; the update moved weights by up to "
              f"{dw(s1, base_sd).max():.2e}); lr {r1:.3e}")
        if loss_rtol:  # one step: the loss sums agree to rounding (a wrong / world is off by the factor world),
            # and the weights p99.99 within VERDICT r04's 1e-5 (measured 6.9e-7 at world 2, 1.7e-6 at world 8)
            assert (dl_w <= loss_rtol).all(), (when, dl_w)
            assert np.percentile(d_w, 99.99) <= 1e-5, (when, np.percentile(d_w, 99.99))
        assert (dl_w <= np.maximum(4 * dl_f, 1e-6)).all(), (when, dl_w, dl_f)
        assert np.percentile(d_w, 99.99) <= max(4 * np.percentile(d_f, 99.99), 1e-6), when
        assert d_w.max() <= max(4 * d_f.max(), 1e-5), when


@pytest.mark.gpu
def test_engine_sees_in_place_weight_writes_between_updates(monkeypatch):
    """a load_state_dict (copy_ into the same storage) between two engine updates must reach the
    second update's forward and backward (the f16 fragment images are re-packed every update): the second update
    equals a fresh engine's update from the loaded weights and the first update's optimizer state, bit for bit.
    Then a torch-path update after the engine (GO1_PPO_ENGINE=0) steps each parameter's Adam state once."""
    d = _fixture()
    monkeypatch.setenv("GO1_PPO_ENGINE", "1")
    alg, out, _ = _storage_update(d, DEV)
    eng = alg._engine
    g = torch.Generator().manual_seed(9)
    w2 = {k: v + 0.05 * torch.randn(v.shape, generator=g).to(v.device) for k, v in alg.actor_critic.state_dict().items()}
    opt_sd = (alg.optimizer.state_dict(), alg.adaptation_module_optimizer.state_dict())
    opt_sd = tuple({"state": {i: {k: (t.clone() if isinstance(t, torch.Tensor) else t) for k, t in s.items()}
                              for i, s in o["state"].items()}, "param_groups": o["param_groups"]} for o in opt_sd)
    lr1 = alg.learning_rate

    def refill(a):
        st = a.storage
        for k in ("observations", "privileged_observations", "observation_histories", "actions", "values",
                  "returns", "actions_log_prob", "advantages", "mu", "sigma", "rewards"):
            getattr(st, k).copy_(torch.from_numpy(d["upd/storage/" + k]))
        st.step = st.num_transitions_per_env

    alg.actor_critic.load_state_dict(w2)
    assert alg.actor_critic.actor_body[0].weight.data_ptr() == eng.params.data_ptr() + 4 * eng.offsets["actor_body.0.weight"]
    refill(alg)
    torch.manual_seed(3)
    loss_a = alg.update()
    sd_a = {k: v.detach().cpu().numpy() for k, v in alg.actor_critic.state_dict().items()}

    ac = R.ActorCritic(261, 2, 261, 12)
    ac.load_state_dict({k: v.cpu() for k, v in w2.items()})
    alg_b = R.PPO(ac, device=DEV, kernels=R.HipRolloutKernels())
    alg_b.optimizer.load_state_dict(opt_sd[0])
    alg_b.adaptation_module_optimizer.load_state_dict(opt_sd[1])
    alg_b.learning_rate = lr1
    T, n = d["gae/rewards_in"].shape
    alg_b.init_storage(n, T, [261], [2], [261], [12])
    refill(alg_b)
    torch.manual_seed(3)
    loss_b = alg_b.update()
    assert alg_b._engine is not eng
    assert loss_a == loss_b
    for k, v in sd_a.items():
        assert np.array_equal(v, alg_b.actor_critic.state_dict()[k].detach().cpu().numpy()), k

    # the torch path after the engine: each parameter's own step, advanced once per optimizer step
    monkeypatch.setenv("GO1_PPO_ENGINE", "0")
    steps0 = float(eng.steps[0])
    refill(alg)
    alg.update()
    n_up = R.PPO_Args.num_learning_epochs * R.PPO_Args.num_mini_batches
    st = [float(s["step"]) for s in alg.optimizer.state.values()]
    assert len(set(st)) == 1 and st[0] == steps0 + n_up, (steps0, st[:3])
    # and back on the engine: it imports the torch path's state
    monkeypatch.setenv("GO1_PPO_ENGINE", "1")
    refill(alg)
    alg.update()
    assert float(eng.steps[0]) == steps0 + 2 * n_up
