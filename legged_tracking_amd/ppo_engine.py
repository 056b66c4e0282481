"""PPO.update on the hand-written HIP update engine (csrc/ppo_update.hip, C ABI include/go1_ppo.h).

`PPOEngine` owns the flat parameter / gradient / Adam-state buffers of an ActorCritic (the module's parameters
become views into the flat parameter buffer, so the state dict, the checkpoints and the fused rollout policy see
every update in place) and runs the mini-batch loop of PPO.update (go1_gym_learn/ppo_cse/ppo.py:98-206):

    per mini-batch:  grad(0) [all-reduce] step(0) grad(1) [all-reduce] step(1)

captured into HIP graphs after the first mini-batch (one graph at world 1; three segments around the two
gradient all-reduces at world > 1, which stay eager RCCL calls).  Hyper-parameters, the adaptive learning rate,
the Adam step counts and the loss sums live on the device: a graph replays correctly after PPO_Args change.

The torch optimizers of rollout.PPO stay the API objects (`PPO.optimizer`, `PPO.adaptation_module_optimizer`):
their per-parameter state entries are views of the engine's Adam state, and a state the caller loaded into them
(`load_state_dict`) is imported before the next update.
"""
import ctypes as C
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GO1_PPO_LIB_OVERRIDE") or os.path.join(HERE, "_build", "libgo1_ppo.so")

NAUX = 8
HIDDEN_A = (256, 128)
HIDDEN = (512, 256, 128)

# state_dict order of the supported ActorCritic, as the engine lays out its flat buffers (go1_ppo.h)
PARAM_NAMES = [f"adaptation_module.{i}.{k}" for i in (0, 2, 4) for k in ("weight", "bias")] + \
              [f"actor_body.{i}.{k}" for i in (0, 2, 4, 6) for k in ("weight", "bias")] + \
              [f"critic_body.{i}.{k}" for i in (0, 2, 4, 6) for k in ("weight", "bias")] + ["std"]
N_ADAPT_TENSORS = 6


class _Dims(C.Structure):
    _fields_ = [("hist", C.c_int32), ("priv", C.c_int32), ("actions", C.c_int32), ("mb", C.c_int32),
                ("rows", C.c_int64)]


class _Bufs(C.Structure):
    _fields_ = [("obs_history", C.c_void_p), ("hist_ld", C.c_int64)] + \
               [(k, C.c_void_p) for k in ("privileged_obs", "actions", "values", "advantages", "returns",
                                          "actions_log_prob", "mu", "sigma", "idx", "params", "grads", "exp_avg",
                                          "exp_avg_sq", "ad_exp_avg", "ad_exp_avg_sq", "steps", "lr", "hyper",
                                          "losses", "work")]


HYPER_FIELDS = ("clip_param", "value_loss_coef", "entropy_coef", "max_grad_norm", "desired_kl",
                "use_clipped_value_loss", "selective", "beta1", "beta2", "eps", "world", "adaptation_lr")

_LIB = []


def load_library(path=None):
    """libgo1_ppo.so through ctypes; raises when the library or the GPU is missing (no CPU fallback).
    `path`: another build of the same source (tools/ppo_gemm_bench.py compares variants)."""
    if _LIB and path is None:
        return _LIB[0]
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"HIP PPO engine library missing: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    lib.go1_ppo_last_error.restype = C.c_char_p
    P = C.POINTER
    lib.go1_ppo_param_count.argtypes = [P(_Dims), P(C.c_int64), P(C.c_int64)]
    lib.go1_ppo_workspace_bytes.argtypes = [P(_Dims), P(C.c_int64)]
    lib.go1_ppo_pack.argtypes = [P(_Dims), P(_Bufs), C.c_void_p]
    for f in ("go1_ppo_grad", "go1_ppo_step"):
        getattr(lib, f).argtypes = [P(_Dims), P(_Bufs), C.c_int32, C.c_void_p]
    lib.go1_ppo_test_linear.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32,
                                        C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]
    lib.go1_ppo_test_wgrad.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p,
                                       C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]
    if path == LIB_PATH:
        _LIB.append(lib)
    return lib


def supported(ac):
    """The engine's architecture: AC_Args' default widths, ELU, latent 1..8, actions 1..16, no decoder."""
    try:
        a, p, c = ac.adaptation_module, ac.actor_body, ac.critic_body
        names = [n for n, _ in ac.named_parameters()]
    except AttributeError:
        return False
    if sorted(names) != sorted(PARAM_NAMES) or len(a) != 5 or len(p) != 7 or len(c) != 7:
        return False
    h, npv = ac.num_obs_history, ac.num_privileged_obs
    na = p[6].out_features
    want = {"adaptation_module.0": (HIDDEN_A[0], h), "adaptation_module.2": (HIDDEN_A[1], HIDDEN_A[0]),
            "adaptation_module.4": (npv, HIDDEN_A[1]), "actor_body.0": (HIDDEN[0], h + npv),
            "actor_body.2": (HIDDEN[1], HIDDEN[0]), "actor_body.4": (HIDDEN[2], HIDDEN[1]),
            "actor_body.6": (na, HIDDEN[2]), "critic_body.0": (HIDDEN[0], h + npv),
            "critic_body.2": (HIDDEN[1], HIDDEN[0]), "critic_body.4": (HIDDEN[2], HIDDEN[1]),
            "critic_body.6": (1, HIDDEN[2])}
    sd = dict(ac.named_parameters())
    ok = all(tuple(sd[k + ".weight"].shape) == v for k, v in want.items())
    acts = [m for seq in (a, p, c) for m in seq if not isinstance(m, torch.nn.Linear)]
    return (ok and 1 <= npv <= 8 and 1 <= na <= 16 and all(isinstance(m, torch.nn.ELU) and m.alpha == 1.0
                                                            for m in acts))


class PPOEngine:
    def __init__(self, alg):
        self.lib = load_library()
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible: the PPO update engine has no CPU fallback")
        self.alg = alg
        ac = alg.actor_critic
        self.device = next(ac.parameters()).device
        self.hist, self.priv = ac.num_obs_history, ac.num_privileged_obs
        self.na = ac.actor_body[6].out_features
        dims = _Dims(hist=self.hist, priv=self.priv, actions=self.na, mb=1, rows=1)
        tot, ad = C.c_int64(), C.c_int64()
        self._chk(self.lib.go1_ppo_param_count(C.byref(dims), C.byref(tot), C.byref(ad)))
        self.n_total, self.n_adapt = tot.value, ad.value
        dev = self.device
        sd = dict(ac.named_parameters())
        self.offsets = {}
        off = 0
        for name in PARAM_NAMES:
            self.offsets[name] = off
            off += sd[name].numel()
        if off != self.n_total or self.offsets[PARAM_NAMES[N_ADAPT_TENSORS]] != self.n_adapt:
            raise RuntimeError("PPO engine: parameter layout mismatch between the module and go1_ppo.h")
        # flat buffers; the module's parameters become views into `params`
        self.params = torch.empty(self.n_total, dtype=torch.float32, device=dev)
        for name in PARAM_NAMES:
            p, o = sd[name], self.offsets[name]
            self.params[o:o + p.numel()].copy_(p.detach().reshape(-1))
            p.data = self.params[o:o + p.numel()].view_as(p)
        self.grads = torch.zeros(NAUX + self.n_total, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(self.n_total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros_like(self.exp_avg)
        self.ad_exp_avg = torch.zeros(self.n_adapt, dtype=torch.float32, device=dev)
        self.ad_exp_avg_sq = torch.zeros_like(self.ad_exp_avg)
        self.steps = torch.zeros(2, dtype=torch.float32, device=dev)
        self.lr = torch.tensor([alg.learning_rate], dtype=torch.float64, device=dev)
        self.hyper = torch.zeros(len(HYPER_FIELDS), dtype=torch.float32, device=dev)
        self.losses = torch.zeros(4, dtype=torch.float64, device=dev)
        self._hyper_host = None
        self._lr_host = float(alg.learning_rate)
        self.work = None
        self.dims = None
        self.bufs = _Bufs()
        self.graphs = None
        self._graph_key = None
        self._import_optimizer_state()
        self._install_optimizer_views()

    # ------------------------------------------------------------------ helpers
    def _chk(self, rc):
        if rc != 0:
            raise RuntimeError(self.lib.go1_ppo_last_error().decode())

    @staticmethod
    def _stream():
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def _param_list(self, adaptation_only=False):
        sd = dict(self.alg.actor_critic.named_parameters())
        names = PARAM_NAMES[:N_ADAPT_TENSORS] if adaptation_only else PARAM_NAMES
        return [(n, sd[n]) for n in names]

    def _views(self, flat, adaptation_only=False):
        out = {}
        for name, p in self._param_list(adaptation_only):
            o = self.offsets[name]
            out[name] = flat[o:o + p.numel()].view_as(p)
        return out

    def _install_optimizer_views(self):
        """torch.optim.Adam-shaped state entries that are views of the engine's state (state_dict works)."""
        alg = self.alg
        for opt, (m1, m2), k, ad in ((alg.optimizer, (self.exp_avg, self.exp_avg_sq), 0, False),
                                     (alg.adaptation_module_optimizer, (self.ad_exp_avg, self.ad_exp_avg_sq), 1, True)):
            v1, v2 = self._views(m1, ad), self._views(m2, ad)
            for name, p in self._param_list(ad):
                opt.state[p] = {"step": self.steps[k], "exp_avg": v1[name], "exp_avg_sq": v2[name]}
        self._state_ptrs = self._optimizer_state_ptrs()

    def release_optimizer_state(self):
        """Give every parameter's optimizer state its own tensors again (copies of the engine's), before a torch
        optimizer steps them: the views share one `step` per optimizer, which a torch Adam would increment once
        per parameter.  The next engine update imports the state back (_sync_external_changes)."""
        alg = self.alg
        for opt, (m1, m2), k, ad in ((alg.optimizer, (self.exp_avg, self.exp_avg_sq), 0, False),
                                     (alg.adaptation_module_optimizer, (self.ad_exp_avg, self.ad_exp_avg_sq), 1, True)):
            g = opt.defaults
            on_dev = bool(g.get("fused") or g.get("capturable"))
            v1, v2 = self._views(m1, ad), self._views(m2, ad)
            for name, p in self._param_list(ad):
                step = self.steps[k].detach().clone()
                opt.state[p] = {"step": step if on_dev else step.cpu(), "exp_avg": v1[name].clone(),
                                "exp_avg_sq": v2[name].clone()}
        self._state_ptrs = None

    def _optimizer_state_ptrs(self):
        alg = self.alg
        return tuple(t.data_ptr() for opt in (alg.optimizer, alg.adaptation_module_optimizer)
                     for s in opt.state.values() for t in s.values() if isinstance(t, torch.Tensor))

    def _import_optimizer_state(self):
        """Copy torch-optimizer state (a previous torch-path update or load_state_dict) into the flat buffers."""
        alg = self.alg
        for opt, (m1, m2), k, ad in ((alg.optimizer, (self.exp_avg, self.exp_avg_sq), 0, False),
                                     (alg.adaptation_module_optimizer, (self.ad_exp_avg, self.ad_exp_avg_sq), 1, True)):
            v1, v2 = self._views(m1, ad), self._views(m2, ad)
            for name, p in self._param_list(ad):
                st = opt.state.get(p)
                if not st:
                    continue
                if "exp_avg" in st and st["exp_avg"].data_ptr() != v1[name].data_ptr():
                    v1[name].copy_(st["exp_avg"].detach().reshape(v1[name].shape))
                    v2[name].copy_(st["exp_avg_sq"].detach().reshape(v2[name].shape))
                if "step" in st:
                    self.steps[k].copy_(torch.as_tensor(st["step"], dtype=torch.float32).reshape(()))

    def _sync_external_changes(self):
        """Parameters or optimizer state replaced outside the engine since the last update."""
        ac = self.alg.actor_critic
        relink = False
        for name, p in self._param_list():
            o = self.offsets[name]
            if p.data_ptr() != self.params.data_ptr() + 4 * o:
                self.params[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.params[o:o + p.numel()].view_as(p)
                relink = True
        if self._optimizer_state_ptrs() != self._state_ptrs:
            self._import_optimizer_state()
            self._install_optimizer_views()
        return ac

    def _write_hyper(self, A, world):
        vals = (A.clip_param, A.value_loss_coef, A.entropy_coef, A.max_grad_norm,
                A.desired_kl if (A.desired_kl is not None and A.schedule == "adaptive") else 0.0,
                1.0 if A.use_clipped_value_loss else 0.0, 1.0 if A.selective_adaptation_module_loss else 0.0,
                0.9, 0.999, 1e-8, float(world), A.adaptation_module_learning_rate)
        vals = tuple(float(v) for v in vals)
        if vals != self._hyper_host:
            self.hyper.copy_(torch.tensor(vals, dtype=torch.float32))
            self._hyper_host = vals
        # Adam betas / eps from the torch optimizers' param groups (the reference's defaults)
        g = self.alg.optimizer.param_groups[0]
        b1, b2 = g.get("betas", (0.9, 0.999))
        eps = g.get("eps", 1e-8)
        if (b1, b2, eps) != (0.9, 0.999, 1e-8):
            v = list(vals)
            v[7:10] = [float(b1), float(b2), float(eps)]
            self.hyper.copy_(torch.tensor(v, dtype=torch.float32))
            self._hyper_host = tuple(v)

    def _bind(self, st, mb):
        rows = st.num_envs * st.num_transitions_per_env
        dims = _Dims(hist=self.hist, priv=self.priv, actions=self.na, mb=mb, rows=rows)
        nb = C.c_int64()
        self._chk(self.lib.go1_ppo_workspace_bytes(C.byref(dims), C.byref(nb)))
        if self.work is None or self.work.numel() < nb.value:
            self.work = torch.zeros(nb.value + 256, dtype=torch.uint8, device=self.device)
            self.graphs = None
        self.dims = dims
        b = self.bufs
        hist = st.observation_histories.flatten(0, 1)
        if hist.stride(1) != 1:
            hist = hist.contiguous()
        self._flat = [hist] + [x.flatten(0, 1).contiguous() for x in (
            st.privileged_observations, st.actions, st.values, st.advantages, st.returns, st.actions_log_prob, st.mu,
            st.sigma)]
        b.obs_history, b.hist_ld = hist.data_ptr(), hist.stride(0)
        for k, t in zip(("privileged_obs", "actions", "values", "advantages", "returns", "actions_log_prob", "mu",
                         "sigma"), self._flat[1:]):
            setattr(b, k, t.data_ptr())
        if getattr(self, "idx", None) is None or self.idx.numel() != mb:
            self.idx = torch.zeros(mb, dtype=torch.int64, device=self.device)
            self.graphs = None
        b.idx = self.idx.data_ptr()
        for k in ("params", "grads", "exp_avg", "exp_avg_sq", "ad_exp_avg", "ad_exp_avg_sq", "steps", "lr", "hyper",
                  "losses"):
            setattr(b, k, getattr(self, k).data_ptr())
        base = self.work.data_ptr()
        b.work = (base + 255) // 256 * 256
        return (mb, rows) + tuple(t.data_ptr() for t in self._flat)

    # ------------------------------------------------------------------ the C-ABI calls
    def pack(self):
        self._chk(self.lib.go1_ppo_pack(C.byref(self.dims), C.byref(self.bufs), self._stream()))

    def grad(self, phase):
        self._chk(self.lib.go1_ppo_grad(C.byref(self.dims), C.byref(self.bufs), phase, self._stream()))

    def step(self, phase):
        self._chk(self.lib.go1_ppo_step(C.byref(self.dims), C.byref(self.bufs), phase, self._stream()))

    def _allreduce(self, n):
        torch.distributed.all_reduce(self.grads[:NAUX + n])

    def _segments(self, world, split):
        """The mini-batch as ("hip", fn) work segments and ("ar", fn) gradient all-reduces between them."""
        if world == 1 and not split:
            return [("hip", lambda: (self.grad(0), self.step(0), self.grad(1), self.step(1)))]
        segs = [("hip", lambda: self.grad(0))]
        if world > 1:
            segs.append(("ar", lambda: self._allreduce(self.n_total)))
        segs.append(("hip", lambda: (self.step(0), self.grad(1))))
        if world > 1:
            segs.append(("ar", lambda: self._allreduce(self.n_adapt)))
        segs.append(("hip", lambda: self.step(1)))
        return segs

    # ------------------------------------------------------------------ PPO.update
    def update(self, A, num_mini_batches, num_epochs, world, use_graph=True, split=False):
        """The mini-batch loop of PPO.update; returns the four loss sums (value, surrogate, adaptation,
        adaptation test) over the mini-batches and the final learning rate."""
        alg = self.alg
        st = alg.storage
        self._sync_external_changes()
        if float(alg.learning_rate) != self._lr_host:  # the caller changed the rate between updates
            self.lr.fill_(float(alg.learning_rate))
        batch = st.num_envs * st.num_transitions_per_env
        mb = batch // num_mini_batches
        key = self._bind(st, mb)
        self._write_hyper(A, world)
        # the f16 fragment images from the current weights, every update: an in-place write to the parameters
        # (load_state_dict, a torch-path update, std.data edits) keeps their storage, so no pointer check sees it
        self.pack()
        self.losses.zero_()
        indices = torch.randperm(num_mini_batches * mb, device=self.device)  # mini_batch_generator's draw
        draw = getattr(self, "_draw", None)
        if draw is None or draw[0].shape != (mb, self.na):
            self._draw = draw = (torch.zeros(mb, self.na, device=self.device),
                                 torch.ones(mb, self.na, device=self.device))
        segs = self._segments(world, split)
        gkey = (key, world, split, self.work.data_ptr(), self.idx.data_ptr())
        if self.graphs is not None and self._graph_key != gkey:
            self.graphs = None
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                self.idx.copy_(indices[i * mb:(i + 1) * mb])
                torch.normal(*draw)  # ac.act's unused sample (ppo.py:110): the reference's torch RNG consumption
                if self.graphs is not None:
                    for kind, g in self.graphs:
                        g() if kind == "ar" else g.replay()
                    continue
                for _, fn in segs:
                    fn()
                if use_graph:
                    self._capture(segs, gkey)
        out = self.losses.cpu().tolist()
        lr = float(self.lr.item())
        self._lr_host = lr
        return out, lr

    def _capture(self, segs, gkey):
        """Capture the HIP segments (all-reduces stay eager callables between them), once the kernels are loaded."""
        torch.cuda.synchronize(self.device)
        side = getattr(self, "_side", None)
        if side is None:
            side = self._side = torch.cuda.Stream(self.device)
        graphs = []
        for kind, fn in segs:
            if kind == "ar":
                graphs.append((kind, fn))
                continue
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                fn()
            graphs.append((kind, g))
        self.graphs = graphs
        self._graph_key = gkey
