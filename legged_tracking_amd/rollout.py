"""PPO rollout over the HIP env step: the go1_gym_learn.ppo_cse API the training script uses.

Mirrors, with the same public names, constructor arguments and parameter names (so
the reference's `ac_weights.pt` state dicts load unchanged):

  AC_Args, ActorCritic     <- go1_gym_learn/ppo_cse/actor_critic.py:9-178
  PPO_Args, PPO            <- go1_gym_learn/ppo_cse/ppo.py:13-206
  RolloutStorage           <- go1_gym_learn/ppo_cse/rollout_storage.py:5-138
  RunnerArgs, Runner       <- go1_gym_learn/ppo_cse/__init__.py:46-357

MI355X mapping: the policy / value / adaptation MLPs are plain GEMM chains on
hipBLASLt (through torch); the per-step transition copy, the GAE scan and the
advantage normalisation are HIP kernels (csrc/rollout.hip, C ABI
include/go1_rollout.h).  With torch.distributed initialised (one process per GPU,
RCCL), the advantage statistics, the gradients and the KL estimate are
all-reduced so that every rank follows the same optimisation trajectory as one
large-batch run.
"""
import contextlib
import copy
import ctypes as C
import os
import time
from collections import deque

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Normal

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GO1_ROLLOUT_LIB_OVERRIDE") or os.path.join(HERE, "_build", "libgo1_rollout.so")


# ----------------------------------------------------------------------------- args
class _Args:
    """Plain mutable argument holder (scripts/train.py assigns attributes)."""


class AC_Args(_Args):
    init_noise_std = 1.0
    actor_hidden_dims = [512, 256, 128]
    critic_hidden_dims = [512, 256, 128]
    activation = "elu"
    adaptation_module_branch_hidden_dims = [256, 128]
    use_decoder = False
    normalize_obs = False


class PPO_Args(_Args):
    value_loss_coef = 1.0
    use_clipped_value_loss = True
    clip_param = 0.2
    entropy_coef = 0.01
    num_learning_epochs = 5
    num_mini_batches = 4
    learning_rate = 1.0e-3
    adaptation_module_learning_rate = 1.0e-3
    num_adaptation_module_substeps = 1
    schedule = "adaptive"
    gamma = 0.99
    lam = 0.95
    desired_kl = 0.01
    max_grad_norm = 1.0
    selective_adaptation_module_loss = False


class RunnerArgs(_Args):
    algorithm_class_name = "RMA"
    num_steps_per_env = 24
    max_iterations = 1500
    save_interval = 400
    save_video_interval = 100
    log_freq = 10
    resume = False
    load_run = -1
    checkpoint = -1
    resume_path = None
    resume_curriculum = True


# ----------------------------------------------------------------------------- native kernels
class _Transition(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("obs", "privileged_obs", "obs_history", "actions", "mu", "sigma",
                                          "actions_log_prob", "values", "rewards", "dones", "time_outs",
                                          "st_obs", "st_privileged_obs", "st_obs_history", "st_actions", "st_mu",
                                          "st_sigma", "st_actions_log_prob", "st_values", "st_rewards",
                                          "st_dones")] + [
        ("num_obs", C.c_int32), ("num_priv", C.c_int32), ("num_obs_history", C.c_int32), ("num_actions", C.c_int32),
        ("time_outs_flag", C.c_void_p), ("time_outs_pending", C.c_void_p), ("time_outs_dst", C.c_void_p),
        ("obs_history_ld", C.c_int64)]


class _PolicyLayer(C.Structure):
    _fields_ = [("w", C.c_void_p), ("b", C.c_void_p), ("wf", C.c_void_p)]


class _PolicyArgs(C.Structure):
    _fields_ = [("obs_history", C.c_void_p), ("privileged_obs", C.c_void_p), ("action_mean", C.c_void_p),
                ("value", C.c_void_p), ("latent", C.c_void_p), ("std", C.c_void_p), ("actions", C.c_void_p),
                ("action_sigma", C.c_void_p), ("log_prob", C.c_void_p), ("rng_seed", C.c_uint64),
                ("rng_step", C.c_uint64), ("env_id_offset", C.c_int32), ("n_envs", C.c_int32),
                ("hist_dim", C.c_int32), ("num_actions", C.c_int32), ("num_priv", C.c_int32),
                ("variant", C.c_int32), ("overflow", C.c_void_p), ("layers", _PolicyLayer * 11),
                ("hist_ld", C.c_int64)]


def _pack_linear(lin):
    """nn.Linear -> (weights split and packed for csrc/rollout.hip's 3xF16 MFMA, bias padded to 16).

    Every weight w is split into hi = f16(w) and lo = f16(w - hi).  Packed as 32-byte records
    [n/16][k/32][lane = 16 q + m][hi r = 0..7, lo r = 0..7] of W[16 t + m][32 g + 8 q + r]: lane
    (m, q) of output tile t reads one record per 32-deep K group g -- its A fragments of
    v_mfma_f32_16x16x32_f16 (row m, k = 8 q .. 8 q + 7) for both halves of the split."""
    W, b = lin.weight.detach().float(), lin.bias.detach().float()
    n, k = W.shape
    npad, kpad = -(-n // 16) * 16, -(-k // 32) * 32
    Wp = torch.zeros(npad, kpad, device=W.device, dtype=torch.float32)
    Wp[:n, :k] = W
    bp = torch.zeros(npad, device=W.device, dtype=torch.float32)
    bp[:n] = b
    hi = Wp.to(torch.float16)
    lo = (Wp - hi.float()).to(torch.float16)
    # [t, m, g, q, r] -> [t, g, q, m, r], then hi and lo side by side in the last dimension
    def frag(x):
        return x.view(npad // 16, 16, kpad // 32, 4, 8).permute(0, 2, 3, 1, 4)
    return torch.cat([frag(hi), frag(lo)], dim=-1).contiguous(), bp


class FusedPolicy:
    """ActorCritic forward for the rollout (act + evaluate) in one HIP kernel
    (csrc/rollout.hip policy_kernel).  Re-pack after every optimiser step."""

    def __init__(self, ac, lib, variant=0):
        self.ac = ac
        self.lib = lib
        self.packed = None
        self.variant = variant  # 0: per-net workgroups of 32 envs, 1: one workgroup of 16 envs (go1_policy_args)
        # workgroups that took the f32 fallback of the range guard (activations beyond f16's range)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=next(ac.parameters()).device)

    @staticmethod
    def supported(ac):
        try:
            a, p, c = ac.adaptation_module, ac.actor_body, ac.critic_body
            shapes = [tuple(m.weight.shape) for m in (a[0], a[2], a[4], p[0], p[2], p[4], p[6], c[0], c[2], c[4],
                                                       c[6])]
        except (IndexError, AttributeError):
            return False
        h, npv = ac.num_obs_history, ac.num_privileged_obs
        want = [(256, h), (128, 256), (npv, 128), (512, h + npv), (256, 512), (128, 256), (None, 128),
                (512, h + npv), (256, 512), (128, 256), (1, 128)]
        ok = all(w[0] in (None, s[0]) and w[1] == s[1] for s, w in zip(shapes, want))
        # any history width for the default launch (inputs streamed in chunks of 288), as long as the
        # 32-wide groups that hold the latent sit in the last chunk (go1_policy_forward checks the same)
        kin, gl, GL = h + npv, h // 32, -(-(h + npv) // 32)
        g_last = 9 * (-(-GL // 9) - 1)
        return (ok and 1 <= npv <= 8 and kin <= 16384 and gl >= g_last and shapes[6][0] <= 16
                and isinstance(a[1], nn.ELU))

    def pack(self):
        ac = self.ac
        mods = [ac.adaptation_module[i] for i in (0, 2, 4)] + [ac.actor_body[i] for i in (0, 2, 4, 6)] + \
               [ac.critic_body[i] for i in (0, 2, 4, 6)]
        self.packed = [_pack_linear(m) for m in mods]
        # the unsplit f32 weights for the range guard's fallback (the module's own tensors: an optimiser
        # step updates them in place; the split copies are re-packed)
        self.wf = [m.weight.detach().float().contiguous() for m in mods]
        self.na = ac.actor_body[6].out_features
        self.np = ac.num_privileged_obs
        self.args = _PolicyArgs(num_actions=self.na, num_priv=self.np, overflow=self.overflow.data_ptr())
        for i, (w, b) in enumerate(self.packed):
            self.args.layers[i].w, self.args.layers[i].b = w.data_ptr(), b.data_ptr()
            self.args.layers[i].wf = self.wf[i].data_ptr()

    def forward(self, obs_history, privileged_obs, sample=None):
        """-> (mean, value, latent) or, with sample = (rng_seed, rng_step, env_id_offset),
        (mean, value, latent, actions, sigma, log_prob): Normal(mean, std) drawn in-kernel."""
        if self.packed is None:
            self.pack()
        h = obs_history.detach()
        p = privileged_obs.detach()
        if h.dim() != 2 or h.stride(1) != 1 or h.stride(0) < h.shape[1]:
            h = h.contiguous()  # row-strided windows (the velocity env's history) are read in place
        if not p.is_contiguous():
            p = p.contiguous()
        n = h.shape[0]
        na = self.na
        dev = h.device
        mean = torch.empty(n, na, device=dev)
        value = torch.empty(n, 1, device=dev)
        latent = torch.empty(n, self.np, device=dev)
        a = self.args
        a.variant = self.variant
        a.obs_history, a.privileged_obs = h.data_ptr(), p.data_ptr()
        a.action_mean, a.value, a.latent = mean.data_ptr(), value.data_ptr(), latent.data_ptr()
        a.n_envs, a.hist_dim, a.hist_ld = n, h.shape[1], h.stride(0)
        out = (mean, value, latent)
        if sample is not None:
            actions = torch.empty(n, na, device=dev)
            sigma = torch.empty(n, na, device=dev)
            logp = torch.empty(n, device=dev)
            self.std = self.ac.std.detach().contiguous()
            a.std, a.actions, a.action_sigma, a.log_prob = (self.std.data_ptr(), actions.data_ptr(),
                                                            sigma.data_ptr(), logp.data_ptr())
            a.rng_seed, a.rng_step, a.env_id_offset = sample
            out = out + (actions, sigma, logp)
        else:
            a.actions = None
        rc = self.lib.go1_policy_forward(C.byref(a), C.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc != 0:
            raise RuntimeError(self.lib.go1_rollout_last_error().decode())
        return out


class HipRolloutKernels:
    """ctypes binding of libgo1_rollout.so; raises when the library or the GPU is missing."""

    def __init__(self):
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP rollout library missing: {LIB_PATH} (run __graft_entry__.build())")
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible: the rollout kernels have no CPU fallback")
        lib = C.CDLL(LIB_PATH)
        lib.go1_rollout_last_error.restype = C.c_char_p
        lib.go1_record_transition.argtypes = [C.POINTER(_Transition), C.c_int32, C.c_float, C.c_void_p]
        lib.go1_gae.argtypes = [C.c_void_p] * 7 + [C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_void_p]
        lib.go1_adv_normalize.argtypes = [C.c_void_p, C.c_void_p, C.c_double, C.c_int64, C.c_void_p]
        lib.go1_policy_forward.argtypes = [C.POINTER(_PolicyArgs), C.c_void_p]
        self.lib = lib

    def _chk(self, rc):
        if rc != 0:
            raise RuntimeError(self.lib.go1_rollout_last_error().decode())

    @staticmethod
    def _s():
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    _SRC = (("obs", "observations"), ("privileged_obs", "privileged_observations"),
            ("obs_history", "observation_histories"), ("actions", "actions"), ("mu", "action_mean"),
            ("sigma", "action_sigma"), ("actions_log_prob", "actions_log_prob"), ("values", "values"),
            ("rewards", "rewards"), ("dones", "dones"), ("time_outs", "time_outs"))

    def record(self, st, step, tr, gamma):
        t = getattr(st, "_tr_struct", None)
        if t is None:
            t = st._tr_struct = _Transition()
            t.num_obs, t.num_priv = st.observations.shape[-1], st.privileged_observations.shape[-1]
            t.num_obs_history, t.num_actions = st.observation_histories.shape[-1], st.actions.shape[-1]
            st._tr_dst = [(k, buf) for k, buf in (
                ("st_obs", st.observations), ("st_privileged_obs", st.privileged_observations),
                ("st_obs_history", st.observation_histories), ("st_actions", st.actions), ("st_mu", st.mu),
                ("st_sigma", st.sigma), ("st_actions_log_prob", st.actions_log_prob), ("st_values", st.values),
                ("st_rewards", st.rewards), ("st_dones", st.dones))]
        keep = []
        for k, name in self._SRC:
            v = tr.get(name)
            if v is None:
                setattr(t, k, None)
                continue
            if v.dtype == torch.bool:
                v = v.view(torch.uint8)
            if k == "obs_history" and v.dim() == 2 and v.stride(1) == 1 and v.stride(0) >= v.shape[1]:
                t.obs_history_ld = v.stride(0)  # a row-strided window is copied row by row
            elif not v.is_contiguous():
                v = v.contiguous()
            if k == "obs_history" and v.is_contiguous():
                t.obs_history_ld = 0
            keep.append(v)
            setattr(t, k, v.data_ptr())
        for k, buf in st._tr_dst:
            setattr(t, k, buf[step].data_ptr())
        d = tr.get("time_outs_deferred")  # (flag, pending, dst) device pointers, or None
        t.time_outs_flag, t.time_outs_pending, t.time_outs_dst = d if d is not None else (None, None, None)
        self._chk(self.lib.go1_record_transition(C.byref(t), st.num_envs, gamma, self._s()))
        return keep

    def gae(self, st, last_values, gamma, lam):
        lv = last_values.detach().contiguous()
        self._chk(self.lib.go1_gae(st.rewards.data_ptr(), st.dones.data_ptr(), st.values.data_ptr(), lv.data_ptr(),
                                   st.returns.data_ptr(), st.advantages.data_ptr(), st.adv_stats.data_ptr(),
                                   st.num_transitions_per_env, st.num_envs, gamma, lam, self._s()))

    def policy(self, ac):
        return FusedPolicy(ac, self.lib) if FusedPolicy.supported(ac) else None

    def normalize(self, st, count):
        self._chk(self.lib.go1_adv_normalize(st.advantages.data_ptr(), st.adv_stats.data_ptr(), float(count),
                                             st.advantages.numel(), self._s()))


# ----------------------------------------------------------------------------- model
def get_activation(name):
    acts = dict(elu=nn.ELU, selu=nn.SELU, relu=nn.ReLU, crelu=nn.ReLU, lrelu=nn.LeakyReLU, tanh=nn.Tanh,
                sigmoid=nn.Sigmoid)
    if name not in acts:
        raise ValueError(f"invalid activation function {name!r}")
    return acts[name]()


_COLSUM_LIB = []  # [ctypes lib or None], loaded on first use


def _colsum(g):
    """Column sums of a (rows, cols) gradient (the bias gradient) with the deterministic HIP kernel
    (go1_colsum); torch's sum(0) off the GPU or without the library."""
    if not g.is_cuda or g.dim() != 2 or not g.is_contiguous() or g.dtype != torch.float32 or g.shape[0] < 64 or \
            os.environ.get("GO1_COLSUM", "1") == "0":
        return g.sum(0)
    if not _COLSUM_LIB:
        lib = None
        if os.path.exists(LIB_PATH):
            lib = C.CDLL(LIB_PATH)
            lib.go1_colsum.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
            lib.go1_rollout_last_error.restype = C.c_char_p
        _COLSUM_LIB.append(lib)
    lib = _COLSUM_LIB[0]
    if lib is None:
        return g.sum(0)
    rows, cols = g.shape
    parts = max(1, min(512 // ((cols + 63) // 64), rows // 256, 64))
    part = torch.empty((parts, cols), dtype=torch.float32, device=g.device)
    out = torch.empty(cols, dtype=torch.float32, device=g.device)
    rc = lib.go1_colsum(g.data_ptr(), rows, cols, part.data_ptr(), parts, out.data_ptr(),
                        C.c_void_p(torch.cuda.current_stream(g.device).cuda_stream))
    if rc != 0:
        raise RuntimeError(lib.go1_rollout_last_error().decode())
    return out


class _LinearSplitK(torch.autograd.Function):
    """y = x W^T + b whose weight gradient is summed over K_SPLIT row chunks of the batch (one batched
    GEMM, then a sum over the chunks): the mini-batch weight gradient dW = dY^T X is a tall-skinny
    reduction (K = 24,576 samples, M x N <= 512 x 263), which one GEMM spreads over only a few dozen
    workgroups of the 256 CUs; the batched form gives each chunk its own tiles.  Same value as
    F.linear's backward up to the f32 summation order."""

    K_SPLIT = 16

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gy @ w if ctx.needs_input_grad[0] else None
        n, S = x.shape[0], _LinearSplitK.K_SPLIT
        if n % S == 0 and n // S >= 256:
            gw = torch.bmm(gy.view(S, n // S, -1).transpose(1, 2), x.view(S, n // S, -1)).sum(0)
        else:
            gw = gy.t() @ x
        return gx, gw, _colsum(gy)


def _mlp_train(seq, x):
    """nn.Sequential of Linear / activation layers evaluated with _LinearSplitK (training mini-batches)."""
    for m in seq:
        x = _LinearSplitK.apply(x, m.weight, m.bias) if isinstance(m, nn.Linear) else m(x)
    return x


def _mlp(sizes, act):
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[i], sizes[i + 1]))
        if i < len(sizes) - 2:
            layers.append(act)
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    """Student/teacher actor-critic (actor_critic.py:21-156): adaptation module
    obs_history -> latent (privileged estimate), actor (obs_history, latent) -> action
    mean, critic (obs_history, privileged_obs) -> value, state-independent std."""

    is_recurrent = False

    def __init__(self, num_obs, num_privileged_obs, num_obs_history, num_actions, **kwargs):
        super().__init__()
        self.decoder = AC_Args.use_decoder
        self.num_obs_history = num_obs_history
        self.num_privileged_obs = num_privileged_obs
        act = get_activation(AC_Args.activation)
        self.adaptation_module = _mlp([num_obs_history, *AC_Args.adaptation_module_branch_hidden_dims,
                                       num_privileged_obs], act)
        self.actor_body = _mlp([num_privileged_obs + num_obs_history, *AC_Args.actor_hidden_dims, num_actions], act)
        self.critic_body = _mlp([num_privileged_obs + num_obs_history, *AC_Args.critic_hidden_dims, 1], act)
        self.std = nn.Parameter(AC_Args.init_noise_std * torch.ones(num_actions))
        self.distribution = None
        self.normalize_obs = AC_Args.normalize_obs
        if self.normalize_obs:
            raise NotImplementedError("normalize_obs is off in the README configuration and not on this path")

    def reset(self, dones=None):
        pass

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def update_distribution(self, observation_history):
        latent = self.adaptation_module(observation_history)
        mean = self.actor_body(torch.cat((observation_history, latent), dim=-1))
        self.distribution = Normal(mean, mean * 0.0 + self.std, validate_args=False)

    def act(self, observation_history, **kwargs):
        self.update_distribution(observation_history)
        return self.distribution.sample()

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def act_expert(self, ob, policy_info={}):
        return self.act_teacher(ob["obs_history"], ob["privileged_obs"])

    def act_inference(self, ob, policy_info={}):
        return self.act_student(ob["obs_history"], policy_info=policy_info)

    def act_student(self, observation_history, policy_info={}):
        latent = self.adaptation_module(observation_history)
        policy_info["latents"] = latent.detach().cpu().numpy()
        return self.actor_body(torch.cat((observation_history, latent), dim=-1))

    def act_teacher(self, observation_history, privileged_info, policy_info={}):
        policy_info["latents"] = privileged_info
        return self.actor_body(torch.cat((observation_history, privileged_info), dim=-1))

    def evaluate(self, observation_history, privileged_observations, **kwargs):
        return self.critic_body(torch.cat((observation_history, privileged_observations), dim=-1))

    def get_student_latent(self, observation_history):
        return self.adaptation_module(observation_history)

    def update_distribution_train(self, observation_history):
        """update_distribution for PPO.update's mini-batches (split-K weight gradients, _LinearSplitK)."""
        latent = _mlp_train(self.adaptation_module, observation_history)
        mean = _mlp_train(self.actor_body, torch.cat((observation_history, latent), dim=-1))
        self.distribution = Normal(mean, mean * 0.0 + self.std, validate_args=False)

    def evaluate_train(self, observation_history, privileged_observations):
        return _mlp_train(self.critic_body, torch.cat((observation_history, privileged_observations), dim=-1))


# ----------------------------------------------------------------------------- storage
class RolloutStorage:
    """Device-resident (T, n, ...) rollout buffers (rollout_storage.py:24-56)."""

    class Transition:
        def __init__(self):
            self.observations = None
            self.privileged_observations = None
            self.observation_histories = None
            self.critic_observations = None
            self.actions = None
            self.rewards = None
            self.dones = None
            self.values = None
            self.actions_log_prob = None
            self.action_mean = None
            self.action_sigma = None
            self.env_bins = None
            self.time_outs = None
            self.time_outs_deferred = None

        def clear(self):
            self.__init__()

    def __init__(self, num_envs, num_transitions_per_env, obs_shape, privileged_obs_shape, obs_history_shape,
                 actions_shape, device="cpu", kernels=None):
        self.device = device
        T, n = num_transitions_per_env, num_envs
        z = lambda *s: torch.zeros(T, n, *s, device=device)  # noqa: E731
        self.obs_shape, self.privileged_obs_shape = obs_shape, privileged_obs_shape
        self.obs_history_shape, self.actions_shape = obs_history_shape, actions_shape
        self.observations = z(*obs_shape)
        self.privileged_observations = z(*privileged_obs_shape)
        self.observation_histories = z(*obs_history_shape)
        self.rewards = z(1)
        self.actions = z(*actions_shape)
        self.dones = z(1).byte()
        self.actions_log_prob = z(1)
        self.values = z(1)
        self.returns = z(1)
        self.advantages = z(1)
        self.mu = z(*actions_shape)
        self.sigma = z(*actions_shape)
        self.env_bins = z(1)
        self.adv_stats = torch.zeros(2, dtype=torch.float64, device=device)
        self.num_transitions_per_env, self.num_envs = T, n
        self.step = 0
        self.kernels = kernels if kernels is not None else HipRolloutKernels()
        self._keep = None

    def add_transitions(self, transition, gamma=0.0):
        if self.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        tr = {k: getattr(transition, k) for k in ("observations", "privileged_observations", "observation_histories",
                                                  "actions", "action_mean", "action_sigma", "actions_log_prob",
                                                  "values", "rewards", "dones", "time_outs")}
        tr["time_outs_deferred"] = getattr(transition, "time_outs_deferred", None)
        self._keep = self.kernels.record(self, self.step, tr, gamma)
        self.step += 1

    def clear(self):
        self.step = 0

    def compute_returns(self, last_values, gamma, lam):
        """GAE (rollout_storage.py:76-90); global normalisation across ranks."""
        self.kernels.gae(self, last_values, gamma, lam)
        count = float(self.advantages.numel())
        if torch.distributed.is_available() and torch.distributed.is_initialized() and \
                torch.distributed.get_world_size() > 1:
            torch.distributed.all_reduce(self.adv_stats)
            count *= torch.distributed.get_world_size()
        self.kernels.normalize(self, count)

    def get_statistics(self):
        done = self.dones.clone()
        done[-1] = 1
        flat_dones = done.permute(1, 0, 2).reshape(-1, 1)
        done_indices = torch.cat((flat_dones.new_tensor([-1], dtype=torch.int64),
                                  flat_dones.nonzero(as_tuple=False)[:, 0]))
        return (done_indices[1:] - done_indices[:-1]).float().mean(), self.rewards.mean()

    def mini_batch_generator(self, num_mini_batches, num_epochs=8, generator=None):
        batch_size = self.num_envs * self.num_transitions_per_env
        mb = batch_size // num_mini_batches
        indices = torch.randperm(num_mini_batches * mb, device=self.device, generator=generator)
        flat = [x.flatten(0, 1) for x in (self.observations, self.observations, self.privileged_observations,
                                         self.observation_histories, self.actions, self.values, self.advantages,
                                         self.returns, self.actions_log_prob, self.mu, self.sigma)]
        bins = self.env_bins.flatten(0, 1)
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                idx = indices[i * mb:(i + 1) * mb]
                b = [x[idx] for x in flat]
                yield (*b, None, bins[idx])


# ----------------------------------------------------------------------------- PPO
def _world():
    d = torch.distributed
    if d.is_available() and d.is_initialized():
        return d.get_world_size()
    return 1


class PPO:
    """PPO with the adaptation-module regression (ppo.py:33-206)."""

    def __init__(self, actor_critic, device="cpu", kernels=None):
        self.device = device
        self.actor_critic = actor_critic.to(device)
        self.storage = None
        self.kernels = kernels
        # On the GPU: fused Adam (one kernel per step instead of a foreach chain), its learning rate a device
        # tensor so that the adaptive schedule (ppo.py:124-136) runs on the device -- no host sync per
        # mini-batch; the rate is computed in f64 as the reference's Python floats are, and the f32 copy the
        # kernel reads is the value the foreach path would cast to.  On the CPU: the reference's path.
        self._dev_lr = torch.device(device).type == "cuda" and os.environ.get("GO1_PPO_FUSED", "1") != "0"
        params = list(self.actor_critic.parameters())
        # The mini-batch step (forward, backward, gradient clip, both Adam steps, the adaptive rate) is
        # captured once into a HIP graph and replayed for every later mini-batch (GO1_PPO_GRAPH=0: eager):
        # it is ~150 small launches whose host issue left the GPU idle between them.  One rank only (the
        # gradient all-reduce stays eager).
        self._graph_on = self._dev_lr and os.environ.get("GO1_PPO_GRAPH", "1") != "0"
        self._graph = None
        self._graph_warm = 0
        if self._dev_lr:
            self._lr64 = torch.tensor(PPO_Args.learning_rate, dtype=torch.float64, device=device)
            self._lr32 = torch.tensor(PPO_Args.learning_rate, dtype=torch.float32, device=device)
            cap = self._graph_on
            self.optimizer = torch.optim.Adam(params, lr=self._lr32, fused=True, capturable=cap)
            self.adaptation_module_optimizer = torch.optim.Adam(params, lr=PPO_Args.adaptation_module_learning_rate,
                                                                fused=True, capturable=cap)
        else:
            self.optimizer = torch.optim.Adam(params, lr=PPO_Args.learning_rate)
            self.adaptation_module_optimizer = torch.optim.Adam(params, lr=PPO_Args.adaptation_module_learning_rate)
        self.transition = RolloutStorage.Transition()
        self.learning_rate = PPO_Args.learning_rate
        self.fused = None  # FusedPolicy once the storage (and its kernels) exist
        self.sample_seed = 0x5EED
        self._sample_step = 0
        self.env_id_offset = 0
        # optional: the record kernel of step t on a side stream, under the policy kernel of step
        # t+1 (they do not depend on each other); the env step of t+1 and every storage reader
        # wait for it (_rec_done).  Measured slower (36.1 against 42.1 M env-steps/s: the
        # cross-stream waits cost more than the 6 us record hides), so off
        self.overlap_record = False
        self._rec_stream, self._rec_done = None, None
        if _world() > 1:  # every rank starts from rank 0's weights
            for p in self.actor_critic.parameters():
                torch.distributed.broadcast(p.data, 0)

    def init_storage(self, num_envs, num_transitions_per_env, actor_obs_shape, privileged_obs_shape,
                     obs_history_shape, action_shape):
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, actor_obs_shape, privileged_obs_shape,
                                      obs_history_shape, action_shape, self.device, kernels=self.kernels)
        pol = getattr(self.storage.kernels, "policy", None)
        self.fused = pol(self.actor_critic) if pol is not None else None
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            self.env_id_offset = torch.distributed.get_rank() * num_envs

    def test_mode(self):
        self.actor_critic.eval()

    def train_mode(self):
        self.actor_critic.train()

    def act(self, obs, privileged_obs, obs_history):
        ac = self.actor_critic
        t = self.transition
        if self.fused is not None and not torch.is_grad_enabled():
            # one kernel: adaptation module + actor + critic + Normal(mean, std) sample + log_prob
            self._sample_step += 1
            mean, values, _, actions, sigma, logp = self.fused.forward(
                obs_history, privileged_obs, sample=(self.sample_seed, self._sample_step, self.env_id_offset))
            self._wait_record()  # after the policy launch: only what follows (the env step) waits
            t.actions, t.values, t.actions_log_prob, t.action_mean, t.action_sigma = actions, values, logp, mean, sigma
            t.observations = obs
            t.critic_observations = obs
            t.privileged_observations = privileged_obs
            t.observation_histories = obs_history
            return t.actions
        else:
            t.actions = ac.act(obs_history).detach()
            t.values = ac.evaluate(obs_history, privileged_obs).detach()
        t.actions_log_prob = ac.get_actions_log_prob(t.actions).detach()
        t.action_mean = ac.action_mean.detach()
        t.action_sigma = ac.action_std.detach()
        t.observations = obs
        t.critic_observations = obs
        t.privileged_observations = privileged_obs
        t.observation_histories = obs_history
        return t.actions

    def process_env_step(self, rewards, dones, infos):
        """Records the transition; the time-out bootstrap r += gamma * V * time_outs
        (ppo.py:85-87) is applied inside the record kernel."""
        t = self.transition
        t.rewards = rewards
        t.dones = dones
        t.time_outs_deferred = None
        deferred = getattr(infos, "deferred_time_outs", None)
        if deferred is not None and "time_outs" in infos:
            # the env's pending extras["time_outs"] rebinding is resolved by the record kernel
            # (no separate sync launch); the tensor it leaves current is the one read here
            t.time_outs, t.time_outs_deferred = deferred()
        else:
            t.time_outs = infos["time_outs"] if "time_outs" in infos else None
        if self.overlap_record and self.fused is not None and rewards.is_cuda and not torch.is_grad_enabled():
            main = torch.cuda.current_stream(rewards.device)
            if self._rec_stream is None:
                self._rec_stream = torch.cuda.Stream(rewards.device)
            side = self._rec_stream
            side.wait_stream(main)  # the step's outputs and the policy's are complete
            with torch.cuda.stream(side):
                self.storage.add_transitions(t, gamma=PPO_Args.gamma)
            for x in (t.observations, t.critic_observations, t.privileged_observations, t.observation_histories,
                      t.actions, t.values, t.actions_log_prob, t.action_mean, t.action_sigma, t.rewards, t.dones,
                      t.time_outs):
                if isinstance(x, torch.Tensor) and x.is_cuda:
                    x.record_stream(side)  # the allocator keeps them until the side stream is past the record
            self._rec_done = torch.cuda.Event()
            self._rec_done.record(side)
        else:
            self.storage.add_transitions(t, gamma=PPO_Args.gamma)
        t.clear()
        self.actor_critic.reset(dones)

    def _wait_record(self):
        """The current stream waits for the last side-stream record (storage readers, the env step)."""
        if self._rec_done is not None:
            torch.cuda.current_stream().wait_event(self._rec_done)
            self._rec_done = None

    def compute_returns(self, last_critic_obs, last_critic_privileged_obs):
        self._wait_record()
        if self.fused is not None and not torch.is_grad_enabled():
            last_values = self.fused.forward(last_critic_obs, last_critic_privileged_obs)[1]
        else:
            last_values = self.actor_critic.evaluate(last_critic_obs, last_critic_privileged_obs).detach()
        self.storage.compute_returns(last_values, PPO_Args.gamma, PPO_Args.lam)

    def _allreduce_grads(self):
        w = _world()
        if w == 1:
            return
        params = [p for p in self.actor_critic.parameters() if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in params])
        torch.distributed.all_reduce(flat)
        flat /= w
        off = 0
        for p in params:
            k = p.numel()
            p.grad.copy_(flat[off:off + k].view_as(p.grad))
            off += k

    def _minibatch_step(self, batch, acc, sample=True):
        """One mini-batch of PPO.update (ppo.py:107-201): the surrogate / value / entropy loss and its Adam step,
        the adaptive learning rate, then the adaptation-module regression step(s).  Loss values accumulate
        into `acc` on the device.  sample=False leaves out ac.act's unused sample (the graphed loop draws it
        outside the graph: torch's generator cannot be advanced inside a HIP capture here)."""
        A = PPO_Args
        ac = self.actor_critic
        (obs_b, critic_obs_b, priv_b, hist_b, act_b, target_v_b, adv_b, ret_b, old_logp_b, old_mu_b,
         old_sigma_b) = batch
        ac.update_distribution_train(hist_b)
        if sample:
            ac.distribution.sample()  # ac.act's (unused) sample: the reference's torch RNG consumption (ppo.py:110)
        logp_b = ac.get_actions_log_prob(act_b)
        value_b = ac.evaluate_train(hist_b, priv_b)
        mu_b, sigma_b, entropy_b = ac.action_mean, ac.action_std, ac.entropy
        if A.desired_kl is not None and A.schedule == "adaptive":
            with torch.inference_mode():
                kl = torch.sum(torch.log(sigma_b / old_sigma_b + 1.0e-5) +
                               (torch.square(old_sigma_b) + torch.square(old_mu_b - mu_b)) /
                               (2.0 * torch.square(sigma_b)) - 0.5, axis=-1)
                kl_mean = torch.mean(kl)
                if _world() > 1:
                    kl_mean = kl_mean.clone()
                    torch.distributed.all_reduce(kl_mean)
                    kl_mean /= _world()
            if self._dev_lr:
                with torch.no_grad():
                    k, lr = kl_mean.double(), self._lr64
                    new = torch.where(k > A.desired_kl * 2.0, torch.clamp(lr / 1.5, min=1e-5),
                                      torch.where((k < A.desired_kl / 2.0) & (k > 0.0),
                                                  torch.clamp(lr * 1.5, max=1e-2), lr))
                    self._lr64.copy_(new)
                    self._lr32.copy_(new)
            else:
                kl_mean = float(kl_mean)
                if kl_mean > A.desired_kl * 2.0:
                    self.learning_rate = max(1e-5, self.learning_rate / 1.5)
                elif A.desired_kl / 2.0 > kl_mean > 0.0:
                    self.learning_rate = min(1e-2, self.learning_rate * 1.5)
                for g in self.optimizer.param_groups:
                    g["lr"] = self.learning_rate
        ratio = torch.exp(logp_b - torch.squeeze(old_logp_b))
        surrogate = -torch.squeeze(adv_b) * ratio
        surrogate_clipped = -torch.squeeze(adv_b) * torch.clamp(ratio, 1.0 - A.clip_param, 1.0 + A.clip_param)
        surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
        if A.use_clipped_value_loss:
            value_clipped = target_v_b + (value_b - target_v_b).clamp(-A.clip_param, A.clip_param)
            value_loss = torch.max((value_b - ret_b).pow(2), (value_clipped - ret_b).pow(2)).mean()
        else:
            value_loss = (ret_b - value_b).pow(2).mean()
        loss = surrogate_loss + A.value_loss_coef * value_loss - A.entropy_coef * entropy_b.mean()
        self.optimizer.zero_grad()
        loss.backward()
        self._allreduce_grads()
        nn.utils.clip_grad_norm_(ac.parameters(), A.max_grad_norm)
        self.optimizer.step()
        acc[0] += value_loss.detach()
        acc[1] += surrogate_loss.detach()
        num_train = int(priv_b.shape[0] // 5 * 4)
        for _ in range(A.num_adaptation_module_substeps):
            pred = _mlp_train(ac.adaptation_module, hist_b)
            with torch.no_grad():
                target = priv_b
            # every column (ppo.py:193: linspace(0, w - 1, w) as an index), or column 0
            sel = 0 if A.selective_adaptation_module_loss else slice(None)
            adapt_loss = F.mse_loss(pred[:num_train, sel], target[:num_train, sel])
            adapt_test = F.mse_loss(pred[num_train:, sel], target[num_train:, sel])
            self.adaptation_module_optimizer.zero_grad()
            adapt_loss.backward()
            self._allreduce_grads()
            self.adaptation_module_optimizer.step()
            acc[2] += adapt_loss.detach()
            acc[3] += adapt_test.detach()

    GRAPH_WARMUP = 3  # eager mini-batches (on a side stream) before the capture: lazy handles and optimizer state

    _ARG_KEYS = ("clip_param", "value_loss_coef", "use_clipped_value_loss", "entropy_coef", "max_grad_norm",
                 "desired_kl", "schedule", "num_adaptation_module_substeps", "selective_adaptation_module_loss")

    def _torch_graph_key(self, mb, flat):
        """What a captured mini-batch step bakes in: the batch size, the storage it gathers from, the PPO_Args
        scalars of the loss / clip / schedule, and the optimizers' state tensors (load_state_dict replaces them)."""
        opt_state = tuple(id(t) for o in (self.optimizer, self.adaptation_module_optimizer)
                          for s in o.state.values() for t in s.values() if isinstance(t, torch.Tensor))
        return (mb, tuple(x.data_ptr() for x in flat), tuple(getattr(PPO_Args, k) for k in self._ARG_KEYS), opt_state)

    def _graphed_minibatches(self, acc):
        """The mini-batch loop of update() with the step replayed from a HIP graph: the batch is gathered inside the
        graph from the storage with a static index buffer, so a mini-batch costs one index copy and one replay."""
        A = PPO_Args
        st = self.storage
        batch = st.num_envs * st.num_transitions_per_env
        mb = batch // A.num_mini_batches
        indices = torch.randperm(A.num_mini_batches * mb, device=self.device)  # mini_batch_generator's draw
        flat = [x.flatten(0, 1) for x in (st.observations, st.observations, st.privileged_observations,
                                         st.observation_histories, st.actions, st.values, st.advantages,
                                         st.returns, st.actions_log_prob, st.mu, st.sigma)]
        key = self._torch_graph_key(mb, flat)
        if self._graph is not None and self._graph_key != key:
            self._graph = None  # new storage, PPO_Args or optimizer state: capture again
            self._graph_warm = 0
        if self._graph is None and self._graph_warm == 0:
            self._graph_idx = torch.empty(mb, dtype=torch.int64, device=self.device)
            self._graph_acc = torch.zeros(4, dtype=torch.float32, device=self.device)
        idx, gacc = self._graph_idx, self._graph_acc
        # ac.act's unused sample per mini-batch, drawn before each step with the same shape: the same torch
        # generator advance as the eager loop's (the values are discarded there too)
        na = st.actions.shape[-1]
        if getattr(self, "_graph_draw", None) is None or self._graph_draw[0].shape != (mb, na):
            self._graph_draw = (torch.zeros(mb, na, device=self.device), torch.ones(mb, na, device=self.device))

        def step():
            # the generator's obs and critic-obs batches (flat[0:2]) are never read by the step (the nets take the
            # history and the privileged obs): not gathered, two index kernels less per mini-batch
            self._minibatch_step([None, None] + [x[idx] for x in flat[2:]], gacc, sample=False)

        # warm-up and capture run on ONE persistent side stream: the parameters' AccumulateGrad nodes are created
        # there and every later backward (warm-up, capture) runs on the same stream (a fresh stream per warm-up
        # mini-batch made torch warn about a stream mismatch of the accumulation)
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        side = self._side
        for _ in range(A.num_learning_epochs):
            for i in range(A.num_mini_batches):
                idx.copy_(indices[i * mb:(i + 1) * mb])
                torch.normal(*self._graph_draw)
                if self._graph is not None:
                    self._graph.replay()
                    continue
                side.wait_stream(torch.cuda.current_stream(self.device))
                if self._graph_warm < self.GRAPH_WARMUP:
                    with torch.cuda.stream(side):
                        step()
                    self._graph_warm += 1
                else:
                    torch.cuda.synchronize(self.device)
                    for p in self.actor_critic.parameters():
                        p.grad = None
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=side):
                        step()
                    self._graph = g
                    self._graph_key = self._torch_graph_key(mb, flat)  # the optimizer state exists by now
                    with torch.cuda.stream(side):
                        g.replay()  # the capture recorded the step without running it
                torch.cuda.current_stream(self.device).wait_stream(side)
        acc += gacc
        gacc.zero_()

    def _engine_on(self):
        """The hand-written HIP update (ppo_engine.PPOEngine, csrc/ppo_update.hip) on the GPU for the default
        architecture; GO1_PPO_ENGINE=0 selects the torch autograd update (A/B)."""
        if torch.device(self.device).type != "cuda" or os.environ.get("GO1_PPO_ENGINE", "1") == "0":
            return False
        from . import ppo_engine
        return ppo_engine.supported(self.actor_critic)

    def update(self):
        A = PPO_Args
        n_up = A.num_learning_epochs * A.num_mini_batches
        n_ad = n_up * A.num_adaptation_module_substeps
        if self._engine_on() and A.num_adaptation_module_substeps == 1:
            from . import ppo_engine
            if getattr(self, "_engine", None) is None:
                self._engine = ppo_engine.PPOEngine(self)
            sums, lr = self._engine.update(A, A.num_mini_batches, A.num_learning_epochs, _world(),
                                           use_graph=self._graph_on,
                                           split=os.environ.get("GO1_PPO_SPLIT", "0") == "1")
            self.learning_rate = lr
            for g in self.optimizer.param_groups:
                if isinstance(g["lr"], torch.Tensor):
                    g["lr"].fill_(lr)
                else:
                    g["lr"] = lr
            if self._dev_lr:
                self._lr64.fill_(lr)
                self._lr32.fill_(lr)
            self.storage.clear()
            if self.fused is not None:
                self.fused.pack()  # the rollout kernel reads the updated weights
            return (sums[0] / n_up, sums[1] / n_up, sums[2] / n_ad, 0.0, 0.0, sums[3] / n_ad, 0.0, 0.0)
        if getattr(self, "_engine", None) is not None:
            self._engine.release_optimizer_state()  # torch's Adam steps per-parameter state of its own
        # the loss means accumulate on the device (ppo.py:186-187, 200-201 call .item() per mini-batch:
        # a host sync each); one copy at the end.
        acc = torch.zeros(4, dtype=torch.float32, device=self.device)  # value, surrogate, adapt, adapt_test
        if self._graph_on and _world() == 1:
            self._graphed_minibatches(acc)
        else:
            gen = self.storage.mini_batch_generator(A.num_mini_batches, A.num_learning_epochs)
            for b in gen:
                self._minibatch_step(b[:11], acc)
        self.storage.clear()
        if self.fused is not None:
            self.fused.pack()  # the rollout kernel reads the updated weights
        mean_value_loss, mean_surrogate_loss, mean_adapt, mean_adapt_test = (float(x) for x in acc.cpu())
        if self._dev_lr:
            self.learning_rate = float(self._lr64)
        return (mean_value_loss / n_up, mean_surrogate_loss / n_up, mean_adapt / n_ad, 0.0, 0.0,
                mean_adapt_test / n_ad, 0.0, 0.0)


# ----------------------------------------------------------------------------- runner
@contextlib.contextmanager
def _rollout_outputs(env):
    """The rollout reads neither the contact forces nor the aux block (ppo_cse/__init__.py:164-214): the step leaves
    both stores out (LeggedRobot.set_output_demand) while it runs, and they are back on afterwards."""
    f = getattr(env, "set_output_demand", None)
    if f is None:
        yield
        return
    f(contact_forces=False, aux=False)
    try:
        yield
    finally:
        f(contact_forces=True, aux=True)


class Runner:
    """Runner (ppo_cse/__init__.py:66-357): rollout of num_steps_per_env env steps per
    iteration, GAE, PPO update, checkpoints (ac_weights.pt + TorchScript adaptation
    module and actor body, the formats scripts/eval.py and the deploy stack read)."""

    def __init__(self, env, device="cpu", runner_args=RunnerArgs, ac_args=AC_Args, log_wandb=False, kernels=None,
                 save_dir=None):
        self.device = device
        self.env = env
        self.runner_args = runner_args
        self.log_wandb = log_wandb
        self.save_dir = save_dir
        ac = ActorCritic(env.num_obs, env.num_privileged_obs, env.num_obs_history, env.num_actions).to(device)
        if runner_args.resume:
            ac.load_state_dict(torch.load(runner_args.resume, map_location=device, weights_only=True))
        self.alg = PPO(ac, device=device, kernels=kernels)
        self.num_steps_per_env = runner_args.num_steps_per_env
        self.alg.init_storage(env.num_train_envs, self.num_steps_per_env, [env.num_obs], [env.num_privileged_obs],
                              [env.num_obs_history], [env.num_actions])
        self.tot_timesteps = 0
        self.tot_time = 0
        self.current_learning_iteration = 0
        self.last_recording_it = -1000
        self.env.reset()

    def rollout(self, obs, privileged_obs, obs_history, update_model=True, eval_expert=False):
        """One iteration's rollout (ppo_cse/__init__.py:164-214)."""
        n_train = self.env.num_train_envs
        rewards = dones = infos = None
        for _ in range(self.num_steps_per_env):
            actions = self.alg.act(obs[:n_train], privileged_obs[:n_train], obs_history[:n_train])
            if n_train < self.env.num_envs:
                ac = self.alg.actor_critic
                extra = ac.act_teacher(obs_history[n_train:], privileged_obs[n_train:]) if eval_expert else \
                    ac.act_student(obs_history[n_train:])
                actions = torch.cat((actions, extra), dim=0)
            obs_dict, rewards, dones, infos = self.env.step(actions)
            obs, privileged_obs, obs_history = obs_dict["obs"], obs_dict["privileged_obs"], obs_dict["obs_history"]
            if update_model:
                self.alg.process_env_step(rewards[:n_train], dones[:n_train], infos)
            if "train/episode" in infos and self.log_wandb:
                import wandb
                info = infos["train/episode"]
                wandb.log({"train": {k: np.mean(v) for k, v in info.items()}})
        return obs, privileged_obs, obs_history, infos

    def learn(self, num_learning_iterations, init_at_random_ep_len=False, eval_freq=100, curriculum_dump_freq=500,
              eval_expert=False, update_model=True):
        n_train = self.env.num_train_envs
        obs_dict = self.env.get_observations()
        obs, privileged_obs, obs_history = (obs_dict[k].to(self.device) for k in ("obs", "privileged_obs",
                                                                                  "obs_history"))
        self.alg.actor_critic.train()
        if init_at_random_ep_len:
            # as in the reference, this lands on the HistoryWrapper, not the env
            self.env.episode_length_buf = torch.randint_like(self.env.episode_length_buf,
                                                             high=int(self.env.max_episode_length))
        for it in range(num_learning_iterations):
            start = time.time()
            with torch.inference_mode(), _rollout_outputs(self.env):
                obs, privileged_obs, obs_history, infos = self.rollout(obs, privileged_obs, obs_history,
                                                                       update_model, eval_expert)
                if update_model:
                    self.alg.compute_returns(obs_history[:n_train], privileged_obs[:n_train])
            if update_model:
                losses = self.alg.update()
            else:
                losses = (0.0,) * 8
            if self.log_wandb:
                import wandb
                keys = ("mean_value_loss", "mean_surrogate_loss", "adaptation_loss", "mean_decoder_loss",
                        "mean_decoder_loss_student", "mean_adaptation_module_test_loss", "mean_decoder_test_loss",
                        "mean_decoder_test_loss_student")
                wandb.log({"metrics": dict(zip(keys, losses))})
            self.tot_timesteps += self.num_steps_per_env * self.env.num_envs
            self.tot_time += time.time() - start
            self.current_learning_iteration = it
            if it % self.runner_args.save_interval == 0:
                self.save(self.checkpoint_dir())
        self.save(self.checkpoint_dir())

    def checkpoint_dir(self):
        """Where the reference's Runner writes checkpoints (ppo_cse/__init__.py:276-279):
        wandb.run.dir/checkpoints with wandb logging, last_run/checkpoints otherwise."""
        if self.save_dir is not None:
            return self.save_dir
        if self.log_wandb:
            import wandb
            return os.path.join(wandb.run.dir, "checkpoints")
        return "last_run/checkpoints"

    def save(self, save_path=None):
        """ac_weights.pt + adaptation_module_latest.jit + body_latest.jit (__init__.py:274-319), uploaded
        with wandb.save when logging to wandb (:294-297)."""
        if _world() > 1 and torch.distributed.get_rank() != 0:
            return
        save_path = save_path or self.checkpoint_dir()
        os.makedirs(save_path, exist_ok=True)
        ac = self.alg.actor_critic
        paths = [os.path.join(save_path, "ac_weights.pt"), os.path.join(save_path, "adaptation_module_latest.jit"),
                 os.path.join(save_path, "body_latest.jit")]
        torch.save(ac.state_dict(), paths[0])
        torch.jit.script(copy.deepcopy(ac.adaptation_module).to("cpu")).save(paths[1])
        torch.jit.script(copy.deepcopy(ac.actor_body).to("cpu")).save(paths[2])
        if self.log_wandb:
            import wandb
            for path in paths:
                wandb.save(path)

    def get_inference_policy(self, device=None):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.act_inference

    def get_expert_policy(self, device=None):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.act_expert
