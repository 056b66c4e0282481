"""Debug: specialised vs generic step kernel (and generic vs generic) -- first step / array that differs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_full_size import _setup, _handle, N, DEV  # noqa: E402
from legged_tracking_amd import config as CF  # noqa: E402

both_generic = len(sys.argv) > 1
cfg, td, dr, ep, rng = _setup(seed=13)
c, ga, k1 = _handle(cfg, td, dr, ep, 0, N)
_, gb, k2 = _handle(cfg, td, dr, ep, 0, N)
gb.specialize(False)
if both_generic:
    ga.specialize(False)
print("spec a/b", ga.specialized, gb.specialized)
scales = CF.reward_scale_vector(CF.derived(cfg)["reward_scales"])
grav, gvec = CF.gravity_state([0.1, -0.3, 0.2])
torch.cuda.synchronize()
del k1, k2
from legged_tracking_amd import native  # noqa: E402
bufs = [dict(dbg=native.debug_buffers(N, c.decimation, DEV), aux=torch.zeros((N, 32), device=DEV),
             log=torch.zeros((N * 16, 18), device=DEV), cnt=torch.zeros(1, dtype=torch.int32, device=DEV),
             div=torch.zeros(1, dtype=torch.int64, device=DEV)) for _ in range(2)]
mode = os.environ.get("MODE", "both")
torch.manual_seed(0)
for t in range(int(os.environ.get("STEPS", "40"))):
    a = torch.randn(N, 12, device=DEV)
    if mode in ("both", "prepared"):
        for g, b in zip((ga, gb), bufs):
            args = g.prepare(dict(obs=g.obs, priv=g.priv, rew=g.rew, reset=g.reset, time_out=g.time_out),
                             aux=b["aux"], diverged_count=b["div"], episode_log=b["log"], log_count=b["cnt"])
            g.step_prepared(args, a, gvec, grav, scales, ("k", t), 5, t, log_tag=t)
        torch.cuda.synchronize()
        sa, sb = ga.state.numpy(), gb.state.numpy()
        d = [k for k in sa if (sa[k] != sb[k]).any()]
        if d:
            print("prepared step", t, "diverges:", d, [np.nonzero((sa[k] != sb[k]).any(axis=1))[0][:4] for k in d])
            break
    if mode in ("both", "plain"):
        for g, b in zip((ga, gb), bufs):
            g.step(a, gvec, grav, scales, rng_seed=6, rng_step=1000 + t, debug=b["dbg"])
    torch.cuda.synchronize()
    sa, sb = ga.state.numpy(), gb.state.numpy()
    bad = {k: (int((sa[k] != sb[k]).any(axis=1).sum()), float(np.abs(sa[k] - sb[k]).max())) for k in sa
           if (sa[k] != sb[k]).any()}
    ob = (ga.obs.cpu().numpy() != gb.obs.cpu().numpy())
    if bad or ob.any():
        envs = np.nonzero(ob.any(axis=1))[0]
        print("step", t, "state diffs (envs, max)", bad, "obs envs", envs[:10], "cols", np.nonzero(ob.any(axis=0))[0][:20])
        for k in bad:
            e = np.nonzero((sa[k] != sb[k]).any(axis=1))[0][:3]
            print("  ", k, "envs", e)
        for k, v in bufs[0]["dbg"].items():
            x, y = v.cpu().numpy(), bufs[1]["dbg"][k].cpu().numpy()
            if (x != y).any():
                if k == "torques":
                    for sub in range(x.shape[0]):
                        dd = (x[sub] != y[sub]).any(axis=1)
                        print("  torques sub", sub, "envs", np.nonzero(dd)[0][:5], "max", np.abs(x[sub] - y[sub]).max())
                print("  dbg", k, x.shape, "max", np.abs(x - y).max(), "envs", np.nonzero((x != y).reshape(x.shape[0], -1).any(axis=1))[0][:5] if x.shape[0] == N else "")
        break
else:
    print("identical over 40 steps")
