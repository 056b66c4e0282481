import sys, time, torch
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_tracking_amd import rollout as R
torch.manual_seed(0)
n, T = 4096, 24
ac = R.ActorCritic(261, 2, 261, 12)
alg = R.PPO(ac, device="cuda:0", kernels=R.HipRolloutKernels())
alg.init_storage(n, T, [261], [2], [261], [12])
st = alg.storage
for k in ("observation_histories", "privileged_observations", "actions", "values", "returns", "advantages", "mu"):
    getattr(st, k).normal_()
st.sigma.fill_(1.0); st.actions_log_prob.fill_(-15.0)
for i in range(4):
    st.step = T
    torch.cuda.synchronize(); t0 = time.perf_counter()
    alg.update()
    torch.cuda.synchronize(); print(f"update {i}: {(time.perf_counter()-t0)*1e3:.2f} ms", flush=True)
