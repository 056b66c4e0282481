"""Lower bound of a layer-per-launch ("weight-stationary") policy forward at the rollout's 4096 envs, against the
fused policy_kernel_split: python tools/policy_ws_bound.py [n_envs] > out.json

A weight-stationary policy keeps each layer's weights resident on the CUs that own it and hands the activations to
the next layer through L2, so the actor path (adaptation module 3 layers -> actor 4 layers: the actor's first layer
needs the latent) is 7 dependent steps: 7 launches, or 7 grid-wide hand-offs inside one.  Measured here:
  * each layer as the PPO engine's 3xF16 MFMA GEMM (xw_kernel through go1_ppo_test_linear, the update's own
    kernel) at n_envs rows: (time of 1 + R launches - time of 1) / R, HIP events;
  * the floor of a dependent launch: a one-element kernel launched back to back on a stream, and the same seven
    times inside a captured HIP graph (per node).
The bound is the sum over the 7 actor-path layers of max(GEMM, graph floor); the critic's 4 layers can share
those launches (the engine groups problems per launch), so they add nothing to it."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_tracking_amd import ppo_engine as PE  # noqa: E402

R = 40
HIST, PRIV, ACT = 261, 2, 12  # HistoryWrapper(TrajectoryTrackingEnv): obs history width, privileged obs, actions
# (name, k, n): n padded to the engine's 128-wide tiles (the output layers are 2 / 12 wide)
ACTOR_PATH = [("adapt L1", HIST, 256), ("adapt L2", 256, 128), ("adapt L3 (latent)", 128, 128),
              ("actor L1", HIST + PRIV, 512), ("actor L2", 512, 256), ("actor L3", 256, 128),
              ("actor L4 (mean)", 128, 128)]


def timed(fn):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(1)
    torch.cuda.synchronize()
    out = []
    for reps in (1, R + 1):
        e0.record(st)
        fn(reps)
        e1.record(st)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return (out[1] - out[0]) / R * 1e3  # us


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    lib = PE.load_library()
    work = torch.zeros(256 << 20, dtype=torch.uint8, device=dev)
    base = (work.data_ptr() + 255) // 256 * 256
    nb = work.numel() - 256
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    layers = []
    for name, k, nn in ACTOR_PATH:
        x = torch.randn(n, k, device=dev, generator=g)
        w = torch.randn(nn, k, device=dev, generator=g) / k ** 0.5
        b = torch.zeros(nn, device=dev)
        y = torch.empty(n, nn, device=dev)

        def run(r):
            rc = lib.go1_ppo_test_linear(x.data_ptr(), n, k, w.data_ptr(), b.data_ptr(), nn, 1, y.data_ptr(), base,
                                         nb, r, s)
            assert rc == 0, rc

        us = timed(run)
        layers.append({"layer": name, "k": k, "n": nn, "gemm_us": us,
                       "f16_tflops": 2.0 * n * k * nn * 3 / us / 1e6})
    # the dependent-launch floor: back to back on the stream, and per node of a captured graph
    one = torch.zeros(1, device=dev)
    stream_us = timed(lambda r: [one.add_(1.0) for _ in range(r)])
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            one.add_(1.0)
    torch.cuda.current_stream().wait_stream(side)
    with torch.cuda.graph(graph):
        for _ in range(len(ACTOR_PATH)):
            one.add_(1.0)
    graph_us = timed(lambda r: [graph.replay() for _ in range(r)]) / len(ACTOR_PATH)
    bound = sum(max(L["gemm_us"], graph_us) for L in layers)
    print(json.dumps({"n_envs": n, "actor_path_layers": layers, "launch_floor_stream_us": stream_us,
                      "launch_floor_graph_node_us": graph_us, "actor_path_bound_us": bound,
                      "what": __doc__.split("\n\n")[0]}, indent=1))


if __name__ == "__main__":
    main()
