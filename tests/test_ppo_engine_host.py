"""Host logic of the PPO update engine's multi-rank path (legged_tracking_amd/ppo_engine.py), on the CPU with gloo.

At world > 1 a mini-batch is three HIP segments with the two gradient all-reduces between them (ppo.py:155-159 and
the adaptation step: every rank follows the same trajectory as one large-batch run):
    grad(0) | all-reduce grads[:AUX + all params] | step(0), grad(1) | all-reduce grads[:AUX + adaptation] | step(1)
The HIP calls are replaced by recorders that write rank-dependent gradients, so the order of the segments, the
slices the all-reduces cover and their sums are checked across two gloo ranks.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

from legged_tracking_amd import ppo_engine as PE


def _fake_engine(rank, n_total, n_adapt, log):
    eng = object.__new__(PE.PPOEngine)
    eng.n_total, eng.n_adapt = n_total, n_adapt
    eng.grads = torch.zeros(PE.NAUX + n_total)

    def grad(phase):
        log.append(("grad", phase))
        if phase == 0:  # every gradient and the aux sums
            eng.grads.copy_(torch.arange(PE.NAUX + n_total, dtype=torch.float32) * (rank + 1))
        else:  # the adaptation slice (and its aux sums) only
            eng.grads[:PE.NAUX + n_adapt] = 1000.0 * (rank + 1)

    def step(phase):
        log.append(("step", phase, eng.grads.clone()))

    eng.grad, eng.step = grad, step
    return eng


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_total, n_adapt = 50, 20
        log = []
        eng = _fake_engine(rank, n_total, n_adapt, log)
        segs = eng._segments(world, split=True)
        kinds = [k for k, _ in segs]
        for _, fn in segs:
            fn()
        out[rank] = (kinds, log)
    finally:
        dist.destroy_process_group()


def test_world2_split_segments_all_reduce_the_right_slices():
    port = 29500 + os.getpid() % 1000
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    n_total, n_adapt = 50, 20
    for rank in range(world):
        kinds, log = res[rank]
        assert kinds == ["hip", "ar", "hip", "ar", "hip"]
        assert [e[:2] for e in log] == [("grad", 0), ("step", 0), ("grad", 1), ("step", 1)]
        g0, g1 = log[1][2], log[3][2]
        base = torch.arange(PE.NAUX + n_total, dtype=torch.float32)
        # phase 0: the whole buffer (aux sums + every gradient) summed over the ranks: (1 + 2) x
        assert torch.equal(g0, base * 3)
        # phase 1: the adaptation slice summed (1000 + 2000); the rest keeps phase 0's all-reduced values
        assert torch.equal(g1[:PE.NAUX + n_adapt], torch.full((PE.NAUX + n_adapt,), 3000.0))
        assert torch.equal(g1[PE.NAUX + n_adapt:], (base * 3)[PE.NAUX + n_adapt:])


@pytest.mark.parametrize("split", [False, True])
def test_world1_segments_have_no_collective(split):
    log = []
    eng = _fake_engine(0, 10, 4, log)
    segs = eng._segments(1, split=split)
    assert all(k == "hip" for k, _ in segs) and len(segs) == (3 if split else 1)
    for _, fn in segs:
        fn()
    assert [e[:2] for e in log] == [("grad", 0), ("step", 0), ("grad", 1), ("step", 1)]
