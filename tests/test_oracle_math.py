"""The isaacgym.torch_utils restatement the fixtures depend on (tests/golden/refstubs/isaacgym/
torch_utils.py; Isaac Gym itself is absent) against the reference's OWN numpy copies of the same
formulas in go1_gym/utils/planner.py:17-78 (quat_apply, quat_from_euler_xyz, quat_apply_inverse,
get_euler_xyz, copysign).  planner.py imports ompl (absent), so the five functions are extracted
from its source with `ast` and compiled alone; nothing else of the module runs.  Also checks the
oracle / kernel f32 forms (oracle/go1_oracle.c quat_rotate_inverse_f, quat_to_rpy_f through a
one-step post-physics replay is covered by the golden fixtures) against the same numpy copies."""
import ast
import importlib.util
import os

import numpy as np
import pytest
import torch

PLANNER = "/root/reference/go1_gym/utils/planner.py"
STUB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "refstubs", "isaacgym", "torch_utils.py")
NAMES = ("quat_apply", "quat_from_euler_xyz", "quat_apply_inverse", "get_euler_xyz", "copysign")

pytestmark = pytest.mark.skipif(not os.path.exists(PLANNER), reason="reference tree absent (GPU box)")


def _planner_funcs():
    tree = ast.parse(open(PLANNER).read(), PLANNER)
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in NAMES]
    assert sorted(f.name for f in fns) == sorted(NAMES)
    mod = ast.Module(body=fns, type_ignores=[])
    ns = {"np": np}
    exec(compile(mod, PLANNER, "exec"), ns)  # noqa: S102 - the five pure-numpy functions only
    return ns


def _stub():
    spec = importlib.util.spec_from_file_location("torch_utils_stub", STUB)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _quats(n, rng):
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    q[:8] = [[0, 0, 0, 1], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0],  # identities / half turns
             [np.sqrt(0.5), 0, 0, np.sqrt(0.5)], [0, np.sqrt(0.5), 0, np.sqrt(0.5)],  # gimbal: pitch = pi/2
             [0, -np.sqrt(0.5), 0, np.sqrt(0.5)], [0, 0, np.sqrt(0.5), np.sqrt(0.5)]]
    return q


def test_quat_apply_and_inverse_match_planner_copies():
    P, S = _planner_funcs(), _stub()
    rng = np.random.default_rng(0)
    q, v = _quats(4096, rng), rng.normal(size=(4096, 3))
    np.testing.assert_allclose(S.quat_apply(torch.from_numpy(q), torch.from_numpy(v)).numpy(), P["quat_apply"](q, v),
                               rtol=1e-12, atol=1e-12)
    # quat_rotate_inverse (torch_utils) == the planner's quat_apply_inverse for unit quaternions
    np.testing.assert_allclose(S.quat_rotate_inverse(torch.from_numpy(q), torch.from_numpy(v)).numpy(),
                               P["quat_apply_inverse"](q, v), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(S.quat_rotate(torch.from_numpy(q), torch.from_numpy(v)).numpy(),
                               P["quat_apply"](q, v), rtol=1e-12, atol=1e-12)


def test_euler_conversions_match_planner_copies():
    P, S = _planner_funcs(), _stub()
    rng = np.random.default_rng(1)
    q = _quats(4096, rng)
    got = [x.numpy() for x in S.get_euler_xyz(torch.from_numpy(q))]
    want = P["get_euler_xyz"](q)
    for g, w in zip(got, want):
        d = np.abs(g - w)
        d = np.minimum(d, 2 * np.pi - d)  # angles mod 2 pi: 0 and 2 pi are the same angle
        # Isaac Gym's copysign builds pi / 2 as a float32 tensor (the stub does the same), the
        # planner's numpy copy in float64: the gimbal-lock rows (|sin p| >= 1) differ by that rounding
        gimbal = np.abs(2.0 * (q[:, 3] * q[:, 1] - q[:, 2] * q[:, 0])) >= 1
        assert d[~gimbal].max() < 1e-9, d[~gimbal].max()
        assert d[gimbal].max() <= abs(float(np.float32(np.pi / 2)) - np.pi / 2) * 1.01
    r, p, y = (rng.uniform(-np.pi, np.pi, 4096) for _ in range(3))
    np.testing.assert_allclose(S.quat_from_euler_xyz(*(torch.from_numpy(x) for x in (r, p, y))).numpy(),
                               P["quat_from_euler_xyz"](r, p, y).T, rtol=1e-12, atol=1e-12)
