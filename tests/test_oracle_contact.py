"""The implicit-contact added mass of the oracle (oracle/go1_oracle.c point_inertia), against a
numpy construction of the same spatial inertia: a point mass matrix Mp (world) at local point lp
of a link with rotation R is, about the link origin in link coordinates,
[[S M S^T, S M], [M S^T, M]] with M = R^T Mp R and S = lp~ (S v = lp x v).  The HIP kernel builds
the same blocks in packed form (go1_step.hip, contact block of phys_substep); tests/test_gpu_parity.py
checks the resulting dynamics against the oracle."""
import ctypes as C

import numpy as np

from oracle import oracle as O


def _skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def _contact_mass(n, cn, cd):
    """Mp = cn n n^T + cd (I - n n^T) (oracle sphere_contact_im, one active layer)."""
    n = n / np.linalg.norm(n)
    return cn * np.outer(n, n) + cd * (np.eye(3) - np.outer(n, n))


def test_point_inertia_matches_spatial_construction():
    lib = O.lib("f64")
    lib.go1o_point_inertia.argtypes = [C.c_void_p] * 4
    rng = np.random.default_rng(4)
    for _ in range(20):
        q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        R = q * np.sign(np.linalg.det(q))
        lp = rng.normal(0, 0.2, 3)
        Mp = _contact_mass(rng.normal(size=3), rng.uniform(0.1, 1.0), rng.uniform(0.0, 0.3))
        out = np.zeros(36)
        args = [np.ascontiguousarray(x, np.float64) for x in (R.ravel(), lp, Mp.ravel())]
        lib.go1o_point_inertia(*(a.ctypes.data for a in args), out.ctypes.data)
        M = R.T @ Mp @ R
        S = _skew(lp)
        want = np.block([[S @ M @ S.T, S @ M], [M @ S.T, M]])
        np.testing.assert_allclose(out.reshape(6, 6), want, rtol=1e-12, atol=1e-14)
        # symmetric positive semi-definite: an added mass never removes inertia
        assert np.allclose(want, want.T) and np.linalg.eigvalsh(want).min() > -1e-12


def test_point_inertia_work_equals_point_kinetic_energy():
    """v^T I v = (v_p)^T Mp v_p for the point velocity v_p = R (v + w x lp) of a spatial velocity (w, v)."""
    lib = O.lib("f64")
    lib.go1o_point_inertia.argtypes = [C.c_void_p] * 4
    rng = np.random.default_rng(5)
    q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
    R = q * np.sign(np.linalg.det(q))
    lp = np.array([0.0, 0.0, -0.213])
    Mp = _contact_mass(np.array([0.1, -0.2, 1.0]), 0.9, 0.3)
    out = np.zeros(36)
    args = [np.ascontiguousarray(x, np.float64) for x in (R.ravel(), lp, Mp.ravel())]
    lib.go1o_point_inertia(*(a.ctypes.data for a in args), out.ctypes.data)
    I6 = out.reshape(6, 6)
    for _ in range(10):
        v6 = rng.normal(size=6)
        vp = R @ (v6[3:] + np.cross(v6[:3], lp))
        np.testing.assert_allclose(v6 @ I6 @ v6, vp @ Mp @ vp, rtol=1e-12)
