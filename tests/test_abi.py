"""C-ABI library: loads without a GPU, exports every entry point of include/go1_mi355x.h,
and its struct layouts match the ctypes mirror (no compute calls)."""
import ctypes as C
import os
import re

import pytest

from legged_tracking_amd import abi, native

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "go1_mi355x.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(go1_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    lib = native.lib()
    names = declared_functions()
    assert "go1_step" in names and "go1_create" in names and len(names) >= 9
    for n in names:
        assert hasattr(lib, n), n


def test_struct_layouts_match_ctypes_mirror():
    lib = native.lib()
    out = (C.c_int64 * 4)()
    lib.go1_abi_sizes(out)
    assert list(out) == [C.sizeof(abi.Go1Config), C.sizeof(abi.Go1State), C.sizeof(abi.Go1Terrain),
                         C.sizeof(abi.Go1StepArgs)]


def test_argument_errors_are_reported_not_thrown():
    lib = native.lib()
    h = C.c_void_p()
    rc = lib.go1_create(None, C.byref(h))
    assert rc == -1
    assert b"null" in lib.go1_last_error()
    bad = abi.Go1Config()
    bad.n_envs = 0
    assert lib.go1_create(C.byref(bad), C.byref(h)) == -1
    assert lib.go1_step(None, None, None) == -1


def test_oracle_library_builds_and_loads():
    from oracle import oracle as O
    O.lib()
    assert O.lib().go1o_abi_version() == abi.GO1_ABI_VERSION
    assert O.lib("f32").go1o_abi_version() == abi.GO1_ABI_VERSION


def test_compiled_model_constants_match_model_block():
    """csrc/go1_model_consts.h (the integrator's compile-time Go1 constants) is generated from
    model.py; go1_create rejects a model block that differs from it, before touching the GPU."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "gen_model_consts.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    from legged_tracking_amd import config as CF
    lib = native.lib()
    h = C.c_void_p()
    cfg = CF.build_abi_config(CF.readme_config(n_envs=16, terrain="single_path", rows=2, cols=2))
    cfg.model[11] = cfg.model[11] * 1.5  # FL hip COM x
    assert lib.go1_create(C.byref(cfg), C.byref(h)) == -1
    assert b"compiled Go1 model" in lib.go1_last_error()
    cfg = CF.build_abi_config(CF.readme_config(n_envs=16, terrain="single_path", rows=2, cols=2))
    cfg.hard_limits[7] = cfg.hard_limits[7] + 0.1
    assert lib.go1_create(C.byref(cfg), C.byref(h)) == -1
    assert b"hard joint limits" in lib.go1_last_error()
