"""bench.py's multi-rank launcher on CPU (gloo): `--gpus N` starts N ranks itself and the
printed line reports the world size the ranks actually saw."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ, **(env or {}))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if env is None or k not in env:
            e.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=120, env=e, cwd=REPO)


def test_launcher_spawns_two_ranks():
    r = _run(["--gpus", "2", "--selftest", "--steps", "5"])
    assert r.returncode == 0, r.stderr
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_size_seen"] == 2
    assert line["ranks"] == [0, 1]
    assert line["config"]["global_envs"] == 2 * 4096


def test_single_rank_selftest():
    r = _run(["--gpus", "1", "--selftest", "--steps", "5"])
    assert r.returncode == 0, r.stderr
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 1


def test_world_size_mismatch_fails_loudly():
    # an external launcher with one rank while --gpus says 2: refuse instead of printing n_gpus 1
    r = _run(["--gpus", "2", "--selftest", "--steps", "5"], env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
