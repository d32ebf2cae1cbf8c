"""bench.py --gpus N measures N ranks however it is started (a bare ``python bench.py --gpus 8``
used to benchmark one rank): without a launcher it runs N rank processes under torch.distributed.run
(decided before any GPU call); with a launcher whose WORLD_SIZE disagrees it exits non-zero."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_plan_launch_rules():
    assert bench.plan_launch(1, {}, [], "bench.py") == ("run", 1)
    how, cmd = bench.plan_launch(4, {}, ["--gpus", "4", "--steps", "3"], "/x/bench.py")
    assert how == "spawn"
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-5:] == ["/x/bench.py", "--gpus", "4", "--steps", "3"]
    assert bench.plan_launch(2, {"WORLD_SIZE": "2"}, [], "b") == ("run", 2)
    assert bench.plan_launch(8, {"WORLD_SIZE": "1"}, [], "b")[0] == "error"
    assert bench.plan_launch(1, {"WORLD_SIZE": "2"}, [], "b")[0] == "error"


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)


def test_bare_bench_spawns_n_ranks():
    r = _run(["--gpus", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["spawned"] for d in lines)


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr
