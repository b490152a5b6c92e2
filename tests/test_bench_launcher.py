"""bench.py's own N-rank launch: ``python bench.py --gpus N`` (the driver's
command form) must run N ranks even without an outer torchrun, start them
before anything touches the GPU, and refuse a WORLD_SIZE that disagrees with
--gpus.  CPU only: the ranks stop at the ZHIP_BENCH_DRY hook, before any
device work."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_plan():
    assert bench.rank_plan(1, {}) == "run"
    assert bench.rank_plan(4, {}) == "launch"
    assert bench.rank_plan(2, {"WORLD_SIZE": "2"}) == "run"
    assert bench.rank_plan(1, {"WORLD_SIZE": "1"}) == "run"
    with pytest.raises(ValueError):
        bench.rank_plan(8, {"WORLD_SIZE": "1"})


def test_launcher_cmd_is_the_driver_form():
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "5"], 8, 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert cmd[-5].endswith("bench.py")


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launches_n_ranks(n):
    env = dict(os.environ, ZHIP_BENCH_DRY="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    assert json.loads(lines[0]) == {"n_gpus": n, "gpus_arg": n}


def test_bench_refuses_mismatched_world():
    env = dict(os.environ, ZHIP_BENCH_DRY="1", WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
