"""bench.py contract on CPU ranks (host-ring "gloo" backend, ATen ConvNet): the driver's two
launch forms - ``python bench.py --gpus N`` (bench starts its own N ranks through ringdp.run) and
``python -m torch.distributed.run ... bench.py --gpus N`` (torchrun agent store -> ringdp's native
TCPStore) - must both yield one JSON line from rank 0 with n_gpus == N and a comm world of N."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, free_port

pytestmark = pytest.mark.slow

ARGS = ["--cpu", "--steps", "2", "--warmup", "1", "--batch-per-rank", "8", "--comm-stats-steps", "1"]


def _run(cmd):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


def _check(res, n):
    assert res["n_gpus"] == n
    assert res["config"]["comm_world_size"] == n
    assert res["config"]["parallelism"] == f"dp{n}"
    assert res["config"]["global_batch"] == 8 * n
    assert res["value"] > 0 and res["ms_per_step"] > 0
    assert res["metric"].startswith("images/sec (whole node) MNIST ConvNet")
    assert "exposed_comm_ms" in res["comm_stats"]
    assert len(res["comm_stats"]["bucket_bytes"]) >= 1


def test_bench_single_rank_runs_comm_path():
    res = _run([sys.executable, "bench.py"] + ARGS)
    _check(res, 1)
    assert "forced" in res["config"]["comm"]  # N=1 runs the same all-reduce path as N>1


def test_bench_self_launches_n_ranks():
    res = _run([sys.executable, "bench.py", "--gpus", "2"] + ARGS)
    _check(res, 2)


def test_bench_under_torchrun_uses_native_store():
    res = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2"] + ARGS)
    _check(res, 2)
