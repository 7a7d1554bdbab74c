"""Multi-process CPU tests of the host-ring backend, DDP, spawn, debug and failure detection.

BASELINE config #1 (ConvNet DDP world_size=2 on CPU via spawn) is test_ddp_equivalence.
"""
import os
import time

import pytest
import torch

import dist_workers as W
from conftest import free_port
from ringdp.multiprocessing import ProcessExitedException, ProcessRaisedException, spawn

pytestmark = pytest.mark.slow


@pytest.mark.parametrize("world", [2, 3, 4])
def test_host_ring_collectives(world):
    spawn(W.collectives_worker, args=(world, free_port()), nprocs=world)


def _reference_train(world, momentum):
    """Single-process training on the full global batch (no DDP)."""
    from ringdp.models import ConvNet
    from ringdp.optim import SGD

    torch.manual_seed(5)  # == rank 0's init in the workers
    model = ConvNet()
    opt = SGD(model.parameters(), lr=0.05, momentum=momentum, nesterov=momentum > 0)
    xs, ys = W._convnet_batches(world, 4, 4)
    for x, y in zip(xs, ys):
        loss = torch.nn.functional.cross_entropy(model(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


@pytest.mark.parametrize("world,momentum,hook,bucket_mb,first_mb", [
    (2, 0.0, "allreduce", 25, None),        # reference W1 settings (plain SGD), BASELINE config #1
    (2, 0.9, "allreduce", 0.1, 0.05),       # several buckets after rebuild
    (3, 0.9, "python", 25, None),           # python comm hook
    (2, 0.0, "bf16", 25, None),             # bf16 wire compression
])
def test_ddp_equivalence(tmp_path, world, momentum, hook, bucket_mb, first_mb):
    spawn(W.ddp_equivalence_worker, args=(world, free_port(), str(tmp_path), momentum, hook, bucket_mb, first_mb),
          nprocs=world)
    res = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    assert all(r["same"] for r in res), "ranks diverged"
    assert all(r["rebuilt"] for r in res)
    ref = _reference_train(world, momentum)
    tol = 2e-2 if hook == "bf16" else 1e-4
    err = float((res[0]["flat"] - ref).abs().max())
    assert err < tol, err
    if bucket_mb < 1:
        assert len(res[0]["buckets"]) > 1


def _reference_join(world, hook, batches=W.JOIN_BATCHES):
    """One process: iteration i averages the gradients of the ranks that still have data over the
    initial world size (the semantics of DDP.join(divide_by_initial_world_size=True))."""
    from ringdp.models import ConvNet
    from ringdp.optim import SGD

    B = 4
    torch.manual_seed(5)
    model = ConvNet()
    opt = SGD(model.parameters(), lr=0.01, momentum=0.9)
    n = batches[:world]
    xs, ys = W._convnet_batches(world, B, max(n))
    for i in range(max(n)):
        loss = 0
        for r in range(world):
            if i < n[r]:
                loss = loss + torch.nn.functional.cross_entropy(model(xs[i][r * B:(r + 1) * B]),
                                                                ys[i][r * B:(r + 1) * B]) / world
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


@pytest.mark.parametrize("world,hook,batches", [(2, "allreduce", W.JOIN_BATCHES), (3, "allreduce", W.JOIN_BATCHES),
                                                (2, "bf16", W.JOIN_BATCHES),
                                                (3, "allreduce", (0, 4, 2))])  # rank 0 joins before iteration 0
def test_join_uneven_inputs(tmp_path, world, hook, batches):
    spawn(W.join_worker, args=(world, free_port(), str(tmp_path), hook, batches), nprocs=world)
    res = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    assert all(r["same"] for r in res), "final model sync from the last joiner failed"
    ref = _reference_join(world, hook, batches)
    err = float((res[0]["flat"] - ref).abs().max())
    assert err < (2e-2 if hook == "bf16" else 1e-4), err


def test_join_throw_on_early_termination(tmp_path):
    spawn(W.join_throw_worker, args=(2, free_port(), str(tmp_path)), nprocs=2)
    res = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(2)]
    assert all(r["raised"] for r in res)


def test_no_sync_accumulates(tmp_path):
    spawn(W.no_sync_worker, args=(2, free_port(), str(tmp_path)), nprocs=2)
    r0, r1 = (torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(2))
    assert torch.allclose(r0["g"], r1["g"])  # synced after the sync step
    assert not torch.allclose(r0["local"], r1["local"])  # but not during no_sync


@pytest.mark.parametrize("find_unused", [False, True])
def test_unused_parameters(tmp_path, find_unused):
    spawn(W.unused_param_worker, args=(2, free_port(), str(tmp_path), find_unused), nprocs=2)
    out = (tmp_path / "r0").read_text()
    if find_unused:
        assert out == "ok"
    else:
        assert out.startswith("error") and "find_unused_parameters" in out


def test_desync_detection(tmp_path):
    spawn(W.desync_worker, args=(2, free_port(), str(tmp_path)), nprocs=2)
    assert (tmp_path / "r0").read_text() == "desync"
    assert (tmp_path / "r1").read_text() == "desync"


def test_dead_peer_detected_within_timeout(tmp_path):
    spawn(W.hang_worker, args=(2, free_port(), str(tmp_path)), nprocs=2)
    res = (tmp_path / "r0").read_text()
    assert res.startswith("error"), res
    assert float(res.split()[1].rstrip("s")) < 15


def test_spawn_ok(tmp_path):
    spawn(W.spawn_ok, args=(str(tmp_path),), nprocs=3)
    assert sorted(os.listdir(tmp_path)) == ["ok0", "ok1", "ok2"]


def test_spawn_propagates_exception():
    t0 = time.time()
    with pytest.raises(ProcessRaisedException) as ei:
        spawn(W.spawn_raise, nprocs=2)
    assert "boom from child 1" in str(ei.value)
    assert time.time() - t0 < 25  # the sleeping peer was terminated


def test_spawn_propagates_exit_code():
    with pytest.raises(ProcessExitedException) as ei:
        spawn(W.spawn_exit, nprocs=2)
    assert ei.value.exit_code == 7 and ei.value.error_index == 0


def test_checkpoint_resume_bitwise(tmp_path):
    from ringdp.multiprocessing import spawn

    spawn(W.checkpoint_resume_worker, args=(2, str(tmp_path / "init"), str(tmp_path)), nprocs=2)
