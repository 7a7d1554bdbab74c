"""CPU rehearsal of tests/test_multigpu_gpu.py: the same multi-rank workers on host-ring ("gloo")
ranks, so the harness logic (equivalence reference, per-step replica checks, bucket-order
agreement under perturbed readiness) is itself tested where no multi-GPU node is available."""
import os

import pytest
import torch

import mgpu_workers as W
from conftest import free_port
from ringdp.multiprocessing import spawn

pytestmark = pytest.mark.slow


def test_collectives_cpu(tmp_path):
    spawn(W.collectives_worker, args=(3, free_port(), str(tmp_path), "cpu"), nprocs=3)
    assert sorted(os.listdir(tmp_path)) == ["r0", "r1", "r2"]


@pytest.mark.parametrize("name,perturb", [("convnet", False), ("convnet", True), ("resnet18", False)])
def test_ddp_equivalence_cpu(tmp_path, name, perturb):
    world = 2
    spawn(W.ddp_train_worker, args=(world, free_port(), str(tmp_path), "cpu", name, False, perturb), nprocs=world)
    res = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    assert all(all(r["same"]) for r in res)
    assert all(r["same_buckets"] for r in res)
    r0 = res[0]
    err = float((r0["ddp"] - r0["ref"]).abs().max())
    upd = float((r0["ref"] - r0["init"]).abs().max())
    assert err <= 1e-4 * upd + 1e-6, (err, upd)
