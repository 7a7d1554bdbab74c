"""One-shot P2P all-reduce (csrc/kernels/p2p.hip) - multi-process on whatever GPUs exist.

Ranks share a GPU when there are fewer GPUs than ranks: the IPC-mapped staging buffers and the
cross-process flag protocol are the same code as on an 8-GPU xGMI node, so a one-GPU box runs the
real multi-process path (RCCL itself refuses two ranks per GPU).  Results must equal the fp32
rank-order sum bit for bit, for fp32 and bf16, sum and average, sizes from 16 B to the slot size,
back-to-back ops of varying size, and hipGraph replays; a missing peer must end the kernel after
its timeout with the error word set (no hang)."""
import os
import subprocess
import sys

import pytest

import p2p_workers as W
from conftest import ROOT, free_port
from ringdp.multiprocessing import spawn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4])
def test_p2p_allreduce_exact(tmp_path, world):
    spawn(W.standalone_worker, args=(world, free_port(), str(tmp_path)), nprocs=world)
    counts = [int((tmp_path / f"r{r}").read_text()) for r in range(world)]
    assert len(set(counts)) == 1 and counts[0] > 60


def test_p2p_allreduce_missing_peer_times_out(tmp_path):
    spawn(W.timeout_worker, args=(2, free_port(), str(tmp_path)), nprocs=2)
    r0 = (tmp_path / "r0").read_text()
    assert r0.startswith("failed=True"), r0
    assert float(r0.split("dt=")[1]) < 10


def test_rccl_pg_routes_small_buckets_to_p2p():
    """World size 1 through the real RcclPG: the P2P path is set up, serves eligible all-reduces
    and DDP buckets (also inside a hipGraph), and RCCL still serves the rest."""
    code = r'''
import os, torch
import ringdp.distributed as dist
from ringdp.models import ConvNet
from ringdp.nn import CrossEntropyLoss
from ringdp.optim import SGD
from ringdp.parallel import DistributedDataParallel as DDP
from ringdp.utils.graph import StepGraph
torch.cuda.set_device(0)
dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
t = torch.arange(4096, dtype=torch.float32, device="cuda")
dist.all_reduce(t, op=dist.ReduceOp.AVG)
pg = dist._default().rccl(0)
assert pg.p2p_max_bytes() == 1 << 20, pg.p2p_max_bytes()
assert torch.equal(t.cpu(), torch.arange(4096, dtype=torch.float32))
big = torch.ones(1 << 19, device="cuda")  # 2 MB > threshold: RCCL
dist.all_reduce(big)
assert torch.all(big == 1)
os.environ["RINGDP_DDP_FORCE_COMM"] = "1"
torch.manual_seed(0)
m = ConvNet().cuda()
ref = ConvNet().cuda(); ref.load_state_dict(m.state_dict())
ddp = DDP(m, device_ids=[0], bucket_cap_mb=0.3, first_bucket_mb=0.3)
opt = SGD(ddp.parameters(), lr=0.05); ropt = SGD(ref.parameters(), lr=0.05)
crit = CrossEntropyLoss()
x = torch.randint(0, 256, (256, 1, 28, 28), dtype=torch.uint8, device="cuda"); y = torch.randint(0, 10, (256,), device="cuda")
def step():
    l = crit(ddp(x), y); opt.zero_grad(set_to_none=True); l.backward(); opt.step(); return l
for _ in range(2):
    step()
g = StepGraph(step, warmup=1).capture()
for _ in range(3):
    g.replay()
for _ in range(6):
    l = crit(ref(x), y); ropt.zero_grad(set_to_none=True); l.backward(); ropt.step()
torch.cuda.synchronize()
for a, b in zip(m.parameters(), ref.parameters()):
    assert torch.equal(a, b), (a - b).abs().max()
print("P2P_OK")
'''
    env = dict(os.environ, RINGDP_P2P_ALLREDUCE_MAX_BYTES=str(1 << 20), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=180)
    assert r.returncode == 0 and "P2P_OK" in r.stdout, r.stderr[-3000:]
