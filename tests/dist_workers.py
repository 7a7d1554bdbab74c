"""Worker bodies for multi-process CPU tests (module-level so the spawn start method can import them)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402


def _init(rank, world, port, backend="gloo", timeout_s=60):
    import datetime

    import ringdp.distributed as dist

    torch.set_num_threads(1)
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s))
    return dist


def collectives_worker(rank, world, port):
    dist = _init(rank, world, port)
    R = dist.ReduceOp
    # all_reduce over dtypes / ops
    for dt in (torch.float32, torch.float64, torch.int64, torch.int32, torch.bfloat16, torch.float16):
        t = torch.full((1000,), rank + 1, dtype=dt)
        dist.all_reduce(t)
        assert torch.all(t == sum(range(1, world + 1))), (dt, t[:4])
    t = torch.tensor([float(rank)])
    dist.all_reduce(t, op=R.MAX)
    assert t.item() == world - 1
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=R.PRODUCT)
    import math
    assert t.item() == math.factorial(world)
    t = torch.tensor([float(rank)] * 7)
    dist.all_reduce(t, op=R.AVG)
    assert torch.allclose(t, torch.full((7,), (world - 1) / 2))
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t, op=R.MIN)
    assert t.item() == 1
    b = torch.tensor([1 << rank], dtype=torch.int64)
    dist.all_reduce(b, op=R.BOR)
    assert b.item() == (1 << world) - 1
    # odd sizes (uneven ring chunks) and empty
    for n in (1, 3, world * 5 + 1, 100003):
        t = torch.arange(n, dtype=torch.float32) * (rank + 1)
        dist.all_reduce(t)
        assert torch.allclose(t, torch.arange(n, dtype=torch.float32) * world * (world + 1) / 2)
    # broadcast from every root
    for root in range(world):
        t = torch.full((33,), float(rank))
        dist.broadcast(t, src=root)
        assert torch.all(t == root)
    big = torch.arange(3_000_000, dtype=torch.float32) if rank == 0 else torch.zeros(3_000_000)
    dist.broadcast(big, 0)
    assert float(big[-1]) == 2_999_999
    # all_gather / all_gather_into_tensor
    outs = [torch.zeros(4) for _ in range(world)]
    dist.all_gather(outs, torch.full((4,), float(rank)))
    assert all(torch.all(o == i) for i, o in enumerate(outs))
    out = torch.zeros(world * 3)
    dist.all_gather_into_tensor(out, torch.full((3,), float(rank)))
    assert torch.equal(out, torch.arange(world).float().repeat_interleave(3))
    # reduce_scatter_tensor
    inp = torch.arange(world * 4, dtype=torch.float32)
    out = torch.zeros(4)
    dist.reduce_scatter_tensor(out, inp)
    assert torch.equal(out, torch.arange(rank * 4, rank * 4 + 4).float() * world)
    # reduce / gather / scatter
    t = torch.ones(5) * (rank + 1)
    dist.reduce(t, dst=world - 1)
    if rank == world - 1:
        assert torch.all(t == world * (world + 1) / 2)
    g = [torch.zeros(2) for _ in range(world)] if rank == 0 else None
    dist.gather(torch.full((2,), float(rank)), g, dst=0)
    if rank == 0:
        assert all(torch.all(x == i) for i, x in enumerate(g))
    s = torch.zeros(3)
    dist.scatter(s, [torch.full((3,), float(i)) for i in range(world)] if rank == 0 else None, src=0)
    assert torch.all(s == rank)
    # all_to_all_single (even and uneven splits)
    inp = torch.arange(world, dtype=torch.float32) + rank * world
    out = torch.zeros(world)
    dist.all_to_all_single(out, inp)
    assert torch.equal(out, torch.tensor([float(r * world + rank) for r in range(world)]))
    in_splits = [r + 1 for r in range(world)]          # send r+1 rows to rank r
    out_splits = [rank + 1] * world                     # receive rank+1 rows from everyone
    inp = torch.cat([torch.full((r + 1, 2), float(rank)) for r in range(world)])
    out = torch.zeros(sum(out_splits), 2)
    dist.all_to_all_single(out, inp, out_splits, in_splits)
    assert torch.equal(out[:, 0], torch.cat([torch.full((rank + 1,), float(r)) for r in range(world)]))
    # point-to-point ring
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    sreq = dist.isend(torch.full((10,), float(rank)), nxt)
    buf = torch.zeros(10)
    dist.recv(buf, prv)
    sreq.wait()
    assert torch.all(buf == prv)
    # async op handles
    w = dist.all_reduce(torch.ones(10), async_op=True)
    w.wait()
    assert w.is_completed()
    # object collectives
    objs = [None] * world
    dist.all_gather_object(objs, {"rank": rank, "s": "x" * rank})
    assert [o["rank"] for o in objs] == list(range(world))
    lst = [f"hello{rank}", rank] if rank == 0 else [None, None]
    dist.broadcast_object_list(lst, src=0)
    assert lst == ["hello0", 0]
    # sub-groups (every rank calls new_group)
    even = dist.new_group([r for r in range(world) if r % 2 == 0])
    if rank % 2 == 0:
        t = torch.ones(3)
        dist.all_reduce(t, group=even)
        assert torch.all(t == len(range(0, world, 2)))
        assert dist.get_rank(even) == rank // 2
    else:
        assert even is dist.GroupMember.NON_GROUP_MEMBER
    dist.barrier()
    dist.monitored_barrier()
    dist.destroy_process_group()


def desync_worker(rank, world, port, result_dir):
    os.environ["RINGDP_DEBUG"] = "1"
    import importlib

    import ringdp.distributed as dist

    importlib.reload(dist)  # pick up the debug flag
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dist.all_reduce(torch.ones(4))  # matched
    try:
        if rank == 0:
            dist.all_reduce(torch.ones(8))
        else:
            dist.broadcast(torch.ones(8), 0)
        ok = "no-error"
    except RuntimeError as e:
        ok = "desync" if "desync" in str(e) else f"other: {e}"
    with open(os.path.join(result_dir, f"r{rank}"), "w") as f:
        f.write(ok)


def hang_worker(rank, world, port, result_dir):
    """rank 1 dies mid-job; rank 0's next collective must fail within the PG timeout."""
    dist = _init(rank, world, port, timeout_s=5)
    dist.all_reduce(torch.ones(10))
    if rank == 1:
        os._exit(0)  # vanish without a collective; spawn treats a clean exit as success
    t0 = time.time()
    try:
        dist.all_reduce(torch.ones(10))
        res = "no-error"
    except Exception as e:  # noqa: BLE001
        res = f"error {time.time() - t0:.1f}s {type(e).__name__}"
    with open(os.path.join(result_dir, f"r{rank}"), "w") as f:
        f.write(res)


def _convnet_batches(world, B, steps, seed=0):
    g = torch.Generator().manual_seed(seed)
    xs = [torch.randn(world * B, 1, 28, 28, generator=g) for _ in range(steps)]
    ys = [torch.randint(0, 10, (world * B,), generator=g) for _ in range(steps)]
    return xs, ys


def ddp_equivalence_worker(rank, world, port, result_dir, momentum, hook, bucket_mb, first_mb):
    """DDP over `world` ranks x B must equal one process over world*B."""
    dist = _init(rank, world, port)
    from ringdp.models import ConvNet
    from ringdp.optim import SGD
    from ringdp.parallel import DistributedDataParallel as DDP
    from ringdp.parallel import comm_hooks

    B, steps = 4, 4
    torch.manual_seed(rank * 1000 + 5)  # different init per rank: DDP must broadcast rank 0's
    model = ConvNet()
    ddp = DDP(model, bucket_cap_mb=bucket_mb, first_bucket_mb=first_mb)
    if hook == "bf16":
        ddp.register_comm_hook(None, comm_hooks.bf16_compress_hook)
    elif hook == "python":
        ddp.register_comm_hook(None, comm_hooks.allreduce_hook)
        ddp._python_hook = None
        def my_hook(state, bucket):
            return dist.all_reduce(bucket.buffer(), op=dist.ReduceOp.AVG, async_op=True)
        ddp.register_comm_hook(None, my_hook)
    opt = SGD(ddp.parameters(), lr=0.05, momentum=momentum, nesterov=momentum > 0)
    xs, ys = _convnet_batches(world, B, steps)
    for i in range(steps):
        x = xs[i][rank * B:(rank + 1) * B]
        y = ys[i][rank * B:(rank + 1) * B]
        loss = torch.nn.functional.cross_entropy(ddp(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    # every rank must hold bit-identical parameters
    allp = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(allp, flat)
    same = all(torch.equal(allp[0], a) for a in allp)
    info = ddp._get_ddp_logging_data()
    torch.save({"flat": flat, "same": same, "buckets": info["bucket_sizes"], "rebuilt": ddp.reducer.rebuilt()},
               os.path.join(result_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def no_sync_worker(rank, world, port, result_dir):
    dist = _init(rank, world, port)
    from ringdp.models import ConvNet
    from ringdp.parallel import DistributedDataParallel as DDP

    torch.manual_seed(0)
    model = ConvNet()
    ddp = DDP(model)
    xs, ys = _convnet_batches(world, 2, 2, seed=3)
    with ddp.no_sync():  # accumulate locally
        loss = torch.nn.functional.cross_entropy(ddp(xs[0][rank * 2:(rank + 1) * 2]), ys[0][rank * 2:(rank + 1) * 2])
        loss.backward()
    local_after_first = model.fc1.bias.grad.clone()
    loss = torch.nn.functional.cross_entropy(ddp(xs[1][rank * 2:(rank + 1) * 2]), ys[1][rank * 2:(rank + 1) * 2])
    loss.backward()
    torch.save({"g": model.fc1.bias.grad.clone(), "local": local_after_first}, os.path.join(result_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def unused_param_worker(rank, world, port, result_dir, find_unused):
    dist = _init(rank, world, port, timeout_s=20)
    from ringdp.parallel import DistributedDataParallel as DDP

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(4, 4)
            self.b = torch.nn.Linear(4, 4)  # unused

        def forward(self, x):
            return self.a(x)

    torch.manual_seed(0)
    net = Net()
    ddp = DDP(net, find_unused_parameters=find_unused)
    res = "ok"
    try:
        ddp(torch.randn(2, 4)).sum().backward()
        ddp(torch.randn(2, 4)).sum().backward()
    except RuntimeError as e:
        res = "error: " + str(e)[:200]
    with open(os.path.join(result_dir, f"r{rank}"), "w") as f:
        f.write(res)
    dist.destroy_process_group()


def spawn_ok(i, path):
    with open(os.path.join(path, f"ok{i}"), "w") as f:
        f.write(str(i))


def spawn_raise(i):
    if i == 1:
        raise ValueError("boom from child 1")
    time.sleep(30)


def spawn_exit(i):
    if i == 0:
        sys.exit(7)
    time.sleep(30)


def checkpoint_resume_worker(rank, world, init_file, out_dir):
    """Train 2 steps, save, 2 more; then a fresh model+optimizer resumes from the checkpoint and
    runs the same 2 steps: the parameters must match bit for bit."""
    import os

    import torch

    import ringdp
    import ringdp.distributed as dist
    from ringdp.models import ConvNet
    from ringdp.optim import SGD
    from ringdp.utils import checkpoint

    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(rank)
    xs = [torch.randn(4, 1, 28, 28, generator=g) for _ in range(4)]
    ys = [torch.randint(0, 10, (4,), generator=g) for _ in range(4)]

    def make():
        torch.manual_seed(0)
        m = ringdp.DistributedDataParallel(ConvNet())
        return m, SGD(m.parameters(), lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-4)

    def step(m, o, i):
        loss = torch.nn.functional.cross_entropy(m(xs[i]), ys[i])
        o.zero_grad()
        loss.backward()
        o.step()

    ckpt = os.path.join(out_dir, "ck.pt")
    m, o = make()
    step(m, o, 0)
    step(m, o, 1)
    checkpoint.save(ckpt, m, o, epoch=3, step=2)
    step(m, o, 2)
    step(m, o, 3)
    ref = [p.detach().clone() for p in m.parameters()]
    m2, o2 = make()
    meta = checkpoint.load(ckpt, m2, o2)
    assert meta == {"epoch": 3, "step": 2}, meta
    step(m2, o2, 2)
    step(m2, o2, 3)
    for a, b in zip(ref, m2.parameters()):
        assert torch.equal(a, b.detach()), (a - b).abs().max()
    # model-only resume: every rank still gets rank 0's meta
    m3, _ = make()
    meta3 = checkpoint.load(ckpt, m3)
    assert meta3 == {"epoch": 3, "step": 2}, (rank, meta3)
    dist.destroy_process_group()


JOIN_BATCHES = (5, 3, 4, 2)


def join_worker(rank, world, port, result_dir, hook, batches=JOIN_BATCHES):
    """Uneven inputs under DDP.join(): rank r trains on batches[r] batches."""
    dist = _init(rank, world, port)
    from ringdp.models import ConvNet
    from ringdp.optim import SGD
    from ringdp.parallel import DistributedDataParallel as DDP
    from ringdp.parallel import comm_hooks

    B = 4
    torch.manual_seed(5)
    model = ConvNet()
    ddp = DDP(model, bucket_cap_mb=0.1, first_bucket_mb=0.05)
    if hook == "bf16":
        ddp.register_comm_hook(None, comm_hooks.bf16_compress_hook)
    opt = SGD(ddp.parameters(), lr=0.01, momentum=0.9)
    steps = max(batches[:world])
    xs, ys = _convnet_batches(world, B, steps)
    with ddp.join():
        for i in range(batches[rank]):
            x = xs[i][rank * B:(rank + 1) * B]
            y = ys[i][rank * B:(rank + 1) * B]
            loss = torch.nn.functional.cross_entropy(ddp(x), y)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    allp = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(allp, flat)
    same = all(torch.equal(allp[0], a) for a in allp)
    torch.save({"flat": flat, "same": same}, os.path.join(result_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def join_throw_worker(rank, world, port, result_dir):
    dist = _init(rank, world, port)
    from ringdp.models import ConvNet
    from ringdp.parallel import DistributedDataParallel as DDP

    torch.manual_seed(5)
    ddp = DDP(ConvNet())
    xs, ys = _convnet_batches(world, 2, 3)
    raised = False
    try:
        with ddp.join(throw_on_early_termination=True):
            for i in range(1 if rank == 0 else 3):
                torch.nn.functional.cross_entropy(ddp(xs[i][:2]), ys[i][:2]).backward()
    except RuntimeError as e:
        raised = "throw_on_early_termination" in str(e)
    torch.save({"raised": raised}, os.path.join(result_dir, f"r{rank}.pt"))
    dist.destroy_process_group()
