"""Workers for tests/test_p2p_allreduce_gpu.py (module level: spawn imports them)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402


def _data(rank, n, dtype, salt):
    g = torch.Generator().manual_seed(1000 * salt + rank)
    return (torch.randn(n, generator=g) * (rank + 1)).to(dtype)


def _expected(world, n, dtype, salt, average):
    acc = _data(0, n, dtype, salt).float()
    for r in range(1, world):
        acc = acc + _data(r, n, dtype, salt).float()  # rank order, fp32: what the kernel does
    if average:
        acc = acc * (1.0 / world)
    return acc.to(dtype)


def standalone_worker(rank, world, port, result_dir):
    from ringdp._native import C

    ngpu = torch.cuda.device_count()
    dev = rank % ngpu  # ranks may share a GPU: IPC works within one device, RCCL would refuse
    torch.cuda.set_device(dev)
    store = C.PrefixStore("t", C.TCPStore("127.0.0.1", port, world, rank == 0, 60000))
    p2p = C.P2PAllReduce(store, rank, world, dev, 1 << 20, 20000)
    checks = 0
    salt = 0
    # sizes: one 16-B vector, sub-segment, multi-segment with a partial tail, the full slot
    for dtype in (torch.float32, torch.bfloat16):
        es = torch.tensor([], dtype=dtype).element_size()
        for nbytes in (16, 4096, 8192, 8192 * 5 + 48, 377408, 1 << 20):
            for average in (False, True):
                salt += 1
                n = nbytes // es
                t = _data(rank, n, dtype, salt).cuda()
                p2p.run(t, average)
                torch.cuda.synchronize()
                want = _expected(world, n, dtype, salt, average)
                assert torch.equal(t.cpu(), want), (dtype, nbytes, average, (t.cpu().float() - want.float()).abs().max())
                checks += 1
    # many back-to-back ops of varying size on one stream (epoch parity per segment, no host sync)
    outs = []
    for k in range(40):
        salt += 1
        n = [64, 20000, 4, 100000][k % 4]
        t = _data(rank, n, torch.float32, salt).cuda()
        p2p.run(t, False)
        outs.append((t, n, salt))
    torch.cuda.synchronize()
    for t, n, s in outs:
        assert torch.equal(t.cpu(), _expected(world, n, torch.float32, s, False))
        checks += 1
    # hipGraph: capture once, replay with fresh inputs copied into the captured tensor
    n = 94352  # ConvNet's first bucket (fp32 elements)
    static = torch.zeros(n, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            p2p.run(static, True)
    for k in range(5):
        salt += 1
        static.copy_(_data(rank, n, torch.float32, salt).cuda())
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(static.cpu(), _expected(world, n, torch.float32, salt, True)), k
        checks += 1
    assert not p2p.failed()
    with open(os.path.join(result_dir, f"r{rank}"), "w") as f:
        f.write(str(checks))


def timeout_worker(rank, world, port, result_dir):
    """Rank 1 skips the second op: rank 0's kernel must give up after its timeout and flag it."""
    from ringdp._native import C

    torch.cuda.set_device(0)
    store = C.PrefixStore("t", C.TCPStore("127.0.0.1", port, world, rank == 0, 60000))
    p2p = C.P2PAllReduce(store, rank, world, 0, 1 << 16, 1500)
    t = torch.ones(1024, device="cuda")
    p2p.run(t, False)
    torch.cuda.synchronize()
    assert torch.all(t == world)
    res = "skipped"
    if rank == 0:
        import time

        t0 = time.time()
        p2p.run(t, False)
        torch.cuda.synchronize()
        res = f"failed={p2p.failed()} dt={time.time() - t0:.2f}"
    store.set(f"done/{rank}", "1")
    store.wait([f"done/{r}" for r in range(world)])
    with open(os.path.join(result_dir, f"r{rank}"), "w") as f:
        f.write(res)
