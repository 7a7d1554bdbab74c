"""Workers for tests/test_xgmi_gpu.py (module level: spawn imports them).

They drive the native XgmiPG directly (no Python collective layer) so every check pins the kernels:
results must equal the fp32 rank-order reference bit for bit."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402


def _data(rank, n, dtype, salt):
    g = torch.Generator().manual_seed(1000 * salt + rank)
    if dtype.is_floating_point:
        return (torch.randn(n, generator=g) * (rank + 1)).to(dtype)
    return torch.randint(-50, 50, (n,), generator=g).to(dtype)


def _expected(world, n, dtype, salt, average):
    """Rank-order sum in fp32 (fp64 for fp64, exact for ints), one rounding: what the kernels do."""
    acc_t = torch.float64 if dtype == torch.float64 else (torch.float32 if dtype.is_floating_point else torch.int64)
    acc = _data(0, n, dtype, salt).to(acc_t)
    for r in range(1, world):
        acc = acc + _data(r, n, dtype, salt).to(acc_t)
    if average:
        acc = acc * (1.0 / world) if dtype.is_floating_point else torch.div(acc, world, rounding_mode="trunc")
    return acc.to(dtype)


def _pg(rank, world, port, timeout_ms=20000):
    from ringdp._native import C

    dev = rank % torch.cuda.device_count()  # ranks share a GPU on a one-GPU box
    torch.cuda.set_device(dev)
    store = C.PrefixStore("t", C.TCPStore("127.0.0.1", port, world, rank == 0, 60000))
    return C, C.XgmiPG(store, rank, world, dev, timeout_ms), dev


def exact_worker(rank, world, port, result_dir):
    # small slots so the test reaches every path: one-shot <= 64 KB, two-shot above, and two-shot in
    # several pieces above world * 1 MB
    os.environ["RINGDP_XGMI_ONESHOT_KB"] = "64"
    os.environ["RINGDP_XGMI_SLOT_MB"] = "1"
    os.environ["RINGDP_XGMI_BLOCKS"] = "32"
    C, pg, dev = _pg(rank, world, port)
    cfg = pg.config()
    assert cfg["oneshot_max"] == 64 << 10 and cfg["slot_bytes"] == 1 << 20, cfg
    R = C.ReduceOp
    checks = 0
    salt = 0

    def allreduce(t, op):
        pg.allreduce([t], op).wait(True)

    # sizes: 16 B, tails that are not a 16-B multiple, one segment, multi-segment, the one-shot limit,
    # two-shot single piece, two-shot with several pieces and a ragged last chunk
    for dtype in (torch.float32, torch.bfloat16):
        es = torch.tensor([], dtype=dtype).element_size()
        for nbytes in (16, 28 if es == 4 else 30, 4096, 8192 * 5 + 48, 64 << 10, 377408, 1 << 20,
                       (3 << 20) + 48, (world << 20) * 2 + 4096 + 16):
            for average in (False, True):
                salt += 1
                n = nbytes // es
                t = _data(rank, n, dtype, salt).cuda()
                allreduce(t, R.AVG if average else R.SUM)
                want = _expected(world, n, dtype, salt, average)
                assert torch.equal(t.cpu(), want), (dtype, nbytes, average, (t.cpu().float() - want.float()).abs().max())
                checks += 1
    # other dtypes and reduce ops
    for dtype in (torch.float16, torch.float64, torch.int32, torch.int64, torch.int8, torch.uint8):
        for n in (5, 1000, 70000):
            salt += 1
            t = _data(rank, n, dtype, salt).cuda()
            allreduce(t, R.SUM)
            assert torch.equal(t.cpu(), _expected(world, n, dtype, salt, False)), (dtype, n)
            checks += 1
    for op, fn in ((R.MAX, torch.maximum), (R.MIN, torch.minimum)):
        for n in (33, 100000):
            salt += 1
            t = _data(rank, n, torch.float32, salt).cuda()
            allreduce(t, op)
            want = _data(0, n, torch.float32, salt)
            for r in range(1, world):
                want = fn(want, _data(r, n, torch.float32, salt))
            assert torch.equal(t.cpu(), want), op
            checks += 1
    # reduce-scatter / all-gather, aligned and ragged per-rank blocks
    for m in (4, 7, 4096, 300001):
        salt += 1
        inp = _data(rank, m * world, torch.float32, salt).cuda()
        out = torch.zeros(m, device="cuda")
        pg.reduce_scatter_tensor(out, inp, R.SUM).wait(True)
        full = _expected(world, m * world, torch.float32, salt, False)
        assert torch.equal(out.cpu(), full[rank * m:(rank + 1) * m]), m
        ag = torch.zeros(m * world, device="cuda")
        pg.allgather_into_tensor(ag, out).wait(True)
        assert torch.equal(ag.cpu(), full), m
        checks += 2
    # back-to-back ops of varying size and kind on one stream, no host sync in between
    outs = []
    for k in range(48):
        salt += 1
        n = [64, 20000, 4, 100000, 400000, 3][k % 6]
        t = _data(rank, n, torch.float32, salt).cuda()
        pg.allreduce([t], R.SUM).wait(False)
        outs.append((t, n, salt))
        if k % 5 == 0:
            pg.barrier().wait(False)
    torch.cuda.synchronize()
    for t, n, s in outs:
        assert torch.equal(t.cpu(), _expected(world, n, torch.float32, s, False))
        checks += 1
    # broadcast from every root; send/recv around the ring
    for root in range(world):
        t = torch.full((5000,), float(rank), device="cuda")
        pg.broadcast([t], root).wait(True)
        assert torch.all(t == root)
        checks += 1
    if world > 1:
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        for n in (3, 70000, 600000):
            buf = torch.zeros(n, device="cuda")
            w1 = pg.send(torch.full((n,), float(rank), device="cuda"), nxt, 0)
            w2 = pg.recv(buf, prv, 0)
            w1.wait(True)
            w2.wait(True)
            assert torch.all(buf == prv), n
            checks += 1
        # unaligned (t[1:] views) messages larger than two P2P slots, two sends posted before their
        # recvs: the scratch staging of an unaligned send must not hold the comm stream
        n = 3 * (1 << 20) // 4
        srcs = [torch.arange(n + 1, device="cuda", dtype=torch.float32) + 1000.0 * rank + 0.5 * j for j in range(2)]
        dsts = [torch.zeros(n + 1, device="cuda") for _ in range(2)]
        ws = [pg.send(srcs[j][1:], nxt, 0) for j in range(2)]
        ws += [pg.recv(dsts[j][1:], prv, 0) for j in range(2)]
        for w in ws:
            w.wait(True)
        for j in range(2):
            exp = torch.arange(n + 1, dtype=torch.float32)[1:] + 1000.0 * prv + 0.5 * j
            assert torch.equal(dsts[j][1:].cpu(), exp), j
            checks += 1
    # hipGraph: capture once (one-shot + two-shot), replay with fresh inputs copied into the captured tensors
    small = torch.zeros(94352 // 8, device="cuda")  # one-shot
    big = torch.zeros(300000, device="cuda")         # two-shot
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            pg.allreduce([small], R.AVG).wait(False)
            pg.allreduce([big], R.SUM).wait(False)
    torch.cuda.synchronize()
    for k in range(5):
        salt += 1
        small.copy_(_data(rank, small.numel(), torch.float32, salt).cuda())
        big.copy_(_data(rank, big.numel(), torch.float32, salt + 1000).cuda())
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(small.cpu(), _expected(world, small.numel(), torch.float32, salt, True)), k
        assert torch.equal(big.cpu(), _expected(world, big.numel(), torch.float32, salt + 1000, False)), k
        checks += 2
    # eager op straight after replays, then replays again (join_into keeps the issue order)
    t = torch.ones(1000, device="cuda")
    pg.allreduce([t], R.SUM).wait(False)
    g.replay()
    torch.cuda.synchronize()
    assert torch.all(t == world)
    assert pg.backend_failure() == "", pg.backend_failure()
    pg.barrier().wait(True)
    pg.shutdown()
    with open(os.path.join(result_dir, f"r{rank}"), "w") as f:
        f.write(str(checks))


def timeout_worker(rank, world, port, result_dir):
    """Rank 1 skips the second op: rank 0's kernel must give up after the timeout and its blocking
    wait must raise instead of returning unreduced data."""
    os.environ["RINGDP_ASYNC_ERROR_HANDLING"] = "0"  # raise instead of tearing the process down
    C, pg, dev = _pg(rank, world, port, timeout_ms=1500)
    t = torch.ones(1024, device="cuda")
    pg.allreduce([t], C.ReduceOp.SUM).wait(True)
    assert torch.all(t == world)
    res = "skipped"
    if rank == 0:
        t0 = time.time()
        try:
            pg.allreduce([t], C.ReduceOp.SUM).wait(True)
            res = "returned"
        except Exception as e:  # noqa: BLE001
            res = f"raised dt={time.time() - t0:.2f} {type(e).__name__}: {e}"
    store = C.PrefixStore("done", C.TCPStore("127.0.0.1", port, world, False, 60000))
    store.set(f"done/{rank}", "1")
    store.wait([f"done/{r}" for r in range(world)])
    with open(os.path.join(result_dir, f"r{rank}"), "w") as f:
        f.write(res)
    os._exit(0)  # the failed group holds a kernel-timeout state; skip its teardown
