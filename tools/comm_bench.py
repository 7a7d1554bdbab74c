#!/usr/bin/env python3
"""All-reduce latency / bandwidth sweep on ringdp's GPU process groups: RCCL, RCCL with its small
all-reduces on the xGMI one-shot kernel, and the "xgmi" backend (ringdp's own kernels for every size).

Sizes default to the DDP buckets that matter here: the ConvNet's two rebuilt
buckets (77 KB, 377 KB) and its whole gradient (455 KB), then 1 / 4 / 25 MB.  For every size and
dtype it times, per rank, a hipGraph of ``--reps`` back-to-back all-reduces (no launch overhead:
what a captured training step sees) and reports the max over ranks as us/op plus algbw
(S/t) and busbw (2(N-1)/N * S/t, the per-GPU ring traffic rate).

  python tools/comm_bench.py --gpus 8                        # launches 8 ranks itself (ringdp.run)
  python tools/comm_bench.py --gpus 8 --sweep                # + NCCL_ALGO / channel variants
  python -m ringdp.run --nproc-per-node 8 tools/comm_bench.py
  python tools/comm_bench.py --gpus 8 --sweep --recommend comm_tuning.json   # + the settings bench.py adopts

The "rccl+xgmi_small" rows exist when RINGDP_P2P_ALLREDUCE_MAX_BYTES is set (this tool sets 4 MiB
unless told otherwise); the crossover between them and the "rccl" rows is the threshold to use for
RINGDP_P2P_ALLREDUCE_MAX_BYTES in training; ``--recommend PATH`` writes that threshold and the fastest RCCL
variant of the sweep as environment settings, which ``bench.py`` adopts at the same world size (its
``--comm-tuning``, default ``comm_tuning.json``).  ``--backend xgmi``: every all-reduce on the xgmi backend
(ranks may share a GPU: rank r uses GPU r % device_count, so a one-GPU box runs --gpus 2/4, which RCCL
refuses).  Rank 0 prints one JSON line per measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SWEEP = [
    {},
    {"NCCL_ALGO": "Ring"},
    {"NCCL_ALGO": "Tree"},
    {"NCCL_PROTO": "LL"},
    {"NCCL_PROTO": "LL128"},
    {"NCCL_MIN_NCHANNELS": "16"},
    {"NCCL_MIN_NCHANNELS": "32"},
]


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--sizes", type=str, default="77312,377408,454720,1048576,4194304,26214400",
                    help="bytes, comma separated")
    ap.add_argument("--dtypes", type=str, default="fp32,bf16")
    ap.add_argument("--reps", type=int, default=20, help="all-reduces per graph")
    ap.add_argument("--iters", type=int, default=20, help="timed graph replays")
    ap.add_argument("--sweep", action="store_true", help="repeat under each RCCL env variant (parent mode)")
    ap.add_argument("--recommend", type=str, default=None,
                    help="write the recommended RINGDP_P2P_ALLREDUCE_MAX_BYTES / RCCL settings (JSON) here")
    ap.add_argument("--backend", type=str, default=None, choices=["rccl", "xgmi"],
                    help="GPU backend (default: RINGDP_GPU_BACKEND, else rccl)")
    return ap.parse_args()


def worker(args):
    import torch

    import ringdp.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if os.environ.get("WORLD_SIZE"):
        dist.init_process_group("nccl")
    else:
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", local)
    probe = torch.zeros(1, device=dev)
    dist.all_reduce(probe)
    pg = dist._default().gpu(local)
    if pg.backend_name() == "xgmi":
        impls = ["xgmi"]
    else:
        impls = ["rccl"] + (["rccl+xgmi_small"] if pg.p2p_max_bytes() > 0 else [])
    variant = {k: os.environ[k] for k in ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS") if k in os.environ}
    # where the numbers were measured: bench.py adopts a recommendation only on the same device / host / RCCL
    ident = {"arch": torch.cuda.get_device_properties(dev).gcnArchName, "host": socket.gethostname(),
             "rccl": ".".join(str(v) for v in torch.cuda.nccl.version())}
    # The first timed measurement of a process ran several times slower whatever its size (ranks sharing
    # a GPU settle their queues / clocks): one untimed pass of the first size goes before the sweep.
    first = max(1, int(args.sizes.split(",")[0]) // 4)
    w = torch.ones(first, dtype=torch.float32, device=dev)
    for _ in range(50):
        dist.all_reduce(w, op=dist.ReduceOp.AVG)
    torch.cuda.synchronize()
    s0 = torch.cuda.Stream()
    g0 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s0), torch.cuda.graph(g0, stream=s0):
        for _ in range(args.reps):
            dist.all_reduce(w, op=dist.ReduceOp.AVG)
    for _ in range(args.iters):
        g0.replay()
    torch.cuda.synchronize()
    dist.barrier()
    del g0
    for dt_name in args.dtypes.split(","):
        dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[dt_name]
        es = torch.tensor([], dtype=dtype).element_size()
        for nbytes in (int(s) for s in args.sizes.split(",")):
            n = max(1, nbytes // es)
            t = torch.ones(n, dtype=dtype, device=dev)
            for impl in impls:
                if impl == "rccl+xgmi_small" and nbytes > pg.p2p_max_bytes():
                    continue
                if impl != "xgmi":
                    pg.set_p2p_enabled(impl == "rccl+xgmi_small")
                for _ in range(3):
                    dist.all_reduce(t, op=dist.ReduceOp.AVG)
                torch.cuda.synchronize()
                s = torch.cuda.Stream()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                    for _ in range(args.reps):
                        dist.all_reduce(t, op=dist.ReduceOp.AVG)
                for _ in range(3):  # warm replays: the first ones pay graph upload / first-touch costs
                    g.replay()
                torch.cuda.synchronize()
                dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.iters):
                    g.replay()
                torch.cuda.synchronize()
                el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
                dist.all_reduce(el, op=dist.ReduceOp.MAX)
                us = float(el.item()) * 1e6 / (args.iters * args.reps)
                ok = bool(torch.all(t == 1).item())  # average of ones stays one
                if rank == 0:
                    algbw = nbytes / (us * 1e-6) / 1e9
                    line = json.dumps({"impl": impl, "world": world, "dtype": dt_name, "bytes": nbytes,
                                       "us_per_op": round(us, 2), "algbw_GBps": round(algbw, 2),
                                       "busbw_GBps": round(algbw * 2 * (world - 1) / max(world, 1), 2),
                                       "correct": ok, "rccl_env": variant, "identity": ident})
                    print(line, flush=True)
                    if os.environ.get("RINGDP_COMM_BENCH_OUT"):  # the parent's --recommend collects these
                        with open(os.environ["RINGDP_COMM_BENCH_OUT"], "a") as f:
                            f.write(line + "\n")
                del g
    if pg.backend_name() != "xgmi":
        pg.set_p2p_enabled(True)
    dist.destroy_process_group()


def recommend(rows, world):
    """Settings for training from the sweep's rows (fp32, correct results only): the RCCL variant with the
    least total time over the measured sizes, and the largest size up to which the xGMI one-shot kernel
    beats RCCL at every size (0: RCCL for every size)."""
    rows = [r for r in rows if r["dtype"] == "fp32" and r["correct"] and r["world"] == world]
    variants = {}
    for r in rows:
        if r["impl"] == "rccl":
            key = json.dumps(r["rccl_env"], sort_keys=True)
            variants.setdefault(key, {})[r["bytes"]] = r["us_per_op"]
    sizes = sorted({b for v in variants.values() for b in v})
    full = {k: v for k, v in variants.items() if sorted(v) == sizes}
    best = min(full, key=lambda k: sum(full[k].values())) if full else "{}"
    env = dict(json.loads(best))
    small = {r["bytes"]: r["us_per_op"] for r in rows if r["impl"] == "rccl+xgmi_small"
             and json.dumps(r["rccl_env"], sort_keys=True) == best}
    thresh = 0
    for b in sizes:
        if b in small and b in full.get(best, {}) and small[b] < full[best][b]:
            thresh = b
        else:
            break
    env["RINGDP_P2P_ALLREDUCE_MAX_BYTES"] = str(thresh)
    idents = {json.dumps(r.get("identity"), sort_keys=True) for r in rows}
    ident = json.loads(idents.pop()) if len(idents) == 1 else None  # mixed or unknown: adopt nowhere
    return {"world": world, "env": env, "identity": ident,
            "evidence": {"rccl_us_by_variant": {k: full[k] for k in full},
                         "xgmi_small_us": small, "chosen_variant": best}}


def main():
    args = parse()
    os.environ.setdefault("RINGDP_P2P_ALLREDUCE_MAX_BYTES", str(4 << 20))
    if args.backend:
        os.environ["RINGDP_GPU_BACKEND"] = args.backend
    if os.environ.get("WORLD_SIZE") is None and (args.gpus > 1 or args.sweep):
        from ringdp.run import launch_local

        argv = [a for a in sys.argv[1:] if a != "--sweep"]
        out = None
        if args.recommend:
            out = os.path.abspath(args.recommend) + ".rows.jsonl"
            if os.path.exists(out):
                os.remove(out)
        rc = 0
        for env in (SWEEP if args.sweep else [{}]):
            env = dict(env, RINGDP_COMM_BENCH_OUT=out) if out else env
            rc = launch_local(os.path.abspath(__file__), argv, args.gpus, env=env) or rc
        if out and os.path.exists(out):
            rows = [json.loads(ln) for ln in open(out) if ln.strip()]
            rec = recommend(rows, args.gpus)
            with open(args.recommend, "w") as f:
                json.dump(rec, f, indent=1)
            print(json.dumps({"recommendation": rec["env"], "path": args.recommend}), flush=True)
        sys.exit(rc)
    worker(args)


if __name__ == "__main__":
    main()
