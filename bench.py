#!/usr/bin/env python3
"""ringdp headline benchmark: MNIST ConvNet DDP training throughput (images/sec, whole job).

Metric/config from BASELINE.json: "images/sec (whole node) MNIST ConvNet at 1/2/4/8 MI355X; DDP
scaling efficiency" - reference workload W1 (ref/launch_dist.py: ConvNet, CrossEntropyLoss,
SGD lr 1e-4, DDP over NCCL, launch-style entrypoint), here on ringdp: bf16 MFMA kernels with fp32
master weights, C++ reducer + RCCL all-reduce over xGMI, fused SGD, whole step in a hipGraph.

Data: synthetic MNIST-shaped uint8 images + labels generated on the device (no dataset download
is possible offline); Normalize((0.1307,),(0.3081,)) is fused into the first conv kernel.
Weights: random init (torch.manual_seed(0), PyTorch default init - identical to the reference).
Scaling: weak (fixed per-rank batch), like the reference.
Per-rank batch: 65536 images (the reference runs 100; `--batch-per-rank 100` reproduces that regime).
The ConvNet is ~44 MFLOP/img, so a 100-image step is launch/latency-bound; 65536 fills 256 CUs and
amortises the 455 KB gradient all-reduce (activations ~3 GB of the 288 GB HBM3E).

Launch (one process per GPU, RCCL over xGMI):
  python bench.py --gpus N ...            N > 1 without WORLD_SIZE in the env: this process starts N
                                          fresh ranks itself (ringdp.run; ref/mpspawn_dist.py:136-140)
                                          and never touches the GPU
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
      bench.py --gpus N ...               the driver's form; ranks read RANK/LOCAL_RANK/WORLD_SIZE
  python -m ringdp.run --nproc-per-node N bench.py --gpus N ...

Comm backend: RCCL (backend "nccl"); RINGDP_GPU_BACKEND=xgmi selects ringdp's own collective
kernels over IPC-mapped peer memory instead (one node; ranks may then share a GPU, rank r using GPU
r % device_count, as ref/launch_dist.py:47 binds devices).

The gradient all-reduce runs at every N, including N=1 (a one-rank communicator, exactly what
upstream DDP does), so every point of the scaling curve executes the same code path;
``--no-force-comm`` skips it at N=1.  After the timed region (never inside it) the bench measures
per-bucket device-timed collective durations over a few eager steps and the step time of a
comm-free graph; their difference to the timed step is the exposed (non-overlapped) comm time.

``--cpu`` runs the same flow on CPU ranks over the native host-ring ("gloo") backend and the ATen
ConvNet: a plumbing rehearsal (BASELINE config #1), not a GPU measurement.

Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import socket
import sys
import time

import torch

METRIC = "images/sec (whole node) MNIST ConvNet at 1/2/4/8 MI355X; DDP scaling efficiency"

# Extra BASELINE.json configs (--model): the deeper families, synthetic data of the named shape.
MODELS = {
    # per-rank batch: throughput plateau on one MI355X (B=32768 16.09M, 49152 16.15M, 65536 16.25M, 131072
    # 16.22M img/s); 65536 also halves the exposed all-reduce share of the step at N > 1
    "convnet": dict(batch=65536, shape=(1, 28, 28), lr=1e-4, momentum=0.0, nesterov=False, wd=0.0,
                    # 455 KB of fp32 grads in two buckets: [fc1 + conv3] is all-reduced while conv2/conv1
                    # backward still run; only the small [conv2 + conv1] bucket is exposed at the end.
                    bucket_mb=0.3, first_bucket_mb=0.3,
                    desc="MNIST ConvNet (ref/launch_dist.py; 113,674 params)"),
    "resnet18": dict(batch=256, shape=(3, 32, 32), lr=0.02, momentum=0.9, nesterov=True, wd=1e-4,
                     desc="ResNet-18 CIFAR-shape (ref/example_mp.py; torchvision tree, 11,181,642 params)"),
    "resnet50": dict(batch=256, shape=(3, 224, 224), lr=0.02, momentum=0.9, nesterov=True, wd=1e-4,
                     desc="ResNet-50 ImageNet-shape (25,557,032 params)"),
    "vit_b_16": dict(batch=128, shape=(3, 224, 224), lr=0.01, momentum=0.9, nesterov=False, wd=0.0,
                     desc="ViT-B/16 ImageNet-shape (86,567,656 params, seq 197)"),
}
NUM_CLASSES = {"convnet": 10, "resnet18": 10, "resnet50": 1000, "vit_b_16": 1000}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", type=str, default="convnet", choices=sorted(MODELS))
    ap.add_argument("--batch-per-rank", type=int, default=None,
                    help="per-rank batch (default: 65536 for the ConvNet, RINGDP_BENCH_BATCH overrides)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--bucket-mb", type=float, default=None, help="bucket cap (default: per model, else 25)")
    ap.add_argument("--first-bucket-mb", type=float, default=None)
    ap.add_argument("--comm-hook", type=str, default="allreduce", choices=["allreduce", "bf16_compress", "fp16_compress"])
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of one hipGraph per step")
    ap.add_argument("--pool", type=int, default=8, help="number of distinct synthetic batches cycled")
    ap.add_argument("--dtype", type=str, default="bf16", choices=["bf16", "fp8", "fp32"],
                    help="fp8: e4m3 linear-layer GEMMs on the block-scaled MFMA (vit_b_16); "
                         "fp32: the ConvNet at the reference's precision (fp32 MFMA kernels)")
    ap.add_argument("--no-force-comm", action="store_true",
                    help="at world size 1 skip the bucket all-reduce (default: run it, the N>1 code path)")
    ap.add_argument("--comm-stream", type=str, default="split", choices=["split", "side", "same"],
                    help="placement of the bucket collectives of the captured step: split (default: the step is "
                         "captured as linear single-stream graph segments cut where buckets become ready, and each "
                         "bucket's collective runs between them on the comm stream, overlapping the rest of "
                         "backward), side (inside one graph on a side stream: a forked graph loses HIP's batched "
                         "launch, +1.2-2 us per kernel) or same (inside one graph on the compute stream: no overlap)")
    ap.add_argument("--comm-tuning", type=str, default=os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                     "comm_tuning.json"),
                    help="settings from tools/comm_bench.py --recommend, adopted when measured at this world size "
                         "(environment variables already set win)")
    ap.add_argument("--comm-stats-steps", type=int, default=20,
                    help="after the timed region: eager steps with device-timed bucket collectives and "
                         "comm-free graph replays for the exposed-comm estimate (0 = skip)")
    ap.add_argument("--cpu", action="store_true",
                    help="CPU ranks on the host-ring ('gloo') backend with the ATen ConvNet (plumbing only)")
    ap.add_argument("--local-rank", "--local_rank", type=int, default=None)
    return ap.parse_args(argv)


def _self_launch(args) -> int:
    """N ranks from one command: fresh interpreters via ringdp.run, before any GPU call here."""
    from ringdp.run import launch_local

    return launch_local(os.path.abspath(__file__), sys.argv[1:], args.gpus)


def _store_agree(dist, key: str, ok: bool, rank: int, world: int) -> bool:
    """Every rank publishes ``ok`` through the native store and reads everyone's.  Used where the
    GPU communicator cannot be trusted (e.g. after a failed hipGraph capture)."""
    st = dist.get_default_store()
    st.set(f"bench/{key}/{rank}", b"1" if ok else b"0")
    keys = [f"bench/{key}/{r}" for r in range(world)]
    st.wait(keys)
    return all(st.get(k) == b"1" for k in keys)


def _identity(dev) -> dict:
    """Where this run executes, as tools/comm_bench.py records it next to its measurements."""
    return {"arch": torch.cuda.get_device_properties(dev).gcnArchName, "host": socket.gethostname(),
            "rccl": ".".join(str(v) for v in torch.cuda.nccl.version())}


def _adopt_comm_tuning(path: str, world: int, here: dict) -> dict:
    """RCCL / small-message settings measured by tools/comm_bench.py --recommend.  Adopted (into the
    environment, before the communicator exists; variables already set win) only when the file was measured
    at this world size on this device type, host and RCCL version - a file left over from another box or
    setup must not silently change this run.  Returns what happened, for the result line."""
    with open(path) as f:
        tun = json.load(f)
    ident = tun.get("identity") or {}
    if int(tun.get("world", -1)) != world:
        return {"adopted": False, "reason": f"measured at world {tun.get('world')}, this run has {world}"}
    bad = [k for k in here if ident.get(k) != here[k]]
    if bad:
        return {"adopted": False, "reason": "identity mismatch: " + ", ".join(
            f"{k} {ident.get(k)!r} != {here[k]!r}" for k in bad)}
    env = {k: os.environ.setdefault(k, str(v)) for k, v in tun.get("env", {}).items()}
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench] adopted {path}: {env}", file=sys.stderr, flush=True)
    return {"adopted": True, "env": env, "identity": here}


def _pack_batch(x: torch.Tensor, y: torch.Tensor):
    """(buffer, x view, y view): copies of x and y in one uint8 buffer (x bytes first, 8-aligned)."""
    nx = x.numel() * x.element_size()
    off = (nx + 7) // 8 * 8
    buf = torch.empty(off + y.numel() * y.element_size(), dtype=torch.uint8, device=x.device)
    xv = buf[:nx].view(x.dtype).view(x.shape)
    yv = buf[off:].view(y.dtype).view(y.shape)
    xv.copy_(x)
    yv.copy_(y)
    return buf, xv, yv


def _phase(msg: str) -> None:
    """One stderr line per bench phase (the JSON line stays the only stdout line): a run that stops
    progressing names the phase it stopped in."""
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def worker(args):
    # RINGDP_BENCH_STACKS_S=N: dump every thread's Python stack after N seconds (hang diagnosis)
    if os.environ.get("RINGDP_BENCH_STACKS_S"):
        faulthandler.dump_traceback_later(float(os.environ["RINGDP_BENCH_STACKS_S"]), repeat=True, file=sys.stderr)
    import ringdp
    import ringdp.distributed as dist
    from ringdp import models
    from ringdp._native import C
    from ringdp.nn import CrossEntropyLoss
    from ringdp.optim import SGD
    from ringdp.parallel import DistributedDataParallel as DDP
    from ringdp.utils.graph import StepGraph

    launched = os.environ.get("WORLD_SIZE") is not None
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", args.local_rank if args.local_rank is not None else 0))
    on_gpu = not args.cpu
    if on_gpu:
        # rank r on GPU r % device_count (device_count() does not initialise the GPU); more ranks than
        # GPUs is only possible on the xgmi backend (RCCL refuses two ranks per GPU)
        ndev = max(torch.cuda.device_count(), 1)
        dev_index = local_rank % ndev
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
        backend = "nccl"
    else:
        dev = torch.device("cpu")
        backend = "gloo"
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // max(world_env, 1)))
    comm_tuning = None
    if on_gpu and args.comm_tuning and os.path.exists(args.comm_tuning):
        comm_tuning = _adopt_comm_tuning(args.comm_tuning, world_env, _identity(dev))
    if launched:
        dist.init_process_group(backend=backend)
    else:
        dist.init_process_group(backend=backend, store=dist.HashStore(), rank=0, world_size=1)
    rank, world = dist.get_rank(), dist.get_world_size()
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but world size is {world}; reporting n_gpus={world}", file=sys.stderr)
    force_comm = world == 1 and not args.no_force_comm
    if force_comm:
        os.environ["RINGDP_DDP_FORCE_COMM"] = "1"  # read by the reducer per bucket launch
    spec = MODELS[args.model]
    B = args.batch_per_rank or int(os.environ.get("RINGDP_BENCH_BATCH", spec["batch"]))
    lr = args.lr if args.lr is not None else spec["lr"]
    if args.model == "convnet" and B <= 4096 and args.bucket_mb is None and args.first_bucket_mb is None:
        # small per-rank batches: the conv2/conv1 backward is too short (~12 us at B=100) to hide the first
        # bucket's collective behind, so one 455 KB bucket (one collective, one latency term) beats two
        args.bucket_mb = args.first_bucket_mb = 1.0
    if args.bucket_mb is None:
        args.bucket_mb = spec.get("bucket_mb", 25.0)
    if args.first_bucket_mb is None:
        args.first_bucket_mb = spec.get("first_bucket_mb")

    if args.dtype == "fp8":
        if args.model != "vit_b_16":
            raise SystemExit("--dtype fp8 is implemented for --model vit_b_16")
        from ringdp.ops.transformer import set_fp8
        set_fp8(True)
    torch.manual_seed(0)
    if args.model == "convnet":
        model = models.ConvNet(precision="fp32" if args.dtype == "fp32" else "bf16").to(dev)
    else:
        if args.dtype == "fp32":
            raise SystemExit("--dtype fp32 is implemented for --model convnet")
        model = getattr(models, args.model)(num_classes=NUM_CLASSES[args.model]).to(dev)
    ddp = DDP(model, device_ids=[dev.index] if on_gpu else None, output_device=dev.index if on_gpu else None,
              bucket_cap_mb=args.bucket_mb, first_bucket_mb=args.first_bucket_mb)
    if args.comm_hook != "allreduce":
        ddp._set_builtin_hook(args.comm_hook)
    crit = CrossEntropyLoss()
    opt = SGD(ddp.parameters(), lr=lr, momentum=spec["momentum"], nesterov=spec["nesterov"],
              weight_decay=spec["wd"])

    ncls = NUM_CLASSES[args.model]
    if args.model == "convnet" and on_gpu:
        pool = [C.synth_u8_images(B, 28, 28, 10, 1000 * rank + i, dev) for i in range(args.pool)]
    elif args.model == "convnet":
        g = torch.Generator().manual_seed(1000 * rank)
        pool = [(torch.randint(0, 256, (B, 1, 28, 28), dtype=torch.uint8, generator=g),
                 torch.randint(0, ncls, (B,), generator=g)) for _ in range(min(args.pool, 2))]
    else:
        g = torch.Generator(device=dev).manual_seed(1000 * rank)
        pool = [(torch.randn((B,) + spec["shape"], device=dev, generator=g),
                 torch.randint(0, ncls, (B,), device=dev, generator=g)) for _ in range(min(args.pool, 4))]
    # Each batch lives in one byte buffer (images, then labels), as a loader's staging buffer would:
    # feeding the captured step is one device copy per step instead of two.
    pool = [_pack_batch(x, y) for x, y in pool]
    static_buf, static_x, static_y = _pack_batch(*pool[0][1:])

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    # d(loss)/d(loss) = 1, allocated once: autograd would otherwise launch a fill kernel per step for the
    # seed gradient (~5 us of a 118 us step at the reference batch)
    seed_grad = torch.ones((), device=dev)

    def step_on(x, y):
        out = ddp(x)
        loss = crit(out, y)
        opt.zero_grad(set_to_none=True)
        loss.backward(seed_grad)
        opt.step()
        return loss

    def static_step():
        return step_on(static_x, static_y)

    def capture():
        """Capture one step into a hipGraph; all ranks agree on the outcome before going on (a
        rank that fell back alone would issue a different collective sequence and hang its peers)."""
        err = None
        graph = None
        try:
            graph = StepGraph(static_step, warmup=2, split_ddp=ddp if split_mode else None).capture()
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
            sync()
        ok = err is None
        if world > 1:
            ok = _store_agree(dist, f"capture{capture.n}", ok, rank, world)
        capture.n += 1
        if ok:
            return graph
        print(f"[bench] rank {rank}: hipGraph capture failed ({err or 'on another rank'})", file=sys.stderr, flush=True)
        if world > 1:
            # Captured-but-never-run collectives may have advanced the communicator's sequence on
            # some ranks only; eager fallback could desynchronise them.  Fail loudly instead.
            sys.stderr.flush()
            os._exit(3)
        return None
    capture.n = 0

    _phase(f"model {args.model} dtype {args.dtype} B={B} world={world}: warmup + capture")
    use_graph = on_gpu and not args.no_graph
    nat_pg = getattr(ddp, "_native_pg", None)
    # fork-free overlap: linear graph segments, bucket collectives between them on the comm stream
    split_mode = (use_graph and (world > 1 or force_comm) and args.comm_stream == "split"
                  and hasattr(nat_pg, "set_same_stream"))
    if use_graph and hasattr(nat_pg, "set_same_stream") and os.environ.get("RINGDP_COMM_SAME_STREAM") is None:
        nat_pg.set_same_stream(args.comm_stream == "same")
    graph = None
    n_warm = max(args.warmup, 3)
    if use_graph:
        # eager warmup (bucket rebuild happens at iteration 1), then capture
        for i in range(2):
            _, x, y = pool[i % len(pool)]
            step_on(x, y)
        if split_mode and len(ddp.reducer.bucket_numels()) < 2:
            # one bucket is ready only at the end of backward: nothing to overlap, and a segment boundary plus a
            # cross-stream wait cost more than the collective on the compute stream inside the one graph
            split_mode = False
            if os.environ.get("RINGDP_COMM_SAME_STREAM") is None:
                nat_pg.set_same_stream(True)
        static_buf.copy_(pool[0][0])
        graph = capture()
        use_graph = graph is not None

    comm_stream_note = None
    if use_graph and (world > 1 or force_comm) and hasattr(nat_pg, "same_stream"):
        if split_mode and graph is not None and graph.segments:
            n_split = sum(1 for p in graph.plan for i in p if i >= 0)
            comm_stream_note = (
                f"comm stream between {len(graph.segments)} linear graph segments for {n_split} bucket(s) "
                "(issued as their gradients are final, overlapping the rest of backward; no fork inside any "
                "graph), the other bucket(s) inline on the compute stream (estimated shorter than a segment "
                "boundary, or the last)" if n_split else
                "compute stream inside the graph (split placement: every bucket collective estimated shorter "
                "than a segment boundary)")
        else:
            comm_stream_note = "compute stream (no overlap)" if nat_pg.same_stream() else \
                "side stream inside the graph (overlaps backward; forked graph)"

    # where each bucket's collective runs in the captured step, and its modelled time (ringdp.utils.comm_model)
    from ringdp.utils import comm_model

    if graph is not None and graph.split_info:
        split_plan = graph.split_info
    else:
        wire = 2 if args.comm_hook != "allreduce" else 4
        same = bool(getattr(nat_pg, "same_stream", lambda: True)()) if use_graph else False
        split_plan = [{"bucket": i, "bytes": wire * n, "est_us": round(comm_model.est_us(wire * n, world), 2),
                       "placement": ("inline (compute stream, one graph)" if same else
                                     "side stream" if use_graph else "side stream (eager)")}
                      for i, n in enumerate(ddp.reducer.bucket_numels())]

    def run_steps(n, g):
        loss = None
        for i in range(n):
            buf, x, y = pool[i % len(pool)]
            if g is not None:
                static_buf.copy_(buf, non_blocking=True)
                loss = g.replay()
            else:
                loss = step_on(x, y)
        return loss

    def timed(n, g):
        sync()
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        loss = run_steps(n, g)
        sync()
        dist.barrier()
        sync()
        el = time.perf_counter() - t0
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()), loss

    sync()
    t_w = time.perf_counter()
    run_steps(n_warm, graph)
    sync()
    # Steady state: the W warmup steps of a short run (e.g. 5 x 2 ms) end before the GPU has left its
    # idle clocks, and the first timed steps then run ~2.5 % slower.  Warmup therefore continues until
    # RINGDP_BENCH_MIN_WARMUP_S of warm steps have run (0 disables); every rank runs the same count (MAX
    # over ranks: the captured step holds collectives).  Reported as "warmup_steps_run".
    min_warm_s = float(os.environ.get("RINGDP_BENCH_MIN_WARMUP_S", "0.5"))
    warm_el = time.perf_counter() - t_w
    extra = 0
    if min_warm_s > 0 and warm_el < min_warm_s:
        extra = min(5000, int((min_warm_s - warm_el) / max(warm_el / n_warm, 1e-6)) + 1)
    if world > 1:
        t_x = torch.tensor([extra], dtype=torch.int64, device=dev)
        dist.all_reduce(t_x, op=dist.ReduceOp.MAX)
        extra = int(t_x.item())
    if extra:
        run_steps(extra, graph)
    n_warm += extra
    _phase(f"timed region: {args.steps} steps")
    elapsed_max, loss = timed(args.steps, graph)
    final_loss = float(loss.item()) if loss is not None else float("nan")
    ms_per_step = 1000.0 * elapsed_max / args.steps
    value = world * B * args.steps / elapsed_max
    if rank == 0 and elapsed_max < 1.0:
        print(f"[bench] note: the timed region is {elapsed_max * 1e3:.1f} ms ({args.steps} steps); "
              "use more --steps for sampling-based observers", file=sys.stderr, flush=True)

    # ------------------------------------------------------------------ comm observability
    nat = ddp._native_pg
    stats = ddp.reducer.stats()
    comm_stats = {"bucket_bytes": [int(s.bytes) for s in stats]}
    def emit(comm_stats, text_only=False):
        n_buckets = len(ddp.reducer.bucket_indices())
        sizes_kb = ",".join(f"{b / 1024:.0f}" for b in comm_stats["bucket_bytes"])
        lib = {"rccl": "RCCL", "xgmi": "ringdp xGMI kernels (IPC peer memory)"}.get(nat.backend_name(), nat.backend_name()) \
            if on_gpu else "host ring (gloo)"
        where = f"collectives on the {comm_stream_note}" if comm_stream_note else (
            "compute stream" if getattr(nat, "same_stream", lambda: False)() else "side HIP stream")
        if world > 1:
            comm = (f"{lib} {args.comm_hook} (avg) over {world} ranks, {n_buckets} bucket(s) [{sizes_kb}] KB, "
                    f"cap {args.bucket_mb} MB, " + where)
        elif force_comm:
            comm = (f"{lib} {args.comm_hook} (avg) over 1 rank, forced so N=1 runs the reducer + collective "
                    f"path of N>1, {where}; {n_buckets} bucket(s) [{sizes_kb}] KB, cap {args.bucket_mb} MB")
        else:
            comm = "none (world_size 1, --no-force-comm)"
        if rank == 0:
            metric = METRIC if args.model == "convnet" else \
                f"images/sec (whole node) {args.model} synthetic DDP training at 1/2/4/8 MI355X"
            if not on_gpu:
                data = "synthetic (host uint8 MNIST-shaped images + labels; random-init weights; CPU plumbing run)"
            elif args.model == "convnet":
                data = "synthetic (on-device uint8 MNIST-shaped images + labels; random-init weights)"
            else:
                data = f"synthetic (on-device N(0,1) {spec['shape']} images + labels; random-init weights)"
            dtype = {"bf16": "bf16", "fp32": "fp32", "fp8": "fp8 (e4m3 linear GEMMs, bf16 attention/norms)"}[args.dtype]
            if not on_gpu:
                dtype = "fp32 (CPU ATen)"
            res = {
                "metric": metric,
                "value": round(value, 1),
                "unit": "images/sec",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "warmup_steps_run": n_warm,
                "ms_per_step": round(ms_per_step, 4),
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": dtype,
                "data": data,
                "config": {
                    "model": spec["desc"],
                    "global_batch": B * world,
                    "per_rank_batch": B,
                    "seq_len": None,
                    "image_shape": list(spec["shape"]),
                    "parallelism": f"dp{world}",
                    "optimizer": f"SGD lr={lr} momentum={spec['momentum']} nesterov={spec['nesterov']} wd={spec['wd']}",
                    "comm": comm,
                    "comm_world_size": int(nat.size()),
                    "comm_backend": nat.backend_name(),
                    "hipgraph": use_graph,
                    "comm_tuning": comm_tuning,
                    "master_weights": "fp32",
                    "device": "cpu" if not on_gpu else torch.cuda.get_device_properties(dev).gcnArchName,
                },
                "comm_stats": comm_stats,
                "final_loss": round(final_loss, 5),
            }
            if world > 1 or force_comm:
                res["split_plan"] = split_plan
                res["modelled_exposed_us"] = comm_model.scaling_model(
                    split_plan, ms_per_step * 1000.0, world, split=bool(graph is not None and graph.split_info))
            if on_gpu and world > torch.cuda.device_count():
                res["config"]["ranks_per_gpu"] = world / torch.cuda.device_count()
            if text_only:
                return json.dumps(res)
            print(json.dumps(res), flush=True)

    # The headline number is already measured: should the comm-statistics phase below stop making
    # progress, a native timer writes the result line without those statistics and ends the rank
    # (every rank arms one; only rank 0's carries the line).
    guard_s = 90.0 + 40.0 * args.comm_stats_steps * ms_per_step / 1000.0
    partial = dict(comm_stats, incomplete=f"comm-statistics phase exceeded {guard_s:.0f} s; statistics omitted")
    line = emit(partial, text_only=True)
    sys.stdout.flush()
    if on_gpu:
        C.exit_guard_arm(guard_s, line + "\n" if line else "")
    if args.comm_stats_steps > 0 and (world > 1 or force_comm):
        S = args.comm_stats_steps
        per_bucket = [[] for _ in stats]
        _phase("comm stats: per-bucket timing")
        if hasattr(nat, "set_timing"):
            nat.set_timing(True)
            for i in range(S):
                _, x, y = pool[i % len(pool)]
                step_on(x, y)
                sync()
                for b, d in enumerate(ddp.reducer.collect_comm_times()):
                    if d >= 0:
                        per_bucket[b].append(d)
            nat.set_timing(False)
            comm_stats["bucket_comm_us"] = [round(sum(v) / len(v), 1) if v else None for v in per_bucket]
            comm_stats["bucket_comm_us_method"] = f"device events around each bucket collective on the comm stream, mean of {S} eager steps"
        # step time without any gradient collective (same graph otherwise): exposed comm estimate
        _phase("comm stats: capture without collectives")
        hook = ddp.reducer.comm_hook()
        ddp.reducer.set_comm_hook(C.CommHook.NONE)
        g2 = capture() if use_graph else None
        _phase("comm stats: interleaved with/without timings")
        ddp.reducer.set_comm_hook(hook)
        # interleave the two variants (with / without collectives) so clock drift cancels
        t_c, t_n = [], []
        for _ in range(3):
            el, _ = timed(S, graph if use_graph else None)
            t_c.append(el)
            ddp.reducer.set_comm_hook(C.CommHook.NONE)
            el, _ = timed(S, g2)
            t_n.append(el)
            ddp.reducer.set_comm_hook(hook)
        ms_c = 1000.0 * min(t_c) / S
        ms_nc = 1000.0 * min(t_n) / S
        comm_stats["step_ms_with_comm"] = round(ms_c, 4)
        comm_stats["step_ms_no_comm"] = round(ms_nc, 4)
        comm_stats["exposed_comm_ms"] = round(ms_c - ms_nc, 4)
        comm_stats["exposed_comm_method"] = (f"best of 3 interleaved {S}-step timings of the same {'graph' if use_graph else 'eager step'} "
                                             f"with and without the bucket collectives (max over ranks)")

    if on_gpu:
        C.exit_guard_cancel()
    emit(comm_stats)
    dist.destroy_process_group()


def main(argv=None):
    args = parse(argv)
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        sys.exit(_self_launch(args))
    worker(args)


if __name__ == "__main__":
    main()
