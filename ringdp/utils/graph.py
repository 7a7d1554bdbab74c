"""hipGraph capture of a whole training step (MI355X-first replacement for a tracing compiler).

A ringdp training step at the reference's shapes is launch-bound: forward,
backward, the bucket all-reduces (RCCL or ringdp's xGMI kernels) on the side stream and the fused
optimizer are a few dozen small launches.  ``StepGraph`` warms the step up on a side stream, drains
every GPU watchdog queue, then captures one step (including the cross-stream event fork/join of the
reducer and the collective kernels) into a hipGraph that ``replay()`` launches with a single call.

Requirements: inputs the step reads must live in static tensors (copy each new batch into
them), DDP bucket rebuild must have happened (warmup >= 2 steps), and the optimizer must use
its graph-safe path (ringdp.optim.SGD flat path: no allocations, lr may be a device tensor).
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional

import torch

from .. import distributed as dist
from .._native import C

ReplayBeacon = getattr(C, "ReplayBeacon", None)


def _gpu_groups() -> List:
    """Every native GPU process group (RCCL or xGMI) of every group."""
    w = dist._world
    return [pg for g in list(w.groups.values()) for pg in list(g._gpu.values())]


def drain_comms():
    """Block until every in-flight GPU collective of every group has completed."""
    for pg in _gpu_groups():
        pg.drain()


class StepGraph:
    """Capture/replay of one training step.

    Watchdog: collectives inside a replay are invisible to the per-op watchdog (they were
    issued once, at capture).  The captured step therefore ends with a beacon node
    (``ReplayBeacon``: a one-thread kernel that writes the count of finished replays into
    host-coherent memory) and ``replay()`` counts issued replays; every GPU group's watchdog
    compares the two with plain loads (``GpuPG.watch_beacon``).  While replays are outstanding
    and none finishes within the group timeout - e.g. a peer died mid-step - the communicator is
    aborted and the process exits non-zero, as for a hung eager collective.  No HIP call is made
    per replay on either thread.  ``RINGDP_GRAPH_WATCHDOG``: unset/``auto`` watches groups with more
    than one rank, ``1`` every group, ``0`` none."""

    def __init__(self, step_fn: Callable[[], Optional[torch.Tensor]], warmup: int = 3, split_ddp=None):
        self.step_fn = step_fn
        self.warmup = warmup
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.output = None
        self._beacon = None
        self._groups: List = []
        # split mode (``split_ddp``: the DistributedDataParallel model whose bucket collectives overlap
        # backward): see capture_split
        self._split = [split_ddp] if split_ddp is not None else []
        self.segments: List[torch.cuda.CUDAGraph] = []
        self.plan: List[List] = []  # plan[k]: what the replay does after segment k (bucket indices / -1 join)

    def capture(self):
        if self._split:
            return self.capture_split()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self.step_fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        drain_comms()
        self.graph = torch.cuda.CUDAGraph()
        dump = os.environ.get("RINGDP_GRAPH_DUMP")  # DOT file of the captured nodes (diagnostics)
        if dump:
            self.graph.enable_debug_mode()
        dev = torch.cuda.current_device()
        mode = os.environ.get("RINGDP_GRAPH_WATCHDOG", "auto")
        watch = []
        if mode != "0":
            # auto: groups with peers only (a one-rank group has no peer to die; its beacon node would
            # only add a launch to the step)
            watch = [pg for pg in _gpu_groups() if pg.device == dev and (mode == "1" or pg.size() > 1)]
        beacon = ReplayBeacon(dev) if watch else None
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            out = self.step_fn()
            if beacon is not None:
                beacon.mark(torch.cuda.current_stream().cuda_stream)
        if dump:
            self.graph.debug_dump(dump)
        # keep only the value: a live autograd graph would pin AccumulateGrad nodes created on the
        # capture stream and make later eager steps on another stream synchronise against them
        self.output = out.detach() if torch.is_tensor(out) else out
        torch.cuda.synchronize()
        for pg in watch:
            pg.watch_beacon(beacon)
        self._beacon = beacon
        self._groups = [pg for pg in _gpu_groups() if pg.device == dev]
        return self

    def capture_split(self):
        """Fork-free overlap of the bucket collectives with backward.

        The step is captured as a chain of linear hipGraph segments on ONE stream (each keeps HIP's
        batched packet launch; a side-stream fork inside a graph costs +1.2-2 us on every kernel): the
        reducer's split hook ends the current segment where a bucket becomes ready (instead of issuing
        its collective) and at the join point.  ``replay()`` launches the segments in order on the
        compute stream and, between them, each split bucket's collective on the process group's comm
        stream (stream-ordered after the segment that produced the gradients, overlapping the next
        segments); before the last bucket's collective and the optimizer the compute stream waits for
        them.  A segment boundary plus two cross-queue waits cost ~15-45 us on MI355X (kernel traces,
        profiles/r05/split/), so a bucket is split off only when its collective is estimated to take
        longer than ``RINGDP_SPLIT_MIN_US`` (30); the others, and always the last bucket (nothing
        follows it to overlap), are captured inline on the compute stream.  The segments share one
        memory pool and always replay in capture order."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self.step_fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        drain_comms()
        pool = torch.cuda.graph_pool_handle()
        segs = [torch.cuda.CUDAGraph()]
        plan: List[List] = [[]]
        ddp = self._split[0]
        nbytes = [4 * n for n in ddp.reducer.bucket_numels()]
        last = len(nbytes) - 1
        world = ddp._native_pg.size()
        min_us = float(os.environ.get("RINGDP_SPLIT_MIN_US", "30"))
        state = {"split": False, "joined": False}

        def est_us(nb):
            # bucket collective estimate: one rank = a local copy (~1.5 TB/s); else a ring over xGMI at
            # ~100 GB/s per rank plus a launch / latency term
            if world <= 1:
                return nb / 1.5e6
            return 10.0 + 2.0 * (world - 1) / world * nb / 1.0e5

        def cut(tag):
            with torch.cuda.stream(s):
                segs[-1].capture_end()
                plan[-1].append(tag)
                segs.append(torch.cuda.CUDAGraph())
                plan.append([])
                segs[-1].capture_begin(pool=pool, capture_error_mode="relaxed")

        def split(idx):
            """True: this bucket's collective runs between segments at replay; False: captured inline."""
            if idx < 0 or idx == last:
                # the join: the earlier buckets' collectives before the optimizer (and before the last
                # bucket's collective, which is captured inline: nothing follows it to overlap)
                if state["split"] and not state["joined"]:
                    cut(-1)
                    state["joined"] = True
                return False
            if est_us(nbytes[idx]) < min_us:  # cheaper than the segment boundary it would need
                return False
            cut(idx)
            state["split"] = True
            return True

        for d in self._split:
            d.reducer.set_capture_split(split)
        try:
            with torch.cuda.stream(s):
                segs[0].capture_begin(pool=pool, capture_error_mode="relaxed")
                try:
                    out = self.step_fn()
                finally:
                    segs[-1].capture_end()
        finally:
            for d in self._split:
                d.reducer.set_capture_split(None)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.segments, self.plan = segs, plan
        self.graph = segs[0]
        self.output = out.detach() if torch.is_tensor(out) else out
        self._groups = [pg for pg in _gpu_groups() if pg.device == torch.cuda.current_device()]
        return self

    def _replay_split(self):
        works = []
        reducer = self._split[0].reducer
        for seg, after in zip(self.segments, self.plan):
            seg.replay()
            for idx in after:
                if idx >= 0:
                    w = reducer.launch_collective(idx)
                    if w is not None:
                        works.append(w)
                else:
                    for w in works:
                        w.wait(False)  # compute stream waits on the comm stream; no host block
                    works = []
        for w in works:
            w.wait(False)
        return self.output

    def replay(self):
        if self.segments:
            if self._groups:
                stream = torch.cuda.current_stream().cuda_stream
                for pg in self._groups:
                    pg.join_into(stream)
            return self._replay_split()
        # an eager collective still running on a group's comm stream must finish before the replay's
        # own collectives of that group start (xGMI kernels reuse slots in issue order); join_into
        # makes no HIP call unless an eager op was issued since the last join
        if self._groups:
            stream = torch.cuda.current_stream().cuda_stream
            for pg in self._groups:
                pg.join_into(stream)
        self.graph.replay()
        if self._beacon is not None:
            self._beacon.issued()
        return self.output
