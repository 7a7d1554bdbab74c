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


def _pack_states() -> List:
    from ..ops.convnet import pack_states

    return pack_states()


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
        self.split_info: List[dict] = []  # per bucket: bytes, modelled collective time, placement
        self._packs: List = []  # ConvNet fragment caches the captured forward may read without packing

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
        watch, beacon = self._watch_beacon()
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
        self._packs = _pack_states()
        return self

    def _watch_beacon(self):
        """(groups to watch, beacon) for a capture on the current device (see the class docstring)."""
        dev = torch.cuda.current_device()
        mode = os.environ.get("RINGDP_GRAPH_WATCHDOG", "auto")
        watch = []
        if mode != "0":
            # auto: groups with peers only (a one-rank group has no peer to die; its beacon node would
            # only add a launch to the step)
            watch = [pg for pg in _gpu_groups() if pg.device == dev and (mode == "1" or pg.size() > 1)]
        return watch, (ReplayBeacon(dev) if watch else None)

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
        longer than ``RINGDP_SPLIT_MIN_US`` (``comm_model.est_us``); the others, and always the last
        bucket (nothing follows it to overlap), are captured inline on the compute stream - except
        after a bucket was split: a later bucket then never goes inline before the join (its collective
        would run on the compute stream while the split one still runs on the comm stream, two
        collectives of one group at once); it is deferred to the next segment boundary instead and
        issued there, in bucket order, on the comm stream.  ``RINGDP_SPLIT_BUCKETS`` (comma list of
        bucket indices) forces the split set (tests).  The segments share one memory pool and always
        replay in capture order.

        Watchdog: the last segment (the one holding the optimizer) ends with the replay beacon, as
        ``capture()``'s graph does, so the collectives captured inline are watched too; the ones issued
        between segments are ordinary eager collectives with their own deadlines."""
        from . import comm_model

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
        hook = ddp.reducer.comm_hook()
        wire = 2 if hook in (C.CommHook.BF16_COMPRESS, C.CommHook.FP16_COMPRESS) else 4
        nbytes = [wire * n for n in ddp.reducer.bucket_numels()]
        last = len(nbytes) - 1
        world = ddp._native_pg.size()
        min_us = float(os.environ.get("RINGDP_SPLIT_MIN_US", str(comm_model.SPLIT_MIN_US)))
        forced = os.environ.get("RINGDP_SPLIT_BUCKETS")
        forced = {int(t) for t in forced.split(",") if t.strip()} if forced is not None else None
        state = {"split": False, "joined": False, "pending": []}
        info = [{"bucket": i, "bytes": nb, "est_us": round(comm_model.est_us(nb, world), 2), "placement": None}
                for i, nb in enumerate(nbytes)]

        def cut(tags):
            with torch.cuda.stream(s):
                segs[-1].capture_end()
                plan[-1].extend(tags)
                segs.append(torch.cuda.CUDAGraph())
                plan.append([])
                segs[-1].capture_begin(pool=pool, capture_error_mode="relaxed")

        def split(idx):
            """True: this bucket's collective runs between segments at replay; False: captured inline."""
            if idx < 0 or idx == last:
                # the join: the earlier buckets' collectives before the optimizer (and before the last
                # bucket's collective, which is captured inline: nothing follows it to overlap)
                if state["split"] and not state["joined"]:
                    cut(state["pending"] + [-1])
                    state["pending"] = []
                    state["joined"] = True
                if idx >= 0:
                    info[idx]["placement"] = "inline (last)"
                return False
            want = (idx in forced) if forced is not None else comm_model.est_us(nbytes[idx], world) >= min_us
            if not want:
                if not state["split"]:  # cheaper than the segment boundary it would need
                    info[idx]["placement"] = "inline"
                    return False
                # a split collective may still run on the comm stream: queue this one behind it
                state["pending"].append(idx)
                info[idx]["placement"] = "deferred to the next boundary"
                return True
            cut(state["pending"] + [idx])
            state["pending"] = []
            state["split"] = True
            info[idx]["placement"] = "split"
            return True

        watch, beacon = self._watch_beacon()
        for d in self._split:
            d.reducer.set_capture_split(split)
        try:
            with torch.cuda.stream(s):
                segs[0].capture_begin(pool=pool, capture_error_mode="relaxed")
                try:
                    out = self.step_fn()
                    if beacon is not None:
                        beacon.mark(s.cuda_stream)
                finally:
                    segs[-1].capture_end()
        finally:
            for d in self._split:
                d.reducer.set_capture_split(None)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        assert not state["pending"], "split capture: deferred buckets never issued"
        self.segments, self.plan = segs, plan
        self.split_info = info
        self.graph = segs[0]
        self.output = out.detach() if torch.is_tensor(out) else out
        for pg in watch:
            pg.watch_beacon(beacon)
        self._beacon = beacon
        self._groups = [pg for pg in _gpu_groups() if pg.device == torch.cuda.current_device()]
        self._packs = _pack_states()
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
        if self._beacon is not None:
            self._beacon.issued()
        return self.output

    def replay(self):
        for st in self._packs:
            # weights changed since the capture behind the captured forward's back (a version bump, or
            # ringdp.ops.convnet.invalidate_pack): rebuild the fragments it reads
            if st.stale():
                st.repack()
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
