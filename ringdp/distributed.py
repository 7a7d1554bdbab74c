"""ringdp.distributed - process-group API on ringdp's native runtime.

API parity target: ``torch.distributed`` as exercised by the reference
(``ref/mpspawn_dist.py:49-54``, ``ref/launch_dist.py:49``, ``ref/example_mp.py:37-42``,
``ref/README.md:36-43,133-134``).  Semantics kept:

* ``init_process_group(backend, init_method, timeout, world_size, rank, store, group_name)``
  with ``env://`` (MASTER_ADDR/MASTER_PORT/RANK/WORLD_SIZE, query string wins), ``tcp://host:port``
  and ``file://path`` rendezvous; rank 0 hosts the TCP store; double init raises; default
  timeouts 10 min (rccl/nccl) / 30 min (host backends).
* ``get_rank/get_world_size/new_group/barrier/all_reduce/broadcast/all_gather/...`` with global
  ranks in src/dst arguments, ``async_op`` returning a Work whose ``wait()`` fences the caller's
  stream (GPU) or blocks (CPU).
* backends: ``"nccl"``/``"rccl"`` -> RCCL over xGMI (GPU tensors), ``"xgmi"`` -> ringdp's own
  collective kernels over IPC-mapped peer memory (GPU tensors, ranks on one node, which may share a
  GPU; ``RINGDP_GPU_BACKEND=xgmi`` makes ``"nccl"`` select it), ``"gloo"``/``"host"`` -> the
  native host ring (CPU tensors; GPU tensors are staged through host memory),
  ``None``/``"cpu:gloo,cuda:nccl"`` -> both, dispatched on the tensor's device.

Native communicators are created lazily on the first collective that needs them (as c10d
does for NCCL), so ``init_process_group`` never needs a GPU.
"""
from __future__ import annotations

import datetime as _dt
import os
import pickle
import sys
import threading
from contextlib import contextmanager
from typing import Any, Dict, List, Optional, Sequence
from urllib.parse import parse_qs, urlparse

import torch

from ._native import C

ReduceOp = C.ReduceOp
Work = C.Work
RingdpError = C.RingdpError
DistTimeoutError = C.DistTimeoutError

TCPStore = C.TCPStore
FileStore = C.FileStore
HashStore = C.HashStore
PrefixStore = C.PrefixStore
Store = C.Store

default_pg_timeout = _dt.timedelta(minutes=30)
default_pg_nccl_timeout = _dt.timedelta(minutes=10)

_GPU_BACKENDS = ("nccl", "rccl")
_GPU_KINDS = ("rccl", "xgmi")  # native GPU process-group kinds


def _gpu_kind_for_nccl() -> str:
    """What "nccl"/"rccl" maps to: RCCL, unless RINGDP_GPU_BACKEND=xgmi selects ringdp's own
    collective kernels over IPC-mapped peer memory (one node; ranks may share a GPU)."""
    v = os.environ.get("RINGDP_GPU_BACKEND", "rccl").strip().lower()
    if v not in _GPU_KINDS:
        raise ValueError(f"ringdp: RINGDP_GPU_BACKEND must be 'rccl' or 'xgmi', got {v!r}")
    return v
_CPU_BACKENDS = ("gloo", "host", "host_ring", "cpu")


class Backend:
    NCCL = "nccl"
    RCCL = "rccl"
    XGMI = "xgmi"  # ringdp's own collective kernels over IPC-mapped peer memory (one node)
    GLOO = "gloo"
    HOST = "host"
    FAKE = "fake"  # collectives are no-ops (upstream fake_pg.py): single-process tests as rank r of N

    @staticmethod
    def normalize(backend: Optional[str]) -> Dict[str, str]:
        """Returns {device_type: native backend} for a user backend string."""
        if backend is None or backend == "undefined":
            return {"cpu": "host", "cuda": _gpu_kind_for_nccl()}
        b = str(backend).lower()
        if ":" in b:
            out = {}
            for part in b.split(","):
                dev, name = part.split(":")
                name = name.strip()
                out[dev.strip()] = (_gpu_kind_for_nccl() if name in _GPU_BACKENDS else
                                    "xgmi" if name == "xgmi" else "host")
            return out
        if b in _GPU_BACKENDS:
            return {"cuda": _gpu_kind_for_nccl()}
        if b in ("xgmi", "ipc"):
            return {"cuda": "xgmi"}
        if b in _CPU_BACKENDS:
            return {"cpu": "host", "cuda": "host"}
        if b == "fake":
            return {"cpu": "fake", "cuda": "fake"}
        raise ValueError(f"ringdp: unknown backend {backend!r} (use 'nccl', 'rccl', 'xgmi', 'gloo', 'host', 'fake')")


def _to_reduce_op(op) -> "C.ReduceOp":
    if isinstance(op, C.ReduceOp):
        return op
    name = getattr(op, "name", None) or str(op).split(".")[-1]
    name = name.upper()
    if name == "PREMUL_SUM":
        raise ValueError("ringdp: PREMUL_SUM is not supported")
    return getattr(C.ReduceOp, name)


# ----------------------------------------------------------------------------- group objects
class _NonMember:
    def __repr__(self):
        return "GroupMember.NON_GROUP_MEMBER"


class GroupMember:
    WORLD = None  # resolved lazily to the default group
    NON_GROUP_MEMBER = _NonMember()


class ProcessGroup:
    """A ringdp process group: global-rank bookkeeping + lazily created native communicators."""

    def __init__(self, store, rank: int, size: int, backends: Dict[str, str], timeout: _dt.timedelta,
                 global_ranks: Sequence[int], name: str, bind_hint: str):
        self._store = store
        self._rank = rank
        self._size = size
        self._backends = backends
        self._timeout = timeout
        self._global_ranks = list(global_ranks)
        self._g2l = {g: i for i, g in enumerate(self._global_ranks)}
        self.group_name = name
        self._bind_hint = bind_hint
        self._host = None
        self._fake = None
        self._gpu: Dict[int, Any] = {}  # device -> native GPU process group (RcclPG / XgmiPG)
        self._lock = threading.Lock()
        self._coll_count = 0
        self.requested_backend: Optional[str] = None  # the user's backend string (get_backend)
        self._kind_agreed = False

    # -- introspection
    def rank(self) -> int:
        return self._rank

    def size(self) -> int:
        return self._size

    def name(self) -> str:
        return self.group_name

    @property
    def ranks(self) -> List[int]:
        return list(self._global_ranks)

    def backend_name(self, device_type: str = "cuda") -> str:
        return self._backends.get(device_type, next(iter(self._backends.values())))

    @property
    def timeout_ms(self) -> int:
        return int(self._timeout.total_seconds() * 1000)

    def __repr__(self):
        return f"ringdp.ProcessGroup(name={self.group_name}, rank={self._rank}, size={self._size}, backends={self._backends})"

    # -- native communicators
    def host(self):
        if self._backends.get("cpu") == "fake":
            return self.native_for(torch.empty(0))[0]
        with self._lock:
            if self._host is None:
                sub = C.PrefixStore(f"{self.group_name}/host", self._store)
                self._host = C.HostRingPG(sub, self._rank, self._size, self.timeout_ms, self._bind_hint)
            return self._host

    def gpu(self, device: int):
        """The native GPU process group of this group on ``device`` (created on first use; collective
        over the group's members)."""
        with self._lock:
            pg = self._gpu.get(device)
            if pg is None:
                kind = self._backends.get("cuda", "rccl")
                if kind not in _GPU_KINDS:
                    kind = "rccl"
                if not torch.cuda.is_available():
                    raise RuntimeError(f"ringdp: the {kind} backend needs a GPU (torch.cuda.is_available() is False)")
                self._agree_gpu_kind(kind)
                sub = C.PrefixStore(f"{self.group_name}/{kind}/{device}", self._store)
                cls = C.RcclPG if kind == "rccl" else C.XgmiPG
                pg = cls(sub, self._rank, self._size, device, self.timeout_ms)
                self._gpu[device] = pg
            return pg

    rccl = gpu  # older name

    def _agree_gpu_kind(self, kind: str) -> None:
        """Every member publishes the GPU backend it resolved (RINGDP_GPU_BACKEND is read per
        process); a mismatch raises here instead of leaving ranks waiting on different store keys."""
        if self._kind_agreed or self._size == 1:
            return
        self._store.set(f"{self.group_name}/gpukind/{self._rank}", kind)
        kinds = {r: self._store.get(f"{self.group_name}/gpukind/{r}").decode() for r in range(self._size)}
        if len(set(kinds.values())) != 1:
            raise RuntimeError(
                f"ringdp: ranks of group {self.group_name} resolved different GPU backends {kinds} "
                "(set RINGDP_GPU_BACKEND identically on every rank)")
        self._kind_agreed = True

    def native_for(self, tensor: torch.Tensor):
        """(native process group, staged-through-host?) for a tensor."""
        dev = "cuda" if tensor.is_cuda else "cpu"
        kind = self._backends.get(dev)
        if kind is None:
            raise RuntimeError(
                f"ringdp: process group {self.group_name} has no backend for {dev} tensors "
                f"(backends={self._backends}); e.g. rccl/nccl only reduces GPU tensors")
        if kind == "fake":
            with self._lock:
                if self._fake is None:
                    self._fake = C.FakePG(self._rank, self._size)
            return self._fake, False
        if kind in _GPU_KINDS:
            return self.gpu(tensor.device.index if tensor.device.index is not None else torch.cuda.current_device()), False
        return self.host(), tensor.is_cuda

    def local_rank_of(self, global_rank: int) -> int:
        try:
            return self._g2l[global_rank]
        except KeyError:
            raise ValueError(f"ringdp: global rank {global_rank} is not part of group {self.group_name}") from None

    def shutdown(self):
        with self._lock:
            self._fake = None
            for pg in self._gpu.values():
                pg.shutdown()
            self._gpu.clear()
            if self._host is not None:
                self._host.shutdown()
                self._host = None


class _World:
    def __init__(self):
        self.default_pg: Optional[ProcessGroup] = None
        self.groups: Dict[str, ProcessGroup] = {}
        self.group_count = 0
        self.store = None
        self.timeout = None
        self.backend = None
        self.bind_hint = "127.0.0.1"


_world = _World()


# ----------------------------------------------------------------------------- rendezvous
def _env_int(name: str) -> Optional[int]:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else None


def _rendezvous(init_method: str, rank: int, world_size: int, timeout: _dt.timedelta):
    """-> (store, rank, world_size, bind_hint).  Mirrors torch/distributed/rendezvous.py."""
    url = urlparse(init_method)
    query = {k: v[-1] for k, v in parse_qs(url.query).items()}
    if "rank" in query:
        rank = int(query["rank"])
    if "world_size" in query:
        world_size = int(query["world_size"])
    tmo_ms = int(timeout.total_seconds() * 1000)
    if url.scheme == "env":
        if rank < 0:
            r = _env_int("RANK")
            if r is None:
                raise ValueError("ringdp env:// rendezvous: RANK is not set (and rank was not given)")
            rank = r
        if world_size < 0:
            w = _env_int("WORLD_SIZE")
            if w is None:
                raise ValueError("ringdp env:// rendezvous: WORLD_SIZE is not set (and world_size was not given)")
            world_size = w
        addr = os.environ.get("MASTER_ADDR")
        port = _env_int("MASTER_PORT")
        if not addr or port is None:
            raise ValueError("ringdp env:// rendezvous: MASTER_ADDR and MASTER_PORT must be set")
        store = _tcp_store(addr, port, rank, world_size, tmo_ms, use_agent=True)
        return store, rank, world_size, addr
    if url.scheme == "tcp":
        if rank < 0 or world_size < 0:
            raise ValueError("ringdp tcp:// rendezvous requires rank and world_size")
        store = _tcp_store(url.hostname, url.port, rank, world_size, tmo_ms, use_agent=False)
        return store, rank, world_size, url.hostname
    if url.scheme == "file":
        if rank < 0 or world_size < 0:
            raise ValueError("ringdp file:// rendezvous requires rank and world_size")
        path = url.path if not url.netloc else url.netloc + url.path
        return C.FileStore(path, world_size, tmo_ms), rank, world_size, "127.0.0.1"
    raise ValueError(f"ringdp: unsupported init_method {init_method!r} (env://, tcp://, file://)")


def _reachable_ip(peer_host: str, peer_port: int) -> str:
    """The local interface address peers use to reach this host: the source address the kernel
    picks for a route to the master (no packet is sent).  Avoids resolving the container
    hostname, which need not resolve."""
    import socket

    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect((peer_host, peer_port))
            return s.getsockname()[0]
    except OSError:
        return peer_host


def _tcp_store(host: str, port: int, rank: int, world_size: int, tmo_ms: int, use_agent: bool):
    if use_agent and os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
        # Started by torchrun: the elastic agent owns MASTER_PORT with its own (c10d) store.  It is
        # used for ONE exchange only: rank 0 starts ringdp's native TCPStore on an ephemeral port
        # and publishes "<ip>:<port>" there; every rank then connects to the native store, which
        # carries all further bootstrap traffic (RCCL unique ids, barriers, debug fingerprints).
        import torch.distributed as tdist

        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        agent = tdist.TCPStore(host, port, world_size, False, _dt.timedelta(milliseconds=tmo_ms))
        key = f"/ringdp/attempt_{attempt}/native_store"
        if rank == 0:
            st = C.TCPStore(host, 0, world_size, True, tmo_ms)
            agent.set(key, f"{_reachable_ip(host, port)}:{st.port}")
        else:
            addr = agent.get(key).decode()
            h, p = addr.rsplit(":", 1)
            st = C.TCPStore(h, int(p), world_size, False, tmo_ms)
        del agent
        return st
    if use_agent and os.environ.get("RINGDP_USE_AGENT_STORE", "0") == "1":
        # Started by `python -m ringdp.launch`: the launcher on node 0 hosts the store on
        # MASTER_PORT; workers are clients, namespaced per restart attempt.
        attempt = os.environ.get("RINGDP_RESTART_COUNT", "0")
        st = C.TCPStore(host, port, world_size, False, tmo_ms)
        return C.PrefixStore(f"attempt_{attempt}", st)
    return C.TCPStore(host, port, world_size, rank == 0, tmo_ms)


def _install_rank_excepthook(rank: int):
    old = sys.excepthook

    def hook(exc_type, exc, tb):
        sys.stderr.write(f"[rank{rank}]: ")
        old(exc_type, exc, tb)

    sys.excepthook = hook


# ----------------------------------------------------------------------------- public: lifecycle
def is_available() -> bool:
    return True


def is_nccl_available() -> bool:
    return True


is_rccl_available = is_nccl_available


def is_gloo_available() -> bool:
    return True


def is_initialized() -> bool:
    return _world.default_pg is not None


def init_process_group(backend: Optional[str] = None, init_method: Optional[str] = None,
                       timeout: Optional[_dt.timedelta] = None, world_size: int = -1, rank: int = -1,
                       store=None, group_name: str = "", pg_options=None, device_id=None) -> None:
    """Initialises the default process group (see module docstring)."""
    if _world.default_pg is not None:
        raise ValueError("trying to initialize the default process group twice!")
    backends = Backend.normalize(backend)
    if timeout is None:
        timeout = default_pg_nccl_timeout if set(backends.values()) <= set(_GPU_KINDS) else default_pg_timeout
    if set(backends.values()) == {"fake"} and store is None and init_method is None:
        # upstream: init_process_group("fake") short-circuits the rendezvous
        if rank < 0 or world_size <= 0:
            raise ValueError("ringdp: the fake backend needs explicit rank and world_size")
        store = C.HashStore()
    if store is not None:
        if init_method is not None:
            raise ValueError("ringdp: cannot specify both init_method and store")
        if rank < 0 or world_size <= 0:
            raise ValueError("ringdp: rank and world_size are required with an explicit store")
        bind_hint = os.environ.get("MASTER_ADDR", "127.0.0.1")
        if not isinstance(store, C.Store):
            store = C.PyStore(store, int(timeout.total_seconds() * 1000))
    else:
        if init_method is None:
            init_method = "env://"
        store, rank, world_size, bind_hint = _rendezvous(init_method, rank, world_size, timeout)
    if not (0 <= rank < world_size):
        raise ValueError(f"ringdp: invalid rank {rank} for world_size {world_size}")
    if isinstance(device_id, torch.device) and device_id.type == "cuda" and device_id.index is not None:
        torch.cuda.set_device(device_id.index)
    root = C.PrefixStore("ringdp", store)
    name = group_name or "default_pg"
    pg = ProcessGroup(root, rank, world_size, backends, timeout, list(range(world_size)), name, bind_hint)
    pg.requested_backend = backend if isinstance(backend, str) else None
    _world.default_pg = pg
    _world.groups = {name: pg}
    _world.group_count = 0
    _world.store = root
    _world.timeout = timeout
    _world.backend = backend
    _world.bind_hint = bind_hint
    GroupMember.WORLD = pg
    if os.environ.get("RINGDP_RANK_EXCEPTHOOK", "1") == "1":
        _install_rank_excepthook(rank)
    if os.environ.get("RINGDP_INIT_BARRIER", os.environ.get("TORCH_DIST_INIT_BARRIER", "0")) == "1":
        _store_barrier(root, "init", rank, world_size, timeout)


def _store_barrier(store, key: str, rank: int, world_size: int, timeout: _dt.timedelta):
    n = store.add(f"barrier/{key}", 1)
    if n == world_size:
        store.set(f"barrier/{key}/done", b"1")
    store.wait([f"barrier/{key}/done"], timeout)


def destroy_process_group(group: Optional[ProcessGroup] = None) -> None:
    if group is None or group is _world.default_pg:
        for g in list(_world.groups.values()):
            g.shutdown()
        _world.__init__()
        GroupMember.WORLD = None
        return
    group.shutdown()
    _world.groups.pop(group.group_name, None)


def _default() -> ProcessGroup:
    if _world.default_pg is None:
        raise RuntimeError("Default process group has not been initialized, please make sure to call "
                           "ringdp.distributed.init_process_group.")
    return _world.default_pg


def _resolve(group) -> ProcessGroup:
    return _default() if group is None else group


def _not_member(group) -> bool:
    return group is GroupMember.NON_GROUP_MEMBER


def get_rank(group: Optional[ProcessGroup] = None) -> int:
    if _not_member(group):
        return -1
    return _resolve(group).rank()


def get_world_size(group: Optional[ProcessGroup] = None) -> int:
    if _not_member(group):
        return -1
    return _resolve(group).size()


def get_backend(group: Optional[ProcessGroup] = None) -> str:
    g = _resolve(group)
    req = g.requested_backend
    if isinstance(req, str) and req and Backend.normalize(req) == g._backends:
        return req.lower()  # upstream returns the name the user asked for ("nccl", even when xgmi serves it)
    kinds = set(g._backends.values())
    if kinds == {"rccl"}:
        return "nccl"
    if kinds == {"xgmi"}:
        return "xgmi"
    if kinds == {"host"}:
        return "gloo"
    if kinds == {"fake"}:
        return "fake"
    return "cpu:gloo,cuda:nccl"


def get_global_rank(group: ProcessGroup, group_rank: int) -> int:
    return group.ranks[group_rank]


def get_group_rank(group: ProcessGroup, global_rank: int) -> int:
    return group.local_rank_of(global_rank)


def get_process_group_ranks(group: ProcessGroup) -> List[int]:
    return _resolve(group).ranks


def new_group(ranks: Optional[Sequence[int]] = None, timeout: Optional[_dt.timedelta] = None,
              backend: Optional[str] = None, pg_options=None, use_local_synchronization: bool = False,
              group_desc: Optional[str] = None):
    """Creates a sub-group.  Every rank of the world must call it with the same ``ranks``."""
    world = _default()
    _world.group_count += 1
    name = f"group_{_world.group_count}"
    ranks = sorted(range(world.size())) if ranks is None else sorted(int(r) for r in ranks)
    if len(set(ranks)) != len(ranks) or any(r < 0 or r >= world.size() for r in ranks):
        raise ValueError(f"ringdp.new_group: invalid ranks {ranks}")
    me = world.rank()
    backends = Backend.normalize(backend) if backend is not None else dict(world._backends)
    # RCCL sub-communicators come from ncclCommSplit of the world's communicator when that exists
    # (every rank takes part in the split, non-members with NCCL_SPLIT_NOCOLOR), otherwise they are
    # created lazily through the store on first use.
    split = {}
    if backends.get("cuda") == "rccl" and os.environ.get("RINGDP_COMM_SPLIT", "1") == "1":
        for dev, parent in sorted(world._gpu.items()):
            if isinstance(parent, C.RcclPG):
                tmo_ms = int(timeout.total_seconds() * 1000) if timeout is not None else 0
                split[dev] = parent.split_with_timeout(ranks, name, tmo_ms)
    if me not in ranks:
        return GroupMember.NON_GROUP_MEMBER
    pg = ProcessGroup(_world.store, ranks.index(me), len(ranks), backends, timeout or world._timeout,
                      ranks, name, _world.bind_hint)
    pg.requested_backend = backend if isinstance(backend, str) else world.requested_backend
    for dev, child in split.items():
        if child is not None:
            pg._gpu[dev] = child
    _world.groups[name] = pg
    return pg


# ----------------------------------------------------------------------------- debug / faults
_fault_spec = os.environ.get("RINGDP_FAULT_INJECT", "")
_debug = os.environ.get("RINGDP_DEBUG", os.environ.get("TORCH_DISTRIBUTED_DEBUG", "")).upper() in ("1", "DETAIL", "INFO")
_coll_counter = 0


def _maybe_fault(group: ProcessGroup):
    """RINGDP_FAULT_INJECT="<global rank>:<n>": that rank hard-exits at its n-th collective."""
    global _coll_counter
    _coll_counter += 1
    if not _fault_spec:
        return
    r, n = _fault_spec.split(":")
    if int(r) == _default().rank() and _coll_counter == int(n):
        sys.stderr.write(f"[ringdp] fault injection: rank {r} exiting at collective {n}\n")
        sys.stderr.flush()
        os._exit(17)


def _fingerprint(op: str, tensors: Sequence[torch.Tensor], extra: str = "") -> str:
    parts = [op, extra]
    for t in tensors:
        parts.append(f"{t.dtype}:{tuple(t.shape)}:{t.device.type}")
    return "|".join(parts)


def _debug_check(group: ProcessGroup, op: str, tensors: Sequence[torch.Tensor], extra: str = ""):
    """RINGDP_DEBUG=1: every rank publishes a fingerprint of each collective and checks that all
    members issued the same op/dtype/shape (c10d ProcessGroupWrapper semantics)."""
    group._coll_count += 1
    seq = group._coll_count
    fp = _fingerprint(op, tensors, extra)
    st = C.PrefixStore(f"{group.group_name}/debug", _world.store)
    st.set(f"{seq}/{group.rank()}", fp)
    keys = [f"{seq}/{r}" for r in range(group.size())]
    st.wait(keys)
    mine = fp
    for r in range(group.size()):
        other = st.get(f"{seq}/{r}").decode()
        if other != mine:
            raise RuntimeError(
                f"ringdp collective desync in group {group.group_name} at collective #{seq}: "
                f"rank {group.rank()} issued [{mine}] but rank {r} issued [{other}]")


def _pre(group: ProcessGroup, op: str, tensors: Sequence[torch.Tensor], extra: str = ""):
    _maybe_fault(group)
    if _debug:
        _debug_check(group, op, tensors, extra)


class _StagedWork:
    """Work for GPU tensors run through the host backend: copy back after completion."""

    def __init__(self, work, pairs):
        self._work = work
        self._pairs = pairs
        self._done = False

    def wait(self, blocking: bool = True):
        if not self._done:
            self._work.wait(True)
            for gpu, cpu in self._pairs:
                gpu.copy_(cpu)
            self._done = True
        return True

    def is_completed(self):
        return self._done or self._work.is_completed()

    def synchronize(self):
        self.wait(True)

    def result(self):
        return [g for g, _ in self._pairs]


def _finish(work, async_op: bool):
    if async_op:
        return work
    work.wait()
    return None


def _stage(ts: Sequence[torch.Tensor], staged: bool):
    if not staged:
        return list(ts), None
    cpus = [t.detach().cpu() for t in ts]
    return cpus, list(zip(ts, cpus))


# ----------------------------------------------------------------------------- collectives
def all_reduce(tensor: torch.Tensor, op=ReduceOp.SUM, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    if _coalesce(g, "all_reduce", tensor, op=op):
        return None
    _pre(g, "all_reduce", [tensor], str(op))
    native, staged = g.native_for(tensor)
    ts, pairs = _stage([tensor], staged)
    w = native.allreduce(ts, _to_reduce_op(op))
    return _finish(_StagedWork(w, pairs) if pairs else w, async_op)


def all_reduce_coalesced(tensors: List[torch.Tensor], op=ReduceOp.SUM, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    _pre(g, "all_reduce_coalesced", tensors, str(op))
    native, staged = g.native_for(tensors[0])
    ts, pairs = _stage(tensors, staged)
    w = native.allreduce_coalesced(ts, _to_reduce_op(op))
    return _finish(_StagedWork(w, pairs) if pairs else w, async_op)


def broadcast(tensor: torch.Tensor, src: int = 0, group=None, async_op: bool = False, group_src: Optional[int] = None):
    if _not_member(group):
        return None
    g = _resolve(group)
    root = group_src if group_src is not None else g.local_rank_of(src)
    if _coalesce(g, "broadcast", tensor, root=root):
        return None
    _pre(g, "broadcast", [tensor], f"root={root}")
    native, staged = g.native_for(tensor)
    ts, pairs = _stage([tensor], staged)
    w = native.broadcast(ts, root)
    return _finish(_StagedWork(w, pairs) if pairs else w, async_op)


def all_gather(tensor_list: List[torch.Tensor], tensor: torch.Tensor, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    _pre(g, "all_gather", [tensor])
    native, staged = g.native_for(tensor)
    if staged:
        outs = [torch.empty_like(tensor, device="cpu") for _ in tensor_list]
        w = native.allgather(outs, tensor.detach().cpu())
        return _finish(_StagedWork(w, list(zip(tensor_list, outs))), async_op)
    w = native.allgather(tensor_list, tensor)
    return _finish(w, async_op)


def all_gather_into_tensor(output_tensor: torch.Tensor, input_tensor: torch.Tensor, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    if _coalesce(g, "all_gather_into_tensor", output_tensor, input_tensor):
        return None
    _pre(g, "all_gather_into_tensor", [output_tensor, input_tensor])
    native, staged = g.native_for(input_tensor)
    (o, i), pairs = _stage([output_tensor, input_tensor], staged)
    w = native.allgather_into_tensor(o, i)
    return _finish(_StagedWork(w, pairs[:1]) if pairs else w, async_op)


def reduce_scatter_tensor(output: torch.Tensor, input: torch.Tensor, op=ReduceOp.SUM, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    if _coalesce(g, "reduce_scatter_tensor", output, input, op=op):
        return None
    _pre(g, "reduce_scatter_tensor", [output, input], str(op))
    native, staged = g.native_for(input)
    (o, i), pairs = _stage([output, input], staged)
    w = native.reduce_scatter_tensor(o, i, _to_reduce_op(op))
    return _finish(_StagedWork(w, pairs[:1]) if pairs else w, async_op)


def reduce_scatter(output: torch.Tensor, input_list: List[torch.Tensor], op=ReduceOp.SUM, group=None, async_op: bool = False):
    flat = torch.cat([t.reshape(-1) for t in input_list])
    out = output.reshape(-1) if output.is_contiguous() else output.contiguous().reshape(-1)
    w = reduce_scatter_tensor(out, flat, op, group, async_op=False)
    if not output.is_contiguous():
        output.copy_(out.view_as(output))
    return None if not async_op else w


def reduce(tensor: torch.Tensor, dst: int = 0, op=ReduceOp.SUM, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    root = g.local_rank_of(dst)
    _pre(g, "reduce", [tensor], f"root={root}|{op}")
    native, staged = g.native_for(tensor)
    ts, pairs = _stage([tensor], staged)
    w = native.reduce(ts[0], root, _to_reduce_op(op))
    return _finish(_StagedWork(w, pairs) if pairs else w, async_op)


def gather(tensor: torch.Tensor, gather_list: Optional[List[torch.Tensor]] = None, dst: int = 0, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    root = g.local_rank_of(dst)
    _pre(g, "gather", [tensor], f"root={root}")
    native, staged = g.native_for(tensor)
    outs = gather_list if gather_list is not None else []
    if staged:
        couts = [torch.empty_like(tensor, device="cpu") for _ in outs]
        w = native.gather(couts, tensor.detach().cpu(), root)
        return _finish(_StagedWork(w, list(zip(outs, couts))), async_op)
    w = native.gather(outs, tensor, root)
    return _finish(w, async_op)


def scatter(tensor: torch.Tensor, scatter_list: Optional[List[torch.Tensor]] = None, src: int = 0, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    root = g.local_rank_of(src)
    _pre(g, "scatter", [tensor], f"root={root}")
    native, staged = g.native_for(tensor)
    ins = scatter_list if scatter_list is not None else []
    if staged:
        cout = torch.empty_like(tensor, device="cpu")
        w = native.scatter(cout, [t.detach().cpu() for t in ins], root)
        return _finish(_StagedWork(w, [(tensor, cout)]), async_op)
    w = native.scatter(tensor, ins, root)
    return _finish(w, async_op)


def all_to_all_single(output: torch.Tensor, input: torch.Tensor, output_split_sizes: Optional[List[int]] = None,
                      input_split_sizes: Optional[List[int]] = None, group=None, async_op: bool = False):
    if _not_member(group):
        return None
    g = _resolve(group)
    _pre(g, "all_to_all_single", [output, input])
    native, staged = g.native_for(input)
    (o, i), pairs = _stage([output, input], staged)
    w = native.alltoall_base(o, i, list(output_split_sizes or []), list(input_split_sizes or []))
    return _finish(_StagedWork(w, pairs[:1]) if pairs else w, async_op)


def all_to_all(output_tensor_list: List[torch.Tensor], input_tensor_list: List[torch.Tensor], group=None, async_op: bool = False):
    inp = torch.cat([t.reshape(-1) for t in input_tensor_list])
    out = torch.empty(sum(t.numel() for t in output_tensor_list), dtype=inp.dtype, device=inp.device)
    all_to_all_single(out, inp, [t.numel() for t in output_tensor_list], [t.numel() for t in input_tensor_list], group)
    off = 0
    for t in output_tensor_list:
        t.copy_(out[off:off + t.numel()].view_as(t))
        off += t.numel()
    return None


def send(tensor: torch.Tensor, dst: int, group=None, tag: int = 0):
    isend(tensor, dst, group, tag).wait()


def recv(tensor: torch.Tensor, src: int, group=None, tag: int = 0) -> int:
    irecv(tensor, src, group, tag).wait()
    return src


def isend(tensor: torch.Tensor, dst: int, group=None, tag: int = 0):
    g = _resolve(group)
    native, staged = g.native_for(tensor)
    t = tensor.detach().cpu() if staged else tensor
    return native.send(t, g.local_rank_of(dst), tag)


def irecv(tensor: torch.Tensor, src: int, group=None, tag: int = 0):
    g = _resolve(group)
    native, staged = g.native_for(tensor)
    if staged:
        c = torch.empty_like(tensor, device="cpu")
        return _StagedWork(native.recv(c, g.local_rank_of(src), tag), [(tensor, c)])
    return native.recv(tensor, g.local_rank_of(src), tag)


class P2POp:
    def __init__(self, op, tensor: torch.Tensor, peer: int, group=None, tag: int = 0):
        self.op, self.tensor, self.peer, self.group, self.tag = op, tensor, peer, group, tag


def batch_isend_irecv(p2p_op_list: List[P2POp]):
    return [op.op(op.tensor, op.peer, op.group, op.tag) for op in p2p_op_list]


def barrier(group=None, async_op: bool = False, device_ids=None):
    """Blocks the host until every member has reached the barrier (c10d semantics)."""
    if _not_member(group):
        return None
    g = _resolve(group)
    _pre(g, "barrier", [])
    use_gpu = g._backends.get("cuda") in _GPU_KINDS and "host" not in g._backends.values() and torch.cuda.is_available()
    if use_gpu:
        dev = device_ids[0] if device_ids else torch.cuda.current_device()
        w = g.gpu(dev).barrier()
    else:
        w = g.host().barrier()
    if async_op:
        return w
    w.wait(True)
    return None


def monitored_barrier(group=None, timeout: Optional[_dt.timedelta] = None, wait_all_ranks: bool = False):
    """Store-based barrier that names the ranks that failed to arrive (c10d monitored_barrier)."""
    g = _resolve(group)
    timeout = timeout or g._timeout
    g._coll_count += 1
    st = C.PrefixStore(f"{g.group_name}/mbarrier/{g._coll_count}", _world.store)
    st.set(f"arrived/{g.rank()}", b"1")
    if g.rank() == 0:
        missing = []
        for r in range(g.size()):
            try:
                st.wait([f"arrived/{r}"], timeout)
            except Exception:
                missing.append(g.ranks[r])
                if not wait_all_ranks:
                    break
        if missing:
            raise RuntimeError(f"ringdp monitored_barrier: ranks {missing} failed to pass the barrier within {timeout}")
        st.set("release", b"1")
    else:
        st.wait(["release"], timeout)


# ----------------------------------------------------------------------------- object collectives
def _obj_device(g: ProcessGroup):
    if "host" in g._backends.values() or not torch.cuda.is_available():
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def _pack(obj, device):
    data = pickle.dumps(obj)
    return torch.frombuffer(bytearray(data), dtype=torch.uint8).to(device), len(data)


def all_gather_object(object_list: List[Any], obj: Any, group=None):
    if _not_member(group):
        return
    g = _resolve(group)
    dev = _obj_device(g)
    t, n = _pack(obj, dev)
    sizes = [torch.zeros(1, dtype=torch.long, device=dev) for _ in range(g.size())]
    all_gather(sizes, torch.tensor([n], dtype=torch.long, device=dev), group=g)
    mx = int(max(int(s.item()) for s in sizes))
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    buf[:n] = t
    outs = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(g.size())]
    all_gather(outs, buf, group=g)
    for i, (o, s) in enumerate(zip(outs, sizes)):
        object_list[i] = pickle.loads(o[: int(s.item())].cpu().numpy().tobytes())


def gather_object(obj: Any, object_gather_list: Optional[List[Any]] = None, dst: int = 0, group=None):
    tmp = [None] * get_world_size(group)
    all_gather_object(tmp, obj, group)
    if get_rank() == dst and object_gather_list is not None:
        object_gather_list[:] = tmp


def broadcast_object_list(object_list: List[Any], src: int = 0, group=None, device=None):
    if _not_member(group):
        return
    g = _resolve(group)
    dev = device or _obj_device(g)
    is_src = _default().rank() == src
    if is_src:
        t, n = _pack(list(object_list), dev)
        size = torch.tensor([n], dtype=torch.long, device=dev)
    else:
        size = torch.zeros(1, dtype=torch.long, device=dev)
    broadcast(size, src, group=g)
    n = int(size.item())
    buf = t if is_src else torch.empty(n, dtype=torch.uint8, device=dev)
    broadcast(buf, src, group=g)
    if not is_src:
        vals = pickle.loads(buf.cpu().numpy().tobytes())
        object_list[:] = vals


def scatter_object_list(scatter_object_output_list: List[Any], scatter_object_input_list: Optional[List[Any]] = None,
                        src: int = 0, group=None):
    objs = list(scatter_object_input_list) if scatter_object_input_list is not None else None
    holder = [objs]
    broadcast_object_list(holder, src=src, group=group)
    scatter_object_output_list[0] = holder[0][get_rank(group)]


# ----------------------------------------------------------------------------- misc helpers
class _CoalescingManager:
    """Collects the collectives issued inside ``_coalescing_manager`` and submits them as one
    native batch (RCCL: a single ncclGroupStart/End, i.e. one fused launch and one completion
    event).  Upstream: ``torch.distributed._coalescing_manager``."""

    _KIND = {"all_reduce": 0, "broadcast": 1, "all_gather_into_tensor": 2, "reduce_scatter_tensor": 3}

    def __init__(self, group: ProcessGroup):
        self.group = group
        self.ops = []
        self.works = []

    def append(self, kind: str, out: torch.Tensor, inp: Optional[torch.Tensor] = None, root: int = 0, op=None):
        self.ops.append((self._KIND[kind], out, inp, root, _to_reduce_op(op if op is not None else ReduceOp.SUM)))

    def flush(self):
        if not self.ops:
            return
        native, staged = self.group.native_for(self.ops[0][1])
        if staged:
            # host backend with GPU tensors: issue one by one through the staging path
            for kind, out, inp, root, op in self.ops:
                if kind == 0:
                    self.works.append(all_reduce(out, op, self.group, async_op=True))
                elif kind == 1:
                    self.works.append(broadcast(out, self.group.ranks[root], self.group, async_op=True))
                elif kind == 2:
                    self.works.append(all_gather_into_tensor(out, inp, self.group, async_op=True))
                else:
                    self.works.append(reduce_scatter_tensor(out, inp, op, self.group, async_op=True))
        else:
            self.works.append(native.coalesced(self.ops))
        self.ops = []

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []


_coalescing = threading.local()


def _coalesce(g: ProcessGroup, kind: str, out, inp=None, root: int = 0, op=None) -> bool:
    """Inside _coalescing_manager for group ``g``: record the op instead of issuing it."""
    cm = getattr(_coalescing, "cm", None)
    if cm is None or cm.group is not g:
        return False
    cm.append(kind, out, inp, root, op)
    return True


@contextmanager
def _coalescing_manager(group=None, device=None, async_ops: bool = False):
    """``with _coalescing_manager(group, async_ops=True) as cm: all_reduce(a); all_reduce(b)``
    issues both as one RCCL group on exit; ``cm.wait()`` then fences the caller's stream
    (``async_ops=False`` waits on exit)."""
    g = _resolve(group)
    if getattr(_coalescing, "cm", None) is not None:
        raise RuntimeError("ringdp: _coalescing_manager cannot be nested")
    cm = _CoalescingManager(g)
    _coalescing.cm = cm
    try:
        yield cm
    finally:
        _coalescing.cm = None
    cm.flush()
    if not async_ops:
        cm.wait()


def get_default_store():
    return _world.store


def native_group(group=None, device: Optional[int] = None):
    """The native communicator that serves ``group`` on ``device`` (GPU) or the host."""
    g = _resolve(group)
    if "fake" in g._backends.values():
        return g.host()
    if device is None:
        return g.host()
    return g.gpu(device)
