"""``python -m ringdp.run`` / ``python -m ringdp.launch``: multi-process launcher.

Parity: ``torch.distributed.run`` (torchrun) and the legacy ``torch.distributed.launch``
(``ref/README.md:341-343``, ``ref/launch_dist.py:45-46``):

* flags ``--nnodes --nproc-per-node/--nproc_per_node --node-rank/--node_rank
  --master-addr/--master_addr --master-port/--master_port --max-restarts --standalone
  --monitor-interval -m/--module --no-python --log-dir``;
* worker env: RANK, LOCAL_RANK, GROUP_RANK, ROLE_RANK, ROLE_NAME, LOCAL_WORLD_SIZE, WORLD_SIZE,
  ROLE_WORLD_SIZE, GROUP_WORLD_SIZE, MASTER_ADDR, MASTER_PORT, TORCHELASTIC_RESTART_COUNT,
  TORCHELASTIC_MAX_RESTARTS, TORCHELASTIC_RUN_ID (+ RINGDP_RESTART_COUNT); OMP_NUM_THREADS=1
  when nproc > 1 and unset;
* ``ringdp.launch`` (legacy) also appends ``--local-rank=N`` to the worker argv unless
  ``--use-env`` is given; ``ringdp.run`` never does;
* the launcher monitors its workers; on the first failure it terminates the rest (SIGTERM, then
  SIGKILL after a grace period) and either restarts the whole local group (``--max-restarts``)
  or exits with the failing worker's code.  Rank 0's process hosts the rendezvous store on
  MASTER_PORT, exactly like a script started by the legacy launcher.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
import uuid
from typing import List, Optional


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def get_args_parser(legacy: bool = False) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="ringdp multi-process launcher (one process per GPU)")
    p.add_argument("--nnodes", type=str, default="1", help="number of nodes (N or MIN:MAX; static only)")
    p.add_argument("--nproc-per-node", "--nproc_per_node", type=str, default="1",
                   help="processes per node: an int, 'gpu' or 'auto'")
    p.add_argument("--node-rank", "--node_rank", type=int, default=0)
    p.add_argument("--master-addr", "--master_addr", type=str, default="127.0.0.1")
    p.add_argument("--master-port", "--master_port", type=int, default=29500)
    p.add_argument("--max-restarts", "--max_restarts", type=int, default=0)
    p.add_argument("--monitor-interval", "--monitor_interval", type=float, default=0.1)
    p.add_argument("--standalone", action="store_true",
                   help="single node: pick a free port on 127.0.0.1")
    p.add_argument("--rdzv-backend", "--rdzv_backend", type=str, default="static")
    p.add_argument("--rdzv-endpoint", "--rdzv_endpoint", type=str, default="")
    p.add_argument("--rdzv-id", "--rdzv_id", type=str, default="none")
    p.add_argument("--run-id", "--run_id", type=str, default=None)
    p.add_argument("--local-addr", "--local_addr", type=str, default=None)
    p.add_argument("--log-dir", "--log_dir", type=str, default=None,
                   help="write each worker's stdout/stderr to <log-dir>/attempt_<k>/<rank>/")
    p.add_argument("--grace-period", type=float, default=10.0)
    p.add_argument("-m", "--module", action="store_true", help="run the script as a python module")
    p.add_argument("--no-python", "--no_python", action="store_true",
                   help="execute the script directly instead of through the interpreter")
    if legacy:
        p.add_argument("--use-env", "--use_env", action="store_true",
                       help="do not pass --local-rank=N in argv (read LOCAL_RANK from env)")
    p.add_argument("training_script", type=str)
    p.add_argument("training_script_args", nargs=argparse.REMAINDER)
    return p


def _nproc(v: str) -> int:
    if v in ("gpu", "auto"):
        try:
            import torch

            n = torch.cuda.device_count()
        except Exception:
            n = 0
        return n if n > 0 else (1 if v == "gpu" else (os.cpu_count() or 1))
    return int(v)


class _Worker:
    def __init__(self, local_rank: int, proc: subprocess.Popen, files):
        self.local_rank = local_rank
        self.proc = proc
        self.files = files


def _start_workers(args, nproc: int, nnodes: int, restart: int, run_id: str, legacy_argv: bool) -> List[_Worker]:
    world = nproc * nnodes
    workers = []
    for lr in range(nproc):
        rank = args.node_rank * nproc + lr
        env = dict(os.environ)
        env.update({
            "RANK": str(rank), "LOCAL_RANK": str(lr), "GROUP_RANK": str(args.node_rank),
            "ROLE_RANK": str(rank), "ROLE_NAME": "default", "LOCAL_WORLD_SIZE": str(nproc),
            "WORLD_SIZE": str(world), "ROLE_WORLD_SIZE": str(world), "GROUP_WORLD_SIZE": str(nnodes),
            "MASTER_ADDR": args.master_addr, "MASTER_PORT": str(args.master_port),
            "TORCHELASTIC_RESTART_COUNT": str(restart), "TORCHELASTIC_MAX_RESTARTS": str(args.max_restarts),
            "TORCHELASTIC_RUN_ID": run_id, "RINGDP_RESTART_COUNT": str(restart),
            "PYTHONUNBUFFERED": "1",
        })
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        if nproc > 1 and "OMP_NUM_THREADS" not in os.environ:
            env["OMP_NUM_THREADS"] = "1"
        if args.no_python:
            cmd = [args.training_script]
        elif args.module:
            cmd = [sys.executable, "-u", "-m", args.training_script]
        else:
            cmd = [sys.executable, "-u", args.training_script]
        if legacy_argv:
            cmd.append(f"--local-rank={lr}")
        cmd += list(args.training_script_args)
        files = None
        stdout = stderr = None
        if args.log_dir:
            d = os.path.join(args.log_dir, f"attempt_{restart}", str(rank))
            os.makedirs(d, exist_ok=True)
            files = (open(os.path.join(d, "stdout.log"), "w"), open(os.path.join(d, "stderr.log"), "w"))
            stdout, stderr = files

        def _preexec():
            try:
                import ctypes

                ctypes.CDLL("libc.so.6").prctl(1, int(signal.SIGTERM))  # PR_SET_PDEATHSIG
            except Exception:
                pass

        proc = subprocess.Popen(cmd, env=env, stdout=stdout, stderr=stderr, preexec_fn=_preexec)
        workers.append(_Worker(lr, proc, files))
    return workers


def _stop_workers(workers: List[_Worker], grace: float):
    for w in workers:
        if w.proc.poll() is None:
            try:
                w.proc.send_signal(signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.monotonic() + grace
    for w in workers:
        try:
            w.proc.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            pass
    for w in workers:
        if w.proc.poll() is None:
            w.proc.kill()
            w.proc.wait()
    for w in workers:
        if w.files:
            for f in w.files:
                f.close()


def _monitor(workers: List[_Worker], interval: float):
    """Returns (ok, failed_worker)."""
    while True:
        alive = False
        for w in workers:
            rc = w.proc.poll()
            if rc is None:
                alive = True
            elif rc != 0:
                return False, w
        if not alive:
            return True, None
        time.sleep(interval)


def run(args, legacy: bool = False) -> int:
    if args.standalone:
        args.master_addr = "127.0.0.1"
        args.master_port = _free_port()
        args.nnodes = "1"
        args.node_rank = 0
    nnodes = int(str(args.nnodes).split(":")[-1])
    nproc = _nproc(args.nproc_per_node)
    if not (0 <= args.node_rank < nnodes):
        raise ValueError(f"--node-rank {args.node_rank} out of range for --nnodes {nnodes}")
    run_id = args.run_id or (args.rdzv_id if args.rdzv_id != "none" else uuid.uuid4().hex[:8])
    legacy_argv = legacy and not getattr(args, "use_env", False)
    restart = 0
    stopping = {"sig": None}

    def _on_signal(signum, frame):
        stopping["sig"] = signum

    old_int = signal.signal(signal.SIGINT, _on_signal)
    old_term = signal.signal(signal.SIGTERM, _on_signal)
    try:
        while True:
            workers = _start_workers(args, nproc, nnodes, restart, run_id, legacy_argv)
            ok, failed = False, None
            while True:
                if stopping["sig"] is not None:
                    _stop_workers(workers, args.grace_period)
                    return 128 + int(stopping["sig"])
                done = True
                for w in workers:
                    rc = w.proc.poll()
                    if rc is None:
                        done = False
                    elif rc != 0:
                        failed = w
                        break
                if failed is not None:
                    break
                if done:
                    ok = True
                    break
                time.sleep(args.monitor_interval)
            if ok:
                _stop_workers(workers, 0)
                return 0
            rc = failed.proc.returncode
            rank = args.node_rank * nproc + failed.local_rank
            sys.stderr.write(f"[ringdp.run] worker rank {rank} (local {failed.local_rank}, pid {failed.proc.pid}) "
                             f"failed with exit code {rc}; terminating the local group\n")
            _stop_workers(workers, args.grace_period)
            if restart >= args.max_restarts:
                return rc if rc and rc > 0 else 1
            restart += 1
            sys.stderr.write(f"[ringdp.run] restarting workers (attempt {restart}/{args.max_restarts})\n")
    finally:
        signal.signal(signal.SIGINT, old_int)
        signal.signal(signal.SIGTERM, old_term)


def main(argv: Optional[List[str]] = None, legacy: bool = False) -> int:
    args = get_args_parser(legacy).parse_args(argv)
    return run(args, legacy=legacy)


def launch_local(script: str, script_args: List[str], nproc: int, master_addr: str = "127.0.0.1",
                 master_port: Optional[int] = None, env: Optional[dict] = None) -> int:
    """Programmatic single-node launch: ``nproc`` fresh interpreters running ``script`` with the
    torchrun env contract; returns the group's exit code.  The calling process never touches the
    GPU (it only forks/execs the workers), so a script can re-launch itself as N ranks
    (``bench.py --gpus N``, ref/mpspawn_dist.py:136-140)."""
    argv = ["--nproc-per-node", str(nproc), "--master-addr", master_addr,
            "--master-port", str(master_port if master_port is not None else _free_port())]
    saved = None
    if env:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return main(argv + [script] + list(script_args))
    finally:
        if saved:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v


if __name__ == "__main__":
    sys.exit(main())
