"""DDP communication hooks (parity: torch/distributed/algorithms/ddp_comm_hooks/default_hooks.py).

The three builtins are recognised by ``DistributedDataParallel.register_comm_hook`` and run
inside the native reducer (no Python on the backward path):

* ``allreduce_hook``       - ncclAvg all-reduce of the fp32 bucket (default);
* ``bf16_compress_hook``   - cast the bucket to bf16 with ringdp's cast kernel, ncclAvg in bf16,
                             cast back (halves xGMI bytes; SURVEY.md §2.7 bf16 column);
* ``fp16_compress_hook``   - same in fp16.

Called directly (e.g. from a user-defined hook) they return an async Work.
"""
from __future__ import annotations

import torch

from .. import distributed as dist


def allreduce_hook(process_group, bucket):
    g = process_group if process_group is not None else dist._default()
    return dist.all_reduce(bucket.buffer(), op=dist.ReduceOp.AVG, group=g, async_op=True)


def _compress(process_group, bucket, dtype):
    g = process_group if process_group is not None else dist._default()
    buf = bucket.buffer()
    wire = buf.to(dtype)
    work = dist.all_reduce(wire, op=dist.ReduceOp.AVG, group=g, async_op=True)

    class _Decompress:
        def wait(self, blocking: bool = False):
            work.wait()
            buf.copy_(wire)
            return True

        def result(self):
            return [buf]

    return _Decompress()


def bf16_compress_hook(process_group, bucket):
    return _compress(process_group, bucket, torch.bfloat16)


def fp16_compress_hook(process_group, bucket):
    return _compress(process_group, bucket, torch.float16)
