"""One rank of a 2-rank xGMI DDP run whose rank 1 dies in the middle of hipGraph replays.

Env: RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun contract), FAULT_TIMEOUT_MS (group
timeout), FAULT_AT (replay index at which rank 1 hard-exits), FAULT_SPLIT (set: the segmented capture,
StepGraph(split_ddp=...), with RINGDP_SPLIT_BUCKETS=<its value> - e.g. "1" or "" for all inline).  Rank 0 keeps replaying: its kernels
wait for a peer that never arrives, give up after the timeout, and the watchdog must end the process
non-zero (SURVEY.md §4.3 Fault row).  Prints "SURVIVED" if rank 0 ever gets past its loop (a bug)."""
import datetime
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ringdp.distributed as dist  # noqa: E402
from ringdp.models import ConvNet  # noqa: E402
from ringdp.nn import CrossEntropyLoss  # noqa: E402
from ringdp.optim import SGD  # noqa: E402
from ringdp.parallel import DistributedDataParallel as DDP  # noqa: E402
from ringdp.utils.graph import StepGraph  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    dev = rank % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    tmo = datetime.timedelta(milliseconds=int(os.environ.get("FAULT_TIMEOUT_MS", "4000")))
    dist.init_process_group("xgmi", timeout=tmo)
    fault_at = int(os.environ.get("FAULT_AT", "3"))
    torch.manual_seed(0)
    model = ConvNet().cuda()
    ddp = DDP(model, device_ids=[dev], bucket_cap_mb=0.1, first_bucket_mb=0.05)
    opt = SGD(ddp.parameters(), lr=0.01)
    crit = CrossEntropyLoss()
    x = torch.randint(0, 256, (64, 1, 28, 28), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda")

    def step():
        loss = crit(ddp(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(2):
        step()
    split = os.environ.get("FAULT_SPLIT")
    if split is not None:
        os.environ["RINGDP_SPLIT_BUCKETS"] = split
    g = StepGraph(step, warmup=1, split_ddp=ddp if split is not None else None).capture()
    if split is not None:
        print(f"rank {rank}: split plan {[b['placement'] for b in g.split_info]}", file=sys.stderr, flush=True)
    for i in range(10_000):
        if rank == 1 and i == fault_at:
            torch.cuda.synchronize()
            print(f"rank 1: exiting at replay {i}", file=sys.stderr, flush=True)
            os._exit(17)
        g.replay()
        if i % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    print("SURVIVED", flush=True)


if __name__ == "__main__":
    main()
