"""One rank whose captured step stalls longer than the process-group timeout: the replay watchdog
(ringdp.utils.graph.StepGraph -> ReplayBeacon + RcclPG.watch_beacon) must abort the communicator and end the
process non-zero.  The stall is a bounded spin kernel (torch.cuda._sleep) captured into the graph,
so nothing on the GPU ever waits forever.  Run by tests/test_watchdog_gpu.py through ringdp.run."""
import datetime
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

import ringdp.distributed as dist  # noqa: E402
from ringdp.models import ConvNet  # noqa: E402
from ringdp.nn import CrossEntropyLoss  # noqa: E402
from ringdp.optim import SGD  # noqa: E402
from ringdp.parallel import DistributedDataParallel as DDP  # noqa: E402
from ringdp.utils.graph import StepGraph  # noqa: E402


def main():
    stall_cycles = int(sys.argv[1])
    # split=<buckets>: the segmented capture (bench.py's default placement) with RINGDP_SPLIT_BUCKETS=<buckets>
    # ("1": bucket 0 inline, bucket 1 between segments, the last inline; "": every bucket inline)
    split = len(sys.argv) > 2 and sys.argv[2].startswith("split=")
    if split:
        os.environ["RINGDP_SPLIT_BUCKETS"] = sys.argv[2][len("split="):]
    os.environ["RINGDP_DDP_FORCE_COMM"] = "1"
    os.environ["RINGDP_GRAPH_WATCHDOG"] = "1"  # one rank: watched only when forced
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group("nccl", timeout=datetime.timedelta(milliseconds=int(os.environ["WD_TIMEOUT_MS"])))
    torch.manual_seed(0)
    model = ConvNet().cuda()
    ddp = DDP(model, device_ids=[torch.cuda.current_device()], bucket_cap_mb=0.1 if split else 25.0,
              first_bucket_mb=0.05 if split else None)
    opt = SGD(ddp.parameters(), lr=1e-3)
    crit = CrossEntropyLoss()
    x = torch.randint(0, 256, (64, 1, 28, 28), dtype=torch.uint8, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda")
    stall = {"on": False}

    def step():
        if stall["on"]:
            torch.cuda._sleep(stall_cycles)
        loss = crit(ddp(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    stall["on"] = True
    g = StepGraph(step, warmup=0, split_ddp=ddp if split else None).capture()
    if split:
        print("split plan", [b["placement"] for b in g.split_info], flush=True)
    print("captured; replaying", flush=True)
    g.replay()
    torch.cuda.synchronize()  # the watchdog ends the process while we wait here
    print("replay finished without the watchdog firing", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
