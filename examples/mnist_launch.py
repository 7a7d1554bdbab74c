"""W1: MNIST ConvNet, launch-style entrypoint - the ringdp version of the reference's
``launch_dist.py`` (ref/launch_dist.py:43-102).

    python -m ringdp.launch --nproc_per_node=8 examples/mnist_launch.py
    python -m ringdp.run --nproc-per-node=8 examples/mnist_launch.py --epochs 1
    # two hosts: --nnodes=2 --node_rank={0,1} --master_addr=<node0> --master_port=22222

RANK / LOCAL_RANK come from the launcher's env (the legacy launcher also passes --local-rank).
The reference builds its DistributedSampler with ``rank=local_rank`` - wrong on >1 node (SURVEY.md
§2.8); here the sampler uses the global rank.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import ringdp  # noqa: E402
import ringdp.distributed as dist  # noqa: E402
from ringdp.data import DataLoader, DeviceLoader, DistributedSampler, mnist_or_synthetic, transforms as T  # noqa: E402
from ringdp.models import ConvNet  # noqa: E402
from ringdp.nn import CrossEntropyLoss  # noqa: E402
from ringdp.optim import SGD  # noqa: E402
from ringdp.utils.logging import WallClock, log, step_line  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--local-rank", "--local_rank", type=int, default=None)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--batch-size", type=int, default=100)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--data", default="./data")
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--max-steps", type=int, default=0)
    p.add_argument("--log-every", type=int, default=100)
    args = p.parse_args(argv)

    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", args.local_rank if args.local_rank is not None else 0))
    use_gpu = torch.cuda.is_available() and not args.cpu
    if use_gpu:
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
    dist.init_process_group("nccl" if use_gpu else "gloo")
    torch.manual_seed(0)
    # the device bound above (the reference uses cuda:local_rank here, which disagrees with set_device(rank %
    # count) whenever local_rank >= device_count - SURVEY §2.8-2)
    device = torch.device("cuda", torch.cuda.current_device()) if use_gpu else torch.device("cpu")
    model = ConvNet().to(device)
    criterion = CrossEntropyLoss()
    optimizer = SGD(model.parameters(), lr=args.lr)
    model = ringdp.DistributedDataParallel(model, device_ids=[device.index] if use_gpu else None,
                                           output_device=device.index if use_gpu else None)
    world = dist.get_world_size()
    if use_gpu:
        data, synthetic = mnist_or_synthetic(args.data)
        sampler = DistributedSampler(data, num_replicas=world, rank=rank)
        loader = DeviceLoader(data, args.batch_size, device, sampler=sampler, out_dtype=torch.uint8)
    else:
        data, synthetic = mnist_or_synthetic(args.data, transform=T.Compose([T.ToTensor(), T.Normalize((0.1307,), (0.3081,))]))
        sampler = DistributedSampler(data, num_replicas=world, rank=rank)
        loader = DataLoader(data, batch_size=args.batch_size, shuffle=False, sampler=sampler, pin_memory=True)
    if synthetic:
        log(f"[note] MNIST not found under {args.data}: using synthetic 1x28x28 data of the same shape")
    clock = WallClock()
    total_step = len(loader)
    log("Total step: ", total_step)
    for epoch in range(args.epochs):
        sampler.set_epoch(epoch)
        for i, (images, labels) in enumerate(loader):
            images = images.to(device, non_blocking=True)
            labels = labels.to(device, non_blocking=True)
            outputs = model(images)
            loss = criterion(outputs, labels)
            optimizer.zero_grad()
            loss.backward()
            optimizer.step()
            if (i + 1) % args.log_every == 0 or args.max_steps and i + 1 == args.max_steps:
                log(step_line(epoch, args.epochs, i, total_step, loss.item()), rank_filter="local")
            if args.max_steps and i + 1 >= args.max_steps:
                break
    log("Training complete in: " + str(clock.elapsed()), rank_filter="local")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
