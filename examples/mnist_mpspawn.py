"""W1: MNIST ConvNet, DDP via ringdp.spawn (one process per GPU) - the ringdp version of the
reference's ``mpspawn_dist.py`` (ref/mpspawn_dist.py:46-145).

    python examples/mnist_mpspawn.py -n 1 -g 2 -nr 0 --epochs 2
    # two hosts: run on each with -n 2 -nr {0,1} and MASTER_ADDR/MASTER_PORT of node 0

Same flags and rank arithmetic (rank = nr * gpus + gpu), same log lines.  Differences, all
MI355X-first: the dataset lives in HBM and each batch is one fused gather kernel
(``DeviceLoader``; the uint8 pixels feed conv1, which fuses ToTensor+Normalize); the model runs on
ringdp's MFMA kernels; gradients are bucket-all-reduced by ringdp's C++ reducer on RCCL.  Without a
GPU (or with ``--cpu``) the same script runs on the host-ring backend ("gloo") with ATen math.
MASTER_ADDR defaults to 127.0.0.1 instead of the reference's hard-coded 172.16.16.5.
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


def train(gpu, args):
    rank = args.nr * args.gpus + gpu
    os.environ["LOCAL_RANK"] = str(gpu)  # log gating on the local rank, like the reference
    print("My rank is: " + str(rank))
    use_gpu = torch.cuda.is_available() and not args.cpu
    dist.init_process_group(backend="nccl" if use_gpu else "gloo", init_method="env://",
                            world_size=args.world_size, rank=rank)
    torch.manual_seed(0)  # identical init on every rank (ref/mpspawn_dist.py:56)
    model = ConvNet()
    if use_gpu:
        torch.cuda.set_device(gpu)
        model.cuda(gpu)
    log("load model sucessfully!")
    batch_size = args.batch_size
    criterion = CrossEntropyLoss()
    optimizer = SGD(model.parameters(), lr=args.lr)
    model = ringdp.DistributedDataParallel(model, device_ids=[gpu] if use_gpu else None)
    log("Sucessfully wrap the model!")

    if use_gpu:
        train_data, synthetic = mnist_or_synthetic(args.data)
        sampler = DistributedSampler(train_data, num_replicas=args.world_size, rank=rank)  # shuffle=True, seed 0 (ref :77-81)
        loader = DeviceLoader(train_data, batch_size, torch.device("cuda", gpu), sampler=sampler,
                              out_dtype=torch.uint8)
    else:
        tf = T.Compose([T.ToTensor(), T.Normalize((0.1307,), (0.3081,))])
        train_data, synthetic = mnist_or_synthetic(args.data, transform=tf)
        sampler = DistributedSampler(train_data, num_replicas=args.world_size, rank=rank)  # shuffle=True, seed 0 (ref :77-81)
        loader = DataLoader(train_data, batch_size=batch_size, shuffle=False, sampler=sampler)
    if synthetic:
        log(f"[note] MNIST not found under {args.data}: using synthetic 1x28x28 data of the same shape")
    log("Load data....done!")

    clock = WallClock()
    total_step = len(loader)
    log("Total step: ", total_step)
    for epoch in range(args.epochs):
        if hasattr(loader, "set_epoch"):
            loader.set_epoch(epoch)
        for i, (images, labels) in enumerate(loader):
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


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("-n", "--nodes", default=1, type=int, metavar="N")
    parser.add_argument("-g", "--gpus", default=1, type=int, help="processes (GPUs) per node")
    parser.add_argument("-nr", "--nr", default=0, type=int, help="ranking within the nodes")
    parser.add_argument("--epochs", default=2, type=int, metavar="N")
    parser.add_argument("--batch-size", default=100, type=int)
    parser.add_argument("--lr", default=1e-4, type=float)
    parser.add_argument("--data", default="./data")
    parser.add_argument("--cpu", action="store_true", help="force the host-ring (gloo) CPU path")
    parser.add_argument("--max-steps", default=0, type=int, help="stop each epoch early (smoke runs)")
    parser.add_argument("--log-every", default=100, type=int)
    args = parser.parse_args(argv)
    args.world_size = args.gpus * args.nodes
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "8888")
    print("Get environment successfully")
    ringdp.spawn(train, nprocs=args.gpus, args=(args,))


if __name__ == "__main__":
    main()
