"""W2: ResNet-18 / CIFAR-10, launch-style entrypoint - the ringdp version of the reference's
``example_launch.py`` (ref/example_launch.py:14-107).

    python -m ringdp.run --nproc-per-node=8 examples/cifar_resnet_launch.py
    python -m ringdp.launch --nproc_per_node=2 examples/cifar_resnet_launch.py --cpu --epochs 1 --max-steps 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import ringdp.distributed as dist  # noqa: E402
from _cifar_train import train  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--local-rank", "--local_rank", type=int, default=None)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--batch-size", type=int, default=128)  # global batch 256 on 2 GPUs, as the reference
    p.add_argument("--lr", type=float, default=0.01 * 2)
    p.add_argument("--workers", type=int, default=4)
    p.add_argument("--data", default="./data")
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--max-steps", type=int, default=0)
    args = p.parse_args(argv)
    local_rank = int(os.environ.get("LOCAL_RANK", args.local_rank if args.local_rank is not None else 0))
    rank = int(os.environ["RANK"])
    use_gpu = torch.cuda.is_available() and not args.cpu
    if use_gpu:
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
    dist.init_process_group(backend="nccl" if use_gpu else "gloo")
    train(local_rank, rank, use_gpu, args)


if __name__ == "__main__":
    main()
