"""W2: ResNet-18 / CIFAR-10, DDP via ringdp.spawn with a ``tcp://`` init URL - the ringdp version of
the reference's ``example_mp.py`` (ref/example_mp.py:15-132).

    python examples/cifar_resnet_mp.py --nodes 1 --ngpus_per_node 8 --dist-url tcp://127.0.0.1:12345
    # CPU plumbing check (host-ring "gloo" backend):
    python examples/cifar_resnet_mp.py --ngpus_per_node 2 --cpu --epochs 1 --max-steps 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import ringdp  # noqa: E402
import ringdp.distributed as dist  # noqa: E402
from _cifar_train import train  # noqa: E402


def train_worker(local_rank, ngpus_per_node, args):
    args.global_rank = args.node_rank * ngpus_per_node + local_rank
    os.environ["LOCAL_RANK"] = str(local_rank)
    use_gpu = torch.cuda.is_available() and not args.cpu
    if use_gpu:
        torch.cuda.set_device(local_rank)
    dist.init_process_group(backend="nccl" if use_gpu else "gloo", init_method=args.dist_url,
                            world_size=args.global_world_size, rank=args.global_rank)
    train(local_rank, args.global_rank, use_gpu, args)


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--nodes", default=1, type=int, help="number of nodes for distributed training")
    parser.add_argument("--ngpus_per_node", default=2, type=int, help="processes (GPUs) per node")
    parser.add_argument("--dist-url", default="tcp://127.0.0.1:12345", type=str, help="rendezvous URL")
    parser.add_argument("--node_rank", default=0, type=int, help="node rank for distributed training")
    parser.add_argument("--epochs", default=5, type=int)
    parser.add_argument("--batch-size", default=256, type=int)
    parser.add_argument("--lr", default=0.01 * 2, type=float)
    parser.add_argument("--workers", default=4, type=int)
    parser.add_argument("--data", default="./data")
    parser.add_argument("--cpu", action="store_true")
    parser.add_argument("--max-steps", default=0, type=int)
    args = parser.parse_args(argv)
    args.global_world_size = args.ngpus_per_node * args.nodes
    ringdp.spawn(train_worker, nprocs=args.ngpus_per_node, args=(args.ngpus_per_node, args))


if __name__ == "__main__":
    main()
