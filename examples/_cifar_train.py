"""Shared W2 training loop (ResNet-18 on CIFAR-10 shapes) for the spawn and launch examples.

Mirrors ref/example_mp.py:44-129 / ref/example_launch.py:17-107: DDP ResNet-18, RandomCrop(32, 4) +
RandomHorizontalFlip + Normalize(CIFAR mean/std), DistributedSampler(shuffle=True) with
set_epoch, SGD(lr=0.01*2, momentum=0.9, weight_decay=1e-4, nesterov=True), running loss / top-1
accuracy printed every 25 steps on global rank 0.
"""
import torch

import ringdp
import ringdp.distributed as dist
from ringdp.data import CIFAR10, DataLoader, DeviceLoader, DistributedSampler, cifar10_or_synthetic, transforms as T
from ringdp.models import resnet18
from ringdp.nn import CrossEntropyLoss
from ringdp.optim import SGD
from ringdp.utils.logging import Meter, log


def train(local_rank: int, global_rank: int, use_gpu: bool, args) -> None:
    # the device the caller bound (set_device): consistent even when local_rank >= device_count
    # (the reference pairs set_device(rank % count) with cuda:local_rank)
    device = torch.device("cuda", torch.cuda.current_device()) if use_gpu else torch.device("cpu")
    print(f"[init] == local rank: {local_rank}, global rank: {global_rank} ==")
    net = resnet18(num_classes=10).to(device)
    net = ringdp.DistributedDataParallel(net, device_ids=[device.index] if use_gpu else None,
                                         output_device=device.index if use_gpu else None)
    mean, std = CIFAR10.mean, CIFAR10.std
    if use_gpu:
        data, synthetic = cifar10_or_synthetic(args.data)
        sampler = DistributedSampler(data, shuffle=True)
        loader = DeviceLoader(data, args.batch_size, device, sampler=sampler, crop_padding=4, hflip=True,
                              mean=mean, std=std, out_dtype=torch.float32, seed=global_rank)
    else:
        tf = T.Compose([T.RandomCrop(32, padding=4), T.RandomHorizontalFlip(), T.ToTensor(), T.Normalize(mean, std)])
        data, synthetic = cifar10_or_synthetic(args.data, transform=tf)
        sampler = DistributedSampler(data, shuffle=True)
        loader = DataLoader(data, batch_size=args.batch_size, num_workers=args.workers, pin_memory=True,
                            sampler=sampler)
    if synthetic:
        log(f"[note] CIFAR-10 not found under {args.data}: using synthetic 3x32x32 data of the same shape")
    criterion = CrossEntropyLoss()
    optimizer = SGD(net.parameters(), lr=args.lr, momentum=0.9, weight_decay=1e-4, nesterov=True)
    log("            =======  Training  ======= \n")
    net.train()
    n_steps = len(loader) if not args.max_steps else min(len(loader), args.max_steps)
    for ep in range(1, args.epochs + 1):
        meter = Meter()
        if hasattr(loader, "set_epoch"):
            loader.set_epoch(ep)
        else:
            sampler.set_epoch(ep)
        for idx, (inputs, targets) in enumerate(loader):
            inputs, targets = inputs.to(device), targets.to(device)
            outputs = net(inputs)
            loss = criterion(outputs, targets)
            optimizer.zero_grad()
            loss.backward()
            optimizer.step()
            meter.update(loss.item(), int(torch.eq(outputs.argmax(dim=1), targets).sum().item()), targets.size(0))
            if (idx + 1) % 25 == 0 or (idx + 1) == n_steps:
                log("   == step: [{:3}/{}] [{}/{}] | loss: {:.3f} | acc: {:6.3f}%".format(
                    idx + 1, len(loader), ep, args.epochs, meter.loss, meter.acc))
            if idx + 1 >= n_steps:
                break
    log("\n            =======  Training Finished  ======= \n")
    dist.destroy_process_group()
