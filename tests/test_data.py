"""Datasets, transforms and loaders (CPU) + the HIP gather/augment kernel (GPU)."""
import os

import numpy as np
import pytest
import torch

from ringdp.data import (CIFAR10, MNIST, DataLoader, DistributedSampler, SyntheticImages, mnist_or_synthetic,
                         transforms as T)
from ringdp.data.datasets import read_idx, write_idx


def _mnist_fixture(tmp_path, n=37):
    rng = np.random.default_rng(0)
    x = rng.integers(0, 256, (n, 28, 28), dtype=np.uint8)
    y = rng.integers(0, 10, (n,), dtype=np.uint8)
    raw = tmp_path / "MNIST" / "raw"
    raw.mkdir(parents=True)
    write_idx(str(raw / "train-images-idx3-ubyte"), x)
    write_idx(str(raw / "train-labels-idx1-ubyte"), y)
    return x, y


def test_idx_roundtrip_and_mnist(tmp_path):
    x, y = _mnist_fixture(tmp_path)
    assert np.array_equal(read_idx(str(tmp_path / "MNIST/raw/train-images-idx3-ubyte")), x)
    ds = MNIST(str(tmp_path), train=True, transform=T.Compose([T.ToTensor(), T.Normalize((0.1307,), (0.3081,))]))
    assert len(ds) == len(x)
    img, t = ds[3]
    assert img.shape == (1, 28, 28) and t == int(y[3])
    ref = (torch.from_numpy(x[3]).float() / 255 - 0.1307) / 0.3081
    torch.testing.assert_close(img[0], ref)
    with pytest.raises(RuntimeError):
        MNIST(str(tmp_path), train=False, download=True)
    _, synth = mnist_or_synthetic(str(tmp_path / "nope"), n_synth=10)
    assert synth


def test_cifar_binary_reader(tmp_path):
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rng = np.random.default_rng(1)
    all_x, all_y = [], []
    for i in range(1, 6):
        y = rng.integers(0, 10, (4,), dtype=np.uint8)
        x = rng.integers(0, 256, (4, 3, 32, 32), dtype=np.uint8)
        rec = np.concatenate([y[:, None], x.reshape(4, -1)], axis=1)
        rec.tofile(str(d / f"data_batch_{i}.bin"))
        all_x.append(x.transpose(0, 2, 3, 1))
        all_y.append(y)
    ds = CIFAR10(str(tmp_path), train=True)
    assert len(ds) == 20
    assert torch.equal(ds.data, torch.from_numpy(np.concatenate(all_x)))
    assert ds.targets.tolist() == np.concatenate(all_y).astype(int).tolist()


def test_transforms_semantics():
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (32, 32, 3), dtype=torch.uint8, generator=g)
    t = T.ToTensor()(img)
    assert t.shape == (3, 32, 32) and t.dtype == torch.float32 and float(t.max()) <= 1.0
    torch.testing.assert_close(t, img.permute(2, 0, 1).float() / 255)
    n = T.Normalize((0.5, 0.4, 0.3), (0.2, 0.2, 0.2))(t)
    torch.testing.assert_close(n[1], (t[1] - 0.4) / 0.2)
    crop = T.RandomCrop(32, padding=4, generator=torch.Generator().manual_seed(3))(img)
    assert crop.shape == (32, 32, 3)
    # every crop is a window of the zero-padded image
    padded = torch.nn.functional.pad(img.permute(2, 0, 1), (4, 4, 4, 4)).permute(1, 2, 0)
    assert any(torch.equal(crop, padded[i:i + 32, j:j + 32]) for i in range(9) for j in range(9))
    flip = T.RandomHorizontalFlip(p=1.0)(img)
    assert torch.equal(flip, img.flip(1))
    assert torch.equal(T.RandomHorizontalFlip(p=0.0)(img), img)


@pytest.mark.parametrize("workers,mode", [(0, "process"), (3, "process"), (3, "thread")])
def test_dataloader_with_distributed_sampler(workers, mode):
    ds = SyntheticImages(103, (28, 28), 10, seed=1, transform=T.ToTensor())
    seen = []
    for rank in range(2):
        s = DistributedSampler(ds, num_replicas=2, rank=rank, shuffle=True, seed=5)
        s.set_epoch(2)
        dl = DataLoader(ds, batch_size=10, sampler=s, num_workers=workers, worker_mode=mode)
        order = list(iter(s))
        got = []
        for xb, yb in dl:
            assert xb.shape[1:] == (1, 28, 28)
            got.append(yb)
        assert len(got) == len(dl) == 6
        assert torch.cat(got).tolist() == ds.targets[order].tolist()
        seen += order
    assert sorted(set(seen)) == list(range(103))
    with pytest.raises(ValueError):
        DataLoader(ds, batch_size=4, shuffle=True, sampler=DistributedSampler(ds, num_replicas=1, rank=0))
    assert len(DataLoader(ds, batch_size=10, drop_last=True)) == 10


class _PidData:
    """Each sample reports the pid of the process that produced it and a draw from torch's RNG."""

    def __init__(self, n, fail_at=None):
        self.n, self.fail_at = n, fail_at

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        if i == self.fail_at:
            raise ValueError(f"bad sample {i}")
        return torch.tensor([i, os.getpid()]), int(torch.randint(0, 1 << 30, ()))


def test_dataloader_worker_processes():
    ds = _PidData(40)
    dl = DataLoader(ds, batch_size=4, num_workers=2, generator=torch.Generator().manual_seed(7))
    ids, pids, draws = [], set(), []
    for xb, rb in dl:
        ids += xb[:, 0].tolist()
        pids |= set(xb[:, 1].tolist())
        draws.append(rb)
    assert ids == list(range(40))                 # sampler order, whatever worker finished first
    assert os.getpid() not in pids and len(pids) == 2  # produced in two separate processes
    # reproducible per-worker seeding: the same generator seed gives the same random draws
    dl2 = DataLoader(ds, batch_size=4, num_workers=2, generator=torch.Generator().manual_seed(7))
    assert torch.equal(torch.cat(draws), torch.cat([r for _, r in dl2]))
    # batch 0 (worker 0) and batch 1 (worker 1) drew from differently seeded streams
    assert not torch.equal(draws[0], draws[1])


def test_dataloader_worker_exception_propagates():
    dl = DataLoader(_PidData(20, fail_at=13), batch_size=4, num_workers=2)
    with pytest.raises(ValueError, match="bad sample 13"):
        for _ in dl:
            pass


def _mix64(z):
    M = (1 << 64) - 1
    z = (z + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def _host_gather_augment(x, y, idx, pad, flip, mean, std, seed):
    """Reference: same per-sample crop/flip choices as the kernel, torchvision op order."""
    out = []
    for b, i in enumerate(idx.tolist()):
        r = _mix64(seed ^ _mix64(b))
        span = 2 * pad + 1
        oy, ox = (r % span, (r >> 16) % span) if pad else (0, 0)
        img = x[i] if x.dim() == 4 else x[i].unsqueeze(-1)
        p = torch.nn.functional.pad(img.permute(2, 0, 1), (pad, pad, pad, pad))
        H, W = img.shape[0], img.shape[1]
        crop = p[:, oy:oy + H, ox:ox + W]
        if flip and ((r >> 40) & 1):
            crop = crop.flip(2)
        t = crop.float() / 255
        m = torch.tensor(mean).view(-1, 1, 1)
        s = torch.tensor(std).view(-1, 1, 1)
        out.append((t - m) / s)
    return torch.stack(out), y[idx]


@pytest.mark.gpu
@pytest.mark.parametrize("shape,pad,flip", [((28, 28), 0, False), ((32, 32, 3), 4, True)])
def test_gather_augment_kernel(shape, pad, flip):
    import ringdp

    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 256, (50, *shape), dtype=torch.uint8, generator=g)
    y = torch.randint(0, 10, (50,), generator=g)
    idx = torch.randperm(50, generator=g)[:17]
    C = 1 if len(shape) == 2 else shape[2]
    mean, std = [0.4914, 0.4822, 0.4465][:C], [0.2023, 0.1994, 0.2010][:C]
    out, yo = ringdp._C.gather_augment(x.cuda(), y.cuda(), idx.cuda(), pad, flip, mean, std, 1234, False,
                                       torch.float32)
    ref, yref = _host_gather_augment(x, y, idx, pad, flip, mean, std, 1234)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(yo.cpu(), yref)
    nhwc, _ = ringdp._C.gather_augment(x.cuda(), y.cuda(), idx.cuda(), pad, flip, mean, std, 1234, True,
                                       torch.bfloat16)
    torch.testing.assert_close(nhwc.float().cpu().permute(0, 3, 1, 2), ref, rtol=1e-2, atol=2e-2)
    raw, _ = ringdp._C.gather_augment(x.cuda(), None, idx.cuda(), 0, False, [], [], 0, False, torch.uint8)
    assert torch.equal(raw.cpu().squeeze(1) if C == 1 else raw.cpu(), x[idx] if C == 1 else x[idx].permute(0, 3, 1, 2))


@pytest.mark.gpu
def test_device_loader_epoch():
    from ringdp.data import DeviceLoader

    ds = SyntheticImages(64, (28, 28), 10, seed=2)
    s = DistributedSampler(ds, num_replicas=2, rank=1, shuffle=True, seed=1)
    dl = DeviceLoader(ds, 8, "cuda", sampler=s, out_dtype=torch.uint8)
    dl.set_epoch(3)
    ys = torch.cat([yb for _, yb in dl]).cpu()
    assert ys.tolist() == ds.targets[list(iter(s))].tolist()
    assert len(dl) == 4
