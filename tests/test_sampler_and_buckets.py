"""DistributedSampler index parity and bucket-assignment parity with upstream PyTorch
(SURVEY.md §4.3 rows 1-2, §2.6/§2.7 measured layouts)."""
import sys

import pytest
import torch
import torch.distributed as tdist
import torch.nn as nn
from torch.utils.data import DistributedSampler as TorchSampler

from ringdp.data import DeviceDistributedSampler, DistributedSampler


@pytest.mark.parametrize("n", [1, 7, 100, 1001, 60000])
@pytest.mark.parametrize("reps", [1, 2, 3, 8])
@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("drop_last", [True, False])
def test_sampler_parity(n, reps, shuffle, drop_last):
    ds = list(range(n))
    for rank in range(reps):
        for seed in (0, 17):
            a = DistributedSampler(ds, num_replicas=reps, rank=rank, shuffle=shuffle, seed=seed, drop_last=drop_last)
            b = TorchSampler(ds, num_replicas=reps, rank=rank, shuffle=shuffle, seed=seed, drop_last=drop_last)
            for epoch in (0, 3):
                a.set_epoch(epoch)
                b.set_epoch(epoch)
                assert list(a) == list(b)
                assert len(a) == len(b)


def test_sampler_rank_validation():
    with pytest.raises(ValueError):
        DistributedSampler(list(range(10)), num_replicas=2, rank=2)
    with pytest.raises(ValueError):
        DistributedSampler(list(range(10)), num_replicas=2, rank=-1)


def test_mnist_steps_per_epoch():
    # 600/300/150/75 steps at ws 1/2/4/8 for 60,000 samples, batch 100
    import math

    for ws, steps in ((1, 600), (2, 300), (4, 150), (8, 75)):
        s = DistributedSampler(range(60000), num_replicas=ws, rank=0)
        assert math.ceil(len(s) / 100) == steps


def test_device_sampler_batches():
    s = DeviceDistributedSampler(list(range(103)), batch_size=10, device="cpu", num_replicas=2, rank=1, seed=4)
    ref = list(TorchSampler(list(range(103)), num_replicas=2, rank=1, seed=4))
    got = torch.cat(list(s.batches())).tolist()
    assert got == ref
    assert s.num_batches() == 6


def _resnet18_like_params():
    # shapes of torchvision resnet18(num_classes=10), registration order
    shapes = [(64, 3, 7, 7), (64,), (64,)]
    def block(cin, cout, down):
        s = [(cout, cin, 3, 3), (cout,), (cout,), (cout, cout, 3, 3), (cout,), (cout,)]
        if down:
            s += [(cout, cin, 1, 1), (cout,), (cout,)]
        return s
    for cin, cout in ((64, 64), (64, 128), (128, 256), (256, 512)):
        down = cin != cout
        shapes += block(cin, cout, down) + block(cout, cout, False)
    shapes += [(10, 512), (10,)]
    return [torch.empty(s) for s in shapes]


@pytest.mark.parametrize("limits", [[sys.maxsize], [1024 * 1024, 25 * 1024 * 1024], [1000, 5000], [64]])
def test_bucket_assignment_parity(limits):
    from ringdp import _C

    cases = [
        [torch.empty(s) for s in [(32, 1, 5, 5), (32,), (64, 32, 3, 3), (64,), (128, 64, 3, 3), (128,), (10, 2048), (10,)]],
        _resnet18_like_params(),
        [torch.empty(100), torch.empty(300, dtype=torch.float64), torch.empty(1000), torch.empty(7, dtype=torch.float64)],
    ]
    for ts in cases:
        assert _C.compute_bucket_assignment_by_size(ts, limits) == tuple(tdist._compute_bucket_assignment_by_size(ts, limits)) or \
            list(_C.compute_bucket_assignment_by_size(ts, limits)) == list(tdist._compute_bucket_assignment_by_size(ts, limits))
        # rebuilt form: reversed ready order + tensor_indices
        order = list(reversed(range(len(ts))))
        mine = _C.compute_bucket_assignment_by_size([ts[i] for i in order], limits, [], order)
        ref = tdist._compute_bucket_assignment_by_size([ts[i] for i in order], limits, [], order)
        assert [list(b) for b in mine[0]] == [list(b) for b in ref[0]]
        assert list(mine[1]) == list(ref[1])


def test_resnet18_rebuilt_buckets_match_survey():
    """ResNet-18 rebuilt buckets are 2,365,450 / 6,623,744 / 2,192,448 elems."""
    from ringdp import _C

    ts = _resnet18_like_params()
    order = list(reversed(range(len(ts))))
    buckets, _ = _C.compute_bucket_assignment_by_size([ts[i] for i in order], [1024 * 1024, 25 * 1024 * 1024], [], order)
    sizes = [sum(ts[i].numel() for i in b) for b in buckets]
    assert sizes == [2365450, 6623744, 2192448]
