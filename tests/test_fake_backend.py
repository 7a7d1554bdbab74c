"""The "fake" backend (upstream torch/testing/_internal/distributed/fake_pg.py): one process acts as
rank r of an N-rank world; collectives complete immediately and leave their tensors untouched."""
import torch

import ringdp.distributed as dist


def test_fake_world_drives_ddp():
    from ringdp.models import ConvNet
    from ringdp.optim import SGD
    from ringdp.parallel import DistributedDataParallel as DDP

    dist.init_process_group("fake", rank=3, world_size=8)
    try:
        assert (dist.get_rank(), dist.get_world_size(), dist.get_backend()) == (3, 8, "fake")
        t = torch.arange(5.0)
        dist.all_reduce(t)
        dist.broadcast(t, src=0)
        assert torch.equal(t, torch.arange(5.0))
        dist.barrier()
        sub = dist.new_group([1, 3, 5])
        assert (dist.get_rank(sub), dist.get_world_size(sub)) == (1, 3)
        torch.manual_seed(0)
        m = ConvNet()
        ddp = DDP(m, bucket_cap_mb=0.1, first_bucket_mb=0.05)
        opt = SGD(ddp.parameters(), lr=0.1)
        before = [p.detach().clone() for p in m.parameters()]
        for _ in range(3):
            ddp(torch.randn(2, 1, 28, 28)).sum().backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
        info = ddp._get_ddp_logging_data()
        assert info["backend_name"] == "fake" and info["world_size"] == 8
        assert ddp.reducer.rebuilt() and len(info["bucket_sizes"]) == 3
        assert any(not torch.equal(a, b) for a, b in zip(before, m.parameters()))
    finally:
        dist.destroy_process_group()
