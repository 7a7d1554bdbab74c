"""ringdp - an MI355X-native (gfx950) data-parallel training framework.

Re-implements the capabilities of the PyTorch distributed tutorial repo
Jackxiini/Pytorch-distributed-learning on PyTorch-ROCm + hand-written CDNA4 HIP kernels + RCCL
over xGMI:

* ``ringdp.distributed``  - init_process_group / collectives (C++ TCP store, RCCL and host-ring
                            process groups, watchdog, debug fingerprints, fault injection)
* ``ringdp.parallel``     - DistributedDataParallel on a C++ bucketed reducer
* ``ringdp.data``         - DistributedSampler (+ on-device variants), datasets, transforms
* ``ringdp.multiprocessing.spawn`` / ``python -m ringdp.run`` / ``python -m ringdp.launch``
* ``ringdp.models``       - ConvNet (MNIST) on fused MFMA kernels; ResNet / ViT families
* ``ringdp.nn`` / ``ringdp.optim`` - cross entropy, fused SGD
"""
from . import distributed  # noqa: F401
from ._native import C as _C  # noqa: F401
from .data import DistributedSampler  # noqa: F401
from .distributed import (  # noqa: F401
    ReduceOp,
    all_gather,
    all_reduce,
    barrier,
    broadcast,
    destroy_process_group,
    get_rank,
    get_world_size,
    init_process_group,
    is_initialized,
    new_group,
)
from .multiprocessing import spawn  # noqa: F401
from .parallel import DistributedDataParallel  # noqa: F401
from . import models, nn, ops, optim  # noqa: F401,E402

__version__ = "0.1.0"
