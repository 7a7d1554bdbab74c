"""``python -m ringdp.launch`` - legacy ``torch.distributed.launch`` contract.

Same launcher as ``ringdp.run`` but, unless ``--use-env`` is given, each worker also receives
``--local-rank=N`` on its command line (``torch/distributed/launch.py:168-180``).
"""
from __future__ import annotations

import sys

from .run import main as _main


def main(argv=None) -> int:
    return _main(argv, legacy=True)


if __name__ == "__main__":
    sys.exit(main())
