"""Median device time of one ConvNet op at batch B (HIP events), for A/B runs of extension variants
(RINGDP_EXT_PATH=<variant .so>).  python tools/op_time.py <op> [B] [iters]  (ops: tools/pmc_run.py)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_run  # noqa: E402  (tools/pmc_run.py: the op table)


def main():
    op = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    fns = pmc_run.build_ops(B)
    fn = fns[op]
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    ts.sort()
    print(json.dumps({"op": op, "B": B, "us_median": round(ts[len(ts) // 2], 1), "us_min": round(ts[0], 1),
                      "ext": os.environ.get("RINGDP_EXT_PATH", "in-tree")}))


if __name__ == "__main__":
    main()
