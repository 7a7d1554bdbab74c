#!/bin/bash
# ws1 ResNet-18 kernel traces, split vs same placement (segment-boundary gaps)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_split2; mkdir -p $O
for m in split same; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$m -o run --output-format csv -- python3 bench.py --model resnet18 --steps 20 --warmup 10 --comm-stats-steps 0 --comm-stream $m > $O/$m.log 2>&1 || { tail -5 $O/$m.log; exit 1; }
  tail -1 $O/$m.log | cut -c1-200
done
RINGDP_COMM_HIGH_PRIORITY=1 timeout -k 10 300 python -u bench.py --model resnet18 --steps 50 --warmup 20 --comm-stream split > $O/hp.json 2>>$O/b.err || exit 1
tail -1 $O/hp.json | cut -c1-200
