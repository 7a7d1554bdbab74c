#!/bin/bash
# bf16 256 kernel: phased vs single-stage-wait pipeline on the ViT shapes (is a phased fp8 port worth it?)
set -o pipefail
O=gpurun_out/r4ad; mkdir -p $O
for ph in 0 1; do
  RINGDP_GEMM256_PHASED=$ph timeout -k 10 200 python -u -c "
import sys, json; sys.argv=['x']; sys.path.insert(0,'tools'); import gemm_bench as gb
for a in [(8192,8192,8192),(25216,3072,768),(25216,768,3072),(25216,2304,768),(25216,768,768)]: print(json.dumps(gb.dense(*a)), flush=True)
" > $O/dense_p$ph.log 2>&1 || exit 1
  echo "phased $ph"; grep shape $O/dense_p$ph.log
done
