#!/bin/bash
# ResNet-50 pointwise conv shapes on the current kernels (fwd+stats / dgrad / wgrad)
set -o pipefail
O=gpurun_out/r4af; mkdir -p $O
timeout -k 10 300 python -u -c "
import sys, json; sys.argv=['x']; sys.path.insert(0,'tools'); import gemm_bench as gb
for a in [(256,56,64,64,1,1),(256,56,64,256,1,1),(256,56,256,64,1,1),(256,28,256,128,1,1),(256,28,128,512,1,1),(256,28,512,128,1,1),(256,14,512,256,1,1),(256,14,256,1024,1,1),(256,14,1024,256,1,1),(256,7,1024,512,1,1),(256,7,512,2048,1,1),(256,7,2048,512,1,1)]:
    print(json.dumps(gb.conv(*a)), flush=True)
" > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
grep shape $O/pw.log
