#!/bin/bash
# ResNet-50: bf16 GEMM routing A/B (256x256 kernel forced) on pointwise shapes and the whole step
set -o pipefail
O=gpurun_out/r4an; mkdir -p $O
for t in 0 256; do
  RINGDP_BF16_TILE=$t timeout -k 10 300 python -u -c "
import sys, json; sys.argv=['x']; sys.path.insert(0,'tools'); import gemm_bench as gb
for a in [(256,56,64,256,1,1),(256,56,256,64,1,1),(256,28,128,512,1,1),(256,28,512,128,1,1),(256,14,256,1024,1,1),(256,14,1024,256,1,1),(256,7,512,2048,1,1),(256,7,2048,512,1,1)]:
    print(json.dumps(gb.conv(*a)), flush=True)
" > $O/pw_$t.log 2>&1 || { tail $O/pw_$t.log; exit 1; }
  echo "tile $t"; grep shape $O/pw_$t.log | cut -c1-200
done
for r in 1 2; do for t in 0 256; do
  RINGDP_BF16_TILE=$t timeout -k 10 300 python -u bench.py --model resnet50 --steps 10 2>>$O/b.err | grep metric | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('tile=$t', d['value'], d['ms_per_step'])" >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
