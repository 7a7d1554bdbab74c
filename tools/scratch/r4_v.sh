#!/bin/bash
# fp8 ViT: 256 fp8 kernel round-fill threshold sweep (bf16 went 0.75 -> 0.55 in round 3)
set -o pipefail
O=gpurun_out/r4v; mkdir -p $O
for r in 1 2; do
for f in 0.75 0.55 0.45; do
  RINGDP_FP8_256_FILL=$f timeout -k 10 300 python bench.py --model vit_b_16 --dtype fp8 --steps 20 > $O/b_fp8_$f.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "fill $f $(tail -1 $O/b_fp8_$f.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
done
done
echo ALLDONE
