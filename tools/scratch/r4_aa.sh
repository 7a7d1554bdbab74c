#!/bin/bash
# bf16 256 GEMM grouped tile order: dense shapes and ViT bf16 / ResNet-50 bench A/B
set -o pipefail
O=gpurun_out/r4aa; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py tests/test_nn_kernels_gpu.py -k "gemm or fp8" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
python3 - > $O/dense.py <<'PY'
PY
for g in 1 4; do
  RINGDP_BF16_GROUP_M=$g timeout -k 10 200 python -u -c "
import sys, json; sys.argv=['x']; sys.path.insert(0,'tools'); import gemm_bench as gb
for a in [(8192,8192,8192),(4096,4096,4096),(25216,3072,768),(25216,768,3072),(25216,2304,768)]: print(json.dumps(gb.dense(*a)), flush=True)
" > $O/dense_g$g.log 2>&1 || exit 1
  echo "group $g"; grep shape $O/dense_g$g.log
done
for r in 1 2; do for g in 1 4; do
  RINGDP_BF16_GROUP_M=$g timeout -k 10 300 python -u bench.py --model vit_b_16 --steps 10 2>>$O/b.err | grep metric | sed "s/^/vit_g$g /" >> $O/ab.txt || exit 1
done; done
for g in 1 4; do
  RINGDP_BF16_GROUP_M=$g timeout -k 10 300 python -u bench.py --model resnet50 --steps 10 2>>$O/b.err | grep metric | sed "s/^/r50_g$g /" >> $O/ab.txt || exit 1
done
echo ALLDONE
cut -c1-120 $O/ab.txt
