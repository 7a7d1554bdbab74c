# r3al: attention dQ kernel recomputing dP (118 VGPRs, 3 waves/SIMD, was 232 / 1) as a prebuilt variant:
# attention + ViT tests on it, then same-box ViT A/B against the tree's extension
set -o pipefail
O=gpurun_out/r3al; mkdir -p $O
RINGDP_EXT_PATH=variants/attn_dq.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nn_kernels_gpu.py -k "attn or attention or vit" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do for v in base attn_dq; do
  RINGDP_EXT_PATH=variants/$v.so timeout -k 10 300 python bench.py --model vit_b_16 --steps 15 --warmup 5 --comm-stats-steps 0 > $O/$v.$r.json 2>$O/$v.$r.err || exit $?
  echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/$v.$r.json)"
done; done
echo ALLDONE
