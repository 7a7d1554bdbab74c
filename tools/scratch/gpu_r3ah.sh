# r3ah: ViT bf16 GEMM routing A/B - default (fill >= 75 %) vs every bf16 GEMM on the 256x256 kernel; fill threshold sweep
set -o pipefail
O=gpurun_out/r3ah; mkdir -p $O
for r in 1 2; do
  for v in default 256; do
    if [ $v = 256 ]; then export RINGDP_BF16_TILE=256; else unset RINGDP_BF16_TILE; fi
    timeout -k 10 300 python bench.py --model vit_b_16 --steps 15 --warmup 5 --comm-stats-steps 0 > $O/vit_$v.$r.json 2>$O/vit_$v.$r.err || exit $?
    echo "$v $r $(grep -o '"ms_per_step": [0-9.]*' $O/vit_$v.$r.json)"
  done
done
unset RINGDP_BF16_TILE
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
RINGDP_BF16_TILE=256 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_vit256 -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 5 --warmup 2 --no-graph --comm-stats-steps 0 > $O/prof_vit256.log 2>&1 || exit $?
echo ALLDONE
