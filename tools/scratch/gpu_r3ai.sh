# r3ai: bf16 256x256 routing fill threshold 0.55 vs 0.75 on ViT, ResNet-50, ResNet-18 (interleaved, 2 rounds)
set -o pipefail
O=gpurun_out/r3ai; mkdir -p $O
for r in 1 2; do
  for m in vit_b_16 resnet50 resnet18; do
    for f in 0.75 0.55; do
      RINGDP_BF16_256_FILL=$f timeout -k 10 300 python bench.py --model $m --steps 15 --warmup 5 --comm-stats-steps 0 > $O/$m.$f.$r.json 2>$O/$m.$f.$r.err || exit $?
      echo "$m fill=$f r$r $(grep -o '"ms_per_step": [0-9.]*' $O/$m.$f.$r.json)"
    done
  done
done
echo ALLDONE
