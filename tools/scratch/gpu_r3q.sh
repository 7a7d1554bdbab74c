# r3q: 128x128 core vs 256x256 kernels per ViT shape (bf16, fp8) after the epilogue fix
set -o pipefail
O=gpurun_out/r3q; mkdir -p $O
timeout -k 10 400 python tools/gemm_tile_probe.py > $O/tiles.jsonl 2>$O/tiles.err || exit $?
cat $O/tiles.jsonl
echo ALLDONE
