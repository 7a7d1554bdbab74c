# r3n: GEMM epilogue with every store sent to a sink (is the ViT-shape loss the HBM writes or the epilogue?)
set -o pipefail
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 300 python tools/gemm_epi_probe.py > $O/epi.jsonl 2>$O/epi.err || exit $?
cat $O/epi.jsonl
echo ALLDONE
