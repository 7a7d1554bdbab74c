# r3i: GEMM epilogue store-mode costs on ViT shapes; two linear graphs joined by external events vs a fork
set -o pipefail
O=gpurun_out/r3i; mkdir -p $O
timeout -k 10 200 python tools/gemm_epi_probe.py > $O/epi.jsonl 2>$O/epi.err || exit $?
cat $O/epi.jsonl
hipcc --offload-arch=gfx950 -O2 tools/graph_ext_probe.hip -o $O/graph_ext_probe || exit $?
for n in 50 200; do timeout -k 10 60 $O/graph_ext_probe $n || exit $?; done
echo ALLDONE
