# r3k: store-pattern probe for the GEMM epilogue (tools/store_pattern_probe.hip)
set -o pipefail
O=gpurun_out/r3k; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 tools/store_pattern_probe.hip -o $O/spp || exit $?
timeout -k 10 60 $O/spp | tee $O/spp.jsonl || exit $?
echo ALLDONE
