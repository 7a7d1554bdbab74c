# r3l: GEMM output-store cache flavours (plain / nt / sc1) x persistent kernel; GEMM tests
set -o pipefail
O=gpurun_out/r3l; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py > $O/gemm_tests.log 2>&1; rc=$?; tail -2 $O/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_epi_probe.py > $O/epi.jsonl 2>$O/epi.err || exit $?
cat $O/epi.jsonl
echo ALLDONE
