# r3y: fp32 GEMM 2-deep prefetch, specialised 2x2 pools: tests, bench, per-kernel trace
set -o pipefail
O=gpurun_out/${RUN:-r3y}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_convnet_fp32_gpu.py > $O/tests.log 2>&1; rc=$?; grep -E "passed|failed|max \|loss" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --dtype fp32 --steps 10 --warmup 3 --comm-stats-steps 0 > $O/b_f32.json 2>$O/b_f32.err || exit $?; grep -o '"value": [0-9.]*' $O/b_f32.json
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f32 -o run --output-format csv -- python3 bench.py --dtype fp32 --steps 3 --warmup 1 --comm-stats-steps 0 > $O/prof_f32.log 2>&1 || exit $?
echo ALLDONE
