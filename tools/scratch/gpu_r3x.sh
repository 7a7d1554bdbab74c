# r3x: fp32 pool kernels (uncapped grids, s2 fwd) tests; BK 16 vs 32 A/B; per-kernel trace of both
set -o pipefail
O=gpurun_out/r3x; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convnet_fp32_gpu.py > $O/tests.log 2>&1; rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
RINGDP_EXT_PATH=variants/f32bk32.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convnet_fp32_gpu.py > $O/tests32.log 2>&1; rc=$?; grep -E "passed|failed" $O/tests32.log | tail -2; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in f32bk16 f32bk32; do
  RINGDP_EXT_PATH=variants/$v.so timeout -k 10 200 python bench.py --dtype fp32 --steps 8 --warmup 3 --comm-stats-steps 0 > $O/$v.$r.json 2>$O/$v.$r.err || exit $?
  echo "$v $r $(grep -o '"value": [0-9.]*' $O/$v.$r.json)"
done; done
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
for v in f32bk16 f32bk32; do
RINGDP_EXT_PATH=variants/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --dtype fp32 --steps 3 --warmup 1 --comm-stats-steps 0 > $O/prof_$v.log 2>&1 || exit $?
done
echo ALLDONE
