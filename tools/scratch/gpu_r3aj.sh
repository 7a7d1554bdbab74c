# r3aj: attention dK/dV kernel with D in LDS + pipelined P loads: attention/ViT tests, ViT bench, kernel stats
set -o pipefail
O=gpurun_out/${RUN:-r3aj}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nn_kernels_gpu.py -k "attn or attention or vit" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --model vit_b_16 --steps 15 --warmup 5 --comm-stats-steps 0 > $O/vit.json 2>$O/vit.err || exit $?; grep -o '"ms_per_step": [0-9.]*' $O/vit.json
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 5 --warmup 2 --no-graph --comm-stats-steps 0 > $O/prof.log 2>&1 || exit $?
grep -E "attn" $O/prof/run_kernel_stats.csv | cut -d, -f1-5
echo ALLDONE
