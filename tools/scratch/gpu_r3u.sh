# r3u: fp32 ConvNet step kernel table (before the fp32 rework)
set -o pipefail
O=gpurun_out/r3u; mkdir -p $O
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_f32 -o run --output-format csv -- python3 bench.py --dtype fp32 --steps 4 --warmup 2 --comm-stats-steps 0 > $O/prof_f32.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $O/prof_f32.log
echo ALLDONE
