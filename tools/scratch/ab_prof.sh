# per-kernel times (rocprofv3 --kernel-trace --stats) of one ConvNet op under extension variants:
#   OP=conv3_fc_bwd_w bash tools/ab_prof.sh v1 v2 ...
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/abprof
S=ringdp/_C.cpython-310-x86_64-linux-gnu.so
for v in "$@"; do
  cp abtest/$v.so $S || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/abp_$v -o run --output-format csv -- python3 tools/pmc_run.py ${OP:-conv3_fc_bwd} ${KB_B:-16384} 10 > gpurun_out/abprof/$v.log 2>&1 || exit 1
  f=$(find /tmp/abp_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; python3 tools/prof_summary.py $f 6
done
