# same-box A/B of prebuilt extension variants (variants/<name>.so via RINGDP_EXT_PATH), interleaved rounds
# usage: bash tools/gpu_ab_variants.sh "<bench args>" name1 name2 ...
set -o pipefail
O=gpurun_out/ab; mkdir -p $O
ARGS="$1"; shift
for r in 1 2 3; do
  for v in "$@"; do
    RINGDP_EXT_PATH=variants/$v.so timeout -k 10 200 python bench.py $ARGS --comm-stats-steps 0 > $O/$v.$r.json 2>$O/$v.$r.err || exit $?
    echo "$v round $r $(grep -o '"ms_per_step": [0-9.]*' $O/$v.$r.json)"
  done
done
echo ALLDONE
