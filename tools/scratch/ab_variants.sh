# A/B timing of extension variants built by tools/build_variant.py: bash tools/ab_variants.sh v1 v2 ...
S=ringdp/_C.cpython-310-x86_64-linux-gnu.so
for v in "$@"; do
  cp abtest/$v.so $S || exit 1
  echo -n "$v "
  timeout -k 10 120 python tools/kbench.py ${KB_B:-16384} 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v['us'] for k, v in d.items() if isinstance(v, dict) and k.startswith(('conv3_fc_bwd', 'conv2_bwd'))}, d['total_us'])" || exit 1
done
