# quick role-split sweep: VAR=RINGDP_C2_DGRAD_FRAC bash tools/split_quick.sh 0.5 0.55 ...
V=${VAR:-RINGDP_C2_DGRAD_FRAC}
for f in "$@"; do
  echo -n "$V=$f "
  env $V=$f timeout -k 10 120 python tools/kbench.py 16384 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v['us'] for k, v in d.items() if isinstance(v, dict) and k.startswith(('conv2_bwd','conv3_fc_bwd'))})"
done
