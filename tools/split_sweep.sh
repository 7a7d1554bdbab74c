for f in 0.5 0.56 0.62 0.68 0.74; do
  echo "C3 $f"; RINGDP_C3_DGRAD_FRAC=$f timeout -k 10 120 python tools/kbench.py 4096 | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['conv3_fc_bwd'], d['conv2_bwd'])" || exit 1
done
for f in 0.44 0.5 0.56 0.62 0.68; do
  echo "C2 $f"; RINGDP_C2_DGRAD_FRAC=$f timeout -k 10 120 python tools/kbench.py 4096 | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['conv3_fc_bwd'], d['conv2_bwd'])" || exit 1
done
