#!/bin/bash
# vectorised bf16 W / W^T cast: tests, cast_t_multi kernel time (rocprofv3 stats) and ViT bench, base vs tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_attn; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "vit or attn" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
for v in base new; do
  if [ $v = base ]; then export RINGDP_EXT_PATH=abv/base.so; else unset RINGDP_EXT_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 10 --warmup 3 --comm-stats-steps 0 > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -1); python tools/prof_summary.py $f 40 > $O/k_$v.md; grep -E "attn_" $O/k_$v.md
done
unset RINGDP_EXT_PATH
for r in 1 2; do
  RINGDP_EXT_PATH=abv/base.so timeout -k 10 300 python -u bench.py --model vit_b_16 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/vit_base$r.json 2>>$O/b.err || exit 1
  timeout -k 10 300 python -u bench.py --model vit_b_16 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/vit_new$r.json 2>>$O/b.err || exit 1
  for f in base new; do tail -1 $O/vit_$f$r.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$f', d['value'], d['ms_per_step'])"; done
done
