#!/bin/bash
# full GPU suite + every model's bench with the round-4 tree
set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for m in "convnet" "resnet18" "resnet50" "vit_b_16"; do
  timeout -k 10 300 python bench.py --model $m --steps 20 > $O/b_$m.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
  echo "$m $(tail -1 $O/b_$m.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --model vit_b_16 --dtype fp8 --steps 20 > $O/b_vit_fp8.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "vit fp8 $(tail -1 $O/b_vit_fp8.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 > $O/b_fp32.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
echo "fp32 $(tail -1 $O/b_fp32.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
echo smoke ok
echo ALLDONE
