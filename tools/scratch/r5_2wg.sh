#!/bin/bash
# two-workgroups-per-CU 256x128 bf16 GEMM: GEMM tests, shape probe (1-WG vs 2-WG), ViT bench with the knob off/on
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_2wg; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
timeout -k 10 300 python -u tools/gemm_2wg_probe.py > $O/probe.jsonl 2>$O/probe.err || { tail -5 $O/probe.err; exit 1; }
cat $O/probe.jsonl
for r in 1 2; do
  for m in 0 2; do
    RINGDP_GEMM_2WG=$m timeout -k 10 300 python -u bench.py --model vit_b_16 --steps 20 --warmup 5 --comm-stats-steps 0 > $O/vit_m$m.$r.json 2>>$O/b.err || exit 1
    tail -1 $O/vit_m$m.$r.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('mode $m', d['value'], d['ms_per_step'])"
  done
done
for m in 0 2; do
  RINGDP_GEMM_2WG=$m timeout -k 10 300 python -u bench.py --model resnet50 --steps 10 --warmup 3 --comm-stats-steps 0 > $O/r50_m$m.json 2>>$O/b.err || exit 1
  tail -1 $O/r50_m$m.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('r50 mode $m', d['value'], d['ms_per_step'])"
done
