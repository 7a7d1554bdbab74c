#!/bin/bash
# op timings under env settings, no tests: r5_ops.sh NAME "OP ENV..." ...  (each arg: op name, then env assignments)
set -o pipefail
export TMPDIR=/tmp
N=$1; shift
O=gpurun_out/$N; mkdir -p $O
SPECS=("$@")
for r in 1 2; do for spec in "${SPECS[@]}"; do
  read -r op envs <<< "$spec"
  echo -n "$op $envs : " | tee -a $O/ops.txt
  env $envs timeout -k 10 120 python tools/op_time.py $op 65536 40 | tee -a $O/ops.txt || exit 1
done; done
