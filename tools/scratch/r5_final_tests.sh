#!/bin/bash
# round-5 evidence (1/2): the full GPU suite + smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5final; mkdir -p $O
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
