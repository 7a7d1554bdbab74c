# r3s: pool2 backward as a scatter over target-position codes: ConvNet tests, benches, conv3 bwd PMC
set -o pipefail
O=gpurun_out/r3s; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py > $O/tests.log 2>&1; rc=$?; grep -E "passed|failed|max \||^l2" $O/tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py > $O/b65536.json 2>$O/b65536.err || exit $?; grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/b65536.json
timeout -k 10 200 python bench.py --batch-per-rank 4096 --steps 100 --warmup 20 > $O/b4096.json 2>$O/b4096.err || exit $?; grep -o '"ms_per_step": [0-9.]*' $O/b4096.json
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 --warmup 20 > $O/b100.json 2>$O/b100.err || exit $?; grep -o '"ms_per_step": [0-9.]*' $O/b100.json
cd /tmp; cd - >/dev/null; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmcB -o run -- python3 tools/pmc_run.py conv3_fc_bwd 65536 3 > $O/pmcB.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/pmc_run.py conv3_fc_bwd 65536 3 > $O/trace.log 2>&1 || exit $?
echo ALLDONE
