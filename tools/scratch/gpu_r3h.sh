# r3h: HIP graph-queue knobs vs the fork penalty; ConvNet launch fusions (pack in conv1, fc1 in conv3, CE 1-block)
set -o pipefail
O=gpurun_out/r3h; mkdir -p $O
for v in "" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  echo "env: $v"; env $v timeout -k 10 120 python tools/graph_fork_probe.py 2>>$O/fork.err || exit $?
done
for v in "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2"; do
  env $v RINGDP_COMM_SAME_STREAM=0 timeout -k 10 200 python bench.py --model resnet18 --steps 50 --warmup 10 --comm-stats-steps 10 > $O/r18_$v.json 2>$O/r18_$v.err || exit $?
  echo "r18 ss=0 $v"; grep -o '"ms_per_step": [0-9.]*\|"step_ms_no_comm": [0-9.]*\|"exposed_comm_ms": [-0-9.]*' $O/r18_$v.json
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convnet_model_gpu.py tests/test_convnet_kernels_gpu.py tests/test_convnet_fp32_gpu.py > $O/cn_tests.log 2>&1; rc=$?; tail -3 $O/cn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 --warmup 20 > $O/b100.json 2>$O/b100.err || exit $?; grep -o '"ms_per_step": [0-9.]*' $O/b100.json
timeout -k 10 200 python bench.py --batch-per-rank 4096 --steps 100 --warmup 20 > $O/b4096.json 2>$O/b4096.err || exit $?; grep -o '"ms_per_step": [0-9.]*' $O/b4096.json
timeout -k 10 200 python bench.py > $O/b65536.json 2>$O/b65536.err || exit $?; grep -o '"ms_per_step": [0-9.]*' $O/b65536.json
cd /tmp; cd - > /dev/null; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_b100 -o run --output-format csv -- python3 bench.py --batch-per-rank 100 --steps 200 --warmup 20 --comm-stats-steps 0 > $O/prof_b100.log 2>&1 || exit $?
echo ALLDONE
