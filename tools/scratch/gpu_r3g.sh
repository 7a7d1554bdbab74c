# r3g: side-stream fork/join cost inside a captured step
set -o pipefail
O=gpurun_out/r3g; mkdir -p $O
timeout -k 10 120 python tools/graph_fork_probe.py > $O/fork_probe.jsonl 2>$O/fork_probe.err || exit $?
cat $O/fork_probe.jsonl
for ss in 1 0; do
  RINGDP_COMM_SAME_STREAM=$ss timeout -k 10 200 python bench.py --model resnet18 --steps 50 --warmup 10 --comm-stats-steps 10 > $O/r18_ss$ss.json 2>$O/r18_ss$ss.err || exit $?
  echo r18 ss=$ss; grep -o '"ms_per_step": [0-9.]*\|"step_ms_no_comm": [0-9.]*\|"exposed_comm_ms": [-0-9.]*' $O/r18_ss$ss.json
  RINGDP_COMM_SAME_STREAM=$ss timeout -k 10 200 python bench.py --batch-per-rank 100 --steps 300 --warmup 20 --comm-stats-steps 20 > $O/b100_ss$ss.json 2>$O/b100_ss$ss.err || exit $?
  echo b100 ss=$ss; grep -o '"ms_per_step": [0-9.]*\|"step_ms_no_comm": [0-9.]*\|"exposed_comm_ms": [-0-9.]*' $O/b100_ss$ss.json
  RINGDP_COMM_SAME_STREAM=$ss timeout -k 10 200 python bench.py --steps 50 --warmup 10 --comm-stats-steps 10 > $O/cn_ss$ss.json 2>$O/cn_ss$ss.err || exit $?
  echo convnet ss=$ss; grep -o '"ms_per_step": [0-9.]*\|"step_ms_no_comm": [0-9.]*\|"exposed_comm_ms": [-0-9.]*' $O/cn_ss$ss.json
done
echo ALLDONE
