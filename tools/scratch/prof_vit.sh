# rocprofv3 kernel stats of the ViT-B/16 step, bf16 and fp8 (eager, short)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for dt in bf16 fp8; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit_$dt -o run --output-format csv -- python bench.py --model vit_b_16 --dtype $dt --steps 6 --warmup 3 --no-graph > gpurun_out/prof_vit_$dt.log 2>&1 || exit 1
  tail -1 gpurun_out/prof_vit_$dt.log
done
