timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_nn_kernels_gpu.py -k "fp8" > gpurun_out/tf.log 2>&1; rc=$?; tail -3 gpurun_out/tf.log; [ $rc -ne 0 ] && exit $rc
for m in 128 256; do echo "tile $m"; RINGDP_FP8_TILE=$m timeout -k 10 120 python tools/gemm_bench.py --vit-fp8 || exit 1; done
