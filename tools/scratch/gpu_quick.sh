mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_convnet_kernels_gpu.py tests/test_convnet_model_gpu.py > gpurun_out/t.log 2>&1; rc=$?; tail -5 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/kbench.py 16384 > gpurun_out/kb.log 2>&1 && tail -1 gpurun_out/kb.log
timeout -k 10 200 python bench.py > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
