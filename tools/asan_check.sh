#!/bin/bash
# AddressSanitizer run of ringdp's host C++ runtime (TCP/File stores, host ring, reducer, bindings)
# under the CPU distributed tests.  CPU only: device code is not sanitized and no GPU is used.
#   tools/asan_check.sh [pytest args...]      (default: store + distributed + launcher tests)
set -eu
cd "$(dirname "$0")/.."
python - <<'PY'
import importlib.util
spec = importlib.util.spec_from_file_location("ringdp_build", "ringdp/_build.py")
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
print(b.build(verbose=True, sanitize="address"))
PY
SO=$(ls build/address/_C*.so)
LIBASAN="$(g++ -print-file-name=libasan.so) $(g++ -print-file-name=libstdc++.so)"  # libstdc++ preloaded so ASan can intercept __cxa_throw
export RINGDP_EXT_PATH=$PWD/$SO
export LD_PRELOAD="$LIBASAN"
# python itself is not instrumented: its arenas look like leaks, so leak checking is off; every
# heap/stack/use-after-free error in the extension aborts the process (halt_on_error=1)
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:protect_shadow_gap=0:print_summary=1
TESTS=${*:-tests/test_store.py tests/test_distributed_cpu.py tests/test_multigpu_cpu.py tests/test_fake_backend.py tests/test_grad_slots.py tests/test_sampler_and_buckets.py}
python -m pytest $TESTS -q -p no:cacheprovider
