#!/bin/bash
# Host-side AddressSanitizer over the engine: the host-ASan build
# of libbabble_hip (make asan: api.cpp, frames.cpp and the launch stubs
# instrumented with -Xarch_host -fsanitize=address; the gfx950 code is the
# regular build's) loaded in place of the in-tree library (BH_LIB_PATH),
# clang's ASan runtime preloaded, over GPU tests that drive every host path:
# inserts and their checks, the pass sequence and per-sync schedules, Reset
# (its transactional allocation included), shard groups, the block
# projection with host hashing, queries.  Run on the GPU box:
#   tools/sanitize_engine.sh [pytest args]
set -euo pipefail
cd "$(dirname "$0")/.."
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export BH_LIB_PATH=$PWD/tools/asan/libbabble_hip.so
test -f "$BH_LIB_PATH" || { echo "missing $BH_LIB_PATH: run make asan" >&2; exit 1; }
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export LD_PRELOAD="$RT"
if [ $# -eq 0 ]; then
  set -- -m gpu -q -x --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_reset.py tests/test_gpu_shard.py \
    tests/test_gpu_frames.py tests/test_gpu_query.py -k "not full_size and not large_properties"
fi
exec python -m pytest -p no:cacheprovider "$@"
