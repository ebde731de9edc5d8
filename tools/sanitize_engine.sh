#!/bin/bash
# Host-side AddressSanitizer over the engine: the host-ASan build
# of libbabble_hip (make asan: api.cpp and frames.cpp built by g++ with
# -fsanitize=address,undefined; the gfx950 kernel objects are the regular
# build's) loaded in place of the in-tree library (BH_LIB_PATH), GCC's ASan
# runtime preloaded, over GPU tests that drive every host path:
# inserts and their checks, the pass sequence and per-sync schedules, Reset
# (its transactional allocation included), shard groups, the block
# projection with host hashing, queries.  Run on the GPU box:
#   tools/sanitize_engine.sh [pytest args]
set -euo pipefail
cd "$(dirname "$0")/.."
RT=$(gcc -print-file-name=libasan.so)
export BH_LIB_PATH=$PWD/tools/asan/libbabble_hip.so
test -f "$BH_LIB_PATH" || { echo "missing $BH_LIB_PATH: run make asan" >&2; exit 1; }
mkdir -p gpurun_out
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:log_path=$PWD/gpurun_out/asan
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=$PWD/gpurun_out/ubsan
export LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}"
if [ $# -eq 0 ]; then
  set -- -m gpu -q -x --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_reset.py tests/test_gpu_shard.py \
    tests/test_gpu_frames.py tests/test_gpu_query.py -k "not full_size and not large_properties"
fi
exec python -m pytest -p no:cacheprovider "$@"
