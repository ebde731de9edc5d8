#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer over the CPU-side native code
# (SURVEY 5): the oracle (oracle/hg_oracle.c) and the DAG generator
# (babble_amd/csrc/dag_gen.c) rebuilt with -fsanitize=address,undefined and
# loaded in place of the regular builds (BH_ORACLE_LIB / BH_GEN_LIB) while the
# CPU test suite runs.  Python itself is not instrumented, so the ASan runtime
# is preloaded and leak detection (which would report the interpreter's
# arenas) is off; any ASan report or UBSan finding aborts the run.
#   tools/sanitize.sh [pytest args]      (default: -m "not gpu" -q)
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle san
mkdir -p build/san
gcc -O1 -g -fno-omit-frame-pointer -fPIC -shared -Wall -Wno-deprecated-declarations \
    -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -o build/san/libbabble_gen.so babble_amd/csrc/dag_gen.c -lcrypto -lpthread
export BH_ORACLE_LIB=$PWD/oracle/_san/liboracle.so
export BH_GEN_LIB=$PWD/build/san/libbabble_gen.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export LD_PRELOAD="$(gcc -print-file-name=libasan.so)"
if [ $# -eq 0 ]; then set -- -m "not gpu" -q; fi
exec python -m pytest tests -p no:cacheprovider "$@"
