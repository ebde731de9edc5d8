#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export BH_SEGMENTS=1
TAG=default timeout -k 10 120 python tools/dbg_lt.py
TAG=combined BH_LT_COMBINED=1 timeout -k 10 120 python tools/dbg_lt.py
TAG=eager BH_EAGER_ROWS=1 timeout -k 10 120 python tools/dbg_lt.py
TAG=seg2 BH_SEGMENTS=2 timeout -k 10 120 python tools/dbg_lt.py
