#!/bin/bash
# round-3 PMC passes: C3, C4 (bench.py) and the Reset bench; SQ + traffic summaries
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.log; done ) &
hb=$!
trap 'kill $hb' EXIT
bash tools/pmc.sh c3 "k_" --cfg 3 && python tools/pmc_sq_summary.py gpurun_out/pmc_c3 128 10000000 > gpurun_out/sq_c3.txt && python tools/pmc_summary.py gpurun_out/pmc_c3 128 10000000 > gpurun_out/traffic_c3.txt &&
bash tools/pmc.sh c4 "k_" --cfg 4 && python tools/pmc_sq_summary.py gpurun_out/pmc_c4 512 20000000 > gpurun_out/sq_c4.txt && python tools/pmc_summary.py gpurun_out/pmc_c4 512 20000000 > gpurun_out/traffic_c4.txt &&
PMC_CMD="python tools/bench_reset.py --steps 1" bash tools/pmc.sh reset "k_" && python tools/pmc_sq_summary.py gpurun_out/pmc_reset 128 1000000 > gpurun_out/sq_reset.txt &&
cp profiles/pmc_sq.json profiles/pmc_traffic.json gpurun_out/ &&
bash tools/prof.sh c3 --cfg 3 --steps 3 --warmup 1 && bash tools/prof.sh c4 --cfg 4 --steps 1 --warmup 1
