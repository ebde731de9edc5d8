#!/bin/bash
# One GPU session: parity tests, smoke, bench.  Stops at the first step that
# faults / aborts / times out (exit >= 124 or signal); test failures (exit 1)
# still let the bench run so one call yields both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal step $name rc=$rc, stopping"; exit $rc
  fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf ;;
    treset) step pytest_reset 600 python -u -m pytest tests/test_gpu_reset.py -m gpu -v --timeout 120 --timeout-method thread -rf ;;
    twide) step pytest_wide 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf -k "wide or 512 or 300 or c4 or C4 or floww" ;;
    tfloww) step pytest_floww 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -rf -x -k "floww" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench2) step bench_c2 600 python bench.py --cfg 2 --steps 3 --warmup 1 ;;
    bench3) step bench_c3 900 python bench.py --cfg 3 --steps 3 --warmup 1 ;;
    serial) step serial 600 env BH_SEG_SERIAL=1 BH_SEG_DEBUG=1 python bench.py --steps 1 --warmup 1 --cpu-sample 0 ;;
    serialrows) step serial_rows 600 env BH_ROUND_ROWS=1 BH_SEG_SERIAL=1 BH_SEG_DEBUG=1 python bench.py --steps 1 --warmup 1 --cpu-sample 0 ;;
    tl) step tl 600 env BH_DIAG=1 BH_TIMELINE=gpurun_out/tl.bin python bench.py --steps 1 --warmup 1 --cpu-sample 0 ;;
    tlg0) step tlg0 600 env BH_ROUND_P8G=0 BH_DIAG=1 BH_TIMELINE=gpurun_out/tlg0.bin python bench.py --steps 1 --warmup 1 --cpu-sample 0 ;;
    bench2q) step bench_c2 600 python bench.py --cfg 2 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench5q) step bench_c5 600 python bench.py --cfg 5 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench3qb) step bench_c3b 900 python bench.py --cfg 3 --steps 3 --warmup 1 --cpu-sample 0 ;;
    tlser) step tlser 600 env BH_SEG_SERIAL=1 BH_DIAG=1 BH_TIMELINE=gpurun_out/tlser.bin python bench.py --steps 1 --warmup 1 --cpu-sample 0 ;;
    tlrows) step tlrows 600 env BH_ROUND_ROWS=1 BH_SEG_SERIAL=1 BH_DIAG=1 BH_TIMELINE=gpurun_out/tlrows.bin python bench.py --steps 1 --warmup 1 --cpu-sample 0 ;;
    bench) step bench 900 python bench.py ;;
    benchrows) step bench_rows 900 env BH_ROUND_ROWS=1 python bench.py --cpu-sample 0 ;;
    bench4tr32) step bench_c4_tr32 1100 env BH_FDT_TR=32 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 ;;
    bench4x16) step bench_c4_x16 1100 env BH_XPOSE_TR=16 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 ;;
    bench4tr64) step bench_c4_tr64 1100 env BH_FDT_TR=64 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 ;;
    bench3p32) step bench_c3_p32 900 env BH_ROUND_P8=0 python bench.py --cfg 3 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench3s16) step bench_c3_s16 900 env BH_SEGMENTS=16 python bench.py --cfg 3 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench3s12) step bench_c3_s12 900 env BH_SEGMENTS=12 python bench.py --cfg 3 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench3s6) step bench_c3_s6 900 env BH_SEGMENTS=6 python bench.py --cfg 3 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench3nolt) step bench_c3_nolt 900 env BH_LOOP_TIMING=0 python bench.py --cfg 3 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench5) step bench_c5 600 python bench.py --cfg 5 --steps 3 --warmup 1 ;;
    bench4) step bench_c4 1100 python bench.py --cfg 4 --steps 1 --warmup 1 ;;
    bench4q) step bench_c4 1100 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 ;;
    bench3g0) step bench_c3_g0 900 env BH_ROUND_P8G=0 python bench.py --cfg 3 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench2g0) step bench_c2_g0 600 env BH_ROUND_P8G=0 python bench.py --cfg 2 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench3q) step bench_c3 900 python bench.py --cfg 3 --steps 3 --warmup 1 --cpu-sample 0 ;;
    bench4i0) step bench_c4_i0 1100 env BH_ROUND_ILP2=0 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 ;;
    bench4g0) step bench_c4_g0 1100 env BH_ROUND_P8G=0 python bench.py --cfg 4 --steps 1 --warmup 1 --cpu-sample 0 ;;
    tround) step pytest_round 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_schedule.py tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -rf ;;
    diag4) step diag_c4 900 env BH_DIAG=1 python bench.py --cfg 4 --steps 1 --warmup 0 --cpu-sample 0 ;;
    diag4old) step diag_c4_old 900 env BH_DIAG=1 BH_FLOWW=1 python bench.py --cfg 4 --steps 1 --warmup 0 --cpu-sample 0 ;;
    diag3) step diag_c3 600 env BH_DIAG=1 python bench.py --cfg 3 --steps 1 --warmup 1 --cpu-sample 0 ;;
    pmc3) step pmc_c3 900 bash tools/pmc.sh c3 "k_" --cfg 3 ;;
    pmc4) step pmc_c4 1100 bash tools/pmc.sh c4 "k_" --cfg 4 ;;
    bresetdiag) step bench_reset_diag 600 env BH_DIAG=1 BH_FIAT_DEBUG=1 python tools/bench_reset.py --n 128 --N 1000000 --block 2 --steps 1 ;;
    bresetdbg) step bench_reset_dbg 600 env BH_FIAT_DEBUG=1 python tools/bench_reset.py --n 128 --N 1000000 --block 2 --steps 1 ;;
    breset) step bench_reset 600 python tools/bench_reset.py --n 128 --N 1000000 --block 2 --out gpurun_out/bench_reset_n128.json ;;
    breset32) step bench_reset32 600 python tools/bench_reset.py --n 32 --N 1000000 --seed 2980 --block 2 --out gpurun_out/bench_reset_n32.json ;;
    profreset) step prof_reset 600 bash -c 'export TMPDIR=/tmp; mkdir -p gpurun_out/prof_reset; rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_reset -o run -- python tools/bench_reset.py --n 128 --N 1000000 --block 2 --steps 1' ;;
    pmct) step pmc_t 900 bash tools/pmc.sh t "k_flow_transpose|k_fd_transpose" --cfg 3 ;;
    prof3) step prof_c3 900 bash tools/prof.sh c3 --cfg 3 --steps 3 --warmup 1 ;;
    prof4) step prof_c4 1100 bash tools/prof.sh c4 --cfg 4 --steps 1 --warmup 1 ;;
  esac
done
