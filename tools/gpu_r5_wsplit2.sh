# round-5: the wide split over the multi-process host transport, then the wide parity suite
set -o pipefail
tag=${1:-wsplit2}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_comm.py -m gpu > gpurun_out/r5_tests_${tag}_comm.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "wide or floww or 160 or 512" > gpurun_out/r5_tests_${tag}_wide.log 2>&1 || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_hip -o run -- python3 bench.py --cpu-sample 0 --steps 2 --warmup 1 > gpurun_out/prof_hip_bench.json 2> gpurun_out/prof_hip_bench.err || exit 3
