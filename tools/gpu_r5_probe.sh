# round-5: k_round2p's shortened probe chain: parity suites, then a same-box A/B against the previous build
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_knobs.py "tests/test_gpu_whole.py::test_c3_whole_dag" -m gpu > gpurun_out/r5_tests_probe.log 2>&1 || exit 1
bash tools/ab_libs.sh 3 - ablibs/head.so > gpurun_out/r5_ab_probe.txt 2>&1 || exit 2
