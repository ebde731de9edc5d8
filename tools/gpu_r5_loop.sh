# round-5: the k_round2p suites (parity, schedules, shards, knobs, comm, whole C3) after a loop change
set -o pipefail
tag=${1:-loop}
timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_shard.py tests/test_gpu_knobs.py tests/test_gpu_comm.py tests/test_gpu_fuzz.py "tests/test_gpu_whole.py::test_c3_whole_dag" -m gpu > gpurun_out/r5_tests_$tag.log 2>&1 || exit 1
