# round-5: the wide coordinate split (n > 128) and the shard / wide suites around it
set -o pipefail
tag=${1:-wsplit}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shard.py -m gpu > gpurun_out/r5_tests_$tag.log 2>&1 || exit 1
