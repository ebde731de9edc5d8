cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
echo "pytest rc=$?"
tail -30 gpurun_out/t1.log
