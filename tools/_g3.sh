cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/t3.log
timeout -k 10 300 python bench.py --steps 3 --cpu-sample 0 > gpurun_out/b3.json 2> gpurun_out/b3.err; echo "bench rc=$?"; cat gpurun_out/b3.json | head -c 600; echo
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --cfg 2 --cpu-sample 0 > gpurun_out/b3_2.json 2> gpurun_out/b3_2.err; echo "2-proc rc=$?"; tail -c 1500 gpurun_out/b3_2.err; cat gpurun_out/b3_2.json | head -c 800
