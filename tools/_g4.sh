cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp NCCL_DEBUG=WARN BH_BENCH_ONE_DEVICE=1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --cfg 2 --cpu-sample 0 > gpurun_out/b4_2.json 2> gpurun_out/b4_2.err; echo "2-proc rc=$?"; grep -v "^\s*$" gpurun_out/b4_2.err | tail -25 | cut -c1-250; cat gpurun_out/b4_2.json | head -c 1500
