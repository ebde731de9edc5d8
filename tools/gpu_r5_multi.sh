# rehearsal of bench.py --gpus 2 on one device (BH_BENCH_ONE_DEVICE=1: gloo), both modes
set -o pipefail
export BH_BENCH_ONE_DEVICE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --events 2000000 > gpurun_out/r5_multi_replicas.json 2> gpurun_out/r5_multi_replicas.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 2 --steps 3 --warmup 1 --events 2000000 --mode shards > gpurun_out/r5_multi_shards.json 2> gpurun_out/r5_multi_shards.err || exit 2
