cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && echo bench ok && \
bash tools/prof.sh c3 --cfg 3 --steps 2 --warmup 1 && echo prof ok && \
bash tools/pmc.sh c3 "k_" --cfg 3 && echo pmc ok
echo "rc=$?"
cat gpurun_out/bench_c3.json
