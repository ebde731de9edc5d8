cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_c3 gpurun_out/pmc_c3
bash tools/prof.sh c3 --cfg 3 --steps 2 --warmup 1 && echo prof ok && \
bash tools/pmc.sh c3 "k_" --cfg 3 && echo pmc ok
