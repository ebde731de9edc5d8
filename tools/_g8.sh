cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for K in 1 8; do echo "K=$K"; BH_SEGMENTS=$K bash tools/ab.sh --steps 3 -- ab_libs/nt.so || exit 1; done
