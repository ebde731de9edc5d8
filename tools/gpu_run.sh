#!/bin/bash
# One GPU session's steps, chained so that the first failure ends it
# (usage: tools/gpu_run.sh TAG STEP...; STEP = tests:<pytest args> |
# bench:<cfg>:<steps>[:env=val,...] | multi:<N>:<cfg>:<events> | prof:<cfg>).
# Output under gpurun_out/<TAG>_*.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out
mkdir -p $out
for step in "$@"; do
  kind=${step%%:*}; arg=${step#*:}
  case $kind in
    tests)
      echo "== tests $arg"
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $arg \
        > $out/${tag}_tests.log 2>&1 || { tail -40 $out/${tag}_tests.log; exit 1; }
      tail -3 $out/${tag}_tests.log ;;
    bench|benchq)
      IFS=: read -r cfg steps envs <<< "$arg"
      name=${tag}_bench_c${cfg}${envs:+_$(echo $envs | tr ',=' '__')}
      echo "== bench cfg$cfg $envs"
      cpu=""; [ $kind = benchq ] && cpu="--cpu-sample 0"
      env $(echo $envs | tr ',' ' ') timeout -k 10 600 python -u bench.py --cfg $cfg --steps $steps --warmup 1 $cpu \
        > $out/$name.json 2> $out/$name.log || { tail -20 $out/$name.log; exit 1; }
      python3 -c "import json,sys; d=json.load(open('$out/$name.json')); print('$name', round(d['value']/1e6,2), 'M ev/s', round(d['ms_per_step'],2), 'ms', d['stages_ms'])" ;;
    multi)
      IFS=: read -r N cfg ev <<< "$arg"
      echo "== one-device multi N=$N cfg$cfg events=$ev"
      BH_BENCH_ONE_DEVICE=1 timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
        --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus $N --steps 3 --warmup 1 --cfg $cfg --events $ev \
        > $out/${tag}_multi$N.json 2> $out/${tag}_multi$N.log || { tail -30 $out/${tag}_multi$N.log; exit 1; }
      tail -c 600 $out/${tag}_multi$N.json ;;
    timeline)
      IFS=: read -r cfg envs <<< "$arg"
      name=${tag}_tl_c${cfg}${envs:+_$(echo $envs | tr ',=' '__')}
      echo "== timeline cfg$cfg $envs"
      env BH_DIAG=1 BH_TIMELINE=$out/$name.bin $(echo $envs | tr ',' ' ') timeout -k 10 600 python -u bench.py --cfg $cfg \
        --steps 1 --warmup 1 --cpu-sample 0 > $out/$name.json 2> $out/$name.log || { tail -20 $out/$name.log; exit 1; }
      python3 tools/timeline.py --tagged $out/$name.bin | tee $out/$name.txt ;;
    prof)
      echo "== rocprofv3 cfg$arg"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_prof -o run -- python3 -u bench.py --cfg $arg --steps 3 --warmup 1 --cpu-sample 0 \
        > $out/${tag}_prof.json 2> $out/${tag}_prof.log || { tail -20 $out/${tag}_prof.log; exit 1; }
      f=$(find $out/${tag}_prof -name '*kernel_stats.csv' | head -1); cp "$f" $out/${tag}_kernel_stats.csv; head -8 $out/${tag}_kernel_stats.csv ;;
  esac
done
echo "== done"
