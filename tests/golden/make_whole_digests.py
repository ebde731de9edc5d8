"""Whole-DAG oracle digests of BASELINE configs (tests/golden/whole_*.json).

The oracle (oracle/hg_oracle.c, the CPU restatement of hashgraph.go) runs
the batch schedule -- every event inserted, then DivideRounds, DecideFame,
DecideRoundReceived, ProcessDecidedRounds once, as BenchmarkConsensus
(hashgraph_test.go:1522-1534) and bench.py do -- over the same seeded DAG
the bench times, and tests/digest.py hashes its outputs.  The GPU test
(tests/test_gpu_whole.py) runs the engine on the same DAG and compares.

  python tests/golden/make_whole_digests.py --cfg 3            # C3, ~10 GB, minutes
  python tests/golden/make_whole_digests.py --cfg 4 --coord16  # C4, ~45 GB, about an hour
  python tests/golden/make_whole_digests.py --n 160 --N 4000000 --seed 0xB16 --lagging 40 --name wide160

--coord16 uses oracle/liboracle16.so (the same source with 16-bit coordinate
storage; it aborts on an index it cannot hold).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=0)
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--N", type=int, default=0)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0)
    ap.add_argument("--lagging", type=int, default=0)
    ap.add_argument("--lag-div", type=int, default=50)
    ap.add_argument("--name", default="")
    ap.add_argument("--coord16", action="store_true")
    args = ap.parse_args()
    if args.coord16:
        subprocess_make("liboracle16.so")
        os.environ["BH_ORACLE_LIB"] = os.path.join(ROOT, "oracle", "liboracle16.so")
    from babble_amd.dag import CONFIGS, Dag
    from digest import oracle_digest
    from oracle_py import Oracle

    if args.cfg:
        c = CONFIGS[args.cfg]
        N = args.N or c["N"]
        d = Dag.config(args.cfg, N=N, sig_mode=0)
        spec = dict(cfg=args.cfg, n=c["n"], N=N, seed=0xBABB1E00 + args.cfg, lagging=c["lagging"], lag_div=50)
        name = args.name or f"c{args.cfg}"
    else:
        d = Dag(args.n, args.N, args.seed, lagging=args.lagging, lag_div=args.lag_div, sig_mode=0)
        spec = dict(cfg=0, n=args.n, N=args.N, seed=args.seed, lagging=args.lagging, lag_div=args.lag_div)
        name = args.name
    import numpy as np
    spec["max_chain"] = int(np.bincount(d.creator, minlength=d.n).max())
    print(f"{name}: n={d.n} N={d.N} longest chain {spec['max_chain']}", flush=True)
    t0 = time.perf_counter()
    o = Oracle(d.n, d.participant_ids, capacity=d.N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    t1 = time.perf_counter()
    print(f"inserted in {t1 - t0:.0f}s", flush=True)
    o.run_consensus()
    t2 = time.perf_counter()
    print(f"consensus in {t2 - t1:.0f}s", flush=True)
    dg = oracle_digest(o)
    dg["spec"] = spec
    dg["oracle"] = dict(lib=os.path.basename(os.environ.get("BH_ORACLE_LIB", "liboracle.so")),
                        insert_s=round(t1 - t0, 1), consensus_s=round(t2 - t1, 1), threads=1)
    out = os.path.join(HERE, f"whole_{name}.json")
    with open(out, "w") as f:
        json.dump(dg, f, indent=1)
    print(f"wrote {out}: {dg['n_ordered']} ordered, {dg['n_blocks']} blocks, last round {dg['stats']['last_round']}")


def subprocess_make(target):
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), target])


if __name__ == "__main__":
    main()
