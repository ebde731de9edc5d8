"""FastSync Reset at scale: a generated DAG runs
consensus with the block projection on; block b's Frame roots
(bh_get_frame_roots, GetFrame hashgraph.go:1125-1231) and the RootEvent
fields of their events build a Reset (bh_reset, hashgraph.go:1324-1369) of a
fresh handle; the frame's events and then every later event (getDiff,
hashgraph_test.go:2776-2795) arrive as wire events; RunConsensus over the
reset hashgraph is timed (whole-DAG recompute per call) beside the plain
hashgraph's run over the same DAG.  Everything runs through the engine; the
oracle parity of Reset is tests/test_gpu_reset.py's job.

  python tools/bench_reset.py --n 128 --N 1000000 --block 2
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def wire(d, pid, ids):
    ids = np.asarray(ids, np.int64)
    op = d.other_parent[ids]
    opc = np.where(op >= 0, pid[d.creator[np.maximum(op, 0)]], -1)
    opi = np.where(op >= 0, d.index[np.maximum(op, 0)], -1)
    return (pid[d.creator[ids]], d.index[ids], d.index[ids] - 1, opc, opi, d.hash.reshape(-1, 32)[ids],
            d.sig_r.reshape(-1, 32)[ids], d.ntx[ids])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=0xBA6)
    ap.add_argument("--block", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    t0 = time.time()
    d = Dag(a.n, a.N, a.seed, sig_mode=0)
    pid = np.asarray(d.participant_ids, np.int64)
    print(f"generated n={a.n} N={a.N} in {time.time() - t0:.1f}s", flush=True)
    # the original hashgraph: consensus, block b's frame and its roots
    hg = Hashgraph(pid, a.N, frames=True)
    assert not np.asarray(hg.insert_dag(d)).any()
    plain = []
    for k in range(a.steps + 1):
        hg.reset_consensus()
        t = time.time()
        hg.run_consensus()
        if k:
            plain.append((time.time() - t) * 1e3)
    res = hg.results()
    blocks = hg.blocks()
    order = hg.consensus_order()
    rr = int(blocks["round_received"][a.block])
    first, cnt = int(blocks["first"][a.block]), int(blocks["count"][a.block])
    frame = order[first:first + cnt]
    roots = hg.frame_roots(rr)
    idx, lt, rnd = d.index, res["lamport"], res["round"]
    hashes = d.hash.reshape(-1, 32)
    nr = [r[0] for r in roots]
    spe = [r[1] for r in roots]
    spi = [int(idx[e]) if e >= 0 else -1 for e in spe]
    splt = [int(lt[e]) if e >= 0 else -1 for e in spe]
    sprd = [int(rnd[e]) if e >= 0 else -1 for e in spe]
    oth = [(p, k, v) for p, r in enumerate(roots) for k, v in r[2]]
    o_root = [p for p, _, _ in oth]
    o_key = np.stack([hashes[k] for _, k, _ in oth]) if oth else np.zeros((0, 32), np.uint8)
    o_cre = [int(pid[d.creator[v]]) for _, _, v in oth]
    o_idx = [int(idx[v]) for _, _, v in oth]
    o_lt = [int(lt[v]) for _, _, v in oth]
    o_rnd = [int(rnd[v]) for _, _, v in oth]
    o_hash = np.stack([hashes[v] for _, _, v in oth]) if oth else np.zeros((0, 32), np.uint8)
    known = np.array(spi, np.int64)
    np.maximum.at(known, d.creator[frame], idx[frame])
    infr = np.zeros(a.N, bool)
    infr[frame] = True
    diff = np.nonzero(~infr & (idx > known[d.creator]))[0]
    F = max(max(nr), max(sprd))
    print(f"block {a.block}: round received {rr}, frame {cnt} events, {len(oth)} Others, F = {F}, "
          f"diff {len(diff)} events", flush=True)
    # the reset hashgraph
    h2 = Hashgraph(pid, a.N)
    h2.reset(rr, a.block, nr, spi, splt, sprd, o_root, o_key, o_cre, o_idx, o_lt, o_rnd, o_hash)
    st_f = h2.insert_events(*wire(d, pid, frame), raise_on_error=False)
    st_d = h2.insert_events(*wire(d, pid, diff), raise_on_error=False)
    runs, stages = [], []
    for k in range(a.steps + 1):
        h2.reset_consensus()
        t = time.time()
        h2.run_consensus()
        if k:
            runs.append((time.time() - t) * 1e3)
            stages.append(h2.stage_ms())
    r2 = h2.results()
    s2 = h2.stats()
    ordered = int(s2.consensus_events)
    n_ev = int(s2.n_events)
    fiat = int((r2["round"] <= F).sum())
    ms = float(np.median(runs))
    out = dict(tool="bench_reset", n=a.n, N=a.N, seed=a.seed, block=a.block, round_received=rr, F=F,
               frame_events=cnt, others=len(oth), inserted=n_ev, rejected=int((st_f != 0).sum() + (st_d != 0).sum()),
               fiat_region_events=fiat, reset_blocks=int(s2.blocks - s2.first_block), plain_blocks=len(blocks["count"]),
               reset_consensus_events=ordered, reset_ms_per_run=ms, reset_events_per_s=n_ev / ms * 1e3,
               reset_stage_ms=[round(float(x), 3) for x in np.median(np.array(stages), axis=0)],
               plain_ms_per_run=float(np.median(plain)), plain_events_per_s=a.N / float(np.median(plain)) * 1e3,
               note="whole reset hashgraph recomputed per RunConsensus (stage 1 includes the k_fiat pass); "
                    "events/s = events the reset hashgraph holds / wall ms of one run_consensus")
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
