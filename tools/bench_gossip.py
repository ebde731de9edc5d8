"""Cost of the live node's schedule: Core.Sync inserts a
gossip batch and calls RunConsensus (node.go:583-603 -> core.go:337-369).
The engine recomputes the passes over the whole DAG on each call, so one
call costs about the batch run over the DAG so far.  This times insert +
RunConsensus per call as the DAG grows and prints one JSON line.
usage: python tools/bench_gossip.py [--n 128] [--events N] [--batch B]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=50_000)
    a = ap.parse_args()
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    d = Dag(a.n, a.events, 0xBABB1E40, sig_mode=0)
    pid = np.asarray(d.participant_ids)
    spi, opc, opi = d.wire()
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    cre = pid[d.creator]
    hg = Hashgraph(pid, a.events)
    calls = []
    for lo in range(0, a.events, a.batch):
        hi = min(a.events, lo + a.batch)
        t0 = time.perf_counter()
        st = hg.insert_events(cre[lo:hi], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi], opi[lo:hi],
                              d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])
        t1 = time.perf_counter()
        hg.run_consensus()
        t2 = time.perf_counter()
        assert not np.asarray(st).any()
        s = hg.stats()
        calls.append({"events": hi, "insert_ms": round((t1 - t0) * 1e3, 2),
                      "consensus_ms": round((t2 - t1) * 1e3, 2), "consensus_events": s.consensus_events})
        print(json.dumps(calls[-1]), file=sys.stderr, flush=True)
    tot = sum(c["insert_ms"] + c["consensus_ms"] for c in calls) / 1e3
    print(json.dumps({"metric": "gossip schedule: insert + RunConsensus per batch, whole-DAG recompute",
                      "n": a.n, "events": a.events, "batch": a.batch, "calls": len(calls),
                      "total_s": round(tot, 3), "events_ordered_per_s": round(calls[-1]["consensus_events"] / tot),
                      "last_call": calls[-1]}))


if __name__ == "__main__":
    main()
