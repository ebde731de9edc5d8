"""Cost of the live node's schedule: Core.Sync inserts a
gossip batch and calls RunConsensus (node.go:583-603 -> core.go:337-369).
The engine keeps its state between calls and a call processes only what
was inserted since the previous one (new events' coordinates, the round
loop from its resume point, fame of pending rounds, frames of newly decided
rounds).  This times insert + RunConsensus per call as the DAG grows and
prints one JSON line; --prefill inserts that many events first with one
call, so the later calls run against a large resident DAG.
usage: python tools/bench_gossip.py [--n 128] [--events N] [--batch B] [--prefill P]"""
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
    ap.add_argument("--prefill", type=int, default=0)
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
    bounds = ([0, a.prefill] if a.prefill else [0]) + list(range(a.prefill + a.batch, a.events, a.batch)) + [a.events]
    for lo, hi in zip(bounds[:-1], bounds[1:]):
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
    inc = calls[1:] if a.prefill else calls
    tot = sum(c["insert_ms"] + c["consensus_ms"] for c in inc) / 1e3
    new = inc[-1]["events"] - (a.prefill if a.prefill else 0)
    cons = np.array([c["consensus_ms"] for c in inc])
    print(json.dumps({"metric": "gossip schedule: insert + RunConsensus per batch (incremental engine)",
                      "n": a.n, "events": a.events, "batch": a.batch, "prefill": a.prefill, "calls": len(inc),
                      "total_s": round(tot, 3), "ns_per_new_event": round(tot * 1e9 / max(new, 1), 1),
                      "consensus_ms_median": float(np.median(cons)), "consensus_ms_max": float(cons.max()),
                      "incremental_calls": hg.pipeline()[1],
                      "prefill_call": calls[0] if a.prefill else None, "last_call": inc[-1]}))


if __name__ == "__main__":
    main()
