"""One rank of a multi-process shard group whose exchange runs over the host
transport (bh_comm_init_transport) on a torch gloo group -- the child
process tests/test_gpu_comm.py starts per rank, all on device 0 (RCCL
refuses two ranks on one GPU; the host transport carries the same bytes at
the same call sites: rank 0's base broadcast, the split's per-segment
send / receive, the replicated exchanges' broadcasts).

Every rank inserts the same DAG in per-sync batches and calls RunConsensus
after each (every pass is collective); rank 0 compares its state with the
oracle's after every call -- the cross-node agreement check of the
reference (node/core_test.go:361-380: every node's blocks and consensus
events are the same) with rank 0 as the node.  Every rank that holds
results (all of them, except the coordinate ranks of a wide split, which
must refuse result queries: they ran no consensus pass) reports a digest of
its whole final state, which the test requires to be the same on every
such rank: the sharded fame rounds and frame sorts reached every rank.
"""
import argparse
import json
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    for k in ("rank", "world", "port", "n", "N", "seed", "lag", "step"):
        ap.add_argument("--" + k, type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=a.world)
    from babble_amd import Hashgraph, HashgraphError
    from babble_amd.dag import Dag
    from digest import engine_digest

    def t(buf):
        return torch.frombuffer(buf, dtype=torch.uint8)

    res = {"rank": a.rank, "ok": False}
    try:
        d = Dag(a.n, a.N, a.seed, lagging=a.lag, sig_mode=0)
        hg = Hashgraph(d.participant_ids, a.N, device=0)
        hg.comm_init_transport(a.rank, a.world, lambda b, p: dist.send(t(b), dst=p),
                               lambda b, p: dist.recv(t(b), src=p), lambda b, r: dist.broadcast(t(b), src=r))
        spi, opc, opi = d.wire()
        pid = d.participant_ids
        opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
        o = None
        if a.rank == 0:
            from oracle_py import Oracle
            from test_gpu_parity import _compare
            o = Oracle(a.n, pid, capacity=a.N)
        args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
        calls = 0
        for lo in range(0, a.N, a.step):
            hi = min(a.N, lo + a.step)
            st = hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi], opi[lo:hi],
                                  d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])
            assert not np.asarray(st).any()
            hg.run_consensus()
            calls += 1
            if o is not None:
                o.insert_dag(*(x[lo:hi] for x in args))
                o.run_consensus()
                _compare(o, hg, f"rank 0 of {a.world} after [0, {hi})")
        res["segments"], res["incremental_calls"] = hg.pipeline()
        res["exchange_ms"] = hg.stage_ms()[5]
        try:
            res["consensus_events"] = int(hg.stats().consensus_events)
            res["digest"] = engine_digest(hg)
            res["stats"] = "returned"
        except HashgraphError as e:
            res["stats"] = f"refused ({e.code})"
            try:  # the other result getters refuse alike (a negated code, not an empty list)
                hg.pending_rounds
                res["pending_rounds"] = "returned"
            except HashgraphError as e2:
                res["pending_rounds"] = f"refused ({e2.code})"
        res["calls"] = calls
        res["ok"] = True
        hg.close()
    except Exception:
        res["error"] = traceback.format_exc()
    with open(a.out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()
    sys.exit(0 if res["ok"] else 1)


if __name__ == "__main__":
    main()
