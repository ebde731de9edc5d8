"""Digests of a whole consensus run (test infrastructure).

A whole-DAG oracle run at BASELINE's sizes takes minutes to an hour on one
core (C3: 10M events, C4: 20M at n = 512), so it is done once, here, by
tests/golden/make_whole_digests.py, and the GPU tests compare the engine's
run of the same seeded DAG against the committed digests.  Every per-event
output is hashed in chunks of CHUNK events, so a mismatch names the chunk;
the consensus order, the blocks, PendingRounds, UndeterminedEvents and the
counters are hashed whole.  Both sides go through `run_digest`, so the
normalisation (dtypes, fame of non-witnesses) is the same by construction.
"""
import hashlib
import json

import numpy as np

CHUNK = 1_000_000

# fixed little-endian dtypes, so the bytes hashed do not depend on the
# producer's array types
_EVENT_KEYS = (("round", "<i4"), ("witness", "<i1"), ("lamport", "<i4"),
               ("round_received", "<i4"), ("fame", "<i1"), ("cons_pos", "<i8"))


def _h(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _chunks(a, dt):
    a = np.asarray(a).astype(dt, copy=False)
    return [_h(a[i:i + CHUNK]) for i in range(0, max(len(a), 1), CHUNK)]


def run_digest(results, order, blocks, pending, stats, undetermined):
    """results: the per-event dict of Oracle.results() / Hashgraph.results();
    blocks: dict round_received / first / count / ntx; pending: [(round,
    decided)]; stats: dict of counters; undetermined: event ids."""
    res = dict(results)
    res["fame"] = np.where(np.asarray(res["witness"]) == 1, res["fame"], -1)
    out = {"events": int(len(res["round"])), "chunk": CHUNK}
    for k, dt in _EVENT_KEYS:
        out[k] = _chunks(res[k], dt)
    out["consensus_order"] = _chunks(order, "<i4")
    out["n_ordered"] = int(len(order))
    out["blocks"] = {k: _h(np.asarray(blocks[k]).astype(dt)) for k, dt in
                     (("round_received", "<i4"), ("first", "<i8"), ("count", "<i8"), ("ntx", "<i8"))}
    out["n_blocks"] = int(len(blocks["round_received"]))
    out["pending_rounds"] = hashlib.sha256(json.dumps([[int(r), bool(d)] for r, d in pending]).encode()).hexdigest()
    out["n_pending"] = len(pending)
    out["undetermined"] = _h(np.asarray(undetermined).astype("<i4"))
    out["n_undetermined"] = int(len(undetermined))
    out["stats"] = {k: int(v) for k, v in stats.items()}
    return out


def oracle_digest(o):
    return run_digest(o.results(), o.consensus_order(), o.blocks(), o.pending_rounds(),
                      dict(last_round=o.last_round(), last_consensus_round=o.last_consensus_round(),
                           consensus_transactions=o.consensus_transactions(),
                           pending_loaded_events=o.pending_loaded_events()),
                      o.undetermined())


def engine_digest(hg):
    st = hg.stats()
    return run_digest(hg.results(), hg.consensus_order(), hg.blocks(), hg.pending_rounds,
                      dict(last_round=st.last_round, last_consensus_round=st.last_consensus_round,
                           consensus_transactions=st.consensus_transactions,
                           pending_loaded_events=st.pending_loaded_events),
                      hg.undetermined_events)


def diff(ref, got):
    """The keys (and chunk numbers) where two digests differ; [] if equal."""
    bad = []
    for k, v in ref.items():
        g = got.get(k)
        if isinstance(v, list) and isinstance(g, list) and len(v) == len(g):
            bad += [f"{k}[chunk {i}]" for i, (a, b) in enumerate(zip(v, g)) if a != b]
        elif v != g:
            bad.append(f"{k}: ref={v} got={g}" if not isinstance(v, (list, dict)) else k)
    return bad
