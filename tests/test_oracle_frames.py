"""Pins the oracle's block projection: the frame roots
of GetFrame (hashgraph.go:1125-1231) against TestGetFrame
(hashgraph_test.go:1565-1670) and TestSparseHashgraphFrames (:2568-2653),
and its Frame / Block JSON against an independent restatement in Python's
json module (tests/frames.py), on the KAT DAGs and on generated DAGs whose
bodies are the Go-JSON bodies their hashes were computed from."""
import pytest

from frames import (base36, block_json, frame_json, kat_event_bytes, matches_fixture,
                    roots_by_name, sha)
from kat import KatDag
from oracle_py import Oracle


def _kat(name):
    d = KatDag(name)
    o = Oracle(d.n, d.participant_ids, capacity=len(d) + 64)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    bodies, sigs = {}, {}
    for e in range(len(d)):
        bodies[e], sigs[e] = kat_event_bytes(d, e)
        o.set_event_bytes(e, bodies[e], sigs[e])
    o.run_consensus()
    return d, o, bodies, sigs


def _check_bytes(o, ids, hashes, index, creator, bodies, sigs):
    res = o.results()
    b = o.blocks()
    order = o.consensus_order()
    assert len(b["round_received"]) > 0
    for bi, rr in enumerate(b["round_received"].tolist()):
        evs = order[b["first"][bi]:b["first"][bi] + b["count"][bi]].tolist()
        want = frame_json(rr, o.frame_roots(rr), evs, creator, ids, hashes, index,
                          res["lamport"], res["round"], bodies, sigs)
        got = o.frame_json(rr)
        assert got == want, (rr, got[:200], want[:200])
        assert o.block_frame_hash(bi) == sha(want)
        assert o.block_json(bi, body_only=True) == block_json(bi, rr, sha(want), evs, bodies, True)
        assert o.block_json(bi) == block_json(bi, rr, sha(want), evs, bodies)


@pytest.mark.parametrize("name", ["kat_consensus", "kat_sparse"])
def test_frame_roots_kat(name):
    d, o, bodies, sigs = _kat(name)
    res = o.results()
    for rr, want in d.expect["frame_roots"].items():
        got = roots_by_name(o.frame_roots(int(rr)), d, res["lamport"], res["round"])
        assert matches_fixture(got, want), (rr, got, want)
    _check_bytes(o, d.participant_ids, d.hashes, d.index, d.creator, bodies, sigs)


def test_frame_hash_needs_every_body():
    """No FrameHash without the bytes of every event of the frame"""
    d = KatDag("kat_consensus")
    o = Oracle(d.n, d.participant_ids, capacity=len(d) + 64)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    for e in range(len(d)):
        if d.names[e] != "f1":  # f1 is in frame 2 (block 1)
            o.set_event_bytes(e, *kat_event_bytes(d, e))
    o.run_consensus()
    assert o.block_frame_hash(0) is not None
    assert o.block_frame_hash(1) is None and o.block_json(1) is None
    assert o.frame_roots(2) is not None


@pytest.mark.parametrize("n,N,seed,lag,step", [(4, 1500, 71, 0, 0), (7, 3000, 72, 2, 0),
                                               (5, 2500, 73, 1, 37)])
def test_frame_bytes_generated(n, N, seed, lag, step):
    """Generated DAGs with the Go-JSON bodies their hashes are SHA-256 of
    (dag_gen.c bg_body_json), batch and per-sync schedules"""
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, lagging=lag, lag_div=40, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    bodies = {e: d.body_json(e) for e in range(N)}
    sigs = {e: (base36(d.sig_r[e]) + "|" + base36(d.sig_s[e])).encode() for e in range(N)}
    assert all(sha(bodies[e]) == bytes(d.hash[e]) for e in range(0, N, 97))
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    for lo in range(0, N, step or N):
        hi = min(N, lo + (step or N))
        o.insert_dag(*(a[lo:hi] for a in args))
        for e in range(lo, hi):
            o.set_event_bytes(e, bodies[e], sigs[e])
        o.run_consensus()
    _check_bytes(o, d.participant_ids, d.hash, d.index, d.creator, bodies, sigs)
