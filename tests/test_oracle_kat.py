"""Pins the CPU oracle against the reference's own known-answer tests
(src/hashgraph/hashgraph_test.go, transcribed in tests/golden/kat_*.json).
Each test cites the Go test it mirrors."""
import numpy as np
import pytest

from kat import KatDag
from oracle_py import UNSET, Oracle


def build(name):
    d = KatDag(name)
    o = Oracle(d.n, d.participant_ids, capacity=len(d) + 64)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    return d, o


def test_ancestry_hashgraph():  # TestAncestor / TestSelfAncestor / TestSee
    d, o = build("kat_hashgraph")
    for x, y, v in d.expect["ancestor"]:
        assert o.see(d.id_of[x], d.id_of[y]) == v, (x, y)
    for x, y, v in d.expect["self_ancestor"]:
        ex, ey = d.id_of[x], d.id_of[y]
        sa = (x == y) or (d.creator[ex] == d.creator[ey] and d.index[ex] >= d.index[ey])
        assert sa == v, (x, y)  # _selfAncestor is pure index arithmetic
    for x, y, v in d.expect["see"]:
        assert o.see(d.id_of[x], d.id_of[y]) == v, (x, y)


def test_lamport_hashgraph():  # TestLamportTimestamp
    d, o = build("kat_hashgraph")
    for e, t in d.expect["lamport"].items():
        assert o.lamport(d.id_of[e]) == t, e


def test_insert_coordinates():  # TestInsertEvent
    d, o = build("kat_round")
    for e, c in d.expect["coordinates"].items():
        la, fd = o.coordinates(d.id_of[e])
        assert la.tolist() == c["la"], e
        assert fd.tolist() == c["fd"], e
    assert o.undetermined().tolist() == d.ids(d.expect["undetermined_after_insert"])
    assert o.pending_loaded_events() == d.expect["pending_loaded_after_insert"]


def test_strongly_see_round_witness():  # TestStronglySee / TestRound / TestWitness
    d, o = build("kat_round")
    for x, y, v in d.expect["strongly_see"]:
        assert o.strongly_see(d.id_of[x], d.id_of[y]) == v, (x, y)
    o.divide_rounds()
    for e, r in d.expect["round"].items():
        assert o.round(d.id_of[e]) == r, e
    for e, w in d.expect["witness"].items():
        assert o.witness(d.id_of[e]) == w, e
    for x, y, diff in d.expect["round_diff"]:
        assert o.round(d.id_of[x]) - o.round(d.id_of[y]) == diff


def test_divide_rounds():  # TestDivideRounds
    d, o = build("kat_round")
    assert o.divide_rounds() == 0
    ex = d.expect["divide_rounds"]
    assert o.last_round() == ex["last_round"]
    res = o.results()
    for r, ws in ex["witnesses"].items():
        got = sorted(d.names[i] for i in np.nonzero((res["round"] == int(r)) & (res["witness"] == 1))[0])
        assert got == sorted(ws)
    assert o.pending_rounds() == [tuple(p) for p in ex["pending_rounds"]]
    for e, (t, r) in ex["lamport_round"].items():
        assert res["lamport"][d.id_of[e]] == t and res["round"][d.id_of[e]] == r, e


def test_consensus_passes():  # TestDivideRoundsBis .. TestProcessDecidedRounds
    d, o = build("kat_consensus")
    ex = d.expect
    o.divide_rounds()
    res = o.results()
    for e, (t, r) in ex["lamport_round"].items():
        assert (res["lamport"][d.id_of[e]], res["round"][d.id_of[e]]) == (t, r), e
    o.decide_fame()
    res = o.results()
    for e, fam in ex["famous"].items():
        assert res["witness"][d.id_of[e]] == 1 and res["fame"][d.id_of[e]] == (1 if fam else 2), e
    assert o.pending_rounds() == [tuple(p) for p in ex["pending_after_fame"]]
    o.decide_round_received()
    res = o.results()
    for i, name in enumerate(d.names):
        want = ex["round_received_by_prefix"].get(name[0], UNSET)
        assert res["round_received"][i] == want, name
    for r, cnt in ex["consensus_events_per_round"].items():
        assert int(np.sum(res["round_received"] == int(r))) == cnt
    assert o.undetermined().tolist() == d.ids(ex["undetermined_after_rr"])
    o.process_decided_rounds()
    order = o.consensus_order()
    assert len(order) == ex["consensus_len"]
    assert o.pending_loaded_events() == ex["pending_loaded"]
    b = o.blocks()
    assert b["round_received"].tolist()[:2] == [1, 2]
    blk0 = [t for e in order[b["first"][0]:b["first"][0] + b["count"][0]] for t in d.txs[e]]
    assert blk0 == ex["blocks"][0]["txs"]
    blk1 = [t for e in order[b["first"][1]:b["first"][1] + b["count"][1]] for t in d.txs[e]]
    assert len(blk1) == ex["blocks"][1]["ntx"] and blk1[1] == ex["blocks"][1]["tx1"]
    assert o.pending_rounds() == [tuple(p) for p in ex["pending_after_process"]]
    # TestGetFrame: frame events = the set, sorted ByLamportTimestamp
    res = o.results()
    for rr, names in ex["frame_events"].items():
        bi = list(b["round_received"]).index(int(rr))
        got = order[b["first"][bi]:b["first"][bi] + b["count"][bi]].tolist()
        ids = d.ids(names)
        want = sorted(ids, key=lambda e: (res["lamport"][e], bytes(d.sig_r[e])))
        assert got == want
    # TestKnown
    known = [int(np.max(d.index[d.creator == c])) for c in range(d.n)]
    assert known == ex["known"]


def test_funky_out_of_order_decision():  # TestFunkyHashgraphFame
    d, o = build("kat_funky")
    o.divide_rounds()
    o.decide_fame()
    assert o.last_round() == d.expect["last_round"]
    assert o.pending_rounds() == [tuple(p) for p in d.expect["pending_after_fame"]]
    o.decide_round_received()
    o.process_decided_rounds()
    assert o.pending_rounds() == [tuple(p) for p in d.expect["pending_after_process"]]


def test_funky_blocks():  # TestFunkyHashgraphBlocks
    d, o = build("kat_funky_full")
    o.run_consensus()
    assert o.last_round() == d.expect["last_round"]
    assert o.pending_rounds() == [tuple(p) for p in d.expect["pending_after_process"]]
    assert o.blocks()["ntx"].tolist()[:3] == d.expect["block_ntx"]


def test_sparse_frames_and_replay():  # initSparseHashgraph + TestSparseHashgraphFrames
    d, o = build("kat_sparse")
    # the replayed plays are all rejected (hashgraph_test.go:2515-2524, :135-137)
    for e in range(4, len(d)):
        rc = o.insert(int(d.creator[e]), int(d.index[e]), int(d.sp[e]), int(d.op[e]),
                      d.hashes[e].tobytes(), d.sig_r[e].tobytes(), int(d.ntx[e]))
        assert rc != 0
    o.run_consensus()
    b = o.blocks()
    assert len(b["ntx"]) >= d.expect["min_blocks"]
    assert b["round_received"].tolist()[:3] == d.expect["block_round_received"]
    order = o.consensus_order()
    for rr, names in d.expect["frame_events_diagram"].items():
        bi = list(b["round_received"]).index(int(rr))
        got = sorted(order[b["first"][bi]:b["first"][bi] + b["count"][bi]].tolist())
        assert got == sorted(d.ids(names)), rr


def test_fork_rejected():  # TestFork
    d, o = build("kat_fork")
    N = o.num_events()
    for c, k, spn, opn, name, tx in d.fx["rejects"]:
        sp = d.id_of[spn] if spn in d.id_of else -1
        op = d.id_of[opn] if opn in d.id_of else (N + 100 if opn else -1)
        assert o.insert(c, k, sp, op, bytes(32), bytes(32), len(tx or [])) != 0, name
    assert o.num_events() == N


@pytest.mark.parametrize("name", ["kat_consensus", "kat_funky_full", "kat_sparse", "kat_round"])
def test_batch_equals_stepwise(name):
    """run_consensus == the four passes called one by one (core.go:335-377)."""
    d, o1 = build(name)
    _, o2 = build(name)
    o1.run_consensus()
    o2.divide_rounds(); o2.decide_fame(); o2.decide_round_received(); o2.process_decided_rounds()
    r1, r2 = o1.results(), o2.results()
    for k in r1:
        assert np.array_equal(r1[k], r2[k]), k


def _state(o):
    return (o.results(), o.consensus_order(), o.blocks(), o.pending_rounds(), o.last_consensus_round(),
            o.consensus_transactions(), o.pending_loaded_events(), o.undetermined())


def _same_state(a, b):
    ra, oa, ba, pa, *sa, ua = a
    rb, ob, bb, pb, *sb, ub = b
    for k in ra:
        assert np.array_equal(ra[k], rb[k]), k
    assert np.array_equal(oa, ob)
    for k in ba:
        assert np.array_equal(ba[k], bb[k]), f"blocks.{k}"
    assert pa == pb and sa == sb
    assert np.array_equal(ua, ub)


@pytest.mark.parametrize("name", ["kat_consensus", "kat_funky_full", "kat_sparse", "kat_round"])
def test_incremental_schedule_equals_batch_kat(name):
    """The live node runs the four passes after every gossip batch
    (node.go:583-603 -> core.go:337-369); on the reference's KAT DAGs that
    schedule -- here the finest one, RunConsensus after every insert -- ends
    in the same state as one batch run.  The engine recomputes the passes
    over the whole DAG on each call, so this is what licenses it as a
    drop-in for the incremental schedule."""
    d, batch = build(name)
    batch.run_consensus()
    inc = Oracle(d.n, d.participant_ids, capacity=len(d) + 64)
    args = (d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    for i in range(len(d)):
        inc.insert_dag(*(a[i:i + 1] for a in args))
        inc.run_consensus()
    _same_state(_state(batch), _state(inc))


@pytest.mark.parametrize("n,N,seed,lag,step", [(4, 3000, 5, 0, 37), (7, 5000, 3, 0, 61), (9, 8000, 14, 3, 250)])
def test_incremental_schedule_equals_batch_random(n, N, seed, lag, step):
    """Same property on seeded gossip DAGs, RunConsensus every `step` events
    (lagging peers keep fame undecided across many calls)."""
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, lagging=lag, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    batch = Oracle(n, d.participant_ids, capacity=N)
    batch.insert_dag(*args)
    batch.run_consensus()
    inc = Oracle(n, d.participant_ids, capacity=N)
    for lo in range(0, N, step):
        inc.insert_dag(*(a[lo:lo + step] for a in args))
        inc.run_consensus()
    _same_state(_state(batch), _state(inc))


def test_queued_trap_fixture_oracle():
    """tests/golden/trap_schedule.json: on the per-sync schedule
    the late witness stays Undefined and the older lagging event is never
    received; one batch run decides both (hashgraph.go:809-815, 984-986)."""
    import json
    import os
    from babble_amd.dag import Dag
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "trap_schedule.json")) as f:
        fx = json.load(f)
    d = Dag(fx["n"], fx["N"], fx["seed"], lagging=fx["lagging"], lag_div=fx["lag_div"], sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    b = Oracle(fx["n"], d.participant_ids, capacity=fx["N"])
    b.insert_dag(*args)
    b.run_consensus()
    o = Oracle(fx["n"], d.participant_ids, capacity=fx["N"])
    for lo in range(0, fx["N"], fx["step"]):
        o.insert_dag(*(a[lo:lo + fx["step"]] for a in args))
        o.run_consensus()
    for which, orc in (("per_sync", o), ("batch", b)):
        res = orc.results()
        for e, want in fx[which]["fame"].items():
            assert res["fame"][int(e)] == want, (which, e)
        for e, want in fx[which]["round_received"].items():
            assert res["round_received"][int(e)] == (UNSET if want is None else want), (which, e)
        assert len(orc.consensus_order()) == fx[which]["consensus_events"], which
    w = fx["trapped_witness"]
    assert o.results()["witness"][w] == 1
