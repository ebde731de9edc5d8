"""The live node's schedule through the engine: RunConsensus after every
gossip batch (node.go:583-603 -> core.go:337-369), the state the Go
Hashgraph keeps between calls, and the RoundInfo query surface.

The reference's Hashgraph is a state machine: InsertEvent only appends to
UndeterminedEvents, each pass updates its own part, and PendingRounds'
`queued` / sticky `decided` flags make the result depend on the call
schedule (hashgraph.go:689-695, 809-815; roundInfo.go:35).  The
oracle replays the Go state machine literally; every comparison here is
against the oracle run on the same schedule, bit-exact."""
import json
import os

import numpy as np
import pytest

from kat import KatDag
from oracle_py import UNSET, Oracle
from test_gpu_parity import _compare, _insert_kat

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _wire_batches(d):
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)

    def batch(lo, hi):
        return (pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi], opi[lo:hi],
                d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])
    return batch


def _schedule(n, N, seed, lagging, lag_div, step, check_every=True):
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, lagging=lagging, lag_div=lag_div, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    batch = _wire_batches(d)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        assert not np.asarray(hg.insert_events(*batch(lo, hi))).any()
        hg.run_consensus()
        if check_every or hi == N:
            _compare(o, hg, f"after events [0, {hi})")
    return d, o, hg


def test_queued_trap_fixture():
    """SURVEY A.12 on a seeded lagging-peer DAG (tests/golden/trap_schedule.json):
    a lagging peer's witness lands in a round that was already processed, so
    it is never queued again -- its fame stays Undefined, its round never
    again reports WitnessesDecided, and an older undetermined event of the
    same peer is never received (hashgraph.go:809-815, 984-986).  The batch
    schedule decides both.  The engine must follow the per-sync schedule."""
    with open(os.path.join(GOLDEN, "trap_schedule.json")) as f:
        fx = json.load(f)
    d, o, hg = _schedule(fx["n"], fx["N"], fx["seed"], fx["lagging"], fx["lag_div"], fx["step"])
    res = hg.results()
    for e, want in fx["per_sync"]["fame"].items():
        assert res["fame"][int(e)] == want, e
    for e, want in fx["per_sync"]["round_received"].items():
        assert res["round_received"][int(e)] == (UNSET if want is None else want), e
    w = int(fx["trapped_witness"])
    info = hg.round_info(int(res["round"][w]))
    assert w in info["witnesses"].tolist() and not info["witnesses_decided"]
    assert not info["pending"]


@pytest.mark.parametrize("n,N,seed,lag,div,step", [
    (5, 4000, 1003, 1, 40, 3),
    (9, 6000, 1014, 3, 80, 7),
    (13, 6000, 1021, 4, 300, 17),
])
def test_lagging_schedules(n, N, seed, lag, div, step):
    """Per-sync schedules with strongly lagging peers, state compared after
    every RunConsensus call."""
    _schedule(n, N, seed, lag, div, step)


def test_state_between_insert_and_run():
    """InsertEvent leaves every pass's results in place: between an insert and
    the next RunConsensus the counters, the consensus order, PendingRounds and
    the per-event fields read what the Go Hashgraph holds at that point
    (undetermined grows by the new events; nothing else changes)."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    n, N, step = 8, 9000, 1500
    d = Dag(n, N, 404, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    batch = _wire_batches(d)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        hg.insert_events(*batch(lo, hi))
        _compare(o, hg, f"after inserting [0, {hi}), before RunConsensus")
        o.run_consensus()
        hg.run_consensus()
        _compare(o, hg, f"after RunConsensus on [0, {hi})")


def test_stepwise_passes_across_calls():
    """The four passes called one at a time on every call of a schedule
    (core.go:337-369 calls them in sequence); the state after EACH pass
    equals the oracle's."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    n, N, step = 6, 5000, 700
    d = Dag(n, N, 505, lagging=1, lag_div=30, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    batch = _wire_batches(d)
    passes = (("divide_rounds", "divide_rounds"), ("decide_fame", "decide_fame"),
              ("decide_round_received", "decide_round_received"),
              ("process_decided_rounds", "process_decided_rounds"))
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        hg.insert_events(*batch(lo, hi))
        for go, ours in passes:
            getattr(o, go)()
            getattr(hg, ours)()
            _compare(o, hg, f"[0, {hi}) after {go}")


def test_stepwise_passes_pipelined(monkeypatch):
    """The passes one at a time through the n <= 128 segment pipeline (the
    persistent loop, witness tables launched from the device's round count,
    DecideFame's device-bounded scatter, no fused DecideRoundReceived): the
    state after each pass equals the oracle's, and the same DAG through
    RunConsensus ends in the same state."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    monkeypatch.setenv("BH_SEGMENTS", "3")
    n, N, step = 128, 30000, 10000
    d = Dag(n, N, 606, lagging=20, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    whole = Hashgraph(d.participant_ids, N)
    batch = _wire_batches(d)
    passes = ("divide_rounds", "decide_fame", "decide_round_received", "process_decided_rounds")
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        hg.insert_events(*batch(lo, hi))
        whole.insert_events(*batch(lo, hi))
        for p in passes:
            getattr(o, p)()
            getattr(hg, p)()
            _compare(o, hg, f"[0, {hi}) after {p}")
        whole.run_consensus()
        _compare(o, whole, f"[0, {hi}) RunConsensus")
    assert hg.pipeline()[0] == 3 and whole.pipeline()[0] == 3


def test_round_info_kat():
    """TestDivideRounds' per-round witness sets (hashgraph_test.go:746-828) and
    TestDecideFame's fame (:1267-1343) through Store.GetRound / RoundInfo;
    GetRound of a missing round is KeyNotFound (inmem_store.go:185-191)."""
    from babble_amd import Hashgraph, HashgraphError
    d = KatDag("kat_round")
    hg = Hashgraph(d.participant_ids, 64)
    _insert_kat(hg, d)
    hg.divide_rounds()
    ex = d.expect["divide_rounds"]
    assert hg.last_round() == ex["last_round"]
    for r, ws in ex["witnesses"].items():
        info = hg.round_info(int(r))
        assert sorted(d.names[i] for i in info["witnesses"]) == sorted(ws), r
        assert info["queued"] and info["pending"]
    with pytest.raises(HashgraphError) as ei:
        hg.round_info(ex["last_round"] + 1)
    assert ei.value.kind == "KeyNotFound"

    d = KatDag("kat_consensus")
    hg = Hashgraph(d.participant_ids, 64)
    _insert_kat(hg, d)
    o = Oracle(d.n, d.participant_ids, capacity=64)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    hg.divide_rounds()
    o.divide_rounds()
    hg.decide_fame()
    o.decide_fame()
    famous = d.expect["famous"]
    seen = set()
    ores = o.results()
    for r in range(hg.last_round() + 1):
        info = hg.round_info(r)
        for w, f in zip(info["witnesses"].tolist(), info["fame"].tolist()):
            assert f == ores["fame"][w], (r, d.names[w])
            name = d.names[w]
            if name in famous:
                assert f == (1 if famous[name] else 2), name
                seen.add(name)
        assert info["witnesses_decided"] == all(f != 0 for f in info["fame"].tolist())
    assert seen == set(famous)
    hg.decide_round_received()
    o.decide_round_received()
    ores = o.results()
    for r in range(hg.last_round() + 1):
        assert hg.round_info(r)["n_consensus"] == int(np.sum(ores["round_received"] == r)), r


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,N,seed,lag,div,step", [
    (128, 60_000, 3067, 40, 60, 500),   # C3's width: k_flow32 + k_round2, fame from ballots
    (200, 60_000, 4146, 60, 60, 400),   # the wide path: k_floww2 + 16-bit k_round_wide, fame from ssw masks
])
def test_per_sync_trap_wide(n, N, seed, lag, div, step):
    """The per-sync schedule at C3's width and on the wide path, state
    compared after EVERY call; seeded so that the A.12 trap occurs (a lagging
    peer's witness lands in a round already processed: never queued again,
    its fame stays Undefined, hashgraph.go:809-815, 984-986).  Every call
    after the first resumes from the previous call's device state."""
    d, o, hg = _schedule(n, N, seed, lag, div, step)
    res = o.results()
    lcr = o.last_consensus_round()
    trapped = np.nonzero((res["witness"] == 1) & (res["fame"] == 0) & (res["round"] < lcr))[0]
    assert len(trapped) >= 1, "the seed no longer produces a trapped witness"
    calls = (N + step - 1) // step
    assert hg.pipeline()[1] >= calls - 2


@pytest.mark.parametrize("n,N,silent,join,step", [(9, 20_000, 4, 12_000, 500), (16, 30_000, 3, 40_000, 1_000)])
def test_schedule_silent_peer(n, N, silent, join, step):
    """A peer with no event at all (join >= N: never) or one that joins late:
    its empty chain must not pin the incremental resume point to round 0
    (k_resume_point only counts the chains a call extends), and every call
    equals the oracle's state."""
    from babble_amd import Hashgraph
    from reset import SilentDag
    d = SilentDag(n, N, 700 + n, silent, join)
    pid = d.participant_ids
    o = Oracle(n, pid, capacity=N)
    hg = Hashgraph(pid, N)
    spi = np.where(d.sp >= 0, d.index - 1, -1)
    opc = np.where(d.op >= 0, pid[d.creator[np.maximum(d.op, 0)]], -1)
    opi = np.where(d.op >= 0, d.index[np.maximum(d.op, 0)], -1)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(d.creator[lo:hi], d.index[lo:hi], d.sp[lo:hi], d.op[lo:hi], d.hashes[lo:hi], d.sig_r[lo:hi],
                     d.ntx[lo:hi])
        o.run_consensus()
        assert not np.asarray(hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc[lo:hi],
                                               opi[lo:hi], d.hashes[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])).any()
        hg.run_consensus()
        _compare(o, hg, f"silent peer, after [0, {hi})")
    # every call but the first and the relayouts (a chain outgrowing its
    # slack: about every 1024 / (step / n) calls here) resumes
    assert hg.pipeline()[1] >= N // step - 1 - (N // step) // (1024 * n // step)
