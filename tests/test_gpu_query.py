"""The Hashgraph's pair predicates through the C-ABI (bh_query_events):
ancestor / selfAncestor / see (TestAncestor, TestSelfAncestor, TestSee,
hashgraph_test.go:204-306), stronglySee (TestStronglySee :611-643) and
roundDiff (TestRoundDiff :713-741) from the transcribed KATs, and every
predicate against the oracle on random pairs of generated DAGs."""
import numpy as np
import pytest

from kat import KatDag
from oracle_py import Oracle
from test_gpu_parity import _insert_kat

pytestmark = pytest.mark.gpu


def _kat(name):
    from babble_amd import Hashgraph
    d = KatDag(name)
    hg = Hashgraph(d.participant_ids, 64)
    _insert_kat(hg, d)
    return d, hg


def _pairs(d, rows):
    return [d.id_of[a] for a, *_ in rows], [d.id_of[b] for _, b, *_ in rows]


def test_query_kat_ancestry():
    d, hg = _kat("kat_hashgraph")  # queried right after insert: coordinates computed on demand
    for kind, key in (("ancestor", "ancestor"), ("self_ancestor", "self_ancestor"), ("see", "see")):
        rows = d.expect[key]
        x, y = _pairs(d, rows)
        got = hg.query(kind, x, y)
        assert got.tolist() == [bool(r[2]) for r in rows], kind


def test_query_kat_strongly_see_and_round_diff():
    from babble_amd import HashgraphError
    d, hg = _kat("kat_round")
    rows = d.expect["strongly_see"]
    x, y = _pairs(d, rows)
    assert hg.query("strongly_see", x, y).tolist() == [bool(r[2]) for r in rows]
    with pytest.raises(HashgraphError) as ei:  # no round before DivideRounds
        hg.query("round_diff", x[:1], y[:1])
    assert ei.value.kind == "State"
    hg.divide_rounds()
    rows = d.expect["round_diff"]
    x, y = _pairs(d, rows)
    assert hg.query("round_diff", x, y).tolist() == [r[2] for r in rows]
    with pytest.raises(HashgraphError) as ei:
        hg.query("see", [0], [len(d) + 3])
    assert ei.value.kind == "KeyNotFound"


@pytest.mark.parametrize("n,N,seed", [(5, 3000, 91), (32, 20000, 92), (100, 30000, 93), (300, 12000, 94)])
def test_query_random_pairs(n, N, seed):
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.divide_rounds()
    hg = Hashgraph(d.participant_ids, N)
    hg.insert_dag(d)
    hg.divide_rounds()
    rng = np.random.default_rng(seed)
    x = rng.integers(0, N, 3000)
    # y near x in insertion order, so that both answers occur
    y = np.clip(x - rng.integers(-200, 2000, 3000), 0, N - 1)
    y[:50] = x[:50]
    same = rng.integers(0, N, 200)
    x = np.concatenate([x, same])
    y = np.concatenate([y, np.array([np.nonzero(d.creator == d.creator[e])[0][0] for e in same])])
    want = {
        "ancestor": [o.see(int(a), int(b)) for a, b in zip(x, y)],
        "self_ancestor": [a == b or (d.creator[a] == d.creator[b] and d.index[a] >= d.index[b]) for a, b in zip(x, y)],
        "strongly_see": [o.strongly_see(int(a), int(b)) for a, b in zip(x, y)],
        "round_diff": [o.round(int(a)) - o.round(int(b)) for a, b in zip(x, y)],
    }
    want["see"] = want["ancestor"]
    for kind, w in want.items():
        got = hg.query(kind, x, y)
        assert got.tolist() == [int(v) if kind == "round_diff" else bool(v) for v in w], kind
    assert 0 < sum(want["strongly_see"]) < len(x) and 0 < sum(want["ancestor"]) < len(x)


@pytest.mark.parametrize("n,N,seed", [(16, 12_000, 95), (160, 12_000, 96)])
def test_query_between_passes(n, N, seed):
    """Go's ancestor / see / stronglySee read the Store and touch no pass
    state: a query right after InsertEvent computes the new
    events' coordinates on the device, then DivideRounds, a query, DecideFame,
    DecideRoundReceived and ProcessDecidedRounds run as in Go, each state
    equal to the oracle's, and the next DivideRounds still resumes from the
    previous call's device state.  (Inserting between DivideRounds and
    DecideRoundReceived is not exercised: Go's DecideRoundReceived then
    memoizes round(x) of the undivided events against the witnesses the Store
    holds at that moment, and Core never interleaves them -- DESIGN.md
    section 2.)"""
    from babble_amd import Hashgraph
    from test_gpu_parity import _compare
    from test_gpu_schedule import _wire_batches
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    batch = _wire_batches(d)
    rng = np.random.default_rng(seed)

    def query(lo, hi):
        x = rng.integers(lo, hi, 300)
        y = np.clip(x - rng.integers(0, 3000, 300), 0, N - 1)
        assert hg.query("strongly_see", x, y).tolist() == [o.strongly_see(int(a), int(b)) for a, b in zip(x, y)]
        assert hg.query("see", x, y).tolist() == [o.see(int(a), int(b)) for a, b in zip(x, y)]

    cuts = [0, N // 3, 2 * N // 3, N]
    for k in range(3):
        lo, hi = cuts[k], cuts[k + 1]
        o.insert_dag(*(a[lo:hi] for a in args))
        hg.insert_events(*batch(lo, hi))
        query(lo, hi)  # coordinates of the new events computed on demand
        for p in ("divide_rounds", "decide_fame", "decide_round_received", "process_decided_rounds"):
            getattr(o, p)()
            getattr(hg, p)()
            if p == "divide_rounds":
                query(lo, hi)
            _compare(o, hg, f"[0, {hi}) after {p}")
    assert hg.pipeline()[1] == 2  # both later DivideRounds resumed
