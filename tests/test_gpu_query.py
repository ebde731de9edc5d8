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
    state: a query between InsertEvent and the next pass computes the new
    events' coordinates on the device, and DecideFame / DecideRoundReceived /
    ProcessDecidedRounds then continue from where DivideRounds left the state
    -- as in Go -- and the next DivideRounds still resumes incrementally."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    from test_gpu_parity import _compare
    from test_gpu_schedule import _wire_batches
    d = Dag(n, N, seed, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    batch = _wire_batches(d)
    h1, h2 = N // 3, 2 * N // 3
    o.insert_dag(*(a[:h1] for a in args))
    hg.insert_events(*batch(0, h1))
    o.run_consensus()
    hg.run_consensus()
    o.insert_dag(*(a[h1:h2] for a in args))
    hg.insert_events(*batch(h1, h2))
    o.divide_rounds()
    hg.divide_rounds()
    o.insert_dag(*(a[h2:] for a in args))
    hg.insert_events(*batch(h2, N))
    rng = np.random.default_rng(seed)
    x = rng.integers(h2, N, 400)
    y = np.clip(x - rng.integers(0, 3000, 400), 0, N - 1)
    got = hg.query("strongly_see", x, y)
    assert got.tolist() == [o.strongly_see(int(a), int(b)) for a, b in zip(x, y)]
    assert hg.query("see", x, y).tolist() == [o.see(int(a), int(b)) for a, b in zip(x, y)]
    for p in ("decide_fame", "decide_round_received", "process_decided_rounds"):
        getattr(o, p)()
        getattr(hg, p)()
        _compare(o, hg, f"after the query, {p}")
    inc = hg.pipeline()[1]
    o.run_consensus()
    hg.run_consensus()
    _compare(o, hg, "next RunConsensus")
    assert hg.pipeline()[1] == inc + 1
