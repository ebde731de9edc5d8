"""Seeded schedule fuzz: random hashgraph shapes and random call schedules
through the engine, state compared with the oracle after every pass.

Each case draws, from its own seed:
  * n (3 ... 200: k_round2 at one, two and four pieces per lane, and the
    wide path past 128), N, lagging peers and how far they lag;
  * a schedule of gossip batches of varying size (one event up to a few
    thousand), and for each batch what Core would do next
    (core.go:337-369): RunConsensus, the four passes one at a time, or
    nothing yet (the next batch arrives first).
The oracle replays the same schedule literally (hashgraph.go's state
machine, `queued` and the sticky PendingRounds flags included), so every
comparison is bit-exact: per-event round, witness, Lamport timestamp, fame,
round received, consensus position, the order, blocks, PendingRounds,
UndeterminedEvents and the counters (test_gpu_parity._compare)."""
import numpy as np
import pytest

from oracle_py import Oracle
from test_gpu_parity import _compare
from test_gpu_schedule import _wire_batches

pytestmark = pytest.mark.gpu

PASSES = ("divide_rounds", "decide_fame", "decide_round_received", "process_decided_rounds")


def _case(seed):
    rng = np.random.default_rng(0xF022 + seed)
    n = int(rng.choice([3, 4, 5, 7, 9, 12, 16, 23, 32, 33, 47, 64, 65, 96, 128, 129, 160, 200]))
    N = int(rng.integers(max(1500, 60 * n), max(12000, min(36000, 180 * n))))  # enough rounds to decide at every n
    lagging = int(rng.integers(0, max(1, n // 3) + 1)) if rng.random() < 0.5 else 0
    lag_div = int(rng.choice([20, 60, 300]))
    return rng, n, N, lagging, lag_div


@pytest.mark.timeout(300)
@pytest.mark.parametrize("seed", range(48))
def test_schedule_fuzz(seed):
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    rng, n, N, lagging, lag_div = _case(seed)
    d = Dag(n, N, 0xF000 + seed, lagging=lagging, lag_div=lag_div, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    batch = _wire_batches(d)
    lo, calls = 0, 0
    while lo < N:
        hi = min(N, lo + int(rng.choice([1, 7, 50, 300, 1000, 2500])))
        o.insert_dag(*(a[lo:hi] for a in args))
        assert not np.asarray(hg.insert_events(*batch(lo, hi))).any()
        what = "run" if hi == N else str(rng.choice(["run", "run", "passes", "wait"]))
        where = f"n={n} N={N} lag={lagging}/{lag_div}: events [0, {hi}), {what}"
        if what == "run":
            o.run_consensus()
            hg.run_consensus()
            _compare(o, hg, where)
        elif what == "passes":
            for name in PASSES:
                getattr(o, name)()
                getattr(hg, name)()
                _compare(o, hg, f"{where}, after {name}")
        lo = hi
        calls += 1
    ordered = hg.stats().consensus_events
    assert ordered == len(o.consensus_order())
    print(f"fuzz {seed}: n={n} N={N} lag={lagging}/{lag_div} calls={calls} ordered={ordered} "
          f"rounds={hg.last_round() + 1} resumed={hg.pipeline()[1]}")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("seed", range(16))
def test_reset_schedule_fuzz(seed):
    """FastSync then gossip (core.go:240-283, then node.go:583-603) on random
    shapes: a fresh hashgraph Reset from a random block's Frame, the frame's
    events, then the diff in random batches as wire events, each followed by
    RunConsensus, the passes one by one, or nothing; every call compared with
    the oracle's Reset restatement (statuses of rejected diff events too)."""
    from babble_amd.dag import Dag
    from reset import DagArrays, ResetInputs, oracle_insert
    from test_gpu_reset import _engine_reset, _oracle_run, _wire
    rng = np.random.default_rng(0x2E5E7 + seed)
    n = int(rng.choice([4, 5, 9, 16, 31, 32, 48, 64, 100, 128, 160]))
    N = int(rng.integers(max(2500, 80 * n), max(9000, min(30000, 200 * n))))
    lag = int(rng.integers(0, max(1, n // 4) + 1)) if rng.random() < 0.4 else 0
    d = DagArrays(Dag(n, N, 0x2E00 + seed, lagging=lag))
    o = _oracle_run(d)
    nb = len(o.blocks()["round_received"])
    assert nb >= 2
    block = int(rng.integers(0, min(nb - 1, 12)))
    rs = ResetInputs(o, d, block)
    o2 = Oracle(d.n, d.participant_ids, capacity=len(d.creator) + 64)
    o2.reset(rs)
    hg = _engine_reset(rs, d, len(d.creator) + 64)
    st_o, st_g = oracle_insert(o2, rs, rs.frame), _wire(hg, d, rs.frame)
    assert np.array_equal(st_o != 0, st_g != 0), "frame inserts"
    o2.run_consensus()
    hg.run_consensus()
    _compare(o2, hg, f"n={n} block {block}: frame")
    diff, lo = rs.diff, 0
    while lo < len(diff):
        hi = min(len(diff), lo + int(rng.choice([1, 20, 200, 1000, 4000])))
        part = diff[lo:hi]
        st_o, st_g = oracle_insert(o2, rs, part), _wire(hg, d, part)
        assert np.array_equal(st_o != 0, st_g != 0), f"diff inserts [{lo}, {hi})"
        what = "run" if hi == len(diff) else str(rng.choice(["run", "run", "passes", "wait"]))
        where = f"n={n} N={N} lag={lag} block {block}: diff [0, {hi}) {what}"
        if what == "run":
            o2.run_consensus()
            hg.run_consensus()
            _compare(o2, hg, where)
        elif what == "passes":
            for name in PASSES:
                getattr(o2, name)()
                getattr(hg, name)()
                _compare(o2, hg, f"{where}, after {name}")
        lo = hi
    print(f"reset fuzz {seed}: n={n} N={N} lag={lag} block={block} diff={len(diff)} "
          f"ordered={hg.stats().consensus_events} resumed={hg.pipeline()[1]}")
