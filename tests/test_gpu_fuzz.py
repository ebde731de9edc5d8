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
