"""Whole-DAG parity at the bench's own sizes, and the wide path's long chains.

* C3 (128 peers, 10M events: the DAG bench.py times) and C4 (512 peers, 20M
  events), every event: the engine's run against the digest of the oracle's
  whole-DAG run of the same seeded DAG (tests/golden/whole_c*.json, written
  by tests/golden/make_whole_digests.py -- minutes of oracle for C3, about an
  hour for C4, so it is done once and committed).  Every per-event output
  (round, witness, Lamport timestamp, fame, round received, consensus
  position) is compared in chunks of 1M events, plus the consensus order,
  the blocks, PendingRounds, UndeterminedEvents and the counters.  The same
  run is also held to the size-independent invariants.
* The wide path's 16-bit rows carry LA + 1 / FD + 1 up to P16_MAXLEN
  (engine.h); chains of the C4 DAG reach 39k events.  Two lag-heavy n = 160
  DAGs put chains past 32,767 (54k: the 16-bit rows' upper half on
  k_floww2 + the 16-bit k_round_wide) and past 65,472 (69.5k: the switch to
  the chunked sweep and the 32-bit rows), against the oracle run live.
* The per-sync schedule at C4's width (n = 512), state compared after every
  one of 100 RunConsensus calls, on a seed where the A.12 trap occurs
  (hashgraph.go:809-815, 984-986).
"""
import json
import os

import numpy as np
import pytest

from digest import diff, engine_digest
from oracle_py import Oracle
from test_gpu_parity import _compare, invariants

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _whole_digest(name, monkeypatch=None, segments=None, reruns=2):
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    with open(os.path.join(GOLDEN, f"whole_{name}.json")) as f:
        ref = json.load(f)
    sp = ref["spec"]
    if segments:
        monkeypatch.setenv("BH_SEGMENTS", str(segments))
    if sp["cfg"]:
        d = Dag.config(sp["cfg"], N=sp["N"], sig_mode=0)
    else:
        d = Dag(sp["n"], sp["N"], sp["seed"], lagging=sp["lagging"], lag_div=sp["lag_div"], sig_mode=0)
    assert int(np.bincount(d.creator, minlength=d.n).max()) == sp["max_chain"], "generator drift"
    hg = Hashgraph(d.participant_ids, d.N)
    assert not hg.insert_dag(d).any()
    want = {k: v for k, v in ref.items() if k not in ("spec", "oracle")}
    # the first run on a fresh handle, then the state bench.py times: each of
    # its steps is bh_reset_consensus + RunConsensus over the resident DAG
    # (BenchmarkConsensus, hashgraph_test.go:1522-1534, reruns the passes on
    # one inserted DAG), where every device table but `blocked` carries over
    # from the previous run
    for run in range(1 + reruns):
        if run:
            hg.reset_consensus()
        hg.run_consensus()
        bad = diff(want, engine_digest(hg))
        assert not bad, f"{name} run {run}: engine differs from the oracle's whole-DAG run at {bad[:12]}"
    return d, hg


@pytest.mark.timeout(900)
def test_c3_whole_dag():
    """The bench's headline DAG, all 10M events, through the default pipeline
    (16 segments from 4M events, the persistent loop), on a fresh handle and
    on two reruns after bh_reset_consensus (the bench's timed step)."""
    d, hg = _whole_digest("c3")
    assert hg.pipeline()[0] == 16 and hg.profile_kernel() == "k_flow32x2"
    assert hg.loop_stats() == (16 * 3, 0)  # one persistent loop per segment and run, no fallback
    invariants(d, hg)


@pytest.mark.timeout(900)
def test_c4_whole_dag():
    """C4, all 20M events (512 peers: k_floww2 and the 16-bit k_round_wide),
    fresh and on two reruns after bh_reset_consensus."""
    if not os.path.exists(os.path.join(GOLDEN, "whole_c4.json")):
        pytest.fail("tests/golden/whole_c4.json missing: run tests/golden/make_whole_digests.py --cfg 4 --coord16")
    d, hg = _whole_digest("c4")
    assert hg.profile_kernel() == "k_floww2"
    invariants(d, hg, ordered=0.9)


def _live(n, N, seed, lag, div, segments=None, monkeypatch=None):
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    if segments:
        monkeypatch.setenv("BH_SEGMENTS", str(segments))
    d = Dag(n, N, seed, lagging=lag, lag_div=div, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    hg = Hashgraph(d.participant_ids, N)
    assert not hg.insert_dag(d).any()
    hg.run_consensus()
    _compare(o, hg, f"n={n} N={N} lag={lag}")
    return d, hg


@pytest.mark.timeout(600)
@pytest.mark.parametrize("N,segments,kernel,lo,hi", [
    (700_000, None, "k_floww2", 32_768, 65_000),      # 16-bit rows' upper half
    (700_000, 4, "k_floww2", 32_768, 65_000),         # ... resumed across segments
    (900_000, None, "k_la_sweep", 65_473, 1 << 20),  # past P16_MAXLEN / k_floww2's chain limit
])
def test_wide_long_chains(N, segments, kernel, lo, hi, monkeypatch):
    d, hg = _live(160, N, 0xB160, 150, 50, segments, monkeypatch)
    longest = int(np.bincount(d.creator, minlength=d.n).max())
    assert lo <= longest <= hi, longest
    assert hg.profile_kernel() == kernel
    if segments:
        assert hg.pipeline()[0] == segments


@pytest.mark.timeout(900)
def test_per_sync_trap_512():
    """C4's width on the live schedule: 100 calls of 1,000 events, state
    compared after every call; seeded so a lagging witness is trapped."""
    from test_gpu_schedule import _schedule
    n, N, step = 512, 100_000, 1_000
    d, o, hg = _schedule(n, N, 5131, 150, 80, step)
    res = o.results()
    lcr = o.last_consensus_round()
    trapped = np.nonzero((res["witness"] == 1) & (res["fame"] == 0) & (res["round"] < lcr))[0]
    assert len(trapped) >= 1, "the seed no longer produces a trapped witness"
    assert hg.pipeline()[1] >= N // step - 2
