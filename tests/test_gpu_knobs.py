"""Every path-changing BH_* switch of the product library that no other
test sets, against the oracle (the switches that select a kernel variant
are parametrised where that variant is tested: test_gpu_parity.py,
test_gpu_shard.py, test_gpu_comm.py).

* BH_NO_GRAPH=1 -- the one-launch-per-iteration loop (BH_ROUND_PERSIST=0)
  launched directly instead of replayed from a captured hipGraph;
* BH_LAYOUT_SLACK -- the chain-major layout's spare rows per chain: small
  slack makes per-sync calls outgrow their regions and lay the chains out
  again (a full pass) every few calls, between incremental ones;
* BH_DIAG=1 with BH_SEG_DEBUG=1 and BH_TIMELINE -- the diagnostic build of
  the kernels (realtime stamps, counters) and the segment pipeline waiting
  for every segment's loop;
* BH_LOOP_TIMING=0 -- no HIP events around the loop (stage 7 reads 0);
* BH_ROUND_F32=0 -- k_round2p's search counting in int32 (sign bits of
  LA - FD) instead of packed f32 with the clamp modifier (the default);
* BH_SEG_RATIO -- the segment pipeline's growth ratio (segment k holds a
  ratio^k share of the events): equal segments (1.0) and steep ones (1.8)
  cut the DAG at other boundaries than the defaults (1.15 above n = 96).
"""
import os

import numpy as np
import pytest

from oracle_py import Oracle
from test_gpu_parity import _compare, _random_parity

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,N,seed,lag,K", [(64, 40_000, 0xD1, 21, 3), (160, 20_000, 0xD2, 2, 1)])
def test_no_graph_per_iteration(monkeypatch, n, N, seed, lag, K):
    monkeypatch.setenv("BH_ROUND_PERSIST", "0")
    monkeypatch.setenv("BH_NO_GRAPH", "1")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    hg = _random_parity(n, N, seed, lag)
    assert hg.loop_stats()[0] == 0  # no persistent launch


@pytest.mark.parametrize("slack,n,N,step", [("0", 24, 30_000, 3_000), ("16", 128, 40_000, 4_000), ("8", 170, 20_000, 2_500)])
def test_layout_slack_relayouts(monkeypatch, slack, n, N, step):
    """Per-sync calls with (almost) no spare rows: chains keep outgrowing
    their regions, so calls alternate between relayouts (full passes) and
    incremental resumes; the state equals the oracle's after every call."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    from test_gpu_schedule import _wire_batches
    monkeypatch.setenv("BH_LAYOUT_SLACK", slack)
    d = Dag(n, N, 0xD3 + n, lagging=2, sig_mode=0)
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
        _compare(o, hg, f"slack {slack} n={n} after [0, {hi})")
    calls = (N + step - 1) // step
    assert hg.pipeline()[1] < calls - 1  # calls after the first laid the chains out again


@pytest.mark.parametrize("n,N,seed,lag,K", [(128, 60_000, 0xD5, 0, 4), (160, 20_000, 0xD6, 2, 1), (9, 8_000, 0xD7, 3, 2)])
def test_diag_build(monkeypatch, tmp_path, n, N, seed, lag, K):
    tl = tmp_path / "timeline.bin"
    monkeypatch.setenv("BH_DIAG", "1")
    monkeypatch.setenv("BH_SEG_DEBUG", "1")
    monkeypatch.setenv("BH_TIMELINE", str(tl))
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    _random_parity(n, N, seed, lag)
    assert tl.exists() and os.path.getsize(tl) > 0


def test_loop_timing_off(monkeypatch):
    monkeypatch.setenv("BH_LOOP_TIMING", "0")
    monkeypatch.setenv("BH_SEGMENTS", "3")
    hg = _random_parity(96, 40_000, 0xD8, 3)
    assert hg.stage_ms()[7] == 0


@pytest.mark.parametrize("n,N,seed,lag,K", [(128, 60_000, 0xD9, 0, 3), (100, 40_000, 0xDA, 4, 1), (7, 6_000, 0xDB, 2, 2)])
def test_round_int32_search(monkeypatch, n, N, seed, lag, K):
    monkeypatch.setenv("BH_ROUND_F32", "0")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    loops, fallbacks = _random_parity(n, N, seed, lag).loop_stats()
    assert loops >= 1 and fallbacks == 0


@pytest.mark.parametrize("ratio,n,N,K", [("1.0", 128, 80_000, 8), ("1.8", 64, 60_000, 6), ("1.32", 32, 50_000, 12)])
def test_segment_ratio(monkeypatch, ratio, n, N, K):
    monkeypatch.setenv("BH_SEG_RATIO", ratio)
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    hg = _random_parity(n, N, 0xDF + K, 2)
    assert hg.pipeline()[0] == K
