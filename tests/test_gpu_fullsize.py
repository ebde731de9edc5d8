"""Whole-DAG parity at BASELINE's sizes, through the segment pipeline.

Every per-event output (round, witness, Lamport timestamp, fame, round
received, consensus position), the consensus order, the blocks,
PendingRounds, UndeterminedEvents and the counters of the engine's run are
compared with the oracle's run on the same events -- not a prefix of a
longer run: the pipelined coordinates of segment s + 1, the round loop's
resume at the last round segment s fixed and the incremental layout are all
on the path these checks cover:

  * C2 (32 peers, 1M events: 12 segments) and C5 (64 peers with 21 lagging,
    2M events: 12 segments), whole;
  * C3's DAG (128 peers, the bench's 10M-event DAG) on its first 2.5M
    events with 5 segments of 500k events -- every chain resumes 4 times at
    real chain lengths (the oracle needs about 25 s for them);
  * C4's DAG (512 peers: k_floww2 + the 16-bit k_round_wide) on its first
    100k events with 4 segments;
  * C2's block projection (FrameHash and block hash of every block, the roots
    of every frame) at 1M events against the oracle's.
"""
import numpy as np
import pytest

from oracle_py import Oracle
from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu


def _whole(cfg, N=None, segments=None, monkeypatch=None, ordered=0.9):
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    if segments:
        monkeypatch.setenv("BH_SEGMENTS", str(segments))
    d = Dag.config(cfg, N=N, sig_mode=0)
    o = Oracle(d.n, d.participant_ids, capacity=d.N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    hg = Hashgraph(d.participant_ids, d.N)
    assert not hg.insert_dag(d).any()
    hg.run_consensus()
    _compare(o, hg, f"cfg{cfg} N={d.N}")
    st = hg.stats()
    assert st.consensus_events > ordered * d.N
    return hg


@pytest.mark.timeout(600)
def test_c2_whole_dag():
    hg = _whole(2)
    assert hg.pipeline()[0] == 12  # the default for >= 1M events at n <= 96


@pytest.mark.timeout(600)
def test_c5_whole_dag():
    hg = _whole(5)
    assert hg.pipeline()[0] == 12  # the default from 1.5M events at n <= 96


@pytest.mark.timeout(900)
def test_c3_multisegment(monkeypatch):
    hg = _whole(3, N=2_500_000, segments=5, monkeypatch=monkeypatch)
    assert hg.pipeline()[0] == 5
    assert hg.profile_kernel() == "k_flow32x2"


@pytest.mark.timeout(600)
def test_c4_wide_segments(monkeypatch):
    hg = _whole(4, N=100_000, segments=4, monkeypatch=monkeypatch, ordered=0.75)
    assert hg.pipeline()[0] == 4
    assert hg.profile_kernel() == "k_floww2"


@pytest.mark.timeout(900)
def test_c2_block_projection():
    """NewBlockFromFrame at C2's size (BASELINE: "full virtual voting + block
    projection"): every block's FrameHash and block hash, every frame's
    roots, and the Frame / Block JSON of every 97th block, byte for byte."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    from frames import sha
    d = Dag.config(2, sig_mode=0)
    N = d.N
    bodies, bo, sigs, so = d.event_bytes()
    o = Oracle(d.n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    braw, sraw = bodies.tobytes(), sigs.tobytes()
    for e in range(N):
        o.set_event_bytes(e, braw[bo[e]:bo[e + 1]], sraw[so[e]:so[e + 1]])
    o.run_consensus()
    hg = Hashgraph(d.participant_ids, N, frames=True)
    assert not np.asarray(hg.insert_dag(d)).any()
    hg._check(hg._L.bh_set_event_bytes(hg._h, 0, N, bodies.ctypes.data, bo.ctypes.data, sigs.ctypes.data,
                                       so.ctypes.data))
    hg.run_consensus()
    _compare(o, hg, "cfg2 frames")
    ob = o.blocks()
    fh, bh, ok = hg.block_hashes()
    assert ok.all() and len(ob["round_received"]) > 1000
    for b, rr in enumerate(ob["round_received"].tolist()):
        assert fh[b].tobytes() == o.block_frame_hash(b), f"FrameHash of block {b} (frame {rr})"
        bj = o.block_json(b)
        assert bh[b].tobytes() == sha(bj), f"block hash {b}"
        assert hg.frame_roots(rr) == o.frame_roots(rr), f"roots of frame {rr}"
        if b % 97 == 0:
            assert hg.frame_json(rr) == o.frame_json(rr), f"frame {rr} JSON"
            assert hg.block_json(b) == bj, f"block {b} JSON"
    # the bench's timed state: bh_reset_consensus + RunConsensus over the
    # resident DAG and event bytes, twice; every hash and per-event output again
    for run in (1, 2):
        hg.reset_consensus()
        hg.run_consensus()
        _compare(o, hg, f"cfg2 frames, rerun {run}")
        fh2, bh2, ok2 = hg.block_hashes()
        assert ok2.all() and (fh2 == fh).all() and (bh2 == bh).all(), f"rerun {run}: block hashes"
        for b in range(0, len(ob["round_received"]), 389):
            rr = int(ob["round_received"][b])
            assert hg.frame_roots(rr) == o.frame_roots(rr), f"rerun {run}: roots of frame {rr}"
