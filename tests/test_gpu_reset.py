"""Reset / FastSync roots through the engine (SURVEY 8(f) row 4;
Hashgraph.Reset hashgraph.go:1324-1369, the Root cases of
docs/fastsync.rst:140-175): a fresh handle is reset from block b of a
hashgraph that ran consensus (its Frame's roots, tests/reset.py), the frame's
events and then the rest of the DAG arrive as wire events, and every output
-- rounds, witnesses, Lamport timestamps, fame, round received, consensus
order, blocks, PendingRounds, UndeterminedEvents, LastConsensusRound,
rejected inserts -- must equal the oracle's Reset restatement (pinned by the
reference's Reset tests in tests/test_oracle_reset.py) on the same inputs.
Covers the reference's Reset DAGs (kat_consensus block 1, the funky and
sparse hashgraphs' blocks 0-2), generated gossip DAGs at n = 4 ... 128
(chain dataflow k_flow32 + k_round2) and n = 160 (k_floww + k_round_wide),
lagging peers (diff events Go rejects), and RunConsensus after every gossip
batch."""
import numpy as np
import pytest

from babble_amd.dag import Dag
from kat import KatDag
from oracle_py import Oracle
from reset import DagArrays, ResetInputs, oracle_insert
from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu


def _oracle_run(d):
    o = Oracle(d.n, d.participant_ids, capacity=len(d.creator) + 64)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    o.run_consensus()
    return o


def _engine_reset(rs, d, cap):
    from babble_amd import Hashgraph
    pid = np.asarray(d.participant_ids, np.int64)
    hg = Hashgraph(pid, cap)
    hg.reset(rs.round_received, rs.block_index, rs.next_round, rs.sp_index, rs.sp_lt, rs.sp_round,
             rs.oth_root, rs.oth_key, pid[np.asarray(rs.oth_creator, np.int64)] if rs.oth_creator else [],
             rs.oth_index, rs.oth_lt, rs.oth_round, rs.oth_hash)
    return hg


def _wire(hg, d, ids):
    """the original events `ids` as wire events (their WireBody never changes)"""
    ids = np.asarray(ids, np.int64)
    if ids.size == 0:
        return np.zeros(0, np.int32)
    pid = np.asarray(d.participant_ids, np.int64)
    cr, ix, sp, op = d.creator[ids], d.index[ids], d.sp[ids], d.op[ids]
    spi = ix - 1  # WireBody.SelfParentIndex (the Root SelfParent.Index for a chain after the Reset)
    opc = np.where(op >= 0, pid[d.creator[np.maximum(op, 0)]], -1)
    opi = np.where(op >= 0, d.index[np.maximum(op, 0)], -1)
    return hg.insert_events(pid[cr], ix, spi, opc, opi, d.hashes[ids], d.sig_r[ids], d.ntx[ids],
                            raise_on_error=False)


def _coords_sample(o2, hg, k=12):
    N = o2.num_events()
    for e in np.unique(np.linspace(0, N - 1, min(N, k)).astype(int)):
        la, fd = o2.coordinates(int(e))
        gla, gfd = hg.coordinates(int(e))
        assert np.array_equal(la, gla) and np.array_equal(fd, gfd), e


def _run_pair(d, block, batches=1, cap_extra=64, tweak=None, expect_inc=True):
    o = _oracle_run(d)
    rs = ResetInputs(o, d, block)
    if tweak:
        tweak(rs)
    o2 = Oracle(d.n, d.participant_ids, capacity=len(d.creator) + cap_extra)
    o2.reset(rs)
    hg = _engine_reset(rs, d, len(d.creator) + cap_extra)
    st_o = oracle_insert(o2, rs, rs.frame)
    st_g = _wire(hg, d, rs.frame)
    assert np.array_equal(st_o != 0, st_g != 0), "frame inserts"
    o2.run_consensus()
    hg.run_consensus()
    _compare(o2, hg, f"block {block} frame")
    diff = rs.diff
    for bi in range(batches):
        part = diff[len(diff) * bi // batches: len(diff) * (bi + 1) // batches]
        st_o = oracle_insert(o2, rs, part)
        st_g = _wire(hg, d, part)
        assert np.array_equal(st_o != 0, st_g != 0), f"diff inserts, batch {bi}"
        o2.run_consensus()
        hg.run_consensus()
        _compare(o2, hg, f"block {block} batch {bi}")
    st = hg.stats()
    assert st.blocks == rs.block_index + 1 + len(o2.blocks()["round_received"])
    _coords_sample(o2, hg)
    if expect_inc and len(diff) >= batches and batches > 1 and len(d.participant_ids) <= 512:
        # the calls after the first resume from the device state (the fiat
        # region again, the round loop from the last round every extended
        # chain fixed); with lagging peers a later batch can bring events
        # whose other-parent only Root.Others knows, and such a call
        # recomputes the whole DAG (k_reset_coords)
        assert hg.pipeline()[1] >= 1
    return o2, hg, rs


def test_reset_from_frame_kat():
    """TestResetFromFrame (hashgraph_test.go:1711-1907) through the engine"""
    d = KatDag("kat_consensus")
    o2, hg, rs = _run_pair(d, 1)
    assert hg.stats().last_consensus_round == rs.round_received


@pytest.mark.parametrize("name", ["kat_funky_full", "kat_sparse"])
@pytest.mark.parametrize("block", [0, 1, 2])
def test_reset_kat(name, block):
    """TestFunkyHashgraphReset / TestSparseHashgraphReset (:2344-2417, :2656-2738)"""
    _run_pair(KatDag(name), block)


@pytest.mark.parametrize("n,N,seed,lag,block,batches", [
    (4, 3000, 0xBA0, 0, 3, 1), (7, 4000, 0xBA1, 0, 5, 4), (16, 8000, 0xBA2, 0, 4, 3),
    (16, 8000, 0xBA3, 5, 2, 1), (32, 8000, 0xBA4, 0, 2, 5), (32, 8000, 0xBA4, 0, 7, 2),
    (64, 30000, 0xBA5, 20, 3, 2), (128, 20000, 0xBA6, 0, 2, 3), (128, 20000, 0xBA6, 0, 3, 2),
    (160, 30000, 0xBA7, 0, 3, 2)])
def test_reset_generated(n, N, seed, lag, block, batches):
    """(some resets progress for many rounds, some stay at the roots' round for
    good -- witnesses received before the frame are not re-inserted -- Go's
    result either way; both run the event-by-event pass over most events)"""
    d = DagArrays(Dag(n, N, seed, lagging=lag))
    _run_pair(d, block, batches, expect_inc=lag == 0)


@pytest.mark.parametrize("n,N,seed,lag,block,batches", [(16, 8000, 0xBA3, 5, 2, 1), (128, 20000, 0xBA6, 0, 3, 2),
                                                        (160, 30000, 0xBA7, 0, 3, 2)])
def test_reset_serial_fiat(monkeypatch, n, N, seed, lag, block, batches):
    """The event-by-event fiat pass (BH_FIAT=serial, k_fiat) against the
    oracle too: the default is the level-synchronous k_fiat_ls"""
    monkeypatch.setenv("BH_FIAT", "serial")
    _run_pair(DagArrays(Dag(n, N, seed, lagging=lag)), block, batches, expect_inc=lag == 0)


@pytest.mark.parametrize("block,p", [(6, 0), (10, 2), (20, 1)])
def test_reset_missing_rounds(block, p):
    """Roots whose NextRounds leave rounds below the block's empty: GetRound
    fails there and events below LastConsensusRound leave UndeterminedEvents
    without a round received (hashgraph.go:968-979)"""
    def tweak(rs):
        L = rs.round_received
        rs.next_round = [max(0, x - 3) if i != p else L - 1 for i, x in enumerate(rs.next_round)]
        rs.sp_round = [min(a, b) for a, b in zip(rs.sp_round, rs.next_round)]
    o2, hg, rs = _run_pair(DagArrays(Dag(8, 4000, 0xBA8)), block, 2, tweak=tweak)
    res = o2.results()
    und = set(o2.undetermined().tolist())
    dropped = [e for e in range(o2.num_events()) if res["round_received"][e] == -2 ** 31 and e not in und]
    assert dropped  # the case is exercised


def test_reset_round_info_and_errors():
    """RoundInfo of the rounds a Reset hashgraph has (and lacks), and the
    rejections bh_reset makes"""
    from babble_amd import Hashgraph
    from babble_amd.hashgraph import HashgraphError
    d = DagArrays(Dag(8, 4000, 0xBA8))
    o2, hg, rs = _run_pair(d, 4)
    res = o2.results()
    for r in range(0, hg.stats().last_round + 1):
        present = bool((res["round"] == r).any())
        if not present:
            with pytest.raises(HashgraphError):
                hg.round_info(r)
            continue
        info = hg.round_info(r)
        want = set(np.nonzero((res["round"] == r) & (res["witness"] == 1))[0].tolist())
        assert set(info["witnesses"].tolist()) == want, r
        assert info["n_events"] == int((res["round"] == r).sum()), r
        assert info["queued"] == (r >= rs.round_received), r
    # a handle that already has events cannot be reset; a root above the block's round is refused
    pid = np.asarray(d.participant_ids, np.int64)
    h2 = Hashgraph(pid, 100)
    with pytest.raises(HashgraphError):
        h2.reset(1, 0, [5] * 8, [-1] * 8, [-1] * 8, [-1] * 8)


@pytest.mark.parametrize("n,N,seed,silent,join", [(5, 60_000, 7, 2, 45_000), (16, 60_000, 8, 9, 50_000)])
def test_reset_high_round_silent_peer(n, N, seed, silent, join):
    """FastSync of a long-running network: Reset from the last
    block before a late-joining peer's first consensus event -- its Root is
    a base Root (SelfParent Round -1, NextRound 0) while the others sit at a
    round in the hundreds or thousands.  The engine's round tables and
    ballots then cover only the rounds the Reset hashgraph can reach (no
    per-round storage from round 0 up), and every output matches the
    oracle's Reset restatement, the silent peer's joining events included."""
    from reset import SilentDag
    d = SilentDag(n, N, seed, silent, join)
    o = _oracle_run(d)
    res = o.results()
    first = int(np.nonzero(d.creator == silent)[0][0])
    rr_first = int(res["round_received"][first])
    b = o.blocks()
    blk = max(i for i, r in enumerate(b["round_received"].tolist()) if r < rr_first)
    rs = ResetInputs(o, d, blk)
    assert rs.sp_index[silent] == -1 and rs.next_round[silent] == 0 and rs.round_received > 100
    # (batches of ~600 events per chain: each fits the chains' layout slack,
    # so every call after the first diff batch resumes incrementally)
    o2, hg, rs = _run_pair(d, blk, batches=6)
    assert (o2.results()["round"][hg.stats().n_events - 1]) > rs.round_received


@pytest.mark.parametrize("frames", [False, True])
def test_reset_allocation_failure(monkeypatch, frames):
    """A bh_reset whose k-th device allocation fails (BH_TEST_FAIL_ALLOC=k,
    for every k up to the call's last allocation) returns the error and
    leaves the handle a fresh one: the same handle then takes the Reset and
    the events and matches the oracle.  With the block projection on, its
    tables and JSON buffers are among the allocations (all made before the
    call commits)."""
    from babble_amd import Hashgraph
    from babble_amd.hashgraph import HashgraphError
    d = DagArrays(Dag(8, 4000, 0xBA8))
    o = _oracle_run(d)
    rs = ResetInputs(o, d, 4)
    pid = np.asarray(d.participant_ids, np.int64)
    args = (rs.round_received, rs.block_index, rs.next_round, rs.sp_index, rs.sp_lt, rs.sp_round,
            rs.oth_root, rs.oth_key, pid[np.asarray(rs.oth_creator, np.int64)] if rs.oth_creator else [],
            rs.oth_index, rs.oth_lt, rs.oth_round, rs.oth_hash)
    kw = dict(self_parent_hash=rs.sp_hash) if frames else {}
    failures = 0
    for k in range(1, 64):
        hg = Hashgraph(pid, len(d.creator) + 64, frames=frames)
        monkeypatch.setenv("BH_TEST_FAIL_ALLOC", str(k))
        try:
            hg.reset(*args, **kw)
            ok = True
        except HashgraphError as e:
            assert e.kind == "Device", e
            ok = False
        monkeypatch.delenv("BH_TEST_FAIL_ALLOC")
        if ok:
            break
        failures += 1
        hg.reset(*args, **kw)  # the failed call changed nothing: the handle takes the Reset now
        o2 = Oracle(d.n, d.participant_ids, capacity=len(d.creator) + 64)
        rs2 = ResetInputs(o, d, 4)
        o2.reset(rs2)
        assert np.array_equal(oracle_insert(o2, rs2, rs2.frame) != 0, _wire(hg, d, rs2.frame) != 0)
        assert np.array_equal(oracle_insert(o2, rs2, rs2.diff) != 0, _wire(hg, d, rs2.diff) != 0)
        o2.run_consensus()
        hg.run_consensus()
        _compare(o2, hg, f"after an injected failure at allocation {k}")
        hg.close()
    assert failures >= (30 if frames else 10)  # every allocation of the call was covered


def _event_bytes(g):
    """EventBody.Marshal() bytes and Signature strings of every event of a
    generated Dag or a KatDag"""
    from frames import kat_event_bytes
    if isinstance(g, KatDag):
        return [list(x) for x in zip(*(kat_event_bytes(g, e) for e in range(len(g))))]
    return [g.body_json(e) for e in range(len(g.creator))], [g.sig_string(e) for e in range(len(g.creator))]


@pytest.mark.parametrize("src,block,batches", [
    ("kat_funky_full", 1, 1), ("kat_sparse", 0, 2), ((4, 3000, 0xBA0), 3, 4), ((7, 4000, 0xBA1), 5, 3),
    ((16, 8000, 0xBA2), 3, 3), ((32, 8000, 0xBA4), 2, 5), ((128, 20000, 0xBA6), 2, 3),
    ((160, 30000, 0xBA7), 3, 2)])
def test_reset_block_projection(src, block, batches):
    """FastSync, then gossip, on a handle with frames (node.go fastForward ->
    Core.FastForward -> Hashgraph.Reset, then RunConsensus per sync): after
    every call, each new block's FrameHash and block hash, the Roots of its
    frame -- the Reset roots (their SelfParent / Others as installed) for the
    peers with no consensus event since the Reset -- and the Frame / Block
    JSON byte for byte equal the oracle's Reset restatement, and Block.Index
    continues from the Reset block's.  At n = 4 and 7 (TestFastSync's
    setting, node_test.go:583-658 with checkGossip :741-771) every block
    body from Index FirstConsensusRound on also equals the original
    network's (tests/test_oracle_reset.py pins that on the oracle)."""
    from babble_amd import Hashgraph
    from frames import sha
    g = KatDag(src) if isinstance(src, str) else Dag(*src)
    d = DagArrays(g)
    bodies, sigs = _event_bytes(g)
    cap = len(d.creator) + 64
    o = Oracle(d.n, d.participant_ids, capacity=cap)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    for e in range(len(d.creator)):
        o.set_event_bytes(e, bodies[e], sigs[e])
    o.run_consensus()
    rs = ResetInputs(o, d, block)
    o2 = Oracle(d.n, d.participant_ids, capacity=cap)
    o2.reset(rs)
    pid = np.asarray(d.participant_ids, np.int64)
    hg = Hashgraph(pid, cap, frames=True)
    hg.reset(rs.round_received, rs.block_index, rs.next_round, rs.sp_index, rs.sp_lt, rs.sp_round,
             rs.oth_root, rs.oth_key, pid[np.asarray(rs.oth_creator, np.int64)] if rs.oth_creator else [],
             rs.oth_index, rs.oth_lt, rs.oth_round, rs.oth_hash, self_parent_hash=rs.sp_hash)
    assert hg.stats().first_block == rs.block_index + 1
    seen = 0
    diff = rs.diff
    calls = [rs.frame] + [diff[len(diff) * b // batches: len(diff) * (b + 1) // batches] for b in range(batches)]
    for c, ids in enumerate(calls):
        n0 = o2.num_events()
        st_o = oracle_insert(o2, rs, ids)
        st_g = _wire(hg, d, ids)
        assert np.array_equal(st_o != 0, st_g != 0), f"inserts of call {c}"
        inv = {v: k for k, v in rs.new_id.items()}
        new = range(n0, o2.num_events())
        for e in new:
            o2.set_event_bytes(e, bodies[inv[e]], sigs[inv[e]])
        hg.set_event_bytes(n0, [bodies[inv[e]] for e in new], [sigs[inv[e]] for e in new])
        o2.run_consensus()
        hg.run_consensus()
        _compare(o2, hg, f"call {c}")
        ob = o2.blocks()
        nb = len(ob["round_received"])
        fh, bh, ok = hg.block_hashes()
        assert len(fh) == nb and ok.all(), f"call {c}"
        for b in range(seen, nb):
            rr = int(ob["round_received"][b])
            assert fh[b].tobytes() == o2.block_frame_hash(b), f"FrameHash of block {b} (frame {rr}), call {c}"
            bj = o2.block_json(b)
            assert bh[b].tobytes() == sha(bj), f"block hash {b}, call {c}"
            assert hg.frame_roots(rr) == o2.frame_roots(rr), f"roots of frame {rr}"
            assert hg.frame_json(rr) == o2.frame_json(rr), f"frame {rr} JSON"
            assert hg.block_json(b) == bj, f"block {b} JSON"
            if d.n <= 7:
                idx = rs.block_index + 1 + b
                if rs.round_received <= idx < len(o.blocks()["round_received"]):
                    assert hg.block_json(b, body_only=True) == o.block_json(idx, body_only=True), idx
        seen = nb
    assert seen > 0
    if batches > 1 and len(diff) >= batches:
        assert hg.pipeline()[1] >= 1
    hg.close()
