"""Block projection on the device: GetFrame roots,
Frame.Marshal / FrameHash and Block.Marshal / block hash, bit-exact against
the oracle (itself pinned by TestGetFrame / TestSparseHashgraphFrames and an
independent Python json restatement, tests/test_oracle_frames.py)."""
import numpy as np
import pytest

from frames import base36, kat_event_bytes, matches_fixture, roots_by_name, sha
from kat import KatDag
from oracle_py import Oracle
from test_gpu_parity import _compare, _insert_kat

pytestmark = pytest.mark.gpu


def _check_projection(o, hg, where="", json_every=1):
    ob = o.blocks()
    gb = hg.blocks()
    assert gb["round_received"].tolist() == ob["round_received"].tolist(), where
    fh, bh, ok = hg.block_hashes()
    for b, rr in enumerate(ob["round_received"].tolist()):
        assert hg.frame_roots(rr) == o.frame_roots(rr), f"{where} roots of frame {rr}"
        want = o.block_frame_hash(b)
        assert bool(ok[b]) == (want is not None), f"{where} block {b}"
        if want is None:
            continue
        assert fh[b].tobytes() == want, f"{where} FrameHash of block {b} (frame {rr})"
        assert bh[b].tobytes() == sha(o.block_json(b)), f"{where} block hash {b}"
        if b % json_every == 0:
            assert hg.frame_json(rr) == o.frame_json(rr), f"{where} frame {rr} JSON"
            assert hg.block_json(b) == o.block_json(b), f"{where} block {b} JSON"
            assert hg.block_json(b, body_only=True) == o.block_json(b, body_only=True)


@pytest.mark.parametrize("name", ["kat_consensus", "kat_sparse", "kat_funky_full"])
def test_frames_kat(name):
    from babble_amd import Hashgraph
    d = KatDag(name)
    hg = Hashgraph(d.participant_ids, 64, frames=True)
    o = Oracle(d.n, d.participant_ids, capacity=len(d) + 64)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    assert not np.asarray(_insert_kat(hg, d)).any()
    bodies, sigs = zip(*(kat_event_bytes(d, e) for e in range(len(d))))
    hg.set_event_bytes(0, bodies, sigs)
    for e in range(len(d)):
        o.set_event_bytes(e, bodies[e], sigs[e])
    hg.run_consensus()
    o.run_consensus()
    _compare(o, hg, name)
    _check_projection(o, hg, name)
    res = hg.results()
    for rr, want in d.expect.get("frame_roots", {}).items():
        got = roots_by_name(hg.frame_roots(int(rr)), d, res["lamport"], res["round"])
        assert matches_fixture(got, want), (rr, got, want)


def _gen(n, N, seed, lag=0, div=40):
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, lagging=lag, lag_div=div, sig_mode=0)
    bodies = [d.body_json(e) for e in range(N)]
    sigs = [(base36(d.sig_r[e]) + "|" + base36(d.sig_s[e])).encode() for e in range(N)]
    return d, bodies, sigs


def _wire(hg, d, lo, hi):
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    return hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi], opi[lo:hi],
                            d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])


@pytest.mark.parametrize("site", ["auto", "device", "host"])
@pytest.mark.parametrize("n,N,seed,lag,step", [(4, 3000, 81, 0, 0), (9, 6000, 82, 2, 0),
                                               (7, 5000, 83, 1, 450), (32, 40000, 84, 0, 0),
                                               (32, 40000, 87, 0, 1500)])
def test_frames_generated(monkeypatch, site, n, N, seed, lag, step):
    """Generated DAGs whose bodies hash to their event hashes; batch and
    per-sync schedules (bytes given with each batch).  The digests of the
    device-built JSON are taken on the device or by the host's SHA-256
    (frames.cpp: a call that emits few frames hashes on the host; site
    forces either), byte-identical either way."""
    if site != "auto":
        monkeypatch.setenv("BH_FRAME_HASH", site)
    from babble_amd import Hashgraph
    d, bodies, sigs = _gen(n, N, seed, lag)
    hg = Hashgraph(d.participant_ids, N, frames=True)
    o = Oracle(n, d.participant_ids, capacity=N)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    step = step or N
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        for e in range(lo, hi):
            o.set_event_bytes(e, bodies[e], sigs[e])
        o.run_consensus()
        assert not np.asarray(_wire(hg, d, lo, hi)).any()
        hg.set_event_bytes(lo, bodies[lo:hi], sigs[lo:hi])
        hg.run_consensus()
    _compare(o, hg)
    _check_projection(o, hg, f"n={n}", json_every=1 if N <= 6000 else 7)


def test_frames_missing_bytes_and_reset():
    """A frame with an event whose bytes were never given has roots but no
    FrameHash; reset_consensus + a second run reproduces every hash."""
    from babble_amd import Hashgraph
    n, N = 5, 4000
    d, bodies, sigs = _gen(n, N, 85)
    hg = Hashgraph(d.participant_ids, N, frames=True)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    hole = 2000
    for e in range(N):
        if e != hole:
            o.set_event_bytes(e, bodies[e], sigs[e])
    o.run_consensus()
    _wire(hg, d, 0, N)
    hg.set_event_bytes(0, bodies[:hole], sigs[:hole])
    hg.set_event_bytes(hole + 1, bodies[hole + 1:], sigs[hole + 1:])
    hg.run_consensus()
    _check_projection(o, hg, "hole", json_every=3)
    fh, bh, ok = hg.block_hashes()
    assert not ok.all() and ok.any()
    hg.reset_consensus()
    hg.run_consensus()
    fh2, bh2, ok2 = hg.block_hashes()
    assert (ok2 == ok).all() and (fh2 == fh).all() and (bh2 == bh).all()


def test_frames_shard_group():
    """Two shards on one device: every shard projects the same blocks."""
    from babble_amd import Hashgraph
    n, N = 8, 8000
    d, bodies, sigs = _gen(n, N, 86)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    for e in range(N):
        o.set_event_bytes(e, bodies[e], sigs[e])
    o.run_consensus()
    hg = Hashgraph(d.participant_ids, N, devices=[0, 0], frames=True)
    _wire(hg, d, 0, N)
    hg.set_event_bytes(0, bodies, sigs)
    hg.run_consensus()
    _check_projection(o, hg, "group", json_every=5)


def test_frames_off_rejects_queries():
    from babble_amd import Hashgraph, HashgraphError
    d = KatDag("kat_consensus")
    hg = Hashgraph(d.participant_ids, 64)
    _insert_kat(hg, d)
    hg.run_consensus()
    with pytest.raises(HashgraphError) as ei:
        hg.frame_roots(1)
    assert ei.value.kind == "State"
