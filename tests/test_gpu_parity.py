"""Parity of the MI355X engine (libbabble_hip through the C ABI) with the CPU
oracle: the reference's known-answer DAGs and seeded synthetic gossip DAGs.
Integer work, so every comparison is bit-exact."""
import numpy as np
import pytest

from kat import KatDag, kat_names
from oracle_py import UNSET, Oracle

pytestmark = pytest.mark.gpu


def _engine(n, ids, cap):
    from babble_amd import Hashgraph
    return Hashgraph(ids, cap)


def _insert_kat(hg, d):
    """KAT play list -> wire form (creator ID, index, sp index, op (ID, index))."""
    pid = d.participant_ids
    spi = np.where(d.sp >= 0, d.index - 1, -1)
    opc = np.where(d.op >= 0, pid[d.creator[np.maximum(d.op, 0)]], -1)
    opi = np.where(d.op >= 0, d.index[np.maximum(d.op, 0)], -1)
    return hg.insert_events(pid[d.creator], d.index, spi, opc, opi, d.hashes, d.sig_r, d.ntx)


def _oracle_kat(d):
    o = Oracle(d.n, d.participant_ids, capacity=len(d) + 64)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    return o


def _compare(o, hg, where=""):
    ref = o.results()
    got = hg.results()
    N = len(ref["round"])
    assert hg.stats().n_events == N
    for k in ("round", "witness", "lamport", "round_received", "cons_pos"):
        bad = np.nonzero(ref[k] != got[k])[0]
        assert len(bad) == 0, f"{where} {k}: {len(bad)} mismatches, first {bad[:8]} ref={ref[k][bad[:8]]} got={got[k][bad[:8]]}"
    fr = np.where(ref["witness"] == 1, ref["fame"], -1)
    bad = np.nonzero(fr != got["fame"])[0]
    assert len(bad) == 0, f"{where} fame: {bad[:8]} ref={fr[bad[:8]]} got={got['fame'][bad[:8]]}"
    assert np.array_equal(o.consensus_order(), hg.consensus_order()), where
    ob, gb = o.blocks(), hg.blocks()
    for k in ("round_received", "first", "count", "ntx"):
        assert np.array_equal(ob[k], gb[k]), f"{where} blocks.{k}"
    assert o.pending_rounds() == hg.pending_rounds, where
    st = hg.stats()
    assert st.last_round == o.last_round()
    lcr = o.last_consensus_round()
    assert st.last_consensus_round == lcr
    assert st.consensus_transactions == o.consensus_transactions()
    assert st.pending_loaded_events == o.pending_loaded_events()
    assert np.array_equal(o.undetermined(), hg.undetermined_events)


@pytest.mark.parametrize("name", [k for k in kat_names() if k != "kat_fork"])
def test_kat_dag_parity(name):
    d = KatDag(name)
    o = _oracle_kat(d)
    o.run_consensus()
    hg = _engine(d.n, d.participant_ids, len(d) + 64)
    st = _insert_kat(hg, d)
    assert not st.any()
    hg.run_consensus()
    _compare(o, hg, name)


def test_kat_stepwise_and_coordinates():
    """TestInsertEvent coordinates + the pass-by-pass states of kat_consensus
    (hashgraph_test.go:436-574, 1207-1520) through the engine."""
    d = KatDag("kat_round")
    hg = _engine(d.n, d.participant_ids, 64)
    _insert_kat(hg, d)
    for e, c in d.expect["coordinates"].items():
        la, fd = hg.coordinates(d.id_of[e])
        assert la.tolist() == c["la"] and fd.tolist() == c["fd"], e
    d = KatDag("kat_consensus")
    hg = _engine(d.n, d.participant_ids, 64)
    _insert_kat(hg, d)
    ex = d.expect
    hg.divide_rounds()
    res = hg.results()
    for e, (t, r) in ex["lamport_round"].items():
        assert (res["lamport"][d.id_of[e]], res["round"][d.id_of[e]]) == (t, r), e
    hg.decide_fame()
    assert hg.pending_rounds == [tuple(p) for p in ex["pending_after_fame"]]
    res = hg.results()
    for e in ex["famous"]:
        assert res["fame"][d.id_of[e]] == 1, e
    hg.decide_round_received()
    assert hg.undetermined_events.tolist() == d.ids(ex["undetermined_after_rr"])
    hg.process_decided_rounds()
    assert len(hg.consensus_order()) == ex["consensus_len"]
    assert hg.pending_loaded_events == ex["pending_loaded"]
    assert hg.pending_rounds == [tuple(p) for p in ex["pending_after_process"]]


def test_kat_fork_rejected():
    """TestFork (hashgraph_test.go:351-398): forks and unknown parents are rejected."""
    from babble_amd import HashgraphError
    d = KatDag("kat_fork")
    hg = _engine(d.n, d.participant_ids, 64)
    _insert_kat(hg, d)
    pid = d.participant_ids
    # second index-0 event of node 2 (self-parent is not its last event)
    with pytest.raises(HashgraphError) as ei:
        hg.insert_event(pid[2], 0, -1, -1, -1, bytes(32), bytes(32), 1)
    assert ei.value.kind in ("SelfParent", "SkippedIndex")
    # other-parent unknown
    with pytest.raises(HashgraphError) as ei:
        hg.insert_event(pid[0], 1, 0, pid[2], 1, bytes(32), bytes(32), 0)
    assert ei.value.kind == "OtherParent"
    assert hg.stats().n_events == 3


def _random_parity(n, N, seed, lagging=0):
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, lagging=lagging, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    hg = _engine(n, d.participant_ids, N)
    st = hg.insert_dag(d)
    assert not st.any()
    hg.run_consensus()
    _compare(o, hg, f"n={n} N={N} seed={seed} lag={lagging}")
    return hg


@pytest.mark.parametrize("n,N,seed,lag", [
    (4, 10_000, 0xBABB1E01, 0),     # C1 shape: coin rounds every 4 rounds of voting
    (3, 3_000, 11, 0),
    (5, 4_000, 12, 0),
    (7, 6_000, 13, 0),
    (9, 8_000, 14, 3),              # lagging peers: long undecided fame, round jumps
    (32, 60_000, 15, 0),            # C2 shape
    (64, 60_000, 16, 21),           # C5 shape (21 lagging)
    (128, 60_000, 17, 0),           # C3 shape
])
def test_random_dag_parity(n, N, seed, lag):
    _random_parity(n, N, seed, lag)


def test_run_twice_and_incremental_batches():
    """Re-running the passes and inserting in several batches gives the batch
    result of the final DAG (schedule: insert all, then the four passes)."""
    from babble_amd.dag import Dag
    n, N = 16, 20_000
    d = Dag(n, N, 99, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    from babble_amd import Hashgraph
    hg = Hashgraph(d.participant_ids, N)
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    for lo, hi in ((0, 5000), (5000, 12345), (12345, N)):
        hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi],
                         opi[lo:hi], d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])
        hg.run_consensus()
    hg.run_consensus()
    _compare(o, hg, "batches")


def test_empty_and_tiny():
    from babble_amd import Hashgraph
    hg = Hashgraph(np.array([5, 9, 11], np.int64), 16)
    hg.run_consensus()
    assert hg.stats().n_events == 0 and len(hg.consensus_order()) == 0
    # three initial events only: one round, nothing decided
    for c, pid in enumerate([5, 9, 11]):
        hg.insert_event(pid, 0, -1, -1, -1, bytes([c + 1] * 32), bytes([c + 1] * 32), 0)
    hg.run_consensus()
    res = hg.results()
    assert res["round"].tolist() == [0, 0, 0] and res["witness"].tolist() == [1, 1, 1]
    assert hg.pending_rounds == [(0, False)]
    assert hg.last_consensus_round is None


def invariants(d, hg, ordered=0.95):
    """Size-independent properties of a whole-DAG run: the Lamport
    recurrence (hashgraph.go:325-379), round monotonicity along both parents
    (_round :205-278), the witness definition (:281-296), the frame sort key
    order (ByLamportTimestamp, event.go:328-347) and block / transaction
    conservation (ProcessDecidedRounds :1041-1122)."""
    res = hg.results()
    lt = res["lamport"]
    sp, op = d.self_parent, d.other_parent
    ltp = np.maximum(np.where(sp >= 0, lt[np.maximum(sp, 0)], -1), np.where(op >= 0, lt[np.maximum(op, 0)], -1))
    assert np.array_equal(lt, ltp + 1)  # _lamportTimestamp
    rnd = res["round"]
    assert np.all(rnd >= np.where(sp >= 0, rnd[np.maximum(sp, 0)], 0))
    assert np.all(rnd >= np.where(op >= 0, rnd[np.maximum(op, 0)], 0))
    wit = res["witness"] == 1
    spr = np.where(sp >= 0, rnd[np.maximum(sp, 0)], -1)
    assert np.array_equal(wit, rnd > spr)  # witness()
    order = hg.consensus_order()
    rr = res["round_received"]
    key_rr = rr[order]
    assert np.all(np.diff(key_rr) >= 0)
    same = np.diff(key_rr) == 0
    assert np.all(np.diff(lt[order])[same] >= 0)
    assert np.all(rr[order] > rnd[order])  # received in a later round
    b = hg.blocks()
    assert b["count"].sum() == len(order)
    assert b["ntx"].sum() == d.ntx[order].sum() == hg.consensus_transactions
    assert len(order) > ordered * d.N
    return res


def test_large_properties():
    """C2 size (1M events, 32 peers): the invariants of a whole-DAG run
    (bit-exact whole-DAG parity at full sizes: test_gpu_fullsize.py,
    test_gpu_whole.py)."""
    from babble_amd.dag import Dag
    from babble_amd import Hashgraph
    n, N = 32, 1_000_000
    d = Dag(n, N, 0xBABB1E02, sig_mode=0)
    hg = Hashgraph(d.participant_ids, N)
    hg.insert_dag(d)
    hg.run_consensus()
    invariants(d, hg)


def test_wide_512_parity():
    """C4's width (512 participants, SM = 342) against the oracle, bit-exact:
    the chunked coordinate sweep, k_round_wide and fame from HBM rows."""
    _random_parity(512, 40_000, 0xBABB1E04, 0)


def _prefix_check(cfg, prefix):
    """Full-size DAG of BASELINE config `cfg` (the DAG bench.py times) through
    the engine, against the oracle on its first `prefix` events.

    Round, witness and Lamport timestamp of an event depend only on its
    ancestors, which precede it in insertion order, so they must agree on
    every prefix event.  A witness's votes depend only on the voters'
    ancestry, so a fame the prefix run decided is the full run's fame; an
    event received in a round the prefix run processed is received there in
    the full run, and those frames -- hence the consensus order and blocks up
    to the prefix run's last processed round -- are identical.  The engine is
    also run on the prefix itself and compared with the oracle in full."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    d = Dag.config(cfg, sig_mode=0)
    N, n = d.N, d.n
    o = Oracle(n, d.participant_ids, capacity=prefix)
    o.insert_dag(*(a[:prefix] for a in (d.creator, d.index, d.self_parent, d.other_parent, d.hash,
                                        d.sig_r, d.ntx)))
    o.run_consensus()
    ref = o.results()
    # the engine on the prefix: full state parity
    hp = Hashgraph(d.participant_ids, prefix)
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    assert not hp.insert_events(pid[d.creator[:prefix]], d.index[:prefix], spi[:prefix], opc_id[:prefix],
                                opi[:prefix], d.hash[:prefix], d.sig_r[:prefix], d.ntx[:prefix]).any()
    hp.run_consensus()
    _compare(o, hp, f"cfg{cfg} prefix {prefix}")
    hp.close()
    # the engine on the whole DAG
    hg = Hashgraph(d.participant_ids, N)
    assert not hg.insert_dag(d).any()
    hg.run_consensus()
    got = hg.results(0, prefix)
    for k in ("round", "witness", "lamport"):
        bad = np.nonzero(ref[k] != got[k])[0]
        assert len(bad) == 0, f"cfg{cfg} {k}: {len(bad)} mismatches, first {bad[:8]}"
    dec = (ref["witness"] == 1) & (ref["fame"] != 0)
    assert dec.sum() > 0
    assert np.array_equal(ref["fame"][dec], got["fame"][dec]), f"cfg{cfg} decided fame"
    rcv = ref["round_received"] != UNSET
    assert np.array_equal(ref["round_received"][rcv], got["round_received"][rcv]), f"cfg{cfg} rr"
    oo = o.consensus_order()
    assert len(oo) > 0.75 * prefix
    assert np.array_equal(oo, hg.consensus_order()[:len(oo)]), f"cfg{cfg} consensus order"
    assert np.array_equal(ref["cons_pos"][rcv], got["cons_pos"][rcv])
    ob, gb = o.blocks(), hg.blocks()
    k = len(ob["round_received"])
    for f in ("round_received", "first", "count", "ntx"):
        assert np.array_equal(ob[f], gb[f][:k]), f"cfg{cfg} blocks.{f}"
    st = hg.stats()
    assert st.consensus_events > 0.95 * N and st.last_consensus_round >= o.last_consensus_round()
    hg.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cfg,prefix", [(3, 200_000), (5, 200_000), (4, 100_000)])
def test_full_size_prefix_parity(cfg, prefix):
    """BASELINE configs C3 (128 peers, 10M events: the bench DAG), C5 (64 peers,
    21 lagging, 2M) and C4 (512 peers, 20M) at full size."""
    _prefix_check(cfg, prefix)


def _wild_dag(n, N, seed, back):
    """A valid DAG that is not gossip-shaped: each event's other-parent is a
    random event of another creator up to `back` events old (Babble accepts
    any known event, checkOtherParent hashgraph.go:417-436).  Exercises
    coordinate parents far outside the engines' on-chip rings."""
    rng = np.random.default_rng(seed)
    creator = np.empty(N, np.int32)
    index = np.empty(N, np.int32)
    sp = np.empty(N, np.int32)
    op = np.empty(N, np.int32)
    last = np.full(n, -1, np.int64)
    cnt = np.zeros(n, np.int32)
    for e in range(N):
        c = e if e < n else int(rng.integers(n))
        creator[e], index[e], sp[e] = c, cnt[c], last[c]
        o = -1
        if e >= n:
            for _ in range(8):
                cand = int(rng.integers(max(0, e - back), e))
                if creator[cand] != c:
                    o = cand
                    break
        op[e] = o
        last[c] = e
        cnt[c] += 1
    hashes = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    sig = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    ntx = (rng.random(N) < 0.5).astype(np.int32)
    return creator, index, sp, op, hashes, sig, ntx


def _wild_parity(n, N, seed, back):
    from babble_amd import Hashgraph
    creator, index, sp, op, hashes, sig, ntx = _wild_dag(n, N, seed, back)
    pid = np.sort(np.random.default_rng(seed + 1).choice(2**31 - 1, n, replace=False)).astype(np.int64)
    o = Oracle(n, pid, capacity=N)
    o.insert_dag(creator, index, sp, op, hashes, sig, ntx)
    o.run_consensus()
    hg = Hashgraph(pid, N)
    spi = np.where(sp >= 0, index - 1, -1)
    opc = np.where(op >= 0, pid[creator[np.maximum(op, 0)]], -1)
    opi = np.where(op >= 0, index[np.maximum(op, 0)], -1)
    st = hg.insert_events(pid[creator], index, spi, opc, opi, hashes, sig, ntx)
    assert not st.any()
    hg.run_consensus()
    _compare(o, hg, f"wild n={n} N={N} back={back}")


def _burst_dag(n, N, seed, burst):
    """Gossip with bursts: now and then one creator emits `burst` events in a
    row (other-parents: recent events of others), so its chain advances
    far more than 31 rows within a round -- the n <= 128 loop's window
    continuation (SM not reached in the staged window) and the hand-off's
    entries past the 64 loaded rows (its wave search)."""
    rng = np.random.default_rng(seed)
    creator = np.empty(N, np.int32)
    index = np.empty(N, np.int32)
    sp = np.empty(N, np.int32)
    op = np.empty(N, np.int32)
    last = np.full(n, -1, np.int64)
    cnt = np.zeros(n, np.int32)
    run_c, run_left = -1, 0
    for e in range(N):
        if e < n:
            c = e
        elif run_left > 0:
            c, run_left = run_c, run_left - 1
        else:
            c = int(rng.integers(n))
            if rng.random() < 0.002:
                run_c, run_left = c, burst
        creator[e], index[e], sp[e] = c, cnt[c], last[c]
        o = -1
        if e >= n:
            for _ in range(8):
                cand = int(rng.integers(max(0, e - 4 * n), e))
                if creator[cand] != c:
                    o = cand
                    break
        op[e] = o
        last[c] = e
        cnt[c] += 1
    hashes = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    sig = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    ntx = (rng.random(N) < 0.5).astype(np.int32)
    return creator, index, sp, op, hashes, sig, ntx


@pytest.mark.parametrize("n,N,seed,burst", [(32, 40_000, 41, 120), (128, 60_000, 42, 200), (100, 50_000, 43, 90)])
def test_burst_dag_parity(n, N, seed, burst):
    from babble_amd import Hashgraph
    creator, index, sp, op, hashes, sig, ntx = _burst_dag(n, N, seed, burst)
    pid = np.sort(np.random.default_rng(seed + 1).choice(2**31 - 1, n, replace=False)).astype(np.int64)
    o = Oracle(n, pid, capacity=N)
    o.insert_dag(creator, index, sp, op, hashes, sig, ntx)
    o.run_consensus()
    hg = Hashgraph(pid, N)
    spi = np.where(sp >= 0, index - 1, -1)
    opc = np.where(op >= 0, pid[creator[np.maximum(op, 0)]], -1)
    opi = np.where(op >= 0, index[np.maximum(op, 0)], -1)
    assert not hg.insert_events(pid[creator], index, spi, opc, opi, hashes, sig, ntx).any()
    hg.run_consensus()
    _compare(o, hg, f"burst n={n} N={N} burst={burst}")
    # the DAG does what it is for: some chain holds more than 31 events of
    # one round (its boundary jumps past the staged window)
    rd = o.results()["round"]
    per = np.bincount(creator.astype(np.int64) * (int(rd.max()) + 2) + (rd.astype(np.int64) + 1))
    assert per.max() > 31


@pytest.mark.parametrize("n,N,seed,back", [
    (8, 30_000, 21, 20_000),     # parents far behind the LDS rings (flow: 64/chain, sweep: 16K)
    (24, 40_000, 22, 3_000),
    (128, 40_000, 23, 30_000),
    (64, 40_000, 24, 5_000),
])
def test_wild_dag_parity(n, N, seed, back):
    _wild_parity(n, N, seed, back)


@pytest.mark.parametrize("n,N,seed,lag", [(32, 40_000, 31, 0), (64, 40_000, 32, 21), (128, 40_000, 33, 0)])
def test_chunk_sweep_parity(monkeypatch, n, N, seed, lag):
    """The chunked coordinate sweep (used above the chain-dataflow limits)
    forced on gossip DAGs the dataflow path would otherwise take."""
    monkeypatch.setenv("BH_SWEEP", "chunk")
    _random_parity(n, N, seed, lag)


def test_chunk_sweep_wild(monkeypatch):
    monkeypatch.setenv("BH_SWEEP", "chunk")
    _wild_parity(8, 30_000, 41, 25_000)


@pytest.mark.parametrize("rows", ["p8", "p8_window", "p8g_tight", "p8_mixed", "p8_single", "p8g_tight_single",
                                  "p16", "p32", "fdt_p8", "fdt_p16", "cols_p8", "cols_p8g_tight", "cols_p16",
                                  "cols2_p8", "cols2_p16", "iter_p8", "iter_p8_mixed", "iter_p8g_tight",
                                  "fallback_p8", "noprestage_p8", "flat_p8_mixed",
                                  "prio_p8", "prio2_p8_mixed", "noreuse_p8", "noreuse_p8g_tight"])
@pytest.mark.parametrize("n,N,seed", [(160, 30_000, 51), (300, 30_000, 52)])
def test_wide_parity(monkeypatch, n, N, seed, rows):
    """More participants than k_round2 / LDS fame support: k_round_wide
    over 8-bit rows -- the default: relative to the shared base B[r-1][i] -
    20 with the candidates' bytes converted once by the workgroup that hands
    them over (cand8); p8_window: relative to each window's first row only
    (BH_ROUND_P8G=0); p8g_tight: a shared base 2 below B[r-1], which many
    windows do not fit, so they fall back to their own base beside windows
    that take the shared one; p8_mixed: a lower spread limit, so windows also
    alternate with the 16-bit fallback -- over 16-bit rows (fd16; n = 300
    has a half-filled last piece) and over the 32-bit rows (BH_NO_P16, the
    path for chains beyond P16_MAXLEN).  *_single: one candidate's search per
    lane group instead of two interleaved (BH_ROUND_ILP2=0, its own tag check
    and cand8 read).  n = 160 / 300 leave the last lanes of a candidate's
    group past the end of its byte row.  The default loop reads its windows
    from the transposed row-major LA and its candidates' FD rows from FDT;
    fdt_*: the same, pinned (BH_WIDE_ROWS=1).  cols_*: the loop over the
    column-major LA (BH_WIDE_COLS=1); cols2_*: the window from the row-major
    LA, the hand-off from la_col (BH_WIDE_COLS=2).  The default 8-bit loop
    runs as one persistent launch (a grid barrier per round), stages its next
    window during the barrier and keeps the rows it shares with the last
    window; iter_*: one launch per round (BH_ROUND_PERSIST=0); fallback_*: the
    persistent loop's barrier gives up at once (BH_PBAR_SPIN=0), the host
    restores the loop's inputs and runs the per-round launches;
    noprestage_*: staging after the barrier; flat_*: the one-counter
    barrier; prio_* / prio2_*: BH_WIDE_PRIO=1 / 2 (the default is 2);
    noreuse_*: every window staged whole (BH_WIN_REUSE=0)."""
    if rows.startswith("noreuse_"):  # every window staged whole (no rows kept from the last one)
        monkeypatch.setenv("BH_WIN_REUSE", "0")
        rows = rows[len("noreuse_"):]
    if rows.startswith("prio"):  # the persistent loop's priority schemes (BH_WIDE_PRIO)
        monkeypatch.setenv("BH_WIDE_PRIO", "2" if rows.startswith("prio2_") else "1")
        rows = rows[rows.index("_") + 1:]
    if rows.startswith("iter_"):
        monkeypatch.setenv("BH_ROUND_PERSIST", "0")
        rows = rows[len("iter_"):]
    if rows.startswith("noprestage_"):  # the next window staged after the barrier, not during it
        monkeypatch.setenv("BH_PRESTAGE", "0")
        rows = rows[len("noprestage_"):]
    if rows.startswith("flat_"):  # the one-counter grid barrier
        monkeypatch.setenv("BH_PBAR", "flat")
        rows = rows[len("flat_"):]
    if rows.startswith("fallback_"):
        monkeypatch.setenv("BH_PBAR_SPIN", "0")
        rows = rows[len("fallback_"):]
    if rows.startswith("cols2_"):
        monkeypatch.setenv("BH_WIDE_COLS", "2")
        rows = rows[len("cols2_"):]
    if rows.startswith("cols_"):
        monkeypatch.setenv("BH_WIDE_COLS", "1")
        rows = rows[len("cols_"):]
    if rows.startswith("fdt_"):
        monkeypatch.setenv("BH_WIDE_ROWS", "1")
        rows = rows[len("fdt_"):]
    if rows.endswith("_single"):
        monkeypatch.setenv("BH_ROUND_ILP2", "0")
        rows = rows[:-len("_single")]
    if rows == "p8_window":
        monkeypatch.setenv("BH_ROUND_P8G", "0")
    if rows == "p8g_tight":
        monkeypatch.setenv("BH_ROUND_P8G", "2")
    if rows == "p8_mixed":
        monkeypatch.setenv("BH_ROUND_P8", "40")
    if rows == "p16":
        monkeypatch.setenv("BH_ROUND_P8", "0")
    if rows == "p32":
        monkeypatch.setenv("BH_NO_P16", "1")
    _random_parity(n, N, seed)


@pytest.mark.parametrize("sweep", ["flow", "chunk"])
@pytest.mark.parametrize("n,N,seed,lag", [(16, 4_000, 61, 2), (128, 20_000, 62, 0)])
def test_coordinates_random(monkeypatch, sweep, n, N, seed, lag):
    """lastAncestors / firstDescendants (hashgraph.go:478-544) of sampled
    events -- every chain's last events included, whose FD entries are
    MaxInt32 for the chains that have not seen them yet -- against the
    oracle, through both coordinate sweeps."""
    from babble_amd.dag import Dag
    if sweep == "chunk":
        monkeypatch.setenv("BH_SWEEP", "chunk")
    d = Dag(n, N, seed, lagging=lag, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    hg = _engine(n, d.participant_ids, N)
    assert not hg.insert_dag(d).any()
    rng = np.random.default_rng(seed)
    last = [int(np.nonzero(d.creator == c)[0][-1]) for c in range(n)]
    first = [int(np.nonzero(d.creator == c)[0][0]) for c in range(n)]
    sample = sorted(set(last + first + rng.integers(0, N, 150).tolist()))
    nmax = 0
    for e in sample:
        la_r, fd_r = o.coordinates(e)
        la_g, fd_g = hg.coordinates(e)
        assert np.array_equal(la_r, la_g), (e, la_r, la_g)
        assert np.array_equal(fd_r, fd_g), (e, fd_r, fd_g)
        nmax += int((np.asarray(fd_r) == 2**31 - 1).sum())
    assert nmax > 0  # the unseen tails were exercised


@pytest.mark.parametrize("n,N,seed,lag", [(16, 4_000, 64, 2), (128, 20_000, 65, 0), (300, 30_000, 66, 0),
                                          (512, 40_000, 67, 0)])
def test_transpose_fd_walk(monkeypatch, n, N, seed, lag):
    """k_flow_transpose's firstDescendants walk (hashgraph.go:520-544 as the
    oracle restates it) through 64-row tiles (n <= 128) and 32-row ones
    (wide), every chain's first and last events included, then consensus
    over the FDT it wrote."""
    from babble_amd.dag import Dag
    if n <= 128:
        monkeypatch.setenv("BH_ROUND_SRC", "rows")  # (the transpose runs, not the la_col loop alone)
    d = Dag(n, N, seed, lagging=lag, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    hg = _engine(n, d.participant_ids, N)
    assert not hg.insert_dag(d).any()
    rng = np.random.default_rng(seed)
    last = [int(np.nonzero(d.creator == c)[0][-1]) for c in range(n)]
    first = [int(np.nonzero(d.creator == c)[0][0]) for c in range(n)]
    sample = sorted(set(last + first + rng.integers(0, N, 120).tolist()))
    for e in sample:
        la_r, fd_r = o.coordinates(e)
        la_g, fd_g = hg.coordinates(e)
        assert np.array_equal(la_r, la_g), (e, la_r, la_g)
        assert np.array_equal(fd_r, fd_g), (e, fd_r, fd_g)
    o.run_consensus()
    hg.run_consensus()
    _compare(o, hg, f"fd walk n={n}")


def test_flow32_lt_fallback(monkeypatch):
    """The one-value k_flow32 (BH_FLOW1=1; the default k_flow32x2 carries LT
    in 32 bits) carries values in 21 bits; Lamport timestamps beyond its
    limit are flagged and recomputed by the two-dword kernel.  A lowered
    limit (BH_FLOW_LTCLAMP, read at handle creation) forces that path on a
    DAG whose timestamps exceed it."""
    monkeypatch.setenv("BH_FLOW1", "1")
    monkeypatch.setenv("BH_FLOW_LTCLAMP", "300")
    hg = _random_parity(16, 20_000, 71, 2)
    assert hg.results()["lamport"].max() > 300


@pytest.mark.parametrize("kernel", ["k_floww2", "k_floww"])
def test_floww_parity_and_lt_fallback(monkeypatch, kernel):
    """The wide dataflow (128 < n <= 512; k_floww2: two values per
    workgroup, k_floww: one, BH_FLOWW=1): parity on random and lagging DAGs
    against the oracle and against the chunked sweep -- n + 1 values odd (one
    three-column workgroup) and even (pairs only) -- then with a lowered LT
    limit that sends the timestamps to the sweep fallback."""
    if kernel == "k_floww":
        monkeypatch.setenv("BH_FLOWW", "1")
    hg = _random_parity(200, 30_000, 74, 0)
    assert hg.profile_kernel() == kernel  # not its watchdog's sweep fallback
    hg = _random_parity(201, 30_000, 78, 2)
    assert hg.profile_kernel() == kernel
    hg = _random_parity(512, 25_000, 75, 3)
    assert hg.profile_kernel() == kernel
    _wild_parity(150, 30_000, 76, 20_000)
    monkeypatch.setenv("BH_FLOW_LTCLAMP", "300")
    hg = _random_parity(160, 20_000, 77, 2)
    assert hg.results()["lamport"].max() > 300


@pytest.mark.parametrize("segments", [None, 4])
def test_floww_watchdog_fallback(monkeypatch, segments):
    """k_floww2's watchdog fires (BH_FLOWW_WATCHDOG=-1: at its first header,
    every launch): the segment pipeline must see the flag before any round
    loop reads the unfinished coordinates and recompute the call through the
    chunked sweep -- in one segment and in four, for a batch and for the
    incremental calls after it."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    monkeypatch.setenv("BH_FLOWW_WATCHDOG", "-1")  # read at handle creation
    if segments:
        monkeypatch.setenv("BH_SEGMENTS", str(segments))
    n, N = 160, 30_000
    d = Dag(n, N, 79, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    for lo, hi in ((0, 20_000), (20_000, 25_000), (25_000, N)):
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        assert not hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi],
                                    opi[lo:hi], d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi]).any()
        hg.run_consensus()
        _compare(o, hg, f"watchdog fallback, events [0, {hi})")
        assert hg.profile_kernel() == "k_la_sweep"


@pytest.mark.parametrize("segments", [None, 8])
@pytest.mark.parametrize("kernel", ["k_flow32x2", "k_flow32"])
def test_flow32_variants(monkeypatch, kernel, segments):
    """The two-value dataflow (k_flow32x2, the default at n <= 128: a
    workgroup carries two LA columns, or a column and LT) and the one-value
    k_flow32 it falls back to for chains past 131,008 events (BH_FLOW1=1
    forces it), whole and through 8 segments: n = 128 (65 workgroups with
    LT inside; k_flow32: LT after the next segment's columns), n = 127 (an
    even value count: no single-column workgroup), n = 64 lagging, and wild
    DAGs whose parents fall far behind the 64-slot rings."""
    if kernel == "k_flow32":
        monkeypatch.setenv("BH_FLOW1", "1")
    if segments:
        monkeypatch.setenv("BH_SEGMENTS", str(segments))
    for n, N, seed, lag in ((128, 80_000, 171, 0), (127, 60_000, 172, 0), (64, 60_000, 173, 21), (5, 20_000, 174, 1)):
        hg = _random_parity(n, N, seed, lag)
        assert hg.profile_kernel() == kernel
        if segments:
            assert hg.pipeline()[0] == min(segments, N // 4096 + 1)  # (segments_for)
    _wild_parity(128, 40_000, 175, 30_000)
    _wild_parity(33, 40_000, 176, 20_000)


def test_flow32_long_chains():
    """Chains past k_flow32x2's 131,008 events (11-bit generations of
    64-slot rings) take the one-value k_flow32 (128-slot rings): a batch,
    then per-sync calls whose chains cross the limit between calls (the
    descriptor format changes with the kernel; each call writes its new
    rows' entries)."""
    from babble_amd.dag import Dag
    from babble_amd import Hashgraph
    n, N = 3, 420_000
    assert int(np.bincount(Dag(n, N, 177, sig_mode=0).creator).max()) > 131_008
    hg = _random_parity(n, N, 177, 0)
    assert hg.profile_kernel() == "k_flow32"
    d = Dag(2, 300_000, 178, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(2, d.participant_ids, capacity=d.N)
    hg = Hashgraph(d.participant_ids, d.N)
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    kernels = set()
    for lo in range(0, d.N, 25_000):
        hi = min(d.N, lo + 25_000)
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        assert not hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi], opi[lo:hi],
                                    d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi]).any()
        hg.run_consensus()
        kernels.add(hg.profile_kernel())
        _compare(o, hg, f"n=2 per-sync, after [0, {hi})")
    assert kernels == {"k_flow32x2", "k_flow32"}


def test_flow64_parity(monkeypatch):
    """The two-dword dataflow kernel (chains of 2^17 .. 2^21 events) forced
    on DAGs the one-dword kernel would take."""
    monkeypatch.setenv("BH_SWEEP", "flow64")
    _random_parity(128, 40_000, 72, 0)
    _wild_parity(24, 30_000, 73, 20_000)


@pytest.mark.parametrize("n,N,seed,lag,step", [(4, 3000, 5, 0, 97), (9, 8000, 14, 3, 400), (32, 30_000, 21, 0, 3000)])
def test_gossip_schedule_every_call(n, N, seed, lag, step):
    """The live node's schedule (node.go:583-603 -> core.go:337-369):
    RunConsensus after every gossip batch.  After EVERY call the engine's
    state (rounds, fame, roundReceived, order, blocks, PendingRounds,
    LastConsensusRound, counters, UndeterminedEvents) equals the oracle run
    on the same schedule."""
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, lagging=lag, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = _engine(n, d.participant_ids, N)
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        st = hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi],
                              opi[lo:hi], d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])
        assert not np.asarray(st).any()
        hg.run_consensus()
        _compare(o, hg, f"after events [0, {hi})")


def test_participant_lookup_rejects_unknown_ids():
    """ParticipantEvents lookups (rolling_index / peers): an unknown creator is
    UnknownParticipant, an unknown other-parent creator is OtherParent; IDs
    spread over the int64 range (the open-addressing table's probing)."""
    from babble_amd import Hashgraph, HashgraphError
    ids = np.array(sorted([0, 3, 11, 12, 13, 1 << 31, 1 << 40, (1 << 62) + 5]), np.int64)
    hg = Hashgraph(ids, 64)
    for c, pid in enumerate(ids):
        hg.insert_event(int(pid), 0, -1, -1, -1, bytes([c + 1] * 32), bytes([c + 1] * 32), 0)
    with pytest.raises(HashgraphError) as ei:
        hg.insert_event(4, 0, -1, -1, -1, bytes(32), bytes(32), 0)
    assert ei.value.kind == "UnknownParticipant"
    with pytest.raises(HashgraphError) as ei:
        hg.insert_event(int(ids[0]), 1, 0, 99, 0, bytes(32), bytes(32), 0)
    assert ei.value.kind == "OtherParent"
    hg.insert_event(int(ids[0]), 1, 0, int(ids[-1]), 0, bytes([77] * 32), bytes([77] * 32), 0)
    assert hg.stats().n_events == len(ids) + 1


@pytest.mark.parametrize("K,n,N,seed,lag", [
    (3, 4, 10_000, 0xBABB1E01, 0),
    (5, 128, 60_000, 91, 0),
    (7, 64, 50_000, 92, 21),
    (2, 32, 40_000, 93, 0),
    (13, 9, 30_000, 94, 3),
    (4, 200, 30_000, 111, 0),    # wide: k_floww2 segments + 16-bit k_round_wide resumes
    (6, 300, 30_000, 112, 5),
    (3, 512, 25_000, 113, 0),
    (5, 129, 30_000, 114, 2),
])
def test_segment_pipeline_parity(monkeypatch, K, n, N, seed, lag):
    """Coordinates of prefix s + 1 overlapped with the round loop on prefix s,
    the loop resuming at the last round the prefix fixed (BH_SEGMENTS=K;
    full-size DAGs take 4 segments by default)."""
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    hg = _random_parity(n, N, seed, lag)
    assert hg.pipeline()[0] == min(K, N // 4096 + 1)  # (segments of at least 4096 events)


@pytest.mark.parametrize("p8", ["p8", "p8_mixed", "p16"])
def test_segment_pipeline_wide_rows(monkeypatch, p8):
    """The wide loop's resumed windows on 8-bit rows, alternating with the
    16-bit fallback, and on 16-bit rows only, through 4 segments"""
    monkeypatch.setenv("BH_SEGMENTS", "4")
    if p8 == "p8_mixed":
        monkeypatch.setenv("BH_ROUND_P8", "40")
    if p8 == "p16":
        monkeypatch.setenv("BH_ROUND_P8", "0")
    hg = _random_parity(160, 30_000, 115, 0)
    assert hg.pipeline()[0] == 4 and hg.profile_kernel() == "k_floww2"


@pytest.mark.parametrize("K", [2, 6])
def test_segment_pipeline_wild(monkeypatch, K):
    """Other-parents far behind the segment start (read back from HBM by the
    resumed dataflow) and chains idle for whole segments."""
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    _wild_parity(24, 40_000, 95, 30_000)
    _wild_parity(128, 40_000, 96, 35_000)
    _wild_parity(170, 30_000, 116, 25_000)  # wide: far parents read back by the resumed k_floww2


def test_segment_pipeline_lt_fallback(monkeypatch):
    monkeypatch.setenv("BH_FLOW1", "1")
    monkeypatch.setenv("BH_SEGMENTS", "4")
    monkeypatch.setenv("BH_FLOW_LTCLAMP", "300")
    hg = _random_parity(16, 20_000, 97, 2)
    assert hg.results()["lamport"].max() > 300


def test_segment_pipeline_schedule(monkeypatch):
    """The per-sync schedule with every call through the segment pipeline."""
    monkeypatch.setenv("BH_SEGMENTS", "3")
    from babble_amd.dag import Dag
    from babble_amd import Hashgraph
    n, N, step = 9, 30_000, 5_000
    d = Dag(n, N, 98, lagging=3, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi], opi[lo:hi],
                         d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])
        hg.run_consensus()
        _compare(o, hg, f"segments, after [0, {hi})")


@pytest.mark.parametrize("n,N,seed,lag,K", [(4, 10_000, 0xBABB1E01, 0, 1), (9, 8_000, 14, 3, 1), (32, 60_000, 15, 0, 3),
                                            (17, 40_000, 31, 5, 4)])
def test_round_solo_parity(monkeypatch, n, N, seed, lag, K):
    """The opt-in resident round loop (k_round_solo, BH_ROUND_SOLO=1: one
    workgroup runs every round, n <= 32) against the oracle, alone and as
    the loop of the segment pipeline; its windows that miss SM continue from
    global memory (the wild DAG)."""
    monkeypatch.setenv("BH_ROUND_SOLO", "1")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    _random_parity(n, N, seed, lag)
    if K == 1:
        _wild_parity(24, 30_000, 73, 20_000)


@pytest.mark.parametrize("variant", ["persist", "tq", "rows"])
@pytest.mark.parametrize("n,N,seed,lag,K", [(4, 10_000, 0xBABB1E01, 0, 1), (9, 8_000, 14, 3, 2), (32, 60_000, 15, 0, 3),
                                            (17, 40_000, 31, 5, 4), (48, 40_000, 37, 6, 2)])
def test_small_n_round_kernels(monkeypatch, variant, n, N, seed, lag, K):
    """k_round2 at n <= 64 (8 lanes per candidate, one or two pieces each,
    8 npad threads): the per-candidate T_q search and the row-probe search
    (BH_ROUND_ROWS=1) against the oracle, alone and inside the segment
    pipeline; the wild DAG's windows that miss SM continue window by window.
    persist: the default one-launch loop (k_round2p); tq / rows: one launch
    per iteration (BH_ROUND_PERSIST=0)."""
    if variant != "persist":
        monkeypatch.setenv("BH_ROUND_PERSIST", "0")
    if variant == "rows":
        monkeypatch.setenv("BH_ROUND_ROWS", "1")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    _random_parity(n, N, seed, lag)
    if K == 1:
        _wild_parity(24, 30_000, 73, 20_000)


@pytest.mark.parametrize("variant", ["persist", "tq", "rows", "eager"])
@pytest.mark.parametrize("n,N,seed,lag,K", [(128, 60_000, 0xB8, 0, 1), (100, 50_000, 0xB9, 4, 3),
                                            (97, 40_000, 0xBA, 0, 2), (72, 30_000, 0xBB, 3, 1)])
def test_round2_la_col(monkeypatch, variant, n, N, seed, lag, K):
    """k_round2 at 64 < npad <= 128 reading only the column-major LA (round
    4): the window staged from la_col 4-row pieces (npad = 100 / 72 leave
    padding columns), the candidates' FD rows searched in la_col at each
    hand-off, lagging peers (hand-offs whose FD entries jump past the 64
    rows loaded), segments resumed at candidates searched from scratch;
    rows: the row-probe search; eager: the segments also build the row-major
    LA and FDT (BH_EAGER_ROWS=1, the round-3 pipeline); persist: the default
    one-launch loop, the others one launch per iteration (BH_ROUND_PERSIST=0)."""
    if variant != "persist":
        monkeypatch.setenv("BH_ROUND_PERSIST", "0")
    if variant == "rows":
        monkeypatch.setenv("BH_ROUND_ROWS", "1")
    if variant == "eager":
        monkeypatch.setenv("BH_EAGER_ROWS", "1")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    _random_parity(n, N, seed, lag)
    if n == 128 and K == 1:
        _wild_parity(128, 40_000, 0xBC, 35_000)


@pytest.mark.parametrize("n,N,seed,lag,K", [(128, 60_000, 0xC0, 0, 1), (100, 50_000, 0xC1, 4, 3),
                                            (32, 40_000, 0xC2, 0, 4), (7, 5_000, 0xC3, 2, 2), (64, 40_000, 0xC4, 21, 1)])
def test_round2_persistent(monkeypatch, n, N, seed, lag, K):
    """The n <= 128 round loop as one launch (k_round2p, the default):
    a grid barrier per iteration, candidates' FD rows and boundaries handed
    over through sc1 stores and loads, every workgroup ending the loop by
    itself -- through segments (resumed candidates), lagging peers, padding
    columns (npad > n) and a 7-chain grid; then incremental calls."""
    monkeypatch.setenv("BH_ROUND_PERSIST", "1")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    loops, fallbacks = _random_parity(n, N, seed, lag).loop_stats()
    assert loops >= 1 and fallbacks == 0
    if n == 128 and K == 1:
        _wild_parity(128, 40_000, 0xC5, 35_000)


@pytest.mark.parametrize("n,N,seed,lag,K", [(128, 500_000, 0xC9, 0, 1), (16, 60_000, 0xCA, 2, 1), (5, 20_000, 0xCB, 1, 2)])
def test_round2_persistent_tag_wrap(monkeypatch, n, N, seed, lag, K):
    """The persistent loop's hand-off words carry the iteration's low 8 bits
    as a tag (k_round2p: a consumer waits for tag == it & 0xFF): loops of
    more than 256 iterations in one launch reuse every tag, so a stale word
    from 256 iterations back must never pass for a fresh one (oracle: 317,
    523 and 897 rounds)."""
    monkeypatch.setenv("BH_ROUND_PERSIST", "1")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    hg = _random_parity(n, N, seed, lag)
    loops, fallbacks = hg.loop_stats()
    assert loops >= 1 and fallbacks == 0
    assert hg.stats().last_round > 256 * K


@pytest.mark.parametrize("n,N,seed,lag,K", [(128, 30_000, 0xC7, 0, 1), (64, 30_000, 0xC8, 21, 3)])
def test_round2_persistent_fallback(monkeypatch, n, N, seed, lag, K):
    """A hand-off wait that gives up (BH_PBAR_SPIN=0: at its first poll that
    finds a word not yet published) ends the persistent loop with ST_ERR = 3; the
    host restores the loop's inputs and runs one launch per iteration, and
    the results are the oracle's."""
    monkeypatch.setenv("BH_ROUND_PERSIST", "1")
    monkeypatch.setenv("BH_PBAR_SPIN", "0")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    loops, fallbacks = _random_parity(n, N, seed, lag).loop_stats()
    assert loops >= 1 and fallbacks >= 1


@pytest.mark.parametrize("fallback", [False, True])
def test_round2_persistent_incremental(monkeypatch, fallback):
    """Per-sync calls through the persistent loop; with fallback, every
    segment's hand-off wait gives up (BH_PBAR_SPIN=0): the loops after the first
    failed one leave at once (ST_PFAIL), and each call is recomputed whole
    with one launch per iteration -- state equal to the oracle's after every
    call either way."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    from test_gpu_schedule import _wire_batches
    monkeypatch.setenv("BH_ROUND_PERSIST", "1")
    if fallback:
        monkeypatch.setenv("BH_PBAR_SPIN", "0")
        monkeypatch.setenv("BH_SEGMENTS", "3")
    n, N, step = 96, 40_000, 5_000
    d = Dag(n, N, 0xC6, lagging=3, sig_mode=0)
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
        _compare(o, hg, f"persistent after [0, {hi})")
    assert (hg.loop_stats()[1] > 0) == fallback


@pytest.mark.parametrize("n,N,seed,lag,K", [(64, 40_000, 0xBD, 21, 4), (128, 60_000, 0xBE, 40, 3)])
def test_lazy_rows_queries(monkeypatch, n, N, seed, lag, K):
    """After a pipelined run that left only the column-major LA, the
    coordinates (LA and FD of every event) and the pair predicates are built
    on demand and equal the oracle's; the next incremental call still
    resumes."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    d = Dag(n, N, seed, lagging=lag, sig_mode=0)
    half = N // 2
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    hg = Hashgraph(d.participant_ids, N)
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    rng = np.random.default_rng(seed)
    prev = 0
    # quarters: the queries after the second call on build only the rows
    # past the ones the previous query built (build_rows), and the older
    # rows' FD entries into the new rows; sampled among the events just
    # before the previous boundary as well
    for lo, hi in ((0, N // 4), (N // 4, half), (half, 3 * N // 4), (3 * N // 4, N)):
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        assert not hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi], opi[lo:hi],
                                    d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi]).any()
        hg.run_consensus()
        _compare(o, hg, f"lazy rows, events [0, {hi})")
        for e in rng.integers(0, hi, 40).tolist() + list(range(max(0, prev - 20), prev)):
            la, fd = hg.coordinates(e)
            ola, ofd = o.coordinates(e)
            assert la.tolist() == ola.tolist() and fd.tolist() == ofd.tolist(), e
        x, y = rng.integers(0, hi, 300), rng.integers(0, hi, 300)
        got = hg.query("strongly_see", x, y)
        assert [bool(v) for v in got] == [o.strongly_see(int(a), int(b)) for a, b in zip(x, y)]
        prev = hi
    assert hg.pipeline()[1] >= 1
