"""Sharded passes through the C ABI: an
in-process shard group on ONE device (device_ids = [0, 0] / [0, 0, 0]) runs
exactly the split kernels and device-to-device exchanges a multi-GPU group
runs over xGMI, and must match the single-shard engine -- and the oracle --
bit for bit: the coordinate split (the default at n <= 128: shards 1 .. G-1
compute LA column ranges and all-gather them per segment, every shard runs
the round loop, fame rounds and frame sorts split between all shards), LA
columns all-gathered unpipelined (BH_SHARD_COORDS=columns) or replicated
coordinates with fame by round ranges and frames sorted by range
(BH_SHARD_COORDS=replicate).  The split at 128 < n <= 512 (k_floww2 on the
coordinate shards, shard 0 transposing each received segment and running
the loop, fame and order alone) is the default from 4 shards and
BH_SHARD_COORDS=split below."""
import numpy as np
import pytest

from oracle_py import Oracle
from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu


def _same_engine(a, b, where):
    ra, rb = a.results(), b.results()
    for k in ra:
        assert np.array_equal(ra[k], rb[k]), f"{where}: {k}"
    assert np.array_equal(a.consensus_order(), b.consensus_order()), where
    ba, bb = a.blocks(), b.blocks()
    for k in ba:
        assert np.array_equal(ba[k], bb[k]), f"{where}: blocks.{k}"
    assert a.pending_rounds == b.pending_rounds, where
    sa, sb = a.stats(), b.stats()
    for f, _ in sa._fields_:
        assert getattr(sa, f) == getattr(sb, f), f"{where}: stats.{f}"


@pytest.mark.parametrize("coords", ["replicate", "columns", "split"])
@pytest.mark.parametrize("n,N,seed,lag,devs", [
    (32, 40_000, 81, 0, [0, 0]),
    (64, 40_000, 82, 21, [0, 0, 0]),
    (128, 60_000, 83, 0, [0, 0]),
    (7, 5_000, 84, 2, [0, 0, 0, 0, 0]),   # more shards than some ranges have items
])
def test_group_matches_single_and_oracle(monkeypatch, coords, n, N, seed, lag, devs):
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    monkeypatch.setenv("BH_SHARD_COORDS", coords)
    d = Dag(n, N, seed, lagging=lag, sig_mode=0)
    one = Hashgraph(d.participant_ids, N)
    grp = Hashgraph(d.participant_ids, N, devices=devs)
    assert not one.insert_dag(d).any() and not grp.insert_dag(d).any()
    one.run_consensus()
    grp.run_consensus()
    _same_engine(one, grp, f"{coords} n={n} shards={len(devs)}")
    assert grp.stage_ms()[5] > 0  # the exchanges ran
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    _compare(o, grp, f"group {coords} vs oracle")


def test_group_wide_chunked():
    """n > 128: the chunked sweep (coordinates always replicated), k_round_wide,
    fame from HBM rows split by round."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    n, N = 160, 20_000
    d = Dag(n, N, 85, sig_mode=0)
    one = Hashgraph(d.participant_ids, N)
    grp = Hashgraph(d.participant_ids, N, devices=[0, 0])
    one.insert_dag(d)
    grp.insert_dag(d)
    one.run_consensus()
    grp.run_consensus()
    _same_engine(one, grp, "wide")


def test_group_per_sync_schedule(monkeypatch):
    """The per-sync schedule with the A.12 trap on a 2-shard group: the
    persistent state (pending flags, trapped witnesses, undetermined events)
    stays identical on every shard across calls."""
    import json
    import os
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    from test_gpu_schedule import GOLDEN, _wire_batches
    monkeypatch.setenv("BH_SHARD_COORDS", "columns")
    with open(os.path.join(GOLDEN, "trap_schedule.json")) as f:
        fx = json.load(f)
    n, N, step = fx["n"], fx["N"], fx["step"] * 7
    d = Dag(n, N, fx["seed"], lagging=fx["lagging"], lag_div=fx["lag_div"], sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    grp = Hashgraph(d.participant_ids, N, devices=[0, 0])
    batch = _wire_batches(d)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        grp.insert_events(*batch(lo, hi))
        grp.run_consensus()
        if hi % (step * 20) == 0 or hi == N:
            _compare(o, grp, f"group after [0, {hi})")


@pytest.mark.parametrize("n,N,step", [(32, 40_000, 10_000), (160, 30_000, 10_000)])
def test_group_pipelined_incremental(monkeypatch, n, N, step):
    """The in-process group -- the handle the Go binding holds for a node with
    G devices -- with replicated coordinates runs the segment pipeline on
    every shard, and its per-sync calls resume from the previous call's
    device state (n = 32: k_flow32 + k_round2; n = 160: k_floww2 +
    k_round_wide), matching the oracle after every call."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    from test_gpu_schedule import _wire_batches
    monkeypatch.setenv("BH_SEGMENTS", "3")
    d = Dag(n, N, 87 + n, lagging=2, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    grp = Hashgraph(d.participant_ids, N, devices=[0, 0])
    batch = _wire_batches(d)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        assert not np.asarray(grp.insert_events(*batch(lo, hi))).any()
        grp.run_consensus()
        _compare(o, grp, f"group n={n} after [0, {hi})")
        assert grp.pipeline()[0] == 3
    assert grp.pipeline()[1] >= N // step - 2  # (a call whose chains outgrow their slack rows lays out anew)


@pytest.mark.parametrize("devs,K", [([0, 0], 3), ([0, 0, 0, 0], 4), ([0, 0, 0], 1)])
@pytest.mark.parametrize("n,N,seed,lag,step", [(128, 60_000, 91, 0, 20_000), (64, 50_000, 92, 21, 10_000),
                                               (24, 40_000, 93, 3, 5_000)])
def test_split_pipeline_incremental(monkeypatch, devs, K, n, N, seed, lag, step):
    """The coordinate split through the segment pipeline and incremental
    calls: 2 / 3 / 4 shards on one device, shard 0 receiving every segment's
    packed LA columns (and rank 1's Lamport timestamps) from the coordinate
    shards; the state equals the oracle's after every call, the calls after
    the first resume, and the receive windows (the exchange) are timed."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    from test_gpu_schedule import _wire_batches
    monkeypatch.setenv("BH_SHARD_COORDS", "split")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    d = Dag(n, N, seed, lagging=lag, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    grp = Hashgraph(d.participant_ids, N, devices=devs)
    batch = _wire_batches(d)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        assert not np.asarray(grp.insert_events(*batch(lo, hi))).any()
        grp.run_consensus()
        _compare(o, grp, f"split {len(devs)} shards n={n} after [0, {hi})")
        assert 1 <= grp.pipeline()[0] <= K  # (segments_for: at most one per 4096 events)
        assert grp.stage_ms()[5] > 0  # the receive windows
    assert grp.pipeline()[1] >= N // step - 2


@pytest.mark.parametrize("coords,devs", [("split", [0, 0]), ("split", [0, 0, 0, 0]), ("replicate", [0, 0])])
def test_group_rerun_after_reset(monkeypatch, coords, devs):
    """The state bench.py times, on a shard group: bh_reset_consensus +
    RunConsensus over the resident DAG, twice, after a first run -- every
    device table but `blocked` carries over between runs -- each equal to the
    oracle's batch run (n = 128, 8 segments: the split's per-segment blocks)."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    monkeypatch.setenv("BH_SHARD_COORDS", coords)
    monkeypatch.setenv("BH_SEGMENTS", "8")
    n, N = 128, 120_000
    d = Dag(n, N, 97, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    grp = Hashgraph(d.participant_ids, N, devices=devs)
    assert not grp.insert_dag(d).any()
    for run in range(3):
        if run:
            grp.reset_consensus()
        grp.run_consensus()
        _compare(o, grp, f"{coords} {len(devs)} shards, run {run}")
        # (four split shards on ONE device each run the 128-workgroup
        # persistent loop: more workgroups than one MI355X holds at once, so
        # a loop may give up waiting for an unplaced workgroup and the call
        # falls back to the unpipelined passes -- exact, as _compare checked;
        # with one rank per GPU no two loops share a device)
        assert grp.pipeline()[0] == 8 or (len(devs) > 2 and grp.loop_stats()[1] > 0)


@pytest.mark.parametrize("rng,seg", [(2, 0), (60, 0), (120, 0), (250, 0), (2, 2), (2, 5)])
def test_split_overflow_chunks(monkeypatch, rng, seg):
    """Chunks whose 64 rows span more than the 16-bit range travel raw in the
    block's overflow slots (BH_SPLIT_RANGE lowers the range so gossip DAGs
    have them); a block that runs out of slots sends the call to the unsplit
    path -- either way the result is the oracle's.  seg > 0: only the blocks
    of segment `seg` on overflow (BH_SPLIT_RANGE_SEG), so the flag is raised
    by a later segment's unpack while earlier segments' persistent loops run
    (every workgroup of a loop decides on the copy k_seg_resume
    took, ST_GATE; the call is a split overflow, not a loop that gave up)."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    monkeypatch.setenv("BH_SHARD_COORDS", "split")
    monkeypatch.setenv("BH_SEGMENTS", "3" if seg == 0 else "8")
    monkeypatch.setenv("BH_SPLIT_RANGE", str(rng))
    monkeypatch.setenv("BH_SPLIT_RANGE_SEG", str(seg))
    n, N = 32, 30_000 if seg == 0 else 60_000
    d = Dag(n, N, 95, lagging=4, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    grp = Hashgraph(d.participant_ids, N, devices=[0, 0, 0])
    assert not grp.insert_dag(d).any()
    fb0 = grp.loop_stats()[1]
    grp.run_consensus()
    _compare(o, grp, f"split, range {rng} from segment {seg}")
    assert grp.loop_stats()[1] == fb0  # no persistent loop gave up (no pbar_spin stall)


@pytest.mark.parametrize("devs,K", [([0, 0], 3), ([0, 0, 0, 0], 4)])
@pytest.mark.parametrize("n,N,seed,lag,step", [(160, 30_000, 101, 2, 10_000), (512, 40_000, 102, 0, 20_000)])
def test_wide_split_pipeline_incremental(monkeypatch, devs, K, n, N, seed, lag, step):
    """The coordinate split at 128 < n <= 512 (BH_SHARD_COORDS=split): the
    coordinate shards run k_floww2 over their LA column ranges and ship each
    segment's packed columns (rank 1 also LT); shard 0 unpacks them,
    transposes the segment into the row-major LA and FDT and runs the 16-bit
    k_round_wide on it -- through the segment pipeline and incremental calls,
    equal to the oracle after every call."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    from test_gpu_schedule import _wire_batches
    monkeypatch.setenv("BH_SHARD_COORDS", "split")
    monkeypatch.setenv("BH_SEGMENTS", str(K))
    d = Dag(n, N, seed, lagging=lag, sig_mode=0)
    args = (d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o = Oracle(n, d.participant_ids, capacity=N)
    grp = Hashgraph(d.participant_ids, N, devices=devs)
    batch = _wire_batches(d)
    for lo in range(0, N, step):
        hi = min(N, lo + step)
        o.insert_dag(*(a[lo:hi] for a in args))
        o.run_consensus()
        assert not np.asarray(grp.insert_events(*batch(lo, hi))).any()
        grp.run_consensus()
        _compare(o, grp, f"wide split {len(devs)} shards n={n} after [0, {hi})")
        assert 1 <= grp.pipeline()[0] <= K
        assert grp.stage_ms()[5] > 0  # the receive windows
    assert grp.pipeline()[1] >= N // step - 2


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0, 0]])
def test_wide_split_matches_single(monkeypatch, devs):
    """A whole DAG at n = 512 through the wide split (default segment count:
    one below 1M events) and then bh_reset_consensus + RunConsensus again
    (the state bench.py times): equal to the single-shard engine and to the
    oracle."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    n, N = 512, 60_000
    d = Dag(n, N, 103, sig_mode=0)
    one = Hashgraph(d.participant_ids, N)
    assert not one.insert_dag(d).any()
    one.run_consensus()
    monkeypatch.setenv("BH_SHARD_COORDS", "split")
    grp = Hashgraph(d.participant_ids, N, devices=devs)
    assert not grp.insert_dag(d).any()
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    for run in range(2):
        if run:
            grp.reset_consensus()
        grp.run_consensus()
        _same_engine(one, grp, f"wide split {len(devs)} shards, run {run}")
        _compare(o, grp, f"wide split vs oracle, run {run}")
        assert grp.stage_ms()[5] > 0


@pytest.mark.parametrize("knob,val", [("BH_FLOWW_WATCHDOG", "-1"), ("BH_FLOW_LTCLAMP", "300")])
def test_wide_split_flags(monkeypatch, knob, val):
    """A coordinate shard's dataflow flags reach shard 0 in its block: the
    k_floww2 watchdog (unfinished columns: the call is recomputed unsplit on
    shard 0) and LT past the dataflow's clamp (the chunked sweep recomputes
    LT) -- either way the oracle's result."""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    monkeypatch.setenv("BH_SHARD_COORDS", "split")
    monkeypatch.setenv("BH_SEGMENTS", "3")
    monkeypatch.setenv(knob, val)  # (read at handle creation)
    n, N = 160, 20_000
    d = Dag(n, N, 104, lagging=2, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    grp = Hashgraph(d.participant_ids, N, devices=[0, 0, 0])
    assert not grp.insert_dag(d).any()
    grp.run_consensus()
    _compare(o, grp, f"wide split, {knob}={val}")
