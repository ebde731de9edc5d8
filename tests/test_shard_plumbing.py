"""The sharding plumbing of DESIGN.md section 7 on the CPU, world_size 2
over gloo: every rank takes its share of the oracle's arrays by the
engine's own split rule (bh_shard_range, exported by libbabble_hip.so and
callable without a GPU) -- LA columns, fame by round (in witness-table
order, ranges by witness offsets), frames of the consensus order (ranges by
frame offsets) -- all-gathers them, reassembles, and must get the
unsharded arrays back byte for byte."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _full_arrays():
    from babble_amd.dag import Dag
    from oracle_py import Oracle
    n, N = 9, 3000
    d = Dag(n, N, 77, lagging=2, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    res = o.results()
    la = np.stack([o.coordinates(e)[0] for e in range(N)])  # [N][n]
    R = o.last_round() + 1
    # witness table: per round, witnesses in chain order (k_wfill's order)
    wofs, wids = [0], []
    for r in range(R):
        w = np.nonzero((res["round"] == r) & (res["witness"] == 1))[0]
        w = w[np.argsort(d.creator[w], kind="stable")]
        wids.extend(w.tolist())
        wofs.append(len(wids))
    wfame = res["fame"][np.array(wids, np.int64)]
    order = o.consensus_order()
    b = o.blocks()
    P = o.last_consensus_round() + 1
    cnt = np.zeros(P, np.int64)
    for rr, c in zip(b["round_received"], b["count"]):
        cnt[rr] = c
    fofs = np.concatenate([[0], np.cumsum(cnt)])
    return dict(la_cols=np.ascontiguousarray(la.T), wfame=wfame, wofs=np.array(wofs), order=order,
                fofs=fofs, R=R, P=P, n=n)


def _gatherv(flat, lo, hi, world):
    """all-gather of [lo, hi) slices of a replicated-layout array"""
    part = torch.from_numpy(np.ascontiguousarray(flat[lo:hi]).astype(np.int64))
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([hi - lo], dtype=torch.int64))
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros(mx, dtype=torch.int64)
    pad[:hi - lo] = part
    outs = [torch.zeros(mx, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(outs, pad)
    return np.concatenate([o[:int(s.item())].numpy() for o, s in zip(outs, sizes)])


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    from babble_amd import shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        f = _full_arrays()
        # LA columns: rank owns columns [c0, c1), each a contiguous run
        c0, c1 = shard_range(f["n"], world, rank)
        cols = f["la_cols"].reshape(-1)
        N = f["la_cols"].shape[1]
        got = _gatherv(cols, c0 * N, c1 * N, world).reshape(f["n"], N)
        ok_la = np.array_equal(got, f["la_cols"])
        # fame: rounds [r0, r1) -> witness entries [wofs[r0], wofs[r1])
        r0, r1 = shard_range(f["R"], world, rank)
        got = _gatherv(f["wfame"], int(f["wofs"][r0]), int(f["wofs"][r1]), world)
        ok_fame = np.array_equal(got, f["wfame"])
        # order: frames [f0, f1) -> positions [fofs[f0], fofs[f1])
        f0, f1 = shard_range(f["P"], world, rank)
        got = _gatherv(f["order"], int(f["fofs"][f0]), int(f["fofs"][f1]), world)
        ok_order = np.array_equal(got, f["order"])
        q.put((rank, ok_la, ok_fame, ok_order, (c0, c1), (r0, r1), (f0, f1)))
    finally:
        dist.destroy_process_group()


def test_shard_gather_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, ok_la, ok_fame, ok_order, cr, rr, fr in out:
        assert ok_la and ok_fame and ok_order, (rank, ok_la, ok_fame, ok_order)
    # the ranges tile their tables
    out.sort()
    assert out[0][4][0] == 0 and out[0][4][1] == out[1][4][0]
    assert out[0][5][1] == out[1][5][0] and out[0][6][1] == out[1][6][0]
