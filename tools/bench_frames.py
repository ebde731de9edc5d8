"""Block projection at benchmark scale: a BASELINE
config's DAG with the Go-JSON bodies its hashes are SHA-256 of, consensus
with bh_config.frames, the projection's device time (stage_ms[6]) per run,
and size-independent checks on the result: for a sample of blocks
SHA-256(Frame JSON) == FrameHash, SHA-256(Block JSON) == block hash (both
recomputed on the host from the bytes the device wrote), the JSON parses
with one root per participant and the frame's events, and the block's
transactions count matches the block's.  Not a headline number: the
projection is outside bench.py's timed step.

  python tools/bench_frames.py --cfg 3 --steps 3
  python tools/bench_frames.py --cfg 3 --N 2000000 --gossip 1600 --calls 40
      (the live node's schedule: a resident DAG, then calls of ~one round of
      events each; the projection of the frames each call emits, per call)
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--N", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--sample", type=int, default=40)
    ap.add_argument("--out", default="")
    ap.add_argument("--gossip", type=int, default=0, help="events per call of a per-sync run (0: batch runs)")
    ap.add_argument("--calls", type=int, default=40)
    a = ap.parse_args()
    from babble_amd import Hashgraph
    from babble_amd.dag import CONFIGS, Dag
    c = CONFIGS[a.cfg]
    N = a.N or c["N"]
    if a.gossip:
        return gossip(a, c, N)
    t = time.time()
    d = Dag.config(a.cfg, N=N, sig_mode=0)
    bodies, bo, sigs, so = d.event_bytes()
    print(f"generated n={c['n']} N={N} in {time.time() - t:.1f}s; bytes {bo[-1] / 1e9:.2f} GB bodies, "
          f"{so[-1] / 1e9:.2f} GB signatures", flush=True)
    hg = Hashgraph(d.participant_ids, N, frames=True)
    assert not np.asarray(hg.insert_dag(d)).any()
    t = time.time()
    L = hg._L
    rc = L.bh_set_event_bytes(hg._h, 0, N, bodies.ctypes.data, bo.ctypes.data, sigs.ctypes.data, so.ctypes.data)
    hg._check(rc)
    print(f"set_event_bytes {time.time() - t:.2f}s", flush=True)
    proj, order = [], []
    for k in range(a.steps + 1):
        hg.reset_consensus()
        hg.run_consensus()
        ms = hg.stage_ms()
        if k:
            proj.append(ms[6])
            order.append(ms[4])
        print(f"run {k}: stages {['%.2f' % x for x in ms]}", flush=True)
    st = hg.stats()
    b = hg.blocks()
    fh, bh, ok = hg.block_hashes()
    assert ok.all(), "every event's bytes were given"
    rng = np.random.default_rng(1)
    nb = len(b["round_received"])
    pick = sorted(set(rng.choice(nb, min(a.sample, nb), replace=False).tolist()) | {0, nb - 1})
    jbytes, tsha = 0, 0.0
    order_ids = hg.consensus_order()
    for i in pick:
        rr = int(b["round_received"][i])
        fj = hg.frame_json(rr)
        t0 = time.perf_counter()
        dig = hashlib.sha256(fj).digest()
        tsha += time.perf_counter() - t0
        jbytes += len(fj)
        assert dig == fh[i].tobytes(), f"FrameHash of block {i}"
        obj = json.loads(fj)
        assert obj["Round"] == rr and len(obj["Roots"]) == c["n"] and len(obj["Events"]) == b["count"][i]
        evs = order_ids[b["first"][i]:b["first"][i] + b["count"][i]]
        assert all(obj["Events"][k]["Body"]["Index"] == int(d.index[e]) for k, e in enumerate(evs[:50]))
        bj = hg.block_json(i)
        assert hashlib.sha256(bj).digest() == bh[i].tobytes(), f"block hash {i}"
        bo_ = json.loads(bj)
        assert len(bo_["Body"]["Transactions"]) == b["ntx"][i]
    frames = st.last_consensus_round + 1
    res = dict(cfg=a.cfg, n=c["n"], N=N, consensus_events=int(st.consensus_events), blocks=int(nb),
               frames=int(frames), projection_ms=float(np.mean(proj)), order_ms=float(np.mean(order)),
               ns_per_consensus_event=float(np.mean(proj)) * 1e6 / max(1, st.consensus_events),
               sample_blocks=len(pick), sample_frame_json_mb=jbytes / 1e6,
               host_sha256_mb_s=jbytes / 1e6 / max(tsha, 1e-9), checks="FrameHash/blockhash/JSON shape ok")
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


def gossip(a, c, N):
    """per-sync projection latency: the first N - calls * gossip events in one
    call, then `calls` calls of `gossip` events; per call the projection's
    device time (stage_ms[6]) and wall time of RunConsensus, the frames it
    emitted, and every emitted FrameHash checked on the host"""
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    d = Dag.config(a.cfg, N=N, sig_mode=0)
    bodies, bo, sigs, so = d.event_bytes()
    hg = Hashgraph(d.participant_ids, N, frames=True)
    spi, opc, opi = d.wire()
    pid = d.participant_ids
    opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
    L = hg._L
    first = N - a.calls * a.gossip
    bounds = [0, first] + [first + a.gossip * (k + 1) for k in range(a.calls)]
    rows, done = [], 0
    for k, (lo, hi) in enumerate(zip(bounds[:-1], bounds[1:])):
        assert not np.asarray(hg.insert_events(pid[d.creator[lo:hi]], d.index[lo:hi], spi[lo:hi], opc_id[lo:hi],
                                               opi[lo:hi], d.hash[lo:hi], d.sig_r[lo:hi], d.ntx[lo:hi])).any()
        bsl, ssl = np.ascontiguousarray(bo[lo:hi + 1]), np.ascontiguousarray(so[lo:hi + 1])  # absolute offsets
        hg._check(L.bh_set_event_bytes(hg._h, lo, hi - lo, bodies.ctypes.data, bsl.ctypes.data,
                                       sigs.ctypes.data, ssl.ctypes.data))
        t0 = time.perf_counter()
        hg.run_consensus()
        wall = (time.perf_counter() - t0) * 1e3
        st = hg.stats()
        nb = st.blocks - done
        fh, bh, ok = hg.block_hashes(done, nb) if nb else (None, None, None)
        b = hg.blocks()
        jb = 0
        for i in range(nb):
            fj = hg.frame_json(int(b["round_received"][done + i]))
            jb += len(fj)
            assert ok[i] and hashlib.sha256(fj).digest() == fh[i].tobytes(), f"FrameHash of block {done + i}"
            assert hashlib.sha256(hg.block_json(done + i)).digest() == bh[i].tobytes()
        done = st.blocks
        if k:
            rows.append(dict(call=k, new_events=hi - lo, blocks=nb, frame_json_kb=round(jb / 1e3, 1),
                             projection_ms=round(hg.stage_ms()[6], 3), run_consensus_ms=round(wall, 3)))
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    with_b = [r for r in rows if r["blocks"]]
    res = dict(cfg=a.cfg, n=c["n"], N=N, gossip=a.gossip, calls=len(rows), calls_with_blocks=len(with_b),
               frame_hash=os.environ.get("BH_FRAME_HASH", "auto"),
               projection_ms_median=float(np.median([r["projection_ms"] for r in with_b])) if with_b else None,
               projection_ms_max=max((r["projection_ms"] for r in with_b), default=None),
               frame_json_kb_median=float(np.median([r["frame_json_kb"] for r in with_b])) if with_b else None,
               run_consensus_ms_median=float(np.median([r["run_consensus_ms"] for r in rows])),
               checks="every emitted FrameHash / block hash recomputed on the host from the device's JSON")
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
