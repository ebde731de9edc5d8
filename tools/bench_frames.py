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
    a = ap.parse_args()
    from babble_amd import Hashgraph
    from babble_amd.dag import CONFIGS, Dag
    c = CONFIGS[a.cfg]
    N = a.N or c["N"]
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


if __name__ == "__main__":
    main()
