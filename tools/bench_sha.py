"""Throughput of the insert-side crypto on the device:
bh_hash_bodies (SHA-256 of Go-JSON event bodies) against hashlib on one host
core, and bh_verify_signatures (ECDSA P-256) on real signatures.  Two JSON
lines.  usage: python tools/bench_sha.py [--events N] [--reps R] [--sigs M]"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=400_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sigs", type=int, default=50_000)
    a = ap.parse_args()
    from babble_amd import Hashgraph
    from babble_amd.dag import Dag
    d = Dag(128, a.events, 0xBABB1E03, sig_mode=0)
    bodies = [d.body_json(e) for e in range(a.events)]
    nbytes = sum(len(b) for b in bodies)
    hg = Hashgraph(np.asarray(d.participant_ids), 64)
    out = hg.hash_bodies(bodies)  # warm-up (allocates the device buffer)
    assert np.array_equal(out, d.hash[:a.events])
    t0 = time.perf_counter()
    for _ in range(a.reps):
        hg.hash_bodies(bodies)
    dt = (time.perf_counter() - t0) / a.reps
    sample = bodies[:50_000]
    t1 = time.perf_counter()
    for b in sample:
        hashlib.sha256(b).digest()
    cpu = len(sample) / (time.perf_counter() - t1)
    print(json.dumps({"metric": "event bodies hashed/sec (SHA-256, host buffers in and out)",
                      "value": a.events / dt, "unit": "bodies/s", "bytes": nbytes,
                      "gb_per_s_pcie_inclusive": nbytes / dt / 1e9,
                      "cpu_hashlib_1core": cpu, "events": a.events}))
    if a.sigs > 0:
        ds = Dag(128, a.sigs, 0xBABB1E03, sig_mode=1)
        pub = np.ascontiguousarray(ds.pubkeys[:, 1:65])
        keys = ds.creator.astype(np.int32)
        ok = hg.verify_signatures(ds.hash, ds.sig_r, ds.sig_s, keys, pub)
        assert ok.all()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            hg.verify_signatures(ds.hash, ds.sig_r, ds.sig_s, keys, pub)
        dt = (time.perf_counter() - t0) / a.reps
        print(json.dumps({"metric": "event signatures verified/sec (ECDSA P-256, host buffers in and out)",
                          "value": a.sigs / dt, "unit": "signatures/s", "signatures": a.sigs}))


if __name__ == "__main__":
    main()
