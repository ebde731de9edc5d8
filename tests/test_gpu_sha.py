"""Insert-side hashing on the device: Event.Hash() =
SHA-256 of the Go-JSON body (event.go:50-56) for a batch of events, against
hashlib and the generator's digests (which tests/test_host.py pins to
Python json + hashlib).  Bit-exact."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _hg(n=4):
    from babble_amd import Hashgraph
    return Hashgraph(np.arange(1, n + 1, dtype=np.int64) * 7919, 64)


def test_sha256_padding_boundaries():
    """Every length around the 55/56/64-byte padding edges, empty input,
    multi-block messages and unaligned offsets."""
    rng = np.random.default_rng(5)
    lens = list(range(0, 140)) + [183, 255, 256, 511, 1000, 4097]
    bodies = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    got = _hg().hash_bodies(bodies)
    for b, g in zip(bodies, got):
        assert g.tobytes() == hashlib.sha256(b).digest(), len(b)


def test_sha256_event_bodies():
    """Go-JSON event bodies of a generated DAG: the digests InsertEvent uses."""
    from babble_amd.dag import Dag
    d = Dag(8, 3000, 91, sig_mode=1)
    ids = list(range(0, 3000, 7))
    bodies = [d.body_json(e) for e in ids]
    got = _hg(8).hash_bodies(bodies)
    for e, b, g in zip(ids, bodies, got):
        assert g.tobytes() == hashlib.sha256(b).digest()
        assert np.array_equal(g, d.hash[e]), e


def test_sha256_empty_batch():
    assert _hg().hash_bodies([]).shape == (0, 32)


def _ecdsa_inputs(n=8, N=2000, seed=93):
    from babble_amd.dag import Dag
    d = Dag(n, N, seed, sig_mode=1)
    pub = np.ascontiguousarray(d.pubkeys[:, 1:65])  # drop the 0x04 prefix
    return d, pub


def test_ecdsa_verify_generator_signatures():
    """Every event signature of a sig_mode=1 DAG verifies (real ECDSA P-256
    signatures over the body digests, pinned by test_host's pure-Python
    verify); the same signatures checked against the wrong key, a flipped
    hash bit, a perturbed s, and out-of-range r / s do not."""
    d, pub = _ecdsa_inputs()
    hg = _hg(8)
    keys = d.creator.astype(np.int32)
    ok = hg.verify_signatures(d.hash, d.sig_r, d.sig_s, keys, pub)
    assert ok.all(), np.nonzero(~ok)[0][:10]
    bad_key = hg.verify_signatures(d.hash, d.sig_r, d.sig_s, (keys + 1) % 8, pub)
    assert not bad_key.any()
    h2 = d.hash.copy()
    h2[:, 31] ^= 1
    assert not hg.verify_signatures(h2, d.sig_r, d.sig_s, keys, pub).any()
    s2 = d.sig_s.copy()
    s2[:, 31] ^= 4
    assert not hg.verify_signatures(d.hash, d.sig_r, s2, keys, pub).any()
    q = bytes.fromhex("FFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551")
    edge = np.zeros((4, 32), np.uint8)
    edge[1] = np.frombuffer(q, np.uint8)  # r = n
    edge[2, 31] = 1
    edge[3] = 0xFF
    for e in range(4):  # r or s in {0, n, 1 (wrong), 2^256-1}
        rr = np.repeat(edge[e:e + 1], 4, 0)
        assert not hg.verify_signatures(d.hash[:4], rr, d.sig_s[:4], keys[:4], pub).any()
        assert not hg.verify_signatures(d.hash[:4], d.sig_r[:4], rr, keys[:4], pub).any()
