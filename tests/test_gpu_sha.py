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
