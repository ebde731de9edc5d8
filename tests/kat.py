"""Known-answer DAG fixtures (tests/golden/kat_*.json) as event arrays."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class KatDag:
    """A transcribed play list.  Hashes and signatures are synthetic: the
    reference tests use random keys, so no assertion depends on them; they
    are fixed here as SHA-256 of the event name."""

    def __init__(self, name):
        with open(os.path.join(GOLDEN, name + ".json")) as f:
            self.fx = json.load(f)
        self.n = self.fx["n"]
        self.expect = self.fx["expect"]
        self.names = []
        self.id_of = {}
        creator, index, sp, op, ntx, txs = [], [], [], [], [], []
        for c, k, spn, opn, name, tx in self.fx["events"]:
            self.id_of[name] = len(self.names)
            self.names.append(name)
            creator.append(c)
            index.append(k)
            sp.append(self.id_of[spn] if spn else -1)
            op.append(self.id_of[opn] if opn else -1)
            ntx.append(len(tx) if tx else 0)
            txs.append(tx or [])
        self.creator = np.array(creator, np.int32)
        self.index = np.array(index, np.int32)
        self.sp = np.array(sp, np.int32)
        self.op = np.array(op, np.int32)
        self.ntx = np.array(ntx, np.int32)
        self.txs = txs
        self.hashes = np.stack([np.frombuffer(hashlib.sha256(n.encode()).digest(), np.uint8)
                                for n in self.names])
        self.sig_r = np.stack([np.frombuffer(hashlib.sha256(b"r" + n.encode()).digest(), np.uint8)
                               for n in self.names])
        self.participant_ids = np.arange(1, self.n + 1, dtype=np.int64) * 1000

    def __len__(self):
        return len(self.names)

    def ids(self, names):
        return [self.id_of[x] for x in names]


def kat_names():
    return sorted(f[:-5] for f in os.listdir(GOLDEN) if f.startswith("kat_") and f.endswith(".json"))
