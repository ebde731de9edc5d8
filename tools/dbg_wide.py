"""Debug aid (round 4): the wide loop over la_col against the oracle on one
DAG; prints the first round boundary B[r][c] that differs.  The variant is
chosen by the environment (BH_ROUND_P8, BH_ROUND_P8G, BH_WIDE_ROWS, ...)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle_py import Oracle  # noqa: E402
from babble_amd import Hashgraph  # noqa: E402
from babble_amd.dag import Dag  # noqa: E402

n, N, seed = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (200, 30000, 74)))
tag = os.environ.get("TAG", "")
d = Dag(n, N, seed, sig_mode=0)
o = Oracle(n, d.participant_ids, capacity=N)
o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
o.run_consensus()
hg = Hashgraph(d.participant_ids, N)
assert not hg.insert_dag(d).any()
hg.run_consensus()
ref, got = o.results()["round"], hg.results()["round"]


def bounds(rnd):
    R = int(rnd.max()) + 1
    B = np.zeros((R + 1, n), np.int64)
    for c in range(n):
        idx = np.nonzero(d.creator == c)[0]
        rr = rnd[idx[np.argsort(d.index[idx])]]
        for r in range(R + 1):
            B[r, c] = np.searchsorted(rr, r)
    return B


bad = np.nonzero(ref != got)[0]
print(tag, "round mismatches", len(bad), "lamport mismatches", int((o.results()["lamport"] != hg.results()["lamport"]).sum()))
if len(bad):
    Br, Bg = bounds(ref), bounds(got)
    R = min(len(Br), len(Bg))
    diff = np.argwhere(Br[:R] != Bg[:R])
    r0 = int(diff[0][0])
    cs = diff[diff[:, 0] == r0][:, 1]
    print(tag, "first differing round", r0, "chains", cs[:10].tolist(), "ref", Br[r0, cs[:10]].tolist(), "got", Bg[r0, cs[:10]].tolist(),
          "prev ref", Br[r0 - 1, cs[:10]].tolist())
