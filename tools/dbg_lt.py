"""debug: Lamport timestamps of a wild DAG through the segment pipeline vs the oracle"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from oracle_py import Oracle
from test_gpu_parity import _wild_dag
from babble_amd import Hashgraph
n, N = 24, 30000
creator, index, sp, op, hashes, sig, ntx = _wild_dag(n, N, 73, 20000)
pid = np.arange(1, n + 1, dtype=np.int64) * 1000
o = Oracle(n, pid, capacity=N); o.insert_dag(creator, index, sp, op, hashes, sig, ntx); o.run_consensus()
hg = Hashgraph(pid, N)
spi = np.where(sp >= 0, index - 1, -1); opc = np.where(op >= 0, pid[creator[np.maximum(op, 0)]], -1); opi = np.where(op >= 0, index[np.maximum(op, 0)], -1)
hg.insert_events(pid[creator], index, spi, opc, opi, hashes, sig, ntx)
hg.run_consensus()
ref, got = o.results()["lamport"], hg.results()["lamport"]
bad = np.nonzero(ref != got)[0]
print(os.environ.get("TAG", ""), "lamport mismatches", len(bad), bad[:5], ref[bad[:5]], got[bad[:5]], "max ref", ref.max())
