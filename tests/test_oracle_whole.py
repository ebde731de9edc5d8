"""The whole-DAG digests' own pins (CPU): the 16-bit-storage oracle build
that made whole_c4.json agrees with the default build, the digest of a run
equals itself across processes, and the committed fixtures describe the
DAGs bench.py times."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")

_SCRIPT = """
import json, os, sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
from babble_amd.dag import Dag
from digest import oracle_digest
from oracle_py import Oracle
d = Dag({n}, {N}, {seed}, lagging={lag}, sig_mode=0)
o = Oracle(d.n, d.participant_ids, capacity=d.N)
o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
o.run_consensus()
print(json.dumps(oracle_digest(o)))
"""


def _digest_with(lib, n, N, seed, lag):
    env = dict(os.environ)
    if lib:
        env["BH_ORACLE_LIB"] = os.path.join(ROOT, "oracle", lib)
    out = subprocess.run([sys.executable, "-c", _SCRIPT.format(root=ROOT, tests=HERE, n=n, N=N, seed=seed, lag=lag)],
                         env=env, check=True, capture_output=True, text=True).stdout
    return json.loads(out)


@pytest.mark.parametrize("n,N,seed,lag", [(8, 20_000, 7, 2), (64, 60_000, 8, 21), (160, 40_000, 9, 0)])
def test_coord16_build_matches(n, N, seed, lag):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle.so", "liboracle16.so"])
    a = _digest_with(None, n, N, seed, lag)
    b = _digest_with("liboracle16.so", n, N, seed, lag)
    assert a == b
    assert a["n_ordered"] > 0.5 * N


@pytest.mark.parametrize("name,cfg", [("c3", 3), ("c4", 4)])
def test_whole_fixtures(name, cfg):
    from babble_amd.dag import CONFIGS
    path = os.path.join(GOLDEN, f"whole_{name}.json")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated yet")
    with open(path) as f:
        fx = json.load(f)
    c = CONFIGS[cfg]
    assert fx["spec"]["cfg"] == cfg and fx["spec"]["n"] == c["n"] and fx["spec"]["N"] == c["N"]
    assert fx["events"] == c["N"] and len(fx["round"]) == (c["N"] + fx["chunk"] - 1) // fx["chunk"]
    assert fx["n_ordered"] > 0.9 * c["N"] and fx["n_blocks"] > 1000
