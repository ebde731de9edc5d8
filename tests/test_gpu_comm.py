"""The multi-process shard group, every rank a process of its own on device 0,
exchanging over the host transport (bh_comm_init_transport) on a torch gloo
group: the same exchange calls at the same sites as the RCCL group of
bench.py --gpus N (rank 0's base broadcast; the coordinate split's
per-segment all-gather at n <= 128 -- one broadcast per coordinate rank --
or its sends to rank 0 at n > 128; the sharded passes' broadcasts per
owner), through the segment pipeline and incremental calls.  Rank 0's state
equals the oracle's after every call (tests/comm_rank.py) -- the reference's
cross-node agreement check (node/core_test.go:361-380) with rank 0 as the
node -- and every rank that holds results ends with the same digest of its
whole state: at n <= 128 every rank ran the loop and a share of the fame
rounds and frame sorts; the coordinate ranks of a wide split refuse result
queries.

"default" runs without BH_SHARD_COORDS: the mode bench.py --gpus N gets
(the split from 3 ranks at n <= 128 and from 4 at n = 512, replicated
coordinates below; fame rounds and frame sorts sharded wherever every rank
holds the rounds).

A block that runs out of overflow slots (BH_SPLIT_RANGE=2: every 64-row
chunk spans more than its 16-bit range) sends the receiving ranks to the
unsplit path mid-call: every segment's exchange is still posted, so no
rank's broadcast or send is left unmatched (the call would hang otherwise)
and the next call runs collectively again.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode,world,n,N,lag,K,step,env", [
    ("default", 2, 128, 60_000, 0, 3, 20_000, {}),  # bench.py's mode at 2 ranks: replicated, passes sharded
    ("default", 3, 128, 40_000, 0, 4, 20_000, {}),  # from 3 ranks: the split, every rank in the loop
    ("default", 4, 128, 40_000, 0, 4, 20_000, {}),
    ("split", 2, 128, 60_000, 0, 3, 20_000, {}),
    ("split", 3, 64, 50_000, 21, 4, 10_000, {}),
    ("split", 3, 32, 30_000, 4, 3, 10_000, {"BH_SPLIT_RANGE": "2"}),  # overflow: unsplit, exchanges matched
    ("split", 3, 32, 30_000, 4, 3, 10_000, {"BH_SPLIT_RANGE": "2", "BH_SPLIT_RANGE_SEG": "2"}),  # a later one
    ("split", 2, 96, 40_000, 3, 3, 8_000, {"BH_ROUND_PERSIST": "0"}),  # loops that wait per segment
    ("split", 3, 160, 30_000, 2, 3, 10_000, {}),  # the wide split: k_floww2 on ranks 1-2, transposes on rank 0
    ("default", 4, 512, 30_000, 0, 3, 15_000, {}),  # n = 512 from 4 ranks: the wide split
    ("default", 2, 512, 30_000, 0, 3, 15_000, {}),  # n = 512 below 4 ranks: replicated, fame / sorts sharded
    ("replicate", 2, 64, 40_000, 3, 3, 10_000, {}),
    ("columns", 2, 32, 30_000, 0, 1, 15_000, {}),
])
def test_multiprocess_group(tmp_path, mode, world, n, N, lag, K, step, env):
    port = _free_port()
    e = dict(os.environ, BH_SEGMENTS=str(K), MASTER_ADDR="127.0.0.1", **env)
    e.pop("BH_SHARD_COORDS", None)
    if mode != "default":
        e["BH_SHARD_COORDS"] = mode
    procs, outs = [], []
    for r in range(world):
        out = tmp_path / f"rank{r}.json"
        outs.append(out)
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(HERE, "comm_rank.py"), "--rank", str(r), "--world", str(world),
             "--port", str(port), "--n", str(n), "--N", str(N), "--seed", str(0xC0 + n), "--lag", str(lag),
             "--step", str(step), "--out", str(out)], env=e))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=420))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail(f"{mode} x{world}: a rank hung (unmatched exchange?)")
    res = [json.loads(o.read_text()) if o.exists() else {"error": "no report"} for o in outs]
    for r, (rc, x) in enumerate(zip(rcs, res)):
        assert rc == 0 and x.get("ok"), f"rank {r}: {x.get('error')}"
    r0 = res[0]
    assert r0["calls"] == (N + step - 1) // step
    assert r0["consensus_events"] > 0
    split = mode == "split" or (mode == "default" and ((n <= 128 and world >= 3) or world >= 4))
    wide_split = split and n > 128
    if split and not env:  # (an overflowed call ends on the unsplit path, which exchanges nothing)
        assert r0["exchange_ms"] > 0  # rank 0's receive windows ran
    for x in res[1:]:
        if wide_split:  # the coordinate ranks of a wide split hold no results
            assert x["stats"].startswith("refused") and x["pending_rounds"].startswith("refused"), x
        else:  # every rank ran the loop: the same state everywhere
            assert x["stats"] == "returned", x
            assert x["digest"] == r0["digest"], f"rank {x['rank']} differs from rank 0"
