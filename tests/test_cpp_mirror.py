"""The C++ host mirror (include/babble_hashgraph.hpp) over the C ABI: the
reference's KAT play lists and a seeded gossip DAG replayed through
tests/cpp/hg_replay, which calls InsertEvent / DivideRounds / DecideFame /
DecideRoundReceived / ProcessDecidedRounds the way hashgraph_test.go calls
*Hashgraph.  Results are compared bit-exact with the CPU oracle."""
import os
import subprocess

import numpy as np
import pytest

from kat import KatDag, kat_names
from oracle_py import UNSET, Oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "hg_replay")


def _build():
    subprocess.check_call(["make", "-s", "-C", ROOT, "tests/cpp/hg_replay"])
    return BIN


def test_mirror_builds_and_links():
    """g++ compiles the header-only mirror against libbabble_hip and every
    entry point resolves (no device call)."""
    out = subprocess.run([_build(), "--link-check"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "link ok" in out.stdout, out.stderr


def _playlist(path, ids, cap, creator_id, index, spi, opc, opi, hashes, sigs, ntx, schedule):
    with open(path, "w") as f:
        f.write("ids " + " ".join(str(int(x)) for x in ids) + "\n")
        f.write(f"cap {cap}\n")
        for i in range(len(creator_id)):
            f.write(f"ev {int(creator_id[i])} {int(index[i])} {int(spi[i])} {int(opc[i])} {int(opi[i])} "
                    f"{bytes(hashes[i]).hex()} {bytes(sigs[i]).hex()} {int(ntx[i])}\n")
        for cmd in schedule:
            f.write(cmd + "\n")


def _run(path):
    out = subprocess.run([_build(), path], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    return out.stdout


def _parse(text, N):
    res = dict(round=np.full(N, UNSET, np.int32), witness=np.zeros(N, np.int8),
               lamport=np.full(N, UNSET, np.int32), round_received=np.full(N, UNSET, np.int32),
               fame=np.full(N, -1, np.int8), cons_pos=np.full(N, -1, np.int64))
    blocks, rejects = [], []
    for line in text.splitlines():
        f = line.split()
        if not f:
            continue
        if f[0] == "stats":
            res["stats"] = tuple(int(x) for x in f[1:])
        elif f[0] == "meta":
            i = int(f[1])
            res["round"][i], res["witness"][i], res["lamport"][i] = int(f[2]), int(f[3]), int(f[4])
            res["round_received"][i], res["fame"][i], res["cons_pos"][i] = int(f[5]), int(f[6]), int(f[7])
        elif f[0] == "order":
            res["order"] = np.array([int(x) for x in f[1:]], np.int32)
        elif f[0] == "pending":
            res["pending"] = [(int(p.split(":")[0]), p.split(":")[1] == "1") for p in f[1:]]
        elif f[0] == "undetermined":
            res["undetermined"] = np.array([int(x) for x in f[1:]], np.int32)
        elif f[0] == "block":
            blocks.append([int(x) for x in f[1:]])
        elif f[0] == "reject":
            rejects.append((int(f[1]), int(f[2])))
    b = np.array(blocks, np.int64).reshape(-1, 5)
    res["blocks"] = dict(round_received=b[:, 1], first=b[:, 2], count=b[:, 3], ntx=b[:, 4])
    res["rejects"] = rejects
    return res


def _compare(o, got, where):
    ref = o.results()
    for k in ("round", "witness", "lamport", "round_received", "cons_pos"):
        bad = np.nonzero(ref[k] != got[k])[0]
        assert len(bad) == 0, f"{where} {k}: {bad[:8]} ref={ref[k][bad[:8]]} got={got[k][bad[:8]]}"
    fr = np.where(ref["witness"] == 1, ref["fame"], -1)
    assert np.array_equal(fr, got["fame"]), where
    assert np.array_equal(o.consensus_order(), got["order"]), where
    ob = o.blocks()
    for k in ("round_received", "first", "count", "ntx"):
        assert np.array_equal(ob[k], got["blocks"][k]), f"{where} blocks.{k}"
    assert o.pending_rounds() == got["pending"], where
    lcr = o.last_consensus_round()
    assert got["stats"] == (lcr, o.consensus_transactions(), o.pending_loaded_events(), o.last_round()), where
    assert np.array_equal(o.undetermined(), got["undetermined"]), where


def _kat_wire(d):
    pid = d.participant_ids
    spi = np.where(d.sp >= 0, d.index - 1, -1)
    opc = np.where(d.op >= 0, pid[d.creator[np.maximum(d.op, 0)]], -1)
    opi = np.where(d.op >= 0, d.index[np.maximum(d.op, 0)], -1)
    return pid[d.creator], d.index, spi, opc, opi


@pytest.mark.gpu
@pytest.mark.parametrize("name", [k for k in kat_names() if k != "kat_fork"])
def test_cpp_mirror_kat(name, tmp_path):
    d = KatDag(name)
    o = Oracle(d.n, d.participant_ids, capacity=len(d) + 64)
    o.insert_dag(d.creator, d.index, d.sp, d.op, d.hashes, d.sig_r, d.ntx)
    o.run_consensus()
    cr, idx, spi, opc, opi = _kat_wire(d)
    p = str(tmp_path / "kat.txt")
    _playlist(p, d.participant_ids, len(d) + 64, cr, idx, spi, opc, opi, d.hashes, d.sig_r, d.ntx,
              ["insert", "divide", "fame", "received", "process", "dump"])
    got = _parse(_run(p), len(d))
    assert not got["rejects"]
    _compare(o, got, name)


@pytest.mark.gpu
def test_cpp_mirror_fork_rejected(tmp_path):
    """TestFork (hashgraph_test.go:351-398) through InsertEvent's error path."""
    d = KatDag("kat_fork")
    cr, idx, spi, opc, opi = _kat_wire(d)
    pid = d.participant_ids
    # append a fork of node 2 (index 0 again) and an event with an unknown other-parent
    cr = np.append(cr, [pid[2], pid[0]])
    idx = np.append(idx, [0, 1])
    spi = np.append(spi, [-1, 0])
    opc = np.append(opc, [-1, pid[2]])
    opi = np.append(opi, [-1, 1])
    z = np.zeros((2, 32), np.uint8)
    p = str(tmp_path / "fork.txt")
    _playlist(p, pid, 64, cr, idx, spi, opc, opi, np.vstack([d.hashes, z]), np.vstack([d.sig_r, z]),
              np.append(d.ntx, [1, 0]), ["insert", "run", "dump"])
    got = _parse(_run(p), len(d))
    kinds = dict(got["rejects"])
    n0 = len(d)
    assert set(kinds) == {n0, n0 + 1}
    assert kinds[n0] in (1, 4)   # BH_ERR_SELF_PARENT / BH_ERR_SKIPPED_INDEX
    assert kinds[n0 + 1] == 2    # BH_ERR_OTHER_PARENT


@pytest.mark.gpu
def test_cpp_mirror_random_dag(tmp_path):
    """A 16-peer gossip DAG, inserted in two batches with a RunConsensus in
    between (the Core schedule), then checked against the batch oracle."""
    from babble_amd.dag import Dag
    n, N = 16, 8000
    d = Dag(n, N, 0xC0FFEE, sig_mode=0)
    o = Oracle(n, d.participant_ids, capacity=N)
    o.insert_dag(d.creator, d.index, d.self_parent, d.other_parent, d.hash, d.sig_r, d.ntx)
    o.run_consensus()
    spi, opc_slot, opi = d.wire()
    pid = d.participant_ids
    opc = np.where(opc_slot >= 0, pid[np.maximum(opc_slot, 0)], -1)
    p = str(tmp_path / "rand.txt")
    half = N // 2
    with open(p, "w") as f:
        f.write("ids " + " ".join(str(int(x)) for x in pid) + f"\ncap {N}\n")

        def evs(lo, hi):
            for i in range(lo, hi):
                f.write(f"ev {int(pid[d.creator[i]])} {int(d.index[i])} {int(spi[i])} {int(opc[i])} "
                        f"{int(opi[i])} {bytes(d.hash[i]).hex()} {bytes(d.sig_r[i]).hex()} {int(d.ntx[i])}\n")
        evs(0, half)
        f.write("insert\nrun\n")
        evs(half, N)
        f.write("insert\nrun\ndump\n")
    got = _parse(_run(p), N)
    assert not got["rejects"]
    _compare(o, got, "cpp random")
