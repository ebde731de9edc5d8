"""Writes tests/golden/kat_*.json: the known-answer DAGs of the reference's
hashgraph tests, transcribed as data (play lists + asserted values).

Source: /root/reference/src/hashgraph/hashgraph_test.go.  Each play is
(creator slot, index, self-parent name, other-parent name, event name, txs),
exactly the `play` struct of hashgraph_test.go:69-77; creator slot i means
the i-th participant in ID-sorted order (hashgraph_test.go:101-103,147-150).
The reference uses random keys, so hashes/signatures are not part of any
assertion; the fixtures only carry names.  Expected values are transcribed
from the cited assertions.  Run: python tests/golden/make_kat_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def initial(n, txs_from_name=False, prefix="e", fmt="{p}{i}"):
    out = []
    for i in range(n):
        name = fmt.format(p=prefix, i=i)
        out.append([i, 0, None, None, name, [name] if txs_from_name else None])
    return out


def play(to, index, sp, op, name, txs=None):
    return [to, index, sp or None, op or None, name, txs]


# Root / RootEvent (root.go:65-96) by name: a RootEvent is [event name or
# "Root" (the base root event NewBaseRootEvent, root.go:73-84), creator slot,
# Index, LamportTimestamp, Round]; next_round None = not asserted
def root(next_round, self_parent, others):
    return {"next_round": next_round, "self_parent": self_parent, "others": others}


def base_root(slot, next_round=0):
    return root(next_round, ["Root", slot, -1, -1, -1], {})


FIXTURES = {}

# --- initHashgraph, hashgraph_test.go:161-202 ------------------------------
FIXTURES["kat_hashgraph"] = {
    "source": "hashgraph_test.go:161-202 (initHashgraph)",
    "n": 3,
    "events": initial(3) + [
        play(0, 1, "e0", "e1", "e01"),
        play(2, 1, "e2", "", "s20"),
        play(1, 1, "e1", "", "s10"),
        play(0, 2, "e01", "", "s00"),
        play(2, 2, "s20", "s00", "e20"),
        play(1, 2, "s10", "e20", "e12"),
    ],
    "expect": {
        # TestAncestor hashgraph_test.go:204-249 (the "" ancestor rows are
        # error cases on a missing key; they have no counterpart with ids)
        "ancestor": [
            ["e01", "e0", True], ["e01", "e1", True], ["s00", "e01", True],
            ["s20", "e2", True], ["e20", "s00", True], ["e20", "s20", True],
            ["e12", "e20", True], ["e12", "s10", True],
            ["s00", "e0", True], ["s00", "e1", True], ["e20", "e01", True],
            ["e20", "e2", True], ["e12", "e1", True], ["e12", "s20", True],
            ["e20", "e0", True], ["e20", "e1", True], ["e20", "e2", True],
            ["e12", "e01", True], ["e12", "e0", True], ["e12", "e1", True],
            ["e12", "e2", True],
            ["e01", "e2", False], ["s00", "e2", False],
        ],
        # TestSelfAncestor hashgraph_test.go:251-281
        "self_ancestor": [
            ["e01", "e0", True], ["s00", "e01", True],
            ["e01", "e1", False], ["e12", "e20", False], ["s20", "e1", False],
            ["e20", "e2", True], ["e12", "e1", True],
            ["e20", "e0", False], ["e12", "e2", False], ["e20", "e01", False],
        ],
        # TestSee hashgraph_test.go:283-306
        "see": [
            ["e01", "e0", True], ["e01", "e1", True], ["e20", "e0", True],
            ["e20", "e01", True], ["e12", "e01", True], ["e12", "e0", True],
            ["e12", "e1", True], ["e12", "s20", True],
        ],
        # TestLamportTimestamp hashgraph_test.go:308-332
        "lamport": {"e0": 0, "e1": 0, "e2": 0, "e01": 1, "s10": 1, "s20": 1,
                    "s00": 2, "e20": 3, "e12": 4},
    },
}

# --- initRoundHashgraph, hashgraph_test.go:400-434 --------------------------
MAX = 2147483647
FIXTURES["kat_round"] = {
    "source": "hashgraph_test.go:400-434 (initRoundHashgraph)",
    "n": 3,
    "events": initial(3) + [
        play(1, 1, "e1", "e0", "e10"),
        play(2, 1, "e2", "", "s20"),
        play(0, 1, "e0", "", "s00"),
        play(2, 2, "s20", "e10", "e21"),
        play(0, 2, "s00", "e21", "e02"),
        play(1, 2, "e10", "", "s10"),
        play(1, 3, "s10", "e02", "f1"),
        play(1, 4, "f1", "", "s11", ["abc"]),
    ],
    "expect": {
        # TestInsertEvent "Check Event Coordinates" hashgraph_test.go:439-543
        "coordinates": {
            "e0": {"fd": [0, 1, 2], "la": [0, -1, -1]},
            "e21": {"fd": [2, 3, 2], "la": [0, 1, 2]},
            "f1": {"fd": [MAX, 3, MAX], "la": [2, 3, 2]},
        },
        # TestInsertEvent "Check UndeterminedEvents" hashgraph_test.go:545-573
        "undetermined_after_insert": ["e0", "e1", "e2", "e10", "s20", "s00",
                                      "e21", "e02", "s10", "f1", "s11"],
        "pending_loaded_after_insert": 4,
        # TestStronglySee hashgraph_test.go:611-643
        "strongly_see": [
            ["e21", "e0", True], ["e02", "e10", True], ["e02", "e0", True],
            ["e02", "e1", True], ["f1", "e21", True], ["f1", "e10", True],
            ["f1", "e0", True], ["f1", "e1", True], ["f1", "e2", True],
            ["s11", "e2", True],
            ["e10", "e0", False], ["e21", "e1", False], ["e21", "e2", False],
            ["e02", "e2", False], ["s11", "e02", False],
        ],
        # TestWitness hashgraph_test.go:645-677
        "witness": {"e0": True, "e1": True, "e2": True, "f1": True,
                    "e10": False, "e21": False, "e02": False},
        # TestRound hashgraph_test.go:679-711
        "round": {"e0": 0, "e1": 0, "e2": 0, "s00": 0, "e10": 0, "s20": 0,
                  "e21": 0, "e02": 0, "s10": 0, "f1": 1, "s11": 1},
        # TestRoundDiff hashgraph_test.go:713-741
        "round_diff": [["f1", "e02", 1], ["e02", "f1", -1], ["e02", "e21", 0]],
        # TestDivideRounds hashgraph_test.go:743-829
        "divide_rounds": {
            "last_round": 1,
            "witnesses": {"0": ["e0", "e1", "e2"], "1": ["f1"]},
            "pending_rounds": [[0, False], [1, False]],
            "lamport_round": {"e0": [0, 0], "e1": [0, 0], "e2": [0, 0],
                              "s00": [1, 0], "e10": [1, 0], "s20": [1, 0],
                              "e21": [2, 0], "e02": [3, 0], "s10": [2, 0],
                              "f1": [4, 1], "s11": [5, 1]},
        },
    },
}

# --- initConsensusHashgraph, hashgraph_test.go:1120-1205 --------------------
FIXTURES["kat_consensus"] = {
    "source": "hashgraph_test.go:1120-1205 (initConsensusHashgraph)",
    "n": 3,
    "events": initial(3) + [
        play(1, 1, "e1", "e0", "e10"),
        play(2, 1, "e2", "e10", "e21", ["e21"]),
        play(2, 2, "e21", "", "e21b"),
        play(0, 1, "e0", "e21b", "e02"),
        play(1, 2, "e10", "e02", "f1"),
        play(1, 3, "f1", "", "f1b", ["f1b"]),
        play(0, 2, "e02", "f1b", "f0"),
        play(2, 3, "e21b", "f1b", "f2"),
        play(1, 4, "f1b", "f0", "f10"),
        play(0, 3, "f0", "e21", "f0x"),
        play(2, 4, "f2", "f10", "f21"),
        play(0, 4, "f0x", "f21", "f02"),
        play(0, 5, "f02", "", "f02b", ["f02b"]),
        play(1, 5, "f10", "f02b", "g1"),
        play(0, 6, "f02b", "g1", "g0"),
        play(2, 5, "f21", "g1", "g2"),
        play(1, 6, "g1", "g0", "g10", ["g10"]),
        play(2, 6, "g2", "g10", "g21"),
        play(0, 7, "g0", "g21", "g02", ["g02"]),
        play(1, 7, "g10", "g02", "h1"),
        play(0, 8, "g02", "h1", "h0"),
        play(2, 7, "g21", "h1", "h2"),
        play(1, 8, "h1", "h0", "h10"),
        play(2, 8, "h2", "h10", "h21"),
        play(0, 9, "h0", "h21", "h02"),
        play(1, 9, "h10", "h02", "i1"),
        play(0, 10, "h02", "i1", "i0"),
        play(2, 9, "h21", "i1", "i2"),
    ],
    "expect": {
        # TestDivideRoundsBis hashgraph_test.go:1207-1265
        "lamport_round": {
            "e0": [0, 0], "e1": [0, 0], "e2": [0, 0], "e10": [1, 0],
            "e21": [2, 0], "e21b": [3, 0], "e02": [4, 0], "f1": [5, 1],
            "f1b": [6, 1], "f0": [7, 1], "f2": [7, 1], "f10": [8, 1],
            "f0x": [8, 1], "f21": [9, 1], "f02": [10, 1], "f02b": [11, 1],
            "g1": [12, 2], "g0": [13, 2], "g2": [13, 2], "g10": [14, 2],
            "g21": [15, 2], "g02": [16, 2], "h1": [17, 3], "h0": [18, 3],
            "h2": [18, 3], "h10": [19, 3], "h21": [20, 3], "h02": [21, 3],
            "i1": [22, 4], "i0": [23, 4], "i2": [23, 4]},
        # TestDecideFame hashgraph_test.go:1267-1344
        "famous": {"e0": True, "e1": True, "e2": True, "f0": True, "f1": True,
                   "f2": True, "g0": True, "g1": True, "g2": True},
        "pending_after_fame": [[0, True], [1, True], [2, True], [3, False], [4, False]],
        # TestDecideRoundReceived hashgraph_test.go:1346-1417: names starting
        # with e -> 1, f -> 2, everything else nil
        "round_received_by_prefix": {"e": 1, "f": 2},
        "consensus_events_per_round": {"0": 0, "1": 7, "2": 9},
        "undetermined_after_rr": ["g1", "g0", "g2", "g10", "g21", "g02", "h1",
                                  "h0", "h2", "h10", "h21", "h02", "i1", "i0", "i2"],
        # TestProcessDecidedRounds hashgraph_test.go:1419-1520
        "consensus_len": 16,
        "pending_loaded": 2,
        "blocks": [{"index": 0, "round_received": 1, "txs": ["e21"]},
                   {"index": 1, "round_received": 2, "ntx": 2, "tx1": "f02b"}],
        "pending_after_process": [[3, False], [4, False]],
        # TestGetFrame hashgraph_test.go:1555-1709 (frame event sets; the test
        # compares against the same set sorted ByLamportTimestamp)
        "frame_events": {
            "1": ["e0", "e1", "e2", "e10", "e21", "e21b", "e02"],
            "2": ["f1", "f1b", "f0", "f2", "f10", "f0x", "f21", "f02", "f02b"]},
        # TestKnown hashgraph_test.go:1536-1553
        "known": [10, 9, 9],
        # TestGetFrame hashgraph_test.go:1565-1670: the roots of frames 1 and
        # 2 (SelfParent and Others; the test does not compare NextRound)
        "frame_roots": {
            "1": [base_root(0, None), base_root(1, None), base_root(2, None)],
            "2": [root(None, ["e02", 0, 1, 4, 0],
                       {"f0": ["f1b", 1, 3, 6, 1], "f0x": ["e21", 2, 1, 2, 0]}),
                  root(None, ["e10", 1, 1, 1, 0], {"f1": ["e02", 0, 1, 4, 0]}),
                  root(None, ["e21b", 2, 2, 3, 0], {"f2": ["f1b", 1, 3, 6, 1]})]},
    },
}

# --- initFunkyHashgraph, hashgraph_test.go:1969-2079 ------------------------
_funky = [
    play(2, 1, "w02", "w03", "a23", ["a23"]),
    play(1, 1, "w01", "a23", "a12", ["a12"]),
    play(0, 1, "w00", "", "a00", ["a00"]),
    play(1, 2, "a12", "a00", "a10", ["a10"]),
    play(2, 2, "a23", "a12", "a21", ["a21"]),
    play(3, 1, "w03", "a21", "w13", ["w13"]),
    play(2, 3, "a21", "w13", "w12", ["w12"]),
    play(1, 3, "a10", "w12", "w11", ["w11"]),
    play(0, 2, "a00", "w11", "w10", ["w10"]),
    play(2, 4, "w12", "w11", "b21", ["b21"]),
    play(3, 2, "w13", "b21", "w23", ["w23"]),
    play(1, 4, "w11", "w23", "w21", ["w21"]),
    play(0, 3, "w10", "", "b00", ["b00"]),
    play(1, 5, "w21", "b00", "c10", ["c10"]),
    play(2, 5, "b21", "c10", "w22", ["w22"]),
    play(0, 4, "b00", "w22", "w20", ["w20"]),
    play(1, 6, "c10", "w20", "w31", ["w31"]),
    play(2, 6, "w22", "w31", "w32", ["w32"]),
    play(0, 5, "w20", "w32", "w30", ["w30"]),
    play(3, 3, "w23", "w32", "w33", ["w33"]),
    play(1, 7, "w31", "w33", "d13", ["d13"]),
    play(0, 6, "w30", "d13", "w40", ["w40"]),
    play(1, 8, "d13", "w40", "w41", ["w41"]),
    play(2, 7, "w32", "w41", "w42", ["w42"]),
    play(3, 4, "w33", "w42", "w43", ["w43"]),
]
_funky_full = [
    play(2, 8, "w42", "w43", "e23", ["e23"]),
    play(1, 9, "w41", "e23", "w51", ["w51"]),
]
FIXTURES["kat_funky"] = {
    "source": "hashgraph_test.go:1969-2153 (initFunkyHashgraph, full=false)",
    "n": 4,
    "events": initial(4, True, "w0", "{p}{i}") + _funky,
    "expect": {
        # TestFunkyHashgraphFame hashgraph_test.go:2081-2153: rounds 1 and 2
        # are decided before round 0; Process must not touch the queue
        "last_round": 4,
        "pending_after_fame": [[0, False], [1, True], [2, True], [3, False], [4, False]],
        "pending_after_process": [[0, False], [1, True], [2, True], [3, False], [4, False]],
    },
}
FIXTURES["kat_funky_full"] = {
    "source": "hashgraph_test.go:1969-2223 (initFunkyHashgraph, full=true)",
    "n": 4,
    "events": initial(4, True, "w0", "{p}{i}") + _funky + _funky_full,
    "expect": {
        # TestFunkyHashgraphBlocks hashgraph_test.go:2155-2223
        "last_round": 5,
        "pending_after_process": [[4, False], [5, False]],
        "block_ntx": [6, 7, 7],
    },
}

# --- initSparseHashgraph, hashgraph_test.go:2419-2529 -----------------------
FIXTURES["kat_sparse"] = {
    "source": "hashgraph_test.go:2419-2654 (initSparseHashgraph)",
    "n": 4,
    "events": initial(4, True, "w0", "{p}{i}") + [
        play(1, 1, "w01", "w00", "e10", ["e10"]),
        play(2, 1, "w02", "e10", "e21", ["e21"]),
        play(3, 1, "w03", "e21", "e32", ["e32"]),
        play(0, 1, "w00", "e32", "w10", ["w10"]),
        play(1, 2, "e10", "w10", "w11", ["w11"]),
        play(0, 2, "w10", "w11", "f01", ["f01"]),
        play(2, 2, "e21", "f01", "w12", ["w12"]),
        play(3, 2, "e32", "w12", "w13", ["w13"]),
        play(1, 3, "w11", "w13", "w21", ["w21"]),
        play(2, 3, "w12", "w21", "w22", ["w22"]),
        play(3, 3, "w13", "w22", "w23", ["w23"]),
        play(1, 4, "w21", "w23", "g13", ["g13"]),
        play(2, 4, "w22", "g13", "w32", ["w32"]),
        play(3, 4, "w23", "w32", "w33", ["w33"]),
        play(1, 5, "g13", "w33", "w31", ["w31"]),
        play(2, 5, "w32", "w31", "h21", ["h21"]),
        play(3, 5, "w33", "h21", "w43", ["w43"]),
        play(1, 6, "w31", "w43", "w41", ["w41"]),
        play(2, 6, "h21", "w41", "w42", ["w42"]),
        play(3, 6, "w43", "w42", "i32", ["i32"]),
        play(1, 7, "w41", "i32", "w51", ["w51"]),
    ],
    # hashgraph_test.go:2515-2524 plays the list a second time; every
    # duplicate insert fails checkSelfParent and is only printed (:135-137)
    "replay_plays": True,
    "expect": {
        # TestSparseHashgraphFrames hashgraph_test.go:2531-2654 fetches blocks
        # 0..2; the frame event sets are from the test's diagram (:2446-2473)
        "min_blocks": 3,
        "block_round_received": [1, 2, 3],
        "frame_events_diagram": {
            "1": ["w00", "w01", "w02", "w03", "e10", "e21", "e32"],
            "2": ["w10", "w11", "f01", "w12", "w13"],
            "3": ["w21", "w22", "w23", "g13"]},
        # the roots it asserts with reflect.DeepEqual (hashgraph_test.go:2568-2653)
        "frame_roots": {
            "1": [base_root(0), base_root(1), base_root(2), base_root(3)],
            "2": [root(1, ["w00", 0, 0, 0, 0], {"w10": ["e32", 3, 1, 3, 0]}),
                  root(1, ["e10", 1, 1, 1, 0], {"w11": ["w10", 0, 1, 4, 1]}),
                  root(1, ["e21", 2, 1, 2, 0], {"w12": ["f01", 0, 2, 6, 1]}),
                  root(1, ["e32", 3, 1, 3, 0], {"w13": ["w12", 2, 2, 7, 1]})],
            "3": [root(1, ["w10", 0, 1, 4, 1], {"f01": ["w11", 1, 2, 5, 1]}),
                  root(2, ["w11", 1, 2, 5, 1], {"w21": ["w13", 3, 2, 8, 1]}),
                  root(2, ["w12", 2, 2, 7, 1], {"w22": ["w21", 1, 3, 9, 2]}),
                  root(2, ["w13", 3, 2, 8, 1], {"w23": ["w22", 2, 3, 10, 2]})]},
    },
}

# --- TestFork, hashgraph_test.go:334-398 ------------------------------------
FIXTURES["kat_fork"] = {
    "source": "hashgraph_test.go:334-398 (TestFork)",
    "n": 3,
    "events": initial(3),
    # (creator, index, sp, op, name, txs, expect_error)
    "rejects": [
        [2, 0, None, None, "a", ["yo"]],  # second index-0 event of node 2
        [0, 1, "e0", "a", "e01", None],   # other-parent a unknown
        [2, 1, "e2", "e01", "e20", None],  # other-parent e01 unknown
    ],
    "expect": {"rejected": ["a", "e01", "e20"]},
}


def main():
    for name, fx in FIXTURES.items():
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(fx, f, indent=1)
    print("wrote", len(FIXTURES), "fixtures")


if __name__ == "__main__":
    main()
