"""FastSync / Reset scenarios built from a hashgraph run.

Follows the reference tests TestResetFromFrame, TestFunkyHashgraphReset and
TestSparseHashgraphReset (hashgraph_test.go:1711-1907, 2344-2417,
2656-2738): take block b of a hashgraph that ran consensus, its Frame
(GetFrame(block.RoundReceived()): roots + sorted events), Reset a fresh
hashgraph from (block, frame) -- Store.Reset(roots), SetBlock,
LastConsensusRound, InsertEvent of the frame's events -- then insert the
"diff" (getDiff, :2776-2795: every event with an Index above the reset
hashgraph's KnownEvents, in topological order) as wire events (ReadWireInfo,
hashgraph.go:1414-1479).

Event ids of the reset hashgraph are insertion positions; an event's
other-parent that the reset hashgraph does not hold is passed as op == -2
with its (creator slot, Index), resolved through Root.Others on insert.

TEST INFRASTRUCTURE ONLY.
"""
import numpy as np


class ResetInputs:
    """Reset inputs for block `block` of oracle `o` (after run_consensus) over
    DAG arrays `d` (creator, index, sp, op, hashes, sig_r, ntx)."""

    def __init__(self, o, d, block):
        b = o.blocks()
        self.block_index = int(block)
        self.round_received = int(b["round_received"][block])
        order = o.consensus_order()
        first, cnt = int(b["first"][block]), int(b["count"][block])
        self.frame = [int(x) for x in order[first:first + cnt]]
        roots = o.frame_roots(self.round_received)
        assert roots is not None
        res = o.results()
        lt, rnd = res["lamport"], res["round"]
        self.next_round = [r[0] for r in roots]
        sp = [r[1] for r in roots]
        self.sp_index = [int(d.index[e]) if e >= 0 else -1 for e in sp]
        self.sp_lt = [int(lt[e]) if e >= 0 else -1 for e in sp]
        self.sp_round = [int(rnd[e]) if e >= 0 else -1 for e in sp]
        # Root.SelfParent.Hash (a base root event's is "Root<id>": zeros here)
        self.sp_hash = np.stack([np.asarray(d.hashes[e], np.uint8) if e >= 0 else np.zeros(32, np.uint8)
                                 for e in sp])
        self.oth_root, self.oth_creator, self.oth_index, self.oth_lt, self.oth_round = [], [], [], [], []
        keys, vals = [], []
        for p, (_, _, oth) in enumerate(roots):
            for key, val in oth:
                self.oth_root.append(p)
                self.oth_creator.append(int(d.creator[val]))
                self.oth_index.append(int(d.index[val]))
                self.oth_lt.append(int(lt[val]))
                self.oth_round.append(int(rnd[val]))
                keys.append(np.asarray(d.hashes[key], np.uint8))
                vals.append(np.asarray(d.hashes[val], np.uint8))
        self.oth_key = np.stack(keys) if keys else np.zeros((0, 32), np.uint8)
        self.oth_hash = np.stack(vals) if vals else np.zeros((0, 32), np.uint8)
        # known after the frame's events: the last Index per creator (or the
        # Root's SelfParent.Index); the diff is every later event
        known = list(self.sp_index)
        for e in self.frame:
            known[int(d.creator[e])] = max(known[int(d.creator[e])], int(d.index[e]))
        self.known = known
        fset = set(self.frame)
        self.diff = [e for e in range(len(d.creator))
                     if e not in fset and int(d.index[e]) > known[int(d.creator[e])]]
        self.d = d

    def root_arrays(self):
        return dict(next_round=self.next_round, sp_index=self.sp_index, sp_lt=self.sp_lt,
                    sp_round=self.sp_round, oth_root=self.oth_root, oth_creator=self.oth_creator,
                    oth_index=self.oth_index, oth_lt=self.oth_lt, oth_round=self.oth_round)

    def events(self, old_ids):
        """Insert arrays (reset-hashgraph ids) for the original events
        old_ids, inserted after every event already mapped; returns
        (dict of arrays, old->new id map updated in place)"""
        d = self.d
        if not hasattr(self, "new_id"):
            self.new_id = {}
        cols = {k: [] for k in ("creator", "index", "sp", "op", "op_creator", "op_index", "ntx")}
        hashes, sigs = [], []
        for e in old_ids:
            s, o = int(d.sp[e]), int(d.op[e])
            cols["creator"].append(int(d.creator[e]))
            cols["index"].append(int(d.index[e]))
            cols["sp"].append(self.new_id.get(s, -1) if s >= 0 else -1)
            if o < 0:
                cols["op"].append(-1)
                cols["op_creator"].append(-1)
                cols["op_index"].append(-1)
            elif o in self.new_id:
                cols["op"].append(self.new_id[o])
                cols["op_creator"].append(int(d.creator[o]))
                cols["op_index"].append(int(d.index[o]))
            else:
                cols["op"].append(-2)
                cols["op_creator"].append(int(d.creator[o]))
                cols["op_index"].append(int(d.index[o]))
            cols["ntx"].append(int(d.ntx[e]))
            hashes.append(np.asarray(d.hashes[e], np.uint8))
            sigs.append(np.asarray(d.sig_r[e], np.uint8))
            self.new_id[e] = len(self.new_id)
        out = {k: np.array(v, np.int32) for k, v in cols.items()}
        out["hashes"] = np.stack(hashes) if hashes else np.zeros((0, 32), np.uint8)
        out["sig_r"] = np.stack(sigs) if sigs else np.zeros((0, 32), np.uint8)
        return out


def oracle_insert(o2, rs, old_ids):
    """insert the original events old_ids into reset oracle o2 one at a time,
    mapping only the accepted ones (a rejected event gets no id, so its
    descendants name it as a missing parent, as in Go); returns statuses"""
    st = np.zeros(len(old_ids), np.int32)
    for i, e in enumerate(old_ids):
        ev = rs.events([e])
        st[i] = o2.insert_ext(ev["creator"], ev["index"], ev["sp"], ev["op"], ev["op_creator"], ev["op_index"],
                              ev["hashes"], ev["sig_r"], ev["ntx"])[0]
        if st[i]:
            del rs.new_id[e]
    return st


class DagArrays:
    """creator / index / sp / op / hashes / sig_r / ntx of a babble_amd.dag.Dag
    or a KatDag under the names ResetInputs reads"""

    def __init__(self, d):
        self.creator, self.index = np.asarray(d.creator), np.asarray(d.index)
        self.sp = np.asarray(getattr(d, "self_parent", getattr(d, "sp", None)))
        self.op = np.asarray(getattr(d, "other_parent", getattr(d, "op", None)))
        self.hashes = np.asarray(getattr(d, "hash", getattr(d, "hashes", None))).reshape(-1, 32)
        self.sig_r = np.asarray(d.sig_r).reshape(-1, 32)
        self.ntx = np.asarray(d.ntx)
        self.participant_ids = np.asarray(d.participant_ids)
        self.n = len(self.participant_ids)


class SilentDag:
    """A gossip DAG in which participant `silent` creates no event before
    insertion position `join` (a peer that joins late): GetFrame gives it a
    base Root (SelfParent Index / Round -1, NextRound 0) in every frame
    before its first consensus event, while the other roots sit at a high
    round -- the FastSync case of a long-running network with a new peer.
    Random other-parents among the active peers' heads; random hashes /
    signature bytes (the engine and the oracle read them as opaque keys)."""

    def __init__(self, n, N, seed, silent, join):
        rng = np.random.default_rng(seed)
        creator, index = np.empty(N, np.int32), np.empty(N, np.int32)
        sp, op = np.empty(N, np.int32), np.empty(N, np.int32)
        last, cnt = np.full(n, -1, np.int64), np.zeros(n, np.int32)
        e = 0
        for c in range(n):
            if c != silent:
                creator[e], index[e], sp[e], op[e] = c, 0, -1, -1
                last[c], cnt[c], e = e, 1, e + 1
        while e < N:
            active = [c for c in range(n) if c != silent or e >= join]
            c = active[int(rng.integers(len(active)))]
            others = [x for x in active if x != c and last[x] >= 0]
            f = others[int(rng.integers(len(others)))]
            creator[e], index[e], sp[e], op[e] = c, cnt[c], last[c], last[f]
            last[c], e = e, e + 1
            cnt[c] += 1
        self.creator, self.index, self.sp, self.op = creator, index, sp, op
        self.hashes = rng.integers(0, 256, (N, 32), dtype=np.uint8)
        self.sig_r = rng.integers(0, 256, (N, 32), dtype=np.uint8)
        self.ntx = (rng.random(N) < 0.5).astype(np.int32)
        self.participant_ids = np.sort(rng.choice(2**31 - 1, n, replace=False)).astype(np.int64)
        self.n = n
        self.silent = silent
