"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the parity checker; nothing in
babble_amd/ imports this module.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = None

UNSET = -(2 ** 31)


def lib():
    global _LIB
    if _LIB is None:
        # BH_ORACLE_LIB: another build of the same source (tools/sanitize.sh:
        # the ASan/UBSan one)
        path = os.environ.get("BH_ORACLE_LIB") or os.path.join(ROOT, "oracle", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(path)
        P, I32, I64, VP = C.c_void_p, C.c_int32, C.c_int64, C.c_void_p
        L.hgo_create.restype = P
        L.hgo_create.argtypes = [I32, VP, I64]
        L.hgo_destroy.argtypes = [P]
        L.hgo_insert.argtypes = [P, I32, I32, I32, I32, VP, VP, I32]
        L.hgo_insert_batch.restype = I64
        L.hgo_insert_batch.argtypes = [P, I64, VP, VP, VP, VP, VP, VP, VP]
        L.hgo_insert_batch_ext.restype = I64
        L.hgo_insert_batch_ext.argtypes = [P, I64, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP]
        L.hgo_reset.argtypes = [P, I32, I64, VP, VP, VP, VP, I32, VP, VP, VP, VP, VP, VP, VP, VP]
        L.hgo_known.argtypes = [P, VP]
        for f in ("hgo_divide_rounds", "hgo_decide_fame", "hgo_decide_round_received",
                  "hgo_process_decided_rounds", "hgo_run_consensus"):
            getattr(L, f).argtypes = [P]
        for f, rt in (("hgo_num_events", I64), ("hgo_last_round", I32),
                      ("hgo_last_consensus_round", I32), ("hgo_consensus_transactions", I64),
                      ("hgo_pending_loaded_events", I64), ("hgo_num_consensus_events", I64),
                      ("hgo_num_undetermined", I64), ("hgo_num_blocks", I64)):
            getattr(L, f).restype = rt
            getattr(L, f).argtypes = [P]
        L.hgo_event_results.argtypes = [P, VP, VP, VP, VP, VP, VP]
        L.hgo_consensus_order.argtypes = [P, VP]
        L.hgo_blocks.argtypes = [P, VP, VP, VP, VP]
        L.hgo_pending_rounds.restype = I32
        L.hgo_pending_rounds.argtypes = [P, VP, VP, I32]
        L.hgo_coordinates.argtypes = [P, I32, VP, VP]
        L.hgo_undetermined.restype = I64
        L.hgo_undetermined.argtypes = [P, VP, I64]
        for f in ("hgo_see", "hgo_strongly_see", "hgo_witness_of"):
            getattr(L, f).argtypes = [P, I32, I32] if f != "hgo_witness_of" else [P, I32]
        L.hgo_round_of.restype = I32
        L.hgo_round_of.argtypes = [P, I32]
        L.hgo_lamport_of.restype = I32
        L.hgo_lamport_of.argtypes = [P, I32]
        L.hgo_set_event_bytes.argtypes = [P, I32, C.c_char_p, I32, C.c_char_p, I32]
        L.hgo_frame_roots.restype = I32
        L.hgo_frame_roots.argtypes = [P, I32, VP, VP, VP, VP, VP, I32]
        L.hgo_frame_json.restype = I64
        L.hgo_frame_json.argtypes = [P, I32, VP, I64]
        L.hgo_block_frame_hash.argtypes = [P, I64, VP]
        L.hgo_block_json.restype = I64
        L.hgo_block_json.argtypes = [P, I64, C.c_int, VP, I64]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    """Hashgraph restated on the CPU; method names follow hashgraph.go."""

    def __init__(self, n, participant_ids=None, capacity=1024):
        self.L = lib()
        self.n = n
        ids = np.asarray(participant_ids if participant_ids is not None else
                         np.arange(1, n + 1) * 1000, dtype=np.int64)
        self._ids = ids
        self.h = self.L.hgo_create(n, _p(ids), int(capacity))

    def close(self):
        if self.h:
            self.L.hgo_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def insert(self, creator, index, sp, op, hash32, sig_r32, ntx):
        h = np.frombuffer(bytes(hash32), dtype=np.uint8)
        r = np.frombuffer(bytes(sig_r32), dtype=np.uint8)
        return self.L.hgo_insert(self.h, creator, index, sp, op, _p(h), _p(r), ntx)

    def insert_dag(self, creator, index, sp, op, hashes, sig_r, ntx):
        a = [np.ascontiguousarray(x, dtype=np.int32) for x in (creator, index, sp, op, ntx)]
        hashes = np.ascontiguousarray(hashes, dtype=np.uint8).reshape(-1, 32)
        sig_r = np.ascontiguousarray(sig_r, dtype=np.uint8).reshape(-1, 32)
        bad = self.L.hgo_insert_batch(self.h, len(a[0]), _p(a[0]), _p(a[1]), _p(a[2]), _p(a[3]),
                                      _p(hashes), _p(sig_r), _p(a[4]))
        if bad:
            raise RuntimeError(f"oracle rejected {bad} events")

    def reset(self, rs):
        """Hashgraph.Reset's Store.Reset + SetBlock + LastConsensusRound
        (the frame's events are inserted next); rs: a ResetInputs"""
        a = {k: np.ascontiguousarray(v, dtype=np.int32) for k, v in rs.root_arrays().items()}
        kh = np.ascontiguousarray(rs.oth_key, dtype=np.uint8).reshape(-1, 32)
        vh = np.ascontiguousarray(rs.oth_hash, dtype=np.uint8).reshape(-1, 32)
        sh = np.ascontiguousarray(rs.sp_hash, dtype=np.uint8).reshape(-1, 32)
        rc = self.L.hgo_reset(self.h, rs.round_received, rs.block_index, _p(a["next_round"]),
                              _p(a["sp_index"]), _p(a["sp_lt"]), _p(a["sp_round"]), len(a["oth_root"]),
                              _p(a["oth_root"]), _p(kh), _p(a["oth_creator"]), _p(a["oth_index"]),
                              _p(a["oth_lt"]), _p(a["oth_round"]), _p(vh), _p(sh))
        if rc:
            raise RuntimeError(f"hgo_reset: {rc}")

    def insert_ext(self, creator, index, sp, op, op_creator, op_index, hashes, sig_r, ntx):
        """insert with other-parents possibly known only through Root.Others
        (op == -2, named by (op_creator, op_index)); returns per-event status"""
        a = [np.ascontiguousarray(x, dtype=np.int32) for x in (creator, index, sp, op, op_creator, op_index, ntx)]
        hashes = np.ascontiguousarray(hashes, dtype=np.uint8).reshape(-1, 32)
        sig_r = np.ascontiguousarray(sig_r, dtype=np.uint8).reshape(-1, 32)
        st = np.zeros(len(a[0]), np.int32)
        self.L.hgo_insert_batch_ext(self.h, len(a[0]), _p(a[0]), _p(a[1]), _p(a[2]), _p(a[3]), _p(a[4]),
                                    _p(a[5]), _p(hashes), _p(sig_r), _p(a[6]), _p(st))
        return st

    def known(self):
        k = np.empty(self.n, np.int32)
        self.L.hgo_known(self.h, _p(k))
        return k

    def divide_rounds(self):
        return self.L.hgo_divide_rounds(self.h)

    def decide_fame(self):
        return self.L.hgo_decide_fame(self.h)

    def decide_round_received(self):
        return self.L.hgo_decide_round_received(self.h)

    def process_decided_rounds(self):
        return self.L.hgo_process_decided_rounds(self.h)

    def run_consensus(self):
        return self.L.hgo_run_consensus(self.h)

    # ---- state ----
    def num_events(self):
        return self.L.hgo_num_events(self.h)

    def last_round(self):
        return self.L.hgo_last_round(self.h)

    def last_consensus_round(self):
        return self.L.hgo_last_consensus_round(self.h)

    def consensus_transactions(self):
        return self.L.hgo_consensus_transactions(self.h)

    def pending_loaded_events(self):
        return self.L.hgo_pending_loaded_events(self.h)

    def results(self):
        N = self.num_events()
        out = dict(round=np.empty(N, np.int32), witness=np.empty(N, np.int8),
                   lamport=np.empty(N, np.int32), round_received=np.empty(N, np.int32),
                   fame=np.empty(N, np.int8), cons_pos=np.empty(N, np.int64))
        self.L.hgo_event_results(self.h, _p(out["round"]), _p(out["witness"]),
                                 _p(out["lamport"]), _p(out["round_received"]),
                                 _p(out["fame"]), _p(out["cons_pos"]))
        return out

    def consensus_order(self):
        k = self.L.hgo_num_consensus_events(self.h)
        ids = np.empty(k, np.int32)
        if k:
            self.L.hgo_consensus_order(self.h, _p(ids))
        return ids

    def blocks(self):
        b = self.L.hgo_num_blocks(self.h)
        rr = np.empty(b, np.int32)
        first = np.empty(b, np.int64)
        cnt = np.empty(b, np.int64)
        ntx = np.empty(b, np.int64)
        if b:
            self.L.hgo_blocks(self.h, _p(rr), _p(first), _p(cnt), _p(ntx))
        return dict(round_received=rr, first=first, count=cnt, ntx=ntx)

    def pending_rounds(self):
        k = self.L.hgo_pending_rounds(self.h, None, None, 0)
        idx = np.empty(max(k, 1), np.int32)
        dec = np.empty(max(k, 1), np.int8)
        self.L.hgo_pending_rounds(self.h, _p(idx), _p(dec), k)
        return [(int(idx[i]), bool(dec[i])) for i in range(k)]

    def coordinates(self, e):
        la = np.empty(self.n, np.int32)
        fd = np.empty(self.n, np.int32)
        self.L.hgo_coordinates(self.h, e, _p(la), _p(fd))
        return la, fd

    def undetermined(self):
        k = self.L.hgo_undetermined(self.h, None, 0)
        ids = np.empty(max(k, 1), np.int32)
        self.L.hgo_undetermined(self.h, _p(ids), k)
        return ids[:k]

    def see(self, x, y):
        return bool(self.L.hgo_see(self.h, x, y))

    def strongly_see(self, x, y):
        return bool(self.L.hgo_strongly_see(self.h, x, y))

    def round(self, x):
        return self.L.hgo_round_of(self.h, x)

    def lamport(self, x):
        return self.L.hgo_lamport_of(self.h, x)

    def witness(self, x):
        return bool(self.L.hgo_witness_of(self.h, x))

    # ---- frames and blocks ----
    def set_event_bytes(self, e, body, sig):
        if self.L.hgo_set_event_bytes(self.h, int(e), bytes(body), len(body), bytes(sig), len(sig)):
            raise ValueError(f"event {e} out of range")

    def frame_roots(self, rr):
        """Roots of frame rr, participant order: [(next_round, self_parent
        event or -1 for the base root, [(key event, value event), ...])]."""
        n = self.n
        nr, sp, no = (np.empty(n, np.int32) for _ in range(3))
        k = self.L.hgo_frame_roots(self.h, rr, _p(nr), _p(sp), _p(no), None, None, 0)
        if k < 0:
            return None
        key = np.empty(max(k, 1), np.int32)
        val = np.empty(max(k, 1), np.int32)
        self.L.hgo_frame_roots(self.h, rr, None, None, None, _p(key), _p(val), k)
        out, o = [], 0
        for p in range(n):
            out.append((int(nr[p]), int(sp[p]),
                        [(int(key[o + j]), int(val[o + j])) for j in range(no[p])]))
            o += int(no[p])
        return out

    def frame_json(self, rr):
        k = self.L.hgo_frame_json(self.h, rr, None, 0)
        if k < 0:
            return None
        buf = np.empty(k, np.uint8)
        self.L.hgo_frame_json(self.h, rr, _p(buf), k)
        return buf.tobytes()

    def block_frame_hash(self, b):
        out = np.empty(32, np.uint8)
        if self.L.hgo_block_frame_hash(self.h, b, _p(out)):
            return None
        return out.tobytes()

    def block_json(self, b, body_only=False):
        k = self.L.hgo_block_json(self.h, b, int(body_only), None, 0)
        if k < 0:
            return None
        buf = np.empty(k, np.uint8)
        self.L.hgo_block_json(self.h, b, int(body_only), _p(buf), k)
        return buf.tobytes()
