"""Hashgraph -- the reference's consensus API, backed by the MI355X engine.

Mirrors the methods node.Core calls on *hashgraph.Hashgraph
(/root/reference/src/hashgraph/hashgraph.go; node/core.go:51-377):

    NewHashgraph            -> Hashgraph(participant_ids, max_events)
    InsertEvent             -> insert_event / insert_events (wire form)
    DivideRounds            -> divide_rounds
    DecideFame              -> decide_fame
    DecideRoundReceived     -> decide_round_received
    ProcessDecidedRounds    -> process_decided_rounds
    UndeterminedEvents, PendingRounds, LastConsensusRound,
    ConsensusTransactions, PendingLoadedEvents  -> properties

Go returns `error`; here the same conditions raise HashgraphError carrying
the Go error kind.  All compute runs in libbabble_hip (HIP kernels); this
module only marshals arrays.
"""
import ctypes as C

import numpy as np

from . import _native

UNSET = -(2 ** 31)


class HashgraphError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_native.ERRORS.get(code, code)}: {msg}")
        self.code = code
        self.kind = _native.ERRORS.get(code, str(code))


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def comm_unique_id():
    """RCCL id for Hashgraph.comm_init (rank 0 makes it, every rank passes it)."""
    L = _native.load()
    buf = (C.c_uint8 * 128)()
    rc = L.bh_comm_unique_id(buf)
    if rc != _native.BH_OK:
        raise HashgraphError(rc, "ncclGetUniqueId failed")
    return bytes(buf)


def shard_range(items, world, rank):
    """[lo, hi) of `items` owned by shard `rank` of `world` -- the engine's
    split rule for LA columns, fame rounds and frames (bh_shard_range)."""
    L = _native.load()
    lo, hi = C.c_int64(), C.c_int64()
    L.bh_shard_range(int(items), int(world), int(rank), C.byref(lo), C.byref(hi))
    return lo.value, hi.value


class Hashgraph:
    def __init__(self, participant_ids, max_events, device=0, devices=None, frames=False):
        """devices: a list of HIP ordinals to shard the passes over in this
        process (repeats allowed: shards sharing one device); None = one
        device, `device`.  frames: keep event hashes / bytes on the device
        and project frames and blocks (GetFrame roots, FrameHash, block
        hashes) at every ProcessDecidedRounds."""
        self._L = _native.load()
        ids = np.ascontiguousarray(participant_ids, dtype=np.int64)
        if np.any(np.diff(ids) <= 0):
            raise ValueError("participant ids must be sorted ascending (peers.go:63-73)")
        self.participant_ids = ids
        self.n = len(ids)
        if devices is not None:
            self._devs = np.ascontiguousarray(devices, dtype=np.int32)
            cfg = _native.Config(self.n, ids.ctypes.data_as(C.POINTER(C.c_int64)), int(max_events),
                                 int(self._devs[0]), len(self._devs),
                                 self._devs.ctypes.data_as(C.POINTER(C.c_int32)), int(bool(frames)))
        else:
            cfg = _native.Config(self.n, ids.ctypes.data_as(C.POINTER(C.c_int64)), int(max_events),
                                 int(device), 0, None, int(bool(frames)))
        h = C.c_void_p()
        rc = self._L.bh_create(C.byref(cfg), C.byref(h))
        if rc != _native.BH_OK:
            raise HashgraphError(rc, "bh_create failed (no HIP device or out of memory)")
        self._h = h

    def comm_init(self, rank, world, uid):
        """Make this handle shard `rank` of `world` processes (RCCL); call
        before inserting events.  Every pass is then collective."""
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._check(self._L.bh_comm_init(self._h, int(rank), int(world), buf))

    def comm_init_transport(self, rank, world, send, recv, broadcast):
        """Make this handle shard `rank` of `world` processes over a host
        transport of the caller's (bh_comm_init_transport): send(buf, peer),
        recv(buf, peer) and broadcast(buf, root) get a writable memoryview of
        the staged bytes and block until done.  Call before inserting
        events; every pass is then collective."""
        def wrap(fn):
            def cb(_ctx, buf, nbytes, peer):
                try:
                    fn(memoryview((C.c_uint8 * nbytes).from_address(buf)).cast("B"), int(peer))
                    return 0
                except Exception:  # the engine reports the failure (BH_ERR_DEVICE)
                    import traceback
                    traceback.print_exc()
                    return 1
            return cb
        t = _native.Transport(None, _native.SEND_FN(wrap(send)), _native.RECV_FN(wrap(recv)),
                              _native.BCAST_FN(wrap(broadcast)))
        self._transport = t  # the callbacks must outlive the handle's calls
        self._check(self._L.bh_comm_init_transport(self._h, int(rank), int(world), C.byref(t)))

    def close(self):
        if getattr(self, "_h", None):
            self._L.bh_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc):
        if rc != _native.BH_OK:
            raise HashgraphError(rc, self._L.bh_last_error(self._h).decode())

    # ---- InsertEvent (hashgraph.go:714-761) ----
    def insert_events(self, creator_id, index, self_parent_index, other_parent_creator_id,
                      other_parent_index, hashes, sig_r, n_transactions, raise_on_error=True):
        """Wire-form batch insert.  Returns the per-event status array (0 = ok)."""
        arrs = [np.ascontiguousarray(a, dtype=dt) for a, dt in (
            (creator_id, np.int64), (index, np.int32), (self_parent_index, np.int32),
            (other_parent_creator_id, np.int64), (other_parent_index, np.int32),
            (hashes, np.uint8), (sig_r, np.uint8), (n_transactions, np.int32))]
        cnt = len(arrs[0])
        if arrs[5].size != cnt * 32 or arrs[6].size != cnt * 32:
            raise ValueError("hash / sig_r must be [count, 32] bytes")
        ev = _native.Events(cnt, *[_ptr(a) for a in arrs])
        status = np.zeros(cnt, np.int32)
        acc = C.c_int64()
        rc = self._L.bh_insert_events(self._h, C.byref(ev), _ptr(status), C.byref(acc))
        if rc != _native.BH_OK and raise_on_error:
            self._check(rc)
        return status

    def insert_event(self, creator_id, index, self_parent_index, other_parent_creator_id,
                     other_parent_index, hash32, sig_r32, n_transactions):
        st = self.insert_events([creator_id], [index], [self_parent_index],
                                [other_parent_creator_id], [other_parent_index],
                                np.frombuffer(bytes(hash32), np.uint8),
                                np.frombuffer(bytes(sig_r32), np.uint8), [n_transactions],
                                raise_on_error=True)
        return int(st[0])

    def insert_dag(self, dag):
        """Insert a babble_amd.dag.Dag (or any object with its arrays)."""
        spi, opc, opi = dag.wire()
        pid = self.participant_ids
        opc_id = np.where(opc >= 0, pid[np.maximum(opc, 0)], -1)
        return self.insert_events(pid[dag.creator], dag.index, spi, opc_id, opi, dag.hash,
                                  dag.sig_r, dag.ntx)

    # ---- consensus passes ----
    def divide_rounds(self):
        self._check(self._L.bh_divide_rounds(self._h))

    def decide_fame(self):
        self._check(self._L.bh_decide_fame(self._h))

    def decide_round_received(self):
        self._check(self._L.bh_decide_round_received(self._h))

    def process_decided_rounds(self):
        self._check(self._L.bh_process_decided_rounds(self._h))

    def run_consensus(self):
        self._check(self._L.bh_run_consensus(self._h))

    def synchronize(self):
        self._check(self._L.bh_synchronize(self._h))

    def reset(self, round_received, block_index, next_round, self_parent_index, self_parent_lamport,
              self_parent_round, other_root=(), other_key=(), other_creator_id=(), other_index=(),
              other_lamport=(), other_round=(), other_hash=(), self_parent_hash=None):
        """Hashgraph.Reset(block, frame) before the frame's events are
        inserted (hashgraph.go:1324-1369): the frame's Roots in participant
        order and their Others flattened (bh_reset); self_parent_hash [n, 32]:
        each Root.SelfParent.Hash (needed with frames=True).  Insert
        frame.Events next, then later events, as wire events."""
        n = len(self.participant_ids)
        per = [np.ascontiguousarray(a, dtype=np.int32) for a in
               (next_round, self_parent_index, self_parent_lamport, self_parent_round)]
        if any(a.size != n for a in per):
            raise ValueError("one root per participant")
        k = len(other_root)
        oth = [np.ascontiguousarray(a, dtype=dt) for a, dt in (
            (other_root, np.int32), (other_key, np.uint8), (other_creator_id, np.int64),
            (other_index, np.int32), (other_lamport, np.int32), (other_round, np.int32),
            (other_hash, np.uint8))]
        if oth[1].size != 32 * k or oth[6].size != 32 * k or any(oth[i].size != k for i in (0, 2, 3, 4, 5)):
            raise ValueError("Others arrays disagree in length")
        oth = [a if a.size else np.zeros(1, a.dtype) for a in oth]
        sph = None
        if self_parent_hash is not None:
            sph = np.ascontiguousarray(self_parent_hash, dtype=np.uint8)
            if sph.size != 32 * n:
                raise ValueError("self_parent_hash must be [n, 32] bytes")
        rt = _native.Roots(int(round_received), int(block_index), *[_ptr(a) for a in per], k,
                           *[_ptr(a) for a in oth], _ptr(sph))
        self._keep_roots = (per, oth, sph)
        self._check(self._L.bh_reset(self._h, C.byref(rt)))

    def reset_consensus(self):
        """Forget every pass's results, keep the events (bh_reset_consensus):
        the next run_consensus recomputes the whole DAG."""
        self._check(self._L.bh_reset_consensus(self._h))

    # ---- state ----
    def stats(self):
        s = _native.Stats()
        self._check(self._L.bh_get_stats(self._h, C.byref(s)))
        return s

    @property
    def last_consensus_round(self):
        r = self.stats().last_consensus_round
        return None if r < 0 else r

    @property
    def consensus_transactions(self):
        return self.stats().consensus_transactions

    @property
    def pending_loaded_events(self):
        return self.stats().pending_loaded_events

    def last_round(self):
        return self.stats().last_round

    @property
    def pending_rounds(self):
        k = self._L.bh_get_pending_rounds(self._h, None, None, 0)
        if k < 0:  # a negated BH_ERR_* (a coordinate rank of a split group holds no rounds)
            self._check(-k)
        idx = np.zeros(max(k, 1), np.int32)
        dec = np.zeros(max(k, 1), np.int8)
        self._L.bh_get_pending_rounds(self._h, _ptr(idx), _ptr(dec), k)
        return [(int(idx[i]), bool(dec[i])) for i in range(k)]

    @property
    def undetermined_events(self):
        k = self._L.bh_get_undetermined(self._h, None, 0)
        if k < 0:
            self._check(-k)
        ids = np.zeros(max(k, 1), np.int32)
        self._L.bh_get_undetermined(self._h, _ptr(ids), k)
        return ids[:k]

    def results(self, first=0, count=None):
        N = self.stats().n_events
        count = N - first if count is None else count
        out = dict(round=np.empty(count, np.int32), witness=np.empty(count, np.int8),
                   lamport=np.empty(count, np.int32), round_received=np.empty(count, np.int32),
                   fame=np.empty(count, np.int8), cons_pos=np.empty(count, np.int64))
        self._check(self._L.bh_get_event_meta(
            self._h, first, count, _ptr(out["round"]), _ptr(out["witness"]), _ptr(out["lamport"]),
            _ptr(out["round_received"]), _ptr(out["fame"]), _ptr(out["cons_pos"])))
        return out

    def consensus_order(self):
        k = self.stats().consensus_events
        ids = np.empty(k, np.int32)
        if k:
            self._check(self._L.bh_get_consensus_order(self._h, 0, k, _ptr(ids)))
        return ids

    def blocks(self):
        st = self.stats()
        b = st.blocks - st.first_block  # blocks this handle made (a Reset starts after the block's Index)
        out = dict(round_received=np.empty(b, np.int32), first=np.empty(b, np.int64),
                   count=np.empty(b, np.int64), ntx=np.empty(b, np.int64))
        if b:
            self._check(self._L.bh_get_blocks(self._h, 0, b, _ptr(out["round_received"]),
                                              _ptr(out["first"]), _ptr(out["count"]),
                                              _ptr(out["ntx"])))
        return out

    def round_info(self, r):
        """Store.GetRound(r) + RoundInfo accessors (inmem_store.go:185-211,
        roundInfo.go:33-128).  Raises HashgraphError(KeyNotFound) for a
        round that does not exist.  Returns a dict with the witnesses (event
        ids, participant order) and their Trilean fame."""
        info = _native.RoundInfo()
        cap = self.n
        wid = np.empty(cap, np.int32)
        fame = np.empty(cap, np.int8)
        self._check(self._L.bh_get_round_info(self._h, int(r), C.byref(info), _ptr(wid), _ptr(fame), cap))
        k = info.n_witnesses
        return dict(round=info.round, n_events=info.n_events, n_consensus=info.n_consensus,
                    witnesses=wid[:k].copy(), fame=fame[:k].copy(), queued=bool(info.queued),
                    witnesses_decided=bool(info.witnesses_decided), pending=bool(info.pending),
                    pending_decided=bool(info.pending_decided))

    def coordinates(self, event_id):
        la = np.empty(self.n, np.int32)
        fd = np.empty(self.n, np.int32)
        self._check(self._L.bh_get_coordinates(self._h, int(event_id), _ptr(la), _ptr(fd)))
        return la, fd

    QUERY = {"ancestor": 0, "self_ancestor": 1, "see": 2, "strongly_see": 3, "round_diff": 4}

    def query(self, kind, x, y):
        """ancestor / self_ancestor / see / strongly_see (bool arrays) or
        round_diff (int32) of the event pairs (x[i], y[i]) (bh_query_events)."""
        xs = np.ascontiguousarray(np.atleast_1d(x), np.int64)
        ys = np.ascontiguousarray(np.atleast_1d(y), np.int64)
        if xs.shape != ys.shape:
            raise ValueError("x and y must pair up")
        out = np.empty(len(xs), np.int32)
        self._check(self._L.bh_query_events(self._h, self.QUERY[kind], len(xs), _ptr(xs), _ptr(ys), _ptr(out)))
        return out if kind == "round_diff" else out.astype(bool)

    def stage_ms(self):
        """[coordinates, rounds, fame, round_received, order, exchange,
        projection, round loop] ms of the last run (device events; exchange:
        host wall time; projection: bh_config.frames only; round loop: its
        launches' device time, overlapped or not)."""
        buf = (C.c_float * 8)()
        k = self._L.bh_get_stage_ms(self._h, buf, 8)
        return [float(buf[i]) for i in range(k)]

    def profile(self):
        it = C.c_int64()
        ms = C.c_float()
        self._check(self._L.bh_get_profile(self._h, C.byref(it), C.byref(ms)))
        return int(it.value), float(ms.value)

    def pipeline(self):
        """(segments the last DivideRounds pipelined over, DivideRounds calls
        so far that resumed from the previous call's device state)"""
        seg = C.c_int32()
        inc = C.c_int64()
        self._check(self._L.bh_get_pipeline(self._h, C.byref(seg), C.byref(inc)))
        return int(seg.value), int(inc.value)

    def loop_stats(self):
        """(round loops run as one persistent launch, of which the grid
        barrier gave up and the per-iteration launches ran them)"""
        pl = C.c_int64()
        fb = C.c_int64()
        self._check(self._L.bh_get_loop_stats(self._h, C.byref(pl), C.byref(fb)))
        return int(pl.value), int(fb.value)

    def profile_kernel(self):
        """Name of the coordinate kernel the last run timed."""
        return self._L.bh_get_profile_kernel(self._h).decode()

    # ---- block projection (bh_config.frames) ----
    def set_event_bytes(self, first, bodies, sigs):
        """EventBody.Marshal() bytes and Signature strings of the inserted
        events [first, first + len(bodies)) (bh_set_event_bytes)."""
        if len(bodies) != len(sigs):
            raise ValueError("one signature per body")
        if not len(bodies):
            return

        def blob(items):
            lens = np.fromiter((len(b) for b in items), np.int64, len(items))
            offs = np.zeros(len(items) + 1, np.int64)
            np.cumsum(lens, out=offs[1:])
            data = np.frombuffer(b"".join(bytes(b) for b in items) or b"\0", np.uint8)
            return data, offs
        bd, bo = blob(bodies)
        sd, so = blob(sigs)
        self._check(self._L.bh_set_event_bytes(self._h, int(first), len(bodies), _ptr(bd), _ptr(bo),
                                               _ptr(sd), _ptr(so)))

    def _neg(self, rc):
        if rc < 0:
            raise HashgraphError(int(-rc), self._L.bh_last_error(self._h).decode())
        return rc

    def frame_roots(self, round_received):
        """GetFrame(r).Roots (hashgraph.go:1125-1231): [(next_round,
        self_parent event or -1 for the base root event, [(key event, value
        event), ...] sorted by key hash)] in peer order."""
        n = self.n
        nr, sp, no = (np.empty(n, np.int32) for _ in range(3))
        k = self._neg(self._L.bh_get_frame_roots(self._h, int(round_received), _ptr(nr), _ptr(sp), _ptr(no),
                                                 None, None, 0))
        key = np.empty(max(k, 1), np.int32)
        val = np.empty(max(k, 1), np.int32)
        self._neg(self._L.bh_get_frame_roots(self._h, int(round_received), None, None, None, _ptr(key),
                                             _ptr(val), k))
        out, o = [], 0
        for p in range(n):
            out.append((int(nr[p]), int(sp[p]), [(int(key[o + j]), int(val[o + j])) for j in range(no[p])]))
            o += int(no[p])
        return out

    def frame_json(self, round_received):
        """Frame.Marshal() of a processed round (frame.go:17-26)."""
        k = self._neg(self._L.bh_get_frame_json(self._h, int(round_received), None, 0))
        buf = np.empty(max(k, 1), np.uint8)
        self._neg(self._L.bh_get_frame_json(self._h, int(round_received), _ptr(buf), k))
        return buf[:k].tobytes()

    def block_hashes(self, first=0, count=None):
        """(frame_hash [m, 32], block_hash [m, 32], valid [m]) of blocks."""
        st = self.stats()
        b = st.blocks - st.first_block  # blocks this handle made (a Reset starts after the block's Index)
        count = b - first if count is None else count
        fh = np.zeros((max(count, 1), 32), np.uint8)
        bh = np.zeros((max(count, 1), 32), np.uint8)
        ok = np.zeros(max(count, 1), np.int8)
        self._check(self._L.bh_get_block_hashes(self._h, int(first), int(count), _ptr(fh), _ptr(bh), _ptr(ok)))
        return fh[:count], bh[:count], ok[:count].astype(bool)

    def block_json(self, b, body_only=False):
        """Block.Marshal() (or BlockBody.Marshal() with body_only) of block b."""
        k = self._neg(self._L.bh_get_block_json(self._h, int(b), int(bool(body_only)), None, 0))
        buf = np.empty(max(k, 1), np.uint8)
        self._neg(self._L.bh_get_block_json(self._h, int(b), int(bool(body_only)), _ptr(buf), k))
        return buf[:k].tobytes()

    def hash_bodies(self, bodies):
        """Event.Hash() (event.go:50-56) of each body on the device: SHA-256
        of the Go-JSON bytes.  bodies: a sequence of bytes; returns [n, 32] u8."""
        lens = np.fromiter((len(b) for b in bodies), np.int64, len(bodies))
        offsets = np.zeros(len(bodies) + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        data = np.frombuffer(b"".join(bodies), np.uint8) if len(bodies) else np.zeros(1, np.uint8)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        out = np.empty((len(bodies), 32), np.uint8)
        self._check(self._L.bh_hash_bodies(self._h, _ptr(data), _ptr(offsets), len(bodies), _ptr(out)))
        return out

    def verify_signatures(self, hashes, sig_r, sig_s, keys, pubkeys):
        """Event.Verify() (event.go:194-209) of a batch on the device: ECDSA
        P-256 with Go ecdsa.Verify semantics.  hashes / sig_r / sig_s: [m, 32]
        u8 big-endian; keys: [m] index into pubkeys [k, 64] (x || y).
        Returns [m] bool."""
        keys = np.ascontiguousarray(keys, np.int32).reshape(-1)
        m = len(keys)
        hashes, sig_r, sig_s = (np.ascontiguousarray(a, np.uint8) for a in (hashes, sig_r, sig_s))
        if any(a.size != 32 * m for a in (hashes, sig_r, sig_s)):
            raise ValueError("hashes / sig_r / sig_s must hold 32 bytes per signature")
        pubkeys = np.ascontiguousarray(pubkeys, np.uint8)
        if pubkeys.size == 0 or pubkeys.size % 64:
            raise ValueError("pubkeys must be [k, 64] bytes (x || y)")
        pubkeys = pubkeys.reshape(-1, 64)
        if m and (keys.min() < 0 or keys.max() >= len(pubkeys)):
            raise ValueError("key index out of range")
        out = np.zeros(m, np.uint8)
        self._check(self._L.bh_verify_signatures(self._h, _ptr(hashes), _ptr(sig_r), _ptr(sig_s), _ptr(keys),
                                                 len(keys), _ptr(pubkeys), len(pubkeys), _ptr(out)))
        return out.astype(bool)
