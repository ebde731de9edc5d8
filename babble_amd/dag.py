"""Synthetic gossip DAG generator (libbabble_gen.so, see csrc/dag_gen.h).

Inputs for the engine and its tests; generation is never timed."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

# BASELINE.json configs; seed = 0xBABB1E00 + cfg
CONFIGS = {
    1: dict(n=4, N=10_000, lagging=0),
    2: dict(n=32, N=1_000_000, lagging=0),
    3: dict(n=128, N=10_000_000, lagging=0),
    4: dict(n=512, N=20_000_000, lagging=0),
    5: dict(n=64, N=2_000_000, lagging=21),
}


class _Params(C.Structure):
    _fields_ = [("n", C.c_int32), ("N", C.c_int64), ("seed", C.c_uint64),
                ("lagging", C.c_int32), ("lag_div", C.c_int32), ("sig_mode", C.c_int32),
                ("threads", C.c_int32), ("tx_prob", C.c_double)]


class _Dag(C.Structure):
    _fields_ = [("n", C.c_int32), ("N", C.c_int64),
                ("participant_ids", C.POINTER(C.c_int64)),
                ("pubkeys", C.POINTER(C.c_uint8)),
                ("creator", C.POINTER(C.c_int32)), ("index", C.POINTER(C.c_int32)),
                ("self_parent", C.POINTER(C.c_int32)), ("other_parent", C.POINTER(C.c_int32)),
                ("ntx", C.POINTER(C.c_int32)),
                ("hash", C.POINTER(C.c_uint8)), ("sig_r", C.POINTER(C.c_uint8)),
                ("sig_s", C.POINTER(C.c_uint8))]


def _lib():
    global _LIB
    if _LIB is None:
        # BH_GEN_LIB: another build of the same source (tools/sanitize.sh)
        path = os.environ.get("BH_GEN_LIB") or os.path.join(_HERE, "libbabble_gen.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make` (or __graft_entry__.build())")
        L = C.CDLL(path)
        L.bg_generate.argtypes = [C.POINTER(_Params), C.POINTER(_Dag)]
        L.bg_free.argtypes = [C.POINTER(_Dag)]
        L.bg_body_json.argtypes = [C.POINTER(_Dag), C.c_int64, C.c_char_p]
        L.bg_body_json.restype = C.c_int32
        L.bg_tx_bytes.argtypes = [C.POINTER(_Dag), C.c_int64, C.c_void_p]
        L.bg_tx_bytes.restype = C.c_int32
        L.bg_sig_string.argtypes = [C.POINTER(_Dag), C.c_int64, C.c_char_p]
        L.bg_sig_string.restype = C.c_int32
        L.bg_event_bytes.argtypes = [C.POINTER(_Dag), C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]
        _LIB = L
    return _LIB


class Dag:
    """Events in topological (insertion) order, SoA numpy arrays.

    creator: participant slot (ID-sorted); index: sequence number;
    self_parent / other_parent: global ids (-1 = Root / none);
    hash, sig_r: [N, 32] uint8 (sig_r big-endian)."""

    def __init__(self, n, N, seed, lagging=0, lag_div=50, sig_mode=1, threads=0, tx_prob=0.5):
        L = _lib()
        p = _Params(n, N, seed, lagging, lag_div, sig_mode, threads, tx_prob)
        d = _Dag()
        rc = L.bg_generate(C.byref(p), C.byref(d))
        if rc:
            raise RuntimeError(f"bg_generate failed rc={rc}")
        self._d = d
        self.n, self.N, self.seed = n, N, seed

        def arr(ptr, cnt, dt):
            return np.ctypeslib.as_array(ptr, shape=(cnt,)).view(dt).copy()

        self.participant_ids = arr(d.participant_ids, n, np.int64)
        self.pubkeys = arr(d.pubkeys, n * 65, np.uint8).reshape(n, 65)
        self.creator = arr(d.creator, N, np.int32)
        self.index = arr(d.index, N, np.int32)
        self.self_parent = arr(d.self_parent, N, np.int32)
        self.other_parent = arr(d.other_parent, N, np.int32)
        self.ntx = arr(d.ntx, N, np.int32)
        self.hash = arr(d.hash, N * 32, np.uint8).reshape(N, 32)
        self.sig_r = arr(d.sig_r, N * 32, np.uint8).reshape(N, 32)
        self.sig_s = arr(d.sig_s, N * 32, np.uint8).reshape(N, 32)

    @classmethod
    def config(cls, cfg, N=None, sig_mode=1, rank=0, **kw):
        c = CONFIGS[cfg]
        return cls(c["n"], N or c["N"], 0xBABB1E00 + cfg + 0x10000 * rank,
                   lagging=c["lagging"], sig_mode=sig_mode, **kw)

    def body_json(self, e):
        buf = C.create_string_buffer(1024)
        k = _lib().bg_body_json(C.byref(self._d), e, buf)
        return buf.raw[:k]

    def sig_string(self, e):
        """Event.Signature: r|s in base 36 (crypto/utils.go:39-41)"""
        buf = C.create_string_buffer(128)
        k = _lib().bg_sig_string(C.byref(self._d), e, buf)
        return buf.raw[:k]

    def event_bytes(self, first=0, count=None):
        """(bodies u8, body_offsets [count+1], sigs u8, sig_offsets) of events
        [first, first + count): the blobs bh_set_event_bytes takes"""
        count = self.N - first if count is None else count
        bodies = np.empty(max(1024 * count, 1), np.uint8)
        sigs = np.empty(max(104 * count, 1), np.uint8)
        bo = np.zeros(count + 1, np.int64)
        so = np.zeros(count + 1, np.int64)
        _lib().bg_event_bytes(C.byref(self._d), first, count, bodies.ctypes.data, bo.ctypes.data,
                              sigs.ctypes.data, so.ctypes.data)
        return bodies[:bo[-1]], bo, sigs[:so[-1]], so

    def tx_bytes(self, e):
        buf = (C.c_uint8 * 64)()
        k = _lib().bg_tx_bytes(C.byref(self._d), e, buf)
        return bytes(buf[:k])

    # wire form (event.go:353-363): parents by (creator slot, index)
    def wire(self):
        sp_index = np.where(self.self_parent >= 0, self.index - 1, -1).astype(np.int32)
        op = self.other_parent
        op_creator = np.where(op >= 0, self.creator[np.maximum(op, 0)], -1).astype(np.int32)
        op_index = np.where(op >= 0, self.index[np.maximum(op, 0)], -1).astype(np.int32)
        return sp_index, op_creator, op_index

    def __del__(self):
        if getattr(self, "_d", None) is not None and _LIB is not None:
            _LIB.bg_free(C.byref(self._d))
            self._d = None
