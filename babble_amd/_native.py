"""ctypes binding of libbabble_hip.so (include/babble_hip.h).

The product path: every call below runs HIP kernels on the MI355X.  There is
no CPU fallback -- if the library or a device is missing this raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# BH_LIB_PATH: an alternative build of the same library (A/B of kernel
# variants in one GPU session); the in-tree build by default
LIB_PATH = os.environ.get("BH_LIB_PATH") or os.path.join(_HERE, "libbabble_hip.so")

BH_OK = 0
ERRORS = {
    1: "SelfParent", 2: "OtherParent", 3: "UnknownParticipant", 4: "SkippedIndex",
    5: "Capacity", 6: "State", 7: "Invalid", 8: "Device", 9: "KeyNotFound",
}

# exported symbols, in include/babble_hip.h order (checked by tests)
SYMBOLS = (
    "bh_create", "bh_destroy", "bh_last_error", "bh_insert_events", "bh_divide_rounds",
    "bh_decide_fame", "bh_decide_round_received", "bh_process_decided_rounds",
    "bh_run_consensus", "bh_synchronize", "bh_reset_consensus", "bh_reset", "bh_get_stats", "bh_get_event_meta",
    "bh_get_consensus_order", "bh_get_blocks", "bh_get_pending_rounds", "bh_get_undetermined",
    "bh_get_round_info", "bh_get_coordinates", "bh_query_events", "bh_get_stage_ms", "bh_get_profile", "bh_get_profile_kernel",
    "bh_get_pipeline", "bh_get_loop_stats", "bh_hash_bodies", "bh_verify_signatures", "bh_set_event_bytes", "bh_get_frame_roots",
    "bh_get_frame_json", "bh_get_block_hashes", "bh_get_block_json", "bh_comm_unique_id", "bh_comm_init", "bh_comm_init_transport",
    "bh_shard_range",
)


class Config(C.Structure):
    _fields_ = [("n_participants", C.c_int32), ("participant_ids", C.POINTER(C.c_int64)),
                ("max_events", C.c_int64), ("device", C.c_int32),
                ("n_devices", C.c_int32), ("device_ids", C.POINTER(C.c_int32)),
                ("frames", C.c_int32)]


# bh_transport: the caller's blocking host-memory send / recv / broadcast
SEND_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int32)
RECV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int32)
BCAST_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int32)


class Transport(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("send", SEND_FN), ("recv", RECV_FN), ("broadcast", BCAST_FN)]


class Events(C.Structure):
    _fields_ = [("count", C.c_int64), ("creator_id", C.c_void_p), ("index", C.c_void_p),
                ("self_parent_index", C.c_void_p), ("other_parent_creator_id", C.c_void_p),
                ("other_parent_index", C.c_void_p), ("hash", C.c_void_p), ("sig_r", C.c_void_p),
                ("n_transactions", C.c_void_p)]


class Roots(C.Structure):
    _fields_ = [("round_received", C.c_int32), ("block_index", C.c_int64),
                ("next_round", C.c_void_p), ("self_parent_index", C.c_void_p),
                ("self_parent_lamport", C.c_void_p), ("self_parent_round", C.c_void_p),
                ("n_others", C.c_int32), ("other_root", C.c_void_p), ("other_key", C.c_void_p),
                ("other_creator_id", C.c_void_p), ("other_index", C.c_void_p),
                ("other_lamport", C.c_void_p), ("other_round", C.c_void_p), ("other_hash", C.c_void_p),
                ("self_parent_hash", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("n_events", C.c_int64), ("last_round", C.c_int32),
                ("last_consensus_round", C.c_int32), ("consensus_events", C.c_int64),
                ("consensus_transactions", C.c_int64), ("pending_loaded_events", C.c_int64),
                ("undetermined_events", C.c_int64), ("blocks", C.c_int64),
                ("pending_rounds", C.c_int32), ("first_block", C.c_int64)]


class RoundInfo(C.Structure):
    _fields_ = [("round", C.c_int32), ("n_events", C.c_int32), ("n_witnesses", C.c_int32),
                ("n_consensus", C.c_int32), ("queued", C.c_int8), ("witnesses_decided", C.c_int8),
                ("pending", C.c_int8), ("pending_decided", C.c_int8)]


_LIB = None


def load():
    """Load libbabble_hip.so; raises if it was not built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `make` or __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    P, VP, I32, I64 = C.c_void_p, C.c_void_p, C.c_int32, C.c_int64
    L.bh_create.argtypes = [C.POINTER(Config), C.POINTER(P)]
    L.bh_create.restype = C.c_int
    L.bh_destroy.argtypes = [P]
    L.bh_last_error.argtypes = [P]
    L.bh_last_error.restype = C.c_char_p
    L.bh_insert_events.argtypes = [P, C.POINTER(Events), VP, C.POINTER(I64)]
    for f in ("bh_divide_rounds", "bh_decide_fame", "bh_decide_round_received",
              "bh_process_decided_rounds", "bh_run_consensus", "bh_synchronize", "bh_reset_consensus"):
        getattr(L, f).argtypes = [P]
        getattr(L, f).restype = C.c_int
    L.bh_get_stats.argtypes = [P, C.POINTER(Stats)]
    L.bh_reset.argtypes = [P, C.POINTER(Roots)]
    L.bh_get_event_meta.argtypes = [P, I64, I64, VP, VP, VP, VP, VP, VP]
    L.bh_get_consensus_order.argtypes = [P, I64, I64, VP]
    L.bh_get_blocks.argtypes = [P, I64, I64, VP, VP, VP, VP]
    L.bh_get_pending_rounds.argtypes = [P, VP, VP, I32]
    L.bh_get_pending_rounds.restype = I32
    L.bh_get_undetermined.argtypes = [P, VP, I64]
    L.bh_get_undetermined.restype = I64
    L.bh_get_round_info.argtypes = [P, I32, C.POINTER(RoundInfo), VP, VP, I32]
    L.bh_get_round_info.restype = C.c_int
    L.bh_get_coordinates.argtypes = [P, I64, VP, VP]
    L.bh_query_events.argtypes = [P, I32, I64, VP, VP, VP]
    L.bh_query_events.restype = C.c_int
    L.bh_get_stage_ms.argtypes = [P, C.POINTER(C.c_float), I32]
    L.bh_get_stage_ms.restype = I32
    L.bh_get_profile.argtypes = [P, C.POINTER(I64), C.POINTER(C.c_float)]
    L.bh_get_profile_kernel.argtypes = [P]
    L.bh_get_profile_kernel.restype = C.c_char_p
    L.bh_get_pipeline.argtypes = [P, C.POINTER(I32), C.POINTER(I64)]
    L.bh_get_pipeline.restype = C.c_int
    L.bh_get_loop_stats.argtypes = [P, C.POINTER(I64), C.POINTER(I64)]
    L.bh_get_loop_stats.restype = C.c_int
    L.bh_hash_bodies.argtypes = [P, VP, VP, I64, VP]
    L.bh_hash_bodies.restype = C.c_int
    L.bh_verify_signatures.argtypes = [P, VP, VP, VP, VP, I64, VP, I32, VP]
    L.bh_verify_signatures.restype = C.c_int
    L.bh_set_event_bytes.argtypes = [P, I64, I64, VP, VP, VP, VP]
    L.bh_set_event_bytes.restype = C.c_int
    L.bh_get_frame_roots.argtypes = [P, I32, VP, VP, VP, VP, VP, I32]
    L.bh_get_frame_roots.restype = I32
    L.bh_get_frame_json.argtypes = [P, I32, VP, I64]
    L.bh_get_frame_json.restype = I64
    L.bh_get_block_hashes.argtypes = [P, I64, I64, VP, VP, VP]
    L.bh_get_block_hashes.restype = C.c_int
    L.bh_get_block_json.argtypes = [P, I64, I32, VP, I64]
    L.bh_get_block_json.restype = I64
    L.bh_comm_unique_id.argtypes = [VP]
    L.bh_comm_unique_id.restype = C.c_int
    L.bh_comm_init.argtypes = [P, I32, I32, VP]
    L.bh_comm_init.restype = C.c_int
    L.bh_comm_init_transport.argtypes = [P, I32, I32, C.POINTER(Transport)]
    L.bh_comm_init_transport.restype = C.c_int
    L.bh_shard_range.argtypes = [I64, I32, I32, C.POINTER(I64), C.POINTER(I64)]
    L.bh_shard_range.restype = None
    _LIB = L
    return L
