/*
 * babble_hip.h -- C ABI of libbabble_hip, the MI355X (gfx950) consensus engine
 * for Babble's hashgraph virtual-voting path.
 *
 * Drop-in boundary: every entry point replaces one method of the reference's
 * Go `Hashgraph` (/root/reference/src/hashgraph/hashgraph.go) as called by
 * node.Core (src/node/core.go).  Plain C types only; one owner per handle;
 * not thread-safe (the reference serialises with Node.coreLock, node.go:27).
 * The cgo binding a maintainer would add is in INTEGRATION.md.
 *
 * Status codes mirror the Go error kinds (common/errors.go:7-15, and the
 * fmt.Errorf messages of hashgraph.go); bh_last_error() gives the message.
 */
#ifndef BABBLE_HIP_H
#define BABBLE_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  BH_OK = 0,
  BH_ERR_SELF_PARENT = 1,   /* "Self-parent not last known event by creator" hashgraph.go:409 */
  BH_ERR_OTHER_PARENT = 2,  /* "Other-parent not known" hashgraph.go:432 */
  BH_ERR_UNKNOWN_PARTICIPANT = 3, /* StoreErr UnknownParticipant (common/errors.go:13) */
  BH_ERR_SKIPPED_INDEX = 4, /* StoreErr SkippedIndex / PassedIndex (rolling index) */
  BH_ERR_CAPACITY = 5,      /* more events than bh_config.max_events */
  BH_ERR_STATE = 6,         /* pass called before its prerequisites */
  BH_ERR_INVALID = 7,       /* bad argument */
  BH_ERR_DEVICE = 8,        /* HIP runtime error / no device / kernel fault */
  BH_ERR_KEY_NOT_FOUND = 9  /* StoreErr KeyNotFound (common/errors.go:8), e.g. GetRound */
};

typedef struct bh_handle bh_handle;

/* NewHashgraph(participants, store, commitCh, logger) (hashgraph.go:47-73)
 * with an InmemStore of capacity max_events (inmem_store.go:27-49). */
typedef struct {
  int32_t n_participants;
  const int64_t *participant_ids; /* peer IDs, ascending (peers.go:63-73, 118-129) */
  int64_t max_events;             /* capacity; the reference's cacheSize must be >= #events */
  int32_t device;                 /* HIP device ordinal (when n_devices <= 1) */
  /* Devices the handle shards its passes over: each
   * holds the whole DAG; coordinate columns, fame rounds and frames are
   * split between them and exchanged device to device.  n_devices <= 1:
   * one device, `device`.  Ordinals may repeat (shards sharing a device). */
  int32_t n_devices;
  const int32_t *device_ids;
  /* Block projection: nonzero keeps every event's hash
   * on the device and accepts its bytes (bh_set_event_bytes); each
   * ProcessDecidedRounds then computes the roots of its frames (GetFrame),
   * and, for frames whose events' bytes are all known, the FrameHash and
   * the hash of the block made from it (NewBlockFromFrame). */
  int32_t frames;
} bh_config;

/* A batch of events in topological order, in the reference's compact wire
 * form (WireBody, event.go:353-363): parents are (creator ID, index) pairs,
 * resolved by the engine exactly like Hashgraph.ReadWireInfo
 * (hashgraph.go:1414-1479).  Buffers stay owned by the caller. */
typedef struct {
  int64_t count;
  const int64_t *creator_id;              /* WireBody.CreatorID */
  const int32_t *index;                   /* WireBody.Index */
  const int32_t *self_parent_index;       /* WireBody.SelfParentIndex, -1 = the Root */
  const int64_t *other_parent_creator_id; /* WireBody.OtherParentCreatorID, -1 = none */
  const int32_t *other_parent_index;      /* WireBody.OtherParentIndex, -1 = none */
  const uint8_t *hash;                    /* [count][32] Event.Hash() = SHA-256(Go-JSON body) */
  const uint8_t *sig_r;                   /* [count][32] big-endian ECDSA r of Event.Signature */
  const int32_t *n_transactions;          /* len(Body.Transactions) */
} bh_events;

int bh_create(const bh_config *cfg, bh_handle **out);
void bh_destroy(bh_handle *h);
const char *bh_last_error(const bh_handle *h);

/* InsertEvent(event, setWireInfo) for each event (hashgraph.go:714-761):
 * checkSelfParent / checkOtherParent / participant-index continuity.  A
 * rejected event is skipped (like createHashgraph, hashgraph_test.go:134-138)
 * and its status written to status[i] (nullable).  Accepted events get
 * consecutive ids (= topologicalIndex).  Signatures are pre-verified inputs.
 * Returns BH_OK if all were accepted, else the first error code. */
int bh_insert_events(bh_handle *h, const bh_events *ev, int32_t *status, int64_t *n_accepted);

/* The consensus passes (node/core.go:335-377), with the Go Hashgraph's
 * state kept between calls: a call after more events were inserted
 * continues from the previous one (coordinates, rounds and fame of the new
 * events and still-pending rounds; frames of newly decided rounds), and the
 * result depends on the call schedule exactly as the reference's does
 * (RoundInfo.queued, PendingRounds' sticky decided flags). */
int bh_divide_rounds(bh_handle *h);           /* hashgraph.go:767-849 (+ coordinates) */
int bh_decide_fame(bh_handle *h);             /* hashgraph.go:852-947 */
int bh_decide_round_received(bh_handle *h);   /* hashgraph.go:951-1036 */
int bh_process_decided_rounds(bh_handle *h);  /* hashgraph.go:1041-1231 */
int bh_run_consensus(bh_handle *h);           /* all four, queued on one stream */
int bh_synchronize(bh_handle *h);             /* wait for queued device work */
/* Forget every pass's results, keep the inserted events: the state of a
 * Hashgraph into which the same events were just inserted
 * (hashgraph_test.go's createHashgraph; what BenchmarkConsensus re-runs).
 * The next RunConsensus recomputes everything; without this call a pass
 * only processes what was inserted since the previous one. */
int bh_reset_consensus(bh_handle *h);

/* Hashgraph.Reset(block, frame) (hashgraph.go:1324-1369; FastSync,
 * node/core.go:240-283) on a fresh handle, before the frame's events are
 * inserted: Store.Reset(frame.Roots), SetBlock(block), LastConsensusRound =
 * block.RoundReceived().  The caller then inserts frame.Events (in frame
 * order) and any later events with bh_insert_events, as Reset and the
 * gossip after it do; an other-parent the engine does not hold is resolved
 * through the creator's Root.Others like ReadWireInfo + checkOtherParent
 * (:1431-1457, 417-436), and rounds / Lamport timestamps follow the Root
 * cases A-F (docs/fastsync.rst:140-175).  Roots are given in participant
 * (ID) order, as Frame.Roots; Others entries flattened, each naming the
 * position of the Root that holds it.  Requires one shard and every
 * NextRound / SelfParent.Round below round_received (as GetFrame's roots
 * are).  Blocks made afterwards have Index block_index + 1 + i.  With
 * bh_config.frames the blocks are projected as GetFrame does on a Reset
 * hashgraph: a participant with no consensus event since the Reset keeps
 * the installed Root whole (InmemStore.LastConsensusEventFrom ->
 * GetRoot, inmem_store.go:136-150), a first event's SelfParent RootEvent
 * is its Root's (createSelfParentRootEvent, hashgraph.go:546-566), and an
 * other-parent the Root's Others names is taken from there
 * (createOtherParentRootEvent :568-578); self_parent_hash then gives each
 * Root.SelfParent.Hash (ignored for Index -1, the base root event
 * "Root<id>"; may be null when frames are off). */
typedef struct {
  int32_t round_received;              /* block.RoundReceived() */
  int64_t block_index;                 /* block.Index() */
  const int32_t *next_round;           /* [n] Root.NextRound */
  const int32_t *self_parent_index;    /* [n] Root.SelfParent.Index */
  const int32_t *self_parent_lamport;  /* [n] Root.SelfParent.LamportTimestamp */
  const int32_t *self_parent_round;    /* [n] Root.SelfParent.Round */
  int32_t n_others;
  const int32_t *other_root;           /* [n_others] position of the Root holding the entry */
  const uint8_t *other_key;            /* [n_others][32] hash of the event keying it (Others[ev.Hex()]) */
  const int64_t *other_creator_id;     /* RootEvent.CreatorID */
  const int32_t *other_index;          /* RootEvent.Index */
  const int32_t *other_lamport;        /* RootEvent.LamportTimestamp */
  const int32_t *other_round;          /* RootEvent.Round */
  const uint8_t *other_hash;           /* [n_others][32] RootEvent.Hash */
  const uint8_t *self_parent_hash;     /* [n][32] Root.SelfParent.Hash bytes (frames; null otherwise) */
} bh_roots;
int bh_reset(bh_handle *h, const bh_roots *roots);

typedef struct {
  int64_t n_events;
  int32_t last_round;             /* Store.LastRound() */
  int32_t last_consensus_round;   /* Hashgraph.LastConsensusRound, -1 = nil */
  int64_t consensus_events;       /* Store.ConsensusEventsCount() */
  int64_t consensus_transactions; /* Hashgraph.ConsensusTransactions */
  int64_t pending_loaded_events;  /* Hashgraph.PendingLoadedEvents */
  int64_t undetermined_events;    /* len(Hashgraph.UndeterminedEvents) */
  int64_t blocks;                 /* Store.LastBlockIndex()+1 (after bh_reset: block_index + 1 + blocks made) */
  int32_t pending_rounds;         /* len(Hashgraph.PendingRounds) */
  int64_t first_block;            /* Index of bh_get_blocks' block 0 (after bh_reset: block_index + 1) */
} bh_stats;
int bh_get_stats(bh_handle *h, bh_stats *out);

/* Per-event private fields (event.go:107-116): round / lamport / rr are
 * INT32_MIN when unset (Go nil); fame = -1 not a witness, 0 Undefined,
 * 1 True, 2 False (roundInfo.go:10-16); consensus_pos = -1 if not ordered. */
int bh_get_event_meta(bh_handle *h, int64_t first, int64_t count, int32_t *round,
                      int8_t *witness, int32_t *lamport, int32_t *round_received,
                      int8_t *fame, int64_t *consensus_pos);
/* consensus order (Store.AddConsensusEvent sequence), event ids */
int bh_get_consensus_order(bh_handle *h, int64_t first, int64_t count, int32_t *ids);
/* Blocks (block.go:100-123): RoundReceived, first consensus position,
 * #events of its Frame, #transactions (concatenated in consensus order). */
int bh_get_blocks(bh_handle *h, int64_t first, int64_t count, int32_t *round_received,
                  int64_t *first_event, int64_t *n_events, int64_t *n_transactions);
/* Hashgraph.PendingRounds: returns the count, fills up to cap entries.
 * A negative return is a negated BH_ERR_* code (-BH_ERR_STATE on a shard
 * that holds no consensus results: a coordinate rank of a wide split) --
 * check it before using the count. */
int32_t bh_get_pending_rounds(bh_handle *h, int32_t *index, int8_t *decided, int32_t cap);
/* Hashgraph.UndeterminedEvents (insertion order): returns the count, fills
 * up to cap ids (ids may be NULL).  Negative: a negated BH_ERR_* code, as
 * for bh_get_pending_rounds. */
int64_t bh_get_undetermined(bh_handle *h, int32_t *ids, int64_t cap);

/* Store.GetRound(r) / RoundWitnesses(r) (inmem_store.go:185-211) and the
 * RoundInfo accessors (roundInfo.go:33-128).  BH_ERR_KEY_NOT_FOUND for a
 * round that does not exist (r < 0 or r > LastRound).  Witnesses are listed
 * in participant (ID) order -- Go returns them in map order -- with their
 * Trilean fame (0 Undefined, 1 True, 2 False) in fame[]; up to cap entries
 * (witness_ids / fame nullable), info->n_witnesses gives the count. */
typedef struct {
  int32_t round;
  int32_t n_events;          /* events whose round is r (RoundInfo.Events also lists the n_consensus ones) */
  int32_t n_witnesses;       /* len(RoundInfo.Witnesses()) */
  int32_t n_consensus;       /* len(RoundInfo.ConsensusEvents()): events received in r */
  int8_t queued;             /* RoundInfo.queued */
  int8_t witnesses_decided;  /* RoundInfo.WitnessesDecided() */
  int8_t pending;            /* r is in Hashgraph.PendingRounds */
  int8_t pending_decided;    /* that entry's Decided flag (0 when not pending) */
} bh_round_info;
int bh_get_round_info(bh_handle *h, int32_t r, bh_round_info *info, int32_t *witness_ids, int8_t *fame,
                      int32_t cap);
/* lastAncestors / firstDescendants indexes of one event (event.go:115-116) */
int bh_get_coordinates(bh_handle *h, int64_t id, int32_t *last_ancestors,
                       int32_t *first_descendants);
/* The Hashgraph's private predicates over event pairs (x[i], y[i]) (event
 * ids), for tests and tools that call them on the Go Hashgraph:
 * BH_Q_ANCESTOR ancestor(x, y) (hashgraph.go:80-118), BH_Q_SELF_ANCESTOR
 * selfAncestor (:120-149), BH_Q_SEE see (:152-157), BH_Q_STRONGLY_SEE
 * stronglySee (:159-191) -> out 1 / 0; BH_Q_ROUND_DIFF roundDiff (:382-395)
 * -> round(x) - round(y) (BH_ERR_STATE before DivideRounds covered the
 * events).  Coordinates are those of every inserted event. */
enum { BH_Q_ANCESTOR = 0, BH_Q_SELF_ANCESTOR = 1, BH_Q_SEE = 2, BH_Q_STRONGLY_SEE = 3, BH_Q_ROUND_DIFF = 4 };
int bh_query_events(bh_handle *h, int32_t kind, int64_t count, const int64_t *x, const int64_t *y, int32_t *out);
/* device milliseconds of the last run, per stage:
 * [0] coordinates+lamport, [1] rounds+witnesses, [2] fame, [3] round received,
 * [4] frames/order/blocks, [5] shard exchanges (host wall time, 0 for one
 * shard), [6] block projection (bh_config.frames: roots, Frame / Block JSON
 * and their hashes; 0 without), [7] the round loop's own device time (its
 * launches summed over the run's loops; [1] is the time the rounds stage
 * adds after the coordinates, less when a pipeline overlaps them); returns
 * the number of entries */
int32_t bh_get_stage_ms(bh_handle *h, float *ms, int32_t cap);
/* kernel statistics of the last run for the roofline report: number of
 * round-loop iterations, coordinate sweep launches' average ms */
int bh_get_profile(bh_handle *h, int64_t *rounds_iterated, float *sweep_ms);
/* name of the coordinate kernel the last run timed ("k_flow32" / "k_flow":
 * chain dataflow; "k_la_sweep": chunked sweep); "" before the first run */
const char *bh_get_profile_kernel(const bh_handle *h);
/* how the last DivideRounds ran (no reference counterpart: engine
 * introspection for tests and reports): the insertion-order segments its
 * coordinate / round-loop pipeline used (1 = unpipelined), and the number of
 * DivideRounds calls so far that resumed from the previous call's device
 * state instead of recomputing the whole DAG */
int bh_get_pipeline(bh_handle *h, int32_t *segments, int64_t *incremental_calls);
/* how the round loops ran so far (engine introspection, no reference
 * counterpart): loops run as one persistent launch (k_round2p, n <= 128),
 * and of those, loops whose grid barrier gave up and that the per-iteration
 * launches then ran from the same inputs */
int bh_get_loop_stats(bh_handle *h, int64_t *persistent_loops, int64_t *persist_fallbacks);
/* SHA-256 of a batch of event bodies on the device:
 * Event.Hash() = SHA-256 of the body's Go-JSON bytes (event.go:50-56), the
 * digest InsertEvent keys, verifies and takes the coin from
 * (hashgraph.go:716-721, 1526-1535).  Body i is bytes[offsets[i] ..
 * offsets[i+1]) (offsets: count + 1 ascending entries); digests receives
 * 32 * count bytes.  Runs on the handle's device and stream, synchronously. */
int bh_hash_bodies(bh_handle *h, const uint8_t *bytes, const int64_t *offsets, int64_t count,
                   uint8_t *digests);
/* ECDSA P-256 verification of a batch of event signatures on the device
 * (SURVEY 8(f) row 2): Event.Verify() (event.go:194-209) -> Go
 * ecdsa.Verify(pub, hash, r, s) (crypto/utils.go:43-51).  Signature i:
 * 32-byte big-endian hash / r / s at 32 * i, signed by public key
 * keys[i] of pubkeys (64 bytes each: x || y big-endian, on the curve);
 * ok[i] = 1 if it verifies, else 0.  Synchronous, on the handle's stream. */
int bh_verify_signatures(bh_handle *h, const uint8_t *hashes, const uint8_t *sig_r, const uint8_t *sig_s,
                         const int32_t *keys, int64_t count, const uint8_t *pubkeys, int32_t n_keys,
                         uint8_t *ok);

/* ---- Block projection (bh_config.frames) ----
 * The bytes Frame.Marshal (frame.go:17-26) needs of events [first, first +
 * count) (already inserted): body i = bodies[body_offsets[i] ..
 * body_offsets[i+1]) is EventBody.Marshal() (event.go:32-39; the Encoder's
 * trailing newline may be included), signature i = sigs[sig_offsets[i] ..
 * sig_offsets[i+1]) is Event.Signature (crypto.EncodeSignature, "r|s" in
 * base 36).  Offsets: count + 1 ascending entries.  Set them before the
 * ProcessDecidedRounds that emits their frame: a frame with an event whose
 * bytes are missing gets roots but no FrameHash. */
int bh_set_event_bytes(bh_handle *h, int64_t first, int64_t count, const uint8_t *bodies,
                       const int64_t *body_offsets, const uint8_t *sigs, const int64_t *sig_offsets);
/* Hashgraph.GetFrame(round_received).Roots (hashgraph.go:1125-1231) of a
 * processed round: per participant (peer order) NextRound, SelfParent (an
 * event id; -1 = the base root event "Root<id>", root.go:73-84) and the
 * number of Others; then the Others of all roots in order, each root's
 * sorted by key hash (Go's JSON map order): key event id -> RootEvent of the
 * value event id (its CreatorID / Index / LamportTimestamp / Round are the
 * event's).  Arrays nullable; up to cap Others.  Returns the total number of
 * Others, or a negative status (-BH_ERR_KEY_NOT_FOUND: not a processed round). */
int32_t bh_get_frame_roots(bh_handle *h, int32_t round_received, int32_t *next_round, int32_t *self_parent,
                           int32_t *n_others, int32_t *other_key, int32_t *other_value, int32_t cap);
/* Frame.Marshal() of a processed round (its Go-JSON bytes, newline
 * included): returns the length and copies up to cap bytes (buf nullable);
 * negative status when unavailable (-BH_ERR_STATE: some event's bytes are
 * missing). */
int64_t bh_get_frame_json(bh_handle *h, int32_t round_received, uint8_t *buf, int64_t cap);
/* Blocks [first, first + count): FrameHash (Block.FrameHash(), block.go:100-
 * 110) and the block's hash (Block.Hash(), block.go:196-205: SHA-256 of
 * Block.Marshal() before any signature is added), 32 bytes each; valid[i]
 * = 0 when the frame's bytes were incomplete (the hashes are then zero).
 * Arrays nullable. */
int bh_get_block_hashes(bh_handle *h, int64_t first, int64_t count, uint8_t *frame_hash, uint8_t *block_hash,
                        int8_t *valid);
/* Block.Marshal() (body_only = 0) or BlockBody.Marshal() (body_only = 1,
 * block.go:21-29 -- what checkGossip compares) of block b: length, up to
 * cap bytes copied; negative status when unavailable. */
int64_t bh_get_block_json(bh_handle *h, int64_t b, int32_t body_only, uint8_t *buf, int64_t cap);

/* Sharding across processes: one shard per process,
 * each holding the whole DAG, joined by an RCCL communicator.  Rank 0 makes
 * the id, every rank passes the same bytes (NCCL_UNIQUE_ID_BYTES = 128)
 * before inserting any event.  Every pass is then collective: all ranks must
 * call the same passes in the same order.  With the coordinate split (the
 * default at n <= 128) only rank 0 holds consensus results: the result
 * getters of ranks > 0 return BH_ERR_STATE. */
int bh_comm_unique_id(uint8_t *id);
int bh_comm_init(bh_handle *h, int32_t rank, int32_t world, const uint8_t *id);
/* The same group over a transport of the caller's (a Go node's own links
 * between its processes; the tests' gloo group): host-memory, blocking
 * point-to-point messages and broadcasts, each returning 0 on success.  The
 * engine stages every exchange through pinned host memory and calls these
 * at exactly the places the RCCL group calls ncclSend / ncclRecv /
 * ncclBroadcast, in the same order on every rank: the call sequence is
 * identical, so a transport that delivers messages between each pair in
 * order suffices.  The struct is copied; ctx is passed back untouched. */
typedef struct bh_transport {
  void *ctx;
  int (*send)(void *ctx, const void *buf, size_t bytes, int32_t peer);
  int (*recv)(void *ctx, void *buf, size_t bytes, int32_t peer);
  int (*broadcast)(void *ctx, void *buf, size_t bytes, int32_t root);
} bh_transport;
int bh_comm_init_transport(bh_handle *h, int32_t rank, int32_t world, const bh_transport *t);
/* The split rule every shard uses for LA columns, fame rounds and frames:
 * shard `rank` of `world` owns [items*rank/world, items*(rank+1)/world). */
void bh_shard_range(int64_t items, int32_t world, int32_t rank, int64_t *lo, int64_t *hi);

#ifdef __cplusplus
}
#endif
#endif
