/*
 * hg_oracle.h -- CPU restatement of Babble v0.4.0's hashgraph consensus passes.
 *
 * TEST INFRASTRUCTURE ONLY.  This oracle is the parity checker for the
 * MI355X engine (libbabble_hip).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path never calls it.
 *
 * It follows the reference Go code control flow literally (recursion with
 * memoisation, the UndeterminedEvents / PendingRounds state machine, the
 * RoundInfo bookkeeping, the DecideFame vote loop), single threaded, because
 * the reference consensus is single threaded (no goroutines in
 * src/hashgraph).  Citations are reference paths (/root/reference/src/...).
 *
 * Parity pin: the Go toolchain is absent, so the reference cannot run here.
 * The restatement is pinned by the known-answer DAG tests of
 * src/hashgraph/hashgraph_test.go transcribed as tests/golden/kat_*.json and
 * checked by tests/test_oracle_kat.py.
 *
 * Roots: base roots (hashgraph/root.go:75-106) for a fresh hashgraph, or a
 * Frame's roots installed by hgo_reset (Hashgraph.Reset, hashgraph.go:
 * 1324-1369; the Root cases A-F of docs/fastsync.rst:140-175).  Frames and
 * FrameHashes are restated for fresh hashgraphs only.
 */
#ifndef HG_ORACLE_H
#define HG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hgo hgo;

/* status codes mirror the Go error kinds (common/errors.go:7-15) */
enum {
  HGO_OK = 0,
  HGO_ERR_SELF_PARENT = 1,   /* "Self-parent not last known event by creator" hashgraph.go:409 */
  HGO_ERR_OTHER_PARENT = 2,  /* "Other-parent not known" hashgraph.go:432 */
  HGO_ERR_BAD_CREATOR = 3,   /* unknown participant */
  HGO_ERR_CAPACITY = 4,
  HGO_ERR_STATE = 5
};

/* participant_ids: peer IDs (FNV-1a-32 of pubkey) sorted ascending
 * (peers/peers.go:63-73).  Slot i of every coordinate vector is participant i. */
hgo *hgo_create(int32_t n, const int64_t *participant_ids, int64_t capacity);
void hgo_destroy(hgo *h);

/* InsertEvent (hashgraph.go:714-761), minus signature verification (the
 * inputs are pre-verified).  sp = global id of the self-parent or
 * -1 for the creator's Root; op = global id of the other-parent or -1 for "".
 * hash: 32-byte SHA-256 of the Go-JSON body; sig_r: 32-byte big-endian ECDSA r.
 * Returns HGO_OK (the event gets the next global id) or an error (rejected). */
int hgo_insert(hgo *h, int32_t creator, int32_t index, int32_t sp, int32_t op,
               const uint8_t *hash32, const uint8_t *sig_r32, int32_t ntx);

/* the same with an other-parent the Store may not hold: op == -2 names it by
 * (op_creator slot, op_index), resolved through the creator's Root.Others as
 * ReadWireInfo + checkOtherParent do (hashgraph.go:1431-1457, 417-436) */
int hgo_insert_ext(hgo *h, int32_t creator, int32_t index, int32_t sp, int32_t op, int32_t op_creator,
                   int32_t op_index, const uint8_t *hash32, const uint8_t *sig_r32, int32_t ntx);
int64_t hgo_insert_batch_ext(hgo *h, int64_t count, const int32_t *creator, const int32_t *index,
                             const int32_t *sp, const int32_t *op, const int32_t *op_creator,
                             const int32_t *op_index, const uint8_t *hash32, const uint8_t *sig_r32,
                             const int32_t *ntx, int32_t *status);

/* Hashgraph.Reset(block, frame) before the frame's events are inserted
 * (fresh hashgraph only): per participant slot the Root's NextRound and
 * SelfParent Index / LamportTimestamp / Round; the Others entries (owning
 * root slot, key event hash, value RootEvent creator slot / Index /
 * LamportTimestamp / Round / Hash); LastConsensusRound = round_received,
 * LastBlockIndex = block_index. */
int hgo_reset(hgo *h, int32_t round_received, int64_t block_index, const int32_t *next_round,
              const int32_t *sp_index, const int32_t *sp_lt, const int32_t *sp_round, int32_t n_others,
              const int32_t *oth_root, const uint8_t *oth_key32, const int32_t *oth_creator,
              const int32_t *oth_index, const int32_t *oth_lt, const int32_t *oth_round,
              const uint8_t *oth_hash32, const uint8_t *sp_hash32 /* [n][32] Root SelfParent hashes, or NULL */);
/* Store.KnownEvents: last Index per participant slot (the Root's
 * SelfParent.Index when it has no event) */
void hgo_known(const hgo *h, int32_t *known);

/* hgo_insert over arrays (test/bench harness convenience); returns the
 * number of rejected events */
int64_t hgo_insert_batch(hgo *h, int64_t count, const int32_t *creator, const int32_t *index,
                         const int32_t *sp, const int32_t *op, const uint8_t *hash32,
                         const uint8_t *sig_r32, const int32_t *ntx);

int hgo_divide_rounds(hgo *h);            /* hashgraph.go:767-849 */
int hgo_decide_fame(hgo *h);              /* hashgraph.go:852-947 */
int hgo_decide_round_received(hgo *h);    /* hashgraph.go:951-1036 */
int hgo_process_decided_rounds(hgo *h);   /* hashgraph.go:1041-1122 */
int hgo_run_consensus(hgo *h);            /* the four, node/core.go:335-377 */

/* ---- queries (test/bench harness) ---- */
int64_t hgo_num_events(const hgo *h);
int32_t hgo_last_round(const hgo *h);                 /* InmemStore.LastRound */
int32_t hgo_last_consensus_round(const hgo *h);       /* -1 == nil */
int64_t hgo_consensus_transactions(const hgo *h);
int64_t hgo_pending_loaded_events(const hgo *h);
int64_t hgo_num_consensus_events(const hgo *h);
int64_t hgo_num_undetermined(const hgo *h);
int64_t hgo_num_blocks(const hgo *h);

/* per-event results; round/lt/rr = INT32_MIN when unset (Go nil pointer);
 * fame: 0 Undefined, 1 True, 2 False (roundInfo.go:10-16) or -1 not a witness;
 * cons_pos = position in the consensus order or -1 */
void hgo_event_results(const hgo *h, int32_t *round, int8_t *witness, int32_t *lt,
                       int32_t *rr, int8_t *fame, int64_t *cons_pos);
/* consensus order (event ids), length hgo_num_consensus_events */
void hgo_consensus_order(const hgo *h, int32_t *ids);
/* blocks: index, round_received, first consensus position, #events, #txs */
void hgo_blocks(const hgo *h, int32_t *round_received, int64_t *first, int64_t *count,
                int64_t *ntx);
/* pending rounds queue */
int32_t hgo_pending_rounds(const hgo *h, int32_t *index, int8_t *decided, int32_t cap);
/* coordinates (lastAncestors / firstDescendants indexes) of one event */
void hgo_coordinates(const hgo *h, int32_t id, int32_t *la, int32_t *fd);
/* UndeterminedEvents queue, in order */
int64_t hgo_undetermined(const hgo *h, int32_t *ids, int64_t cap);
/* ---- frames and blocks (GetFrame hashgraph.go:1125-1231, frame.go,
 * root.go, block.go) ---- */
/* The bytes Frame.Marshal needs of event e: its Go-JSON body
 * (EventBody.Marshal, event.go:32-39; the trailing newline is dropped) and
 * its Signature string.  Optional: without them no FrameHash is computed. */
int hgo_set_event_bytes(hgo *h, int32_t e, const uint8_t *body, int32_t body_len, const uint8_t *sig,
                        int32_t sig_len);
/* Roots of frame rr (a processed round), participant order: NextRound,
 * SelfParent (event id, -1 = the base root event), number of Others; then
 * the Others (key event -> RootEvent of the value event) of all roots in
 * order, each root's sorted by key hash.  Returns the total number of
 * Others, -1 if the frame has no roots. */
int32_t hgo_frame_roots(const hgo *h, int32_t rr, int32_t *next_round, int32_t *sp, int32_t *n_others,
                        int32_t *oth_key, int32_t *oth_val, int32_t cap);
/* Frame.Marshal of frame rr (with the Encoder's newline): returns its
 * length and copies up to cap bytes; -1 if unavailable */
int64_t hgo_frame_json(hgo *h, int32_t rr, uint8_t *buf, int64_t cap);
/* FrameHash of block blk (SHA-256 of its frame's JSON); -1 if unavailable */
int hgo_block_frame_hash(const hgo *h, int64_t blk, uint8_t *out32);
/* Block.Marshal (no signatures) or, body_only, BlockBody.Marshal of block blk */
int64_t hgo_block_json(hgo *h, int64_t blk, int body_only, uint8_t *buf, int64_t cap);
/* primitives, exposed for the ancestry known-answer tests */
int hgo_see(hgo *h, int32_t x, int32_t y);
int hgo_strongly_see(hgo *h, int32_t x, int32_t y);
int32_t hgo_round_of(hgo *h, int32_t x);
int32_t hgo_lamport_of(hgo *h, int32_t x);
int hgo_witness_of(hgo *h, int32_t x);

#ifdef __cplusplus
}
#endif
#endif
