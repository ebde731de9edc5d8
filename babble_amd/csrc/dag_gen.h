/*
 * dag_gen.h -- deterministic synthetic gossip DAG generator (bench/test input).
 *
 * Emits events exactly as Babble would create them:
 *  - participant keys: P-256 private key_i = SHA-256("babble-hip" || seed || i)
 *    mod q; ID = FNV-1a-32 of the 65-byte uncompressed public key
 *    (peers/peer.go:194-205, common/hash32.go:5-11); participants sorted by ID
 *    (peers/peers.go:63-73);
 *  - initial events: Index 0, parents ["Root<id>", ""], nil payloads
 *    (node/core_test.go:42-46);
 *  - gossip: `to` creates an event with self-parent = its head, other-parent =
 *    `from`'s head, index = seq+1 (node/core.go:285-313); peer choice excludes
 *    self and the last peer (node/peer_selector.go:39-55);
 *  - body hash: SHA-256 of Go encoding/json of EventBody + "\n"
 *    (hashgraph/event.go:32-56);
 *  - signature: ECDSA P-256 with deterministic nonce k = SHA-256(seed||hash)
 *    mod q, encoded r|s base 36 (crypto/utils.go:39-51).  sig_mode 0 replaces
 *    the EC math by r = SHA-256("r"||seed||hash) mod q (same distribution of
 *    the tie-break key, no verifiable signature) for very large DAGs.
 * Generation is not part of any timed region.
 */
#ifndef BABBLE_DAG_GEN_H
#define BABBLE_DAG_GEN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t n;          /* participants */
  int64_t N;          /* total events, including the n initial events */
  uint64_t seed;      /* e.g. 0xBABB1E00 + cfg */
  int32_t lagging;    /* number of lagging peers (C5: 21) */
  int32_t lag_div;    /* lagging peers are picked with weight 1/lag_div (C5: 50) */
  int32_t sig_mode;   /* 1 = deterministic ECDSA, 0 = synthetic r */
  int32_t threads;    /* worker threads for signatures (0 = auto) */
  double tx_prob;     /* probability of one transaction per event (0.5) */
} bg_params;

typedef struct {
  int32_t n;
  int64_t N;
  int64_t *participant_ids;   /* [n] ascending */
  uint8_t *pubkeys;           /* [n][65] in slot order */
  /* events in topological (insertion) order */
  int32_t *creator;           /* participant slot */
  int32_t *index;             /* Index in the creator's sequence */
  int32_t *self_parent;       /* global id, -1 = Root */
  int32_t *other_parent;      /* global id, -1 = "" */
  int32_t *ntx;               /* 0 or 1 transactions */
  uint8_t *hash;              /* [N][32] SHA-256 of the Go-JSON body */
  uint8_t *sig_r;             /* [N][32] big-endian r */
  uint8_t *sig_s;             /* [N][32] big-endian s */
} bg_dag;

int bg_generate(const bg_params *p, bg_dag *out);
void bg_free(bg_dag *d);
/* transaction bytes of event e (deterministic); returns length (<= 64) */
int32_t bg_tx_bytes(const bg_dag *d, int64_t e, uint8_t *buf64);
/* Go-JSON body of event e (for tests), returns length; buf must hold 1024 B */
int32_t bg_body_json(const bg_dag *d, int64_t e, char *buf);
/* FNV-1a-32 (common/hash32.go) */
/* Event.Signature of event e: crypto.EncodeSignature(r, s) = r and s in
 * base 36, lower case, joined by '|' (crypto/utils.go:39-41); returns the
 * length (at most 101) */
int32_t bg_sig_string(const bg_dag *d, int64_t e, char *buf);
/* bodies (EventBody.Marshal, with its newline) and signature strings of
 * events [first, first + count), concatenated; offsets get count + 1
 * entries each.  Buffers: at least 1024 * count and 104 * count bytes. */
void bg_event_bytes(const bg_dag *d, int64_t first, int64_t count, uint8_t *bodies, int64_t *body_offsets,
                    uint8_t *sigs, int64_t *sig_offsets);
uint32_t bg_fnv1a32(const uint8_t *data, int64_t len);

#ifdef __cplusplus
}
#endif
#endif
