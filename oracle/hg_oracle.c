/*
 * hg_oracle.c -- CPU restatement of the reference hashgraph consensus path.
 *
 * TEST INFRASTRUCTURE ONLY (see hg_oracle.h).  Used by tests/ as the parity
 * checker and by bench.py as the "CPU restatement of reference Go path,
 * 1 thread" baseline.  Never linked into libbabble_hip.
 *
 * Every function cites the Go code it restates (paths under
 * /root/reference/src).  Hash-string keys of the Go code become dense event
 * ids (insertion order == topologicalIndex, hashgraph.go:731-732); the LRU
 * memo caches become plain memo arrays (the reference runs batch consensus
 * with cacheSize >= #events, so nothing is ever evicted).
 */
#include "hg_oracle.h"

#include <limits.h>
#include <openssl/sha.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define UNSET INT32_MIN
#define FD_NONE INT32_MAX /* math.MaxInt32, hashgraph.go:447 */

/* Storage of the coordinate vectors.  The default keeps each Index as an
 * int32.  -DHGO_COORD16 (liboracle16.so, for whole-DAG digests of C4:
 * 512 x 20M events x 2 vectors would need 82 GB as int32) stores them as
 * uint16 -- LA as index + 1 (so -1 is 0), FD as the index or 0xFFFF for
 * MaxInt32 -- and aborts on an index it cannot hold.  Only the storage
 * changes; every comparison sees the decoded int32 values. */
#ifdef HGO_COORD16
typedef uint16_t coord_t;
#define COORD_MAX_INDEX 65533
static inline int32_t la_get(const coord_t *r, int32_t i) { return (int32_t)r[i] - 1; }
static inline void la_put(coord_t *r, int32_t i, int32_t v) { r[i] = (coord_t)(v + 1); }
static inline int32_t fd_get(const coord_t *r, int32_t i) { return r[i] == 0xFFFF ? FD_NONE : (int32_t)r[i]; }
static inline void fd_put(coord_t *r, int32_t i, int32_t v) { r[i] = v == FD_NONE ? (coord_t)0xFFFF : (coord_t)v; }
#else
typedef int32_t coord_t;
#define COORD_MAX_INDEX INT32_MAX
static inline int32_t la_get(const coord_t *r, int32_t i) { return r[i]; }
static inline void la_put(coord_t *r, int32_t i, int32_t v) { r[i] = v; }
static inline int32_t fd_get(const coord_t *r, int32_t i) { return r[i]; }
static inline void fd_put(coord_t *r, int32_t i, int32_t v) { r[i] = v; }
#endif

enum { TRI_UNDEFINED = 0, TRI_TRUE = 1, TRI_FALSE = 2 }; /* roundInfo.go:10-16 */

typedef struct {
  int32_t id;
  uint8_t witness;
  uint8_t famous; /* Trilean */
  uint8_t consensus;
} round_event; /* roundInfo.go:29-33 */

typedef struct {
  int exists;
  int queued; /* roundInfo.go:35 */
  round_event *ev;
  int32_t len, cap;
} round_info; /* roundInfo.go:33-42 */

typedef struct {
  int32_t index;
  int8_t decided;
} pending_round; /* roundInfo.go:22-25 */

struct hgo {
  int32_t n, sm;
  int64_t *pids;
  int64_t cap, N;
  /* event bodies */
  int32_t *creator, *index, *sp, *op, *ntx;
  uint8_t *hash, *sigr;
  /* coordinates: lastAncestors / firstDescendants indexes, [N][n]
   * (coord_t: see the storage note below) */
  coord_t *la, *fd;
  /* memo caches (hashgraph.go:36-40) */
  int32_t *round_memo, *lt_memo;
  /* Event private fields (event.go:107-116): nil == UNSET */
  int32_t *ev_round, *ev_lt, *ev_rr;
  /* RoundInfo.Events is a Go map keyed by event hash: an event has at most two
   * entries (its own round, and its round-received), indexed here for O(1)
   * lookup like the map */
  int32_t *ent_round[2], *ent_slot[2];
  /* participant event chains (ParticipantEventsCache) */
  int32_t **chain;
  int32_t *chain_len, *chain_cap;
  /* hashgraph state (hashgraph.go:19-34) */
  int32_t *und;
  int64_t und_len;
  pending_round *pend;
  int32_t pend_len, pend_cap;
  int has_lcr;
  int32_t lcr;
  int64_t consensus_txs, pending_loaded;
  /* InmemStore rounds / consensus / blocks (inmem_store.go) */
  round_info *rounds;
  int32_t rounds_cap;
  int32_t last_round;
  int32_t *cons;
  int64_t ncons;
  int64_t *cons_pos;
  int32_t *blk_rr;
  int64_t *blk_first, *blk_count, *blk_ntx;
  int64_t nblocks, blk_cap;
  /* frames cache (InmemStore.GetFrame/SetFrame, inmem_store.go:254-270) */
  int8_t *frame_done;
  int64_t *frame_first, *frame_len;
  int32_t *frame_ev;
  int64_t frame_ev_len;
  /* Frame roots (GetFrame, hashgraph.go:1150-1218), per frame round */
  struct frame_roots **roots;
  /* InmemStore.lastConsensusEvents (inmem_store.go:178-183): per slot, -1 = none */
  int32_t *last_cons;
  /* event bytes for Frame.Marshal (frame.go:17-26): Go-JSON body (no
   * trailing newline) and the Signature string, per event; optional */
  uint8_t **body, **sig;
  int32_t *body_len, *sig_len;
  /* FrameHash of each block (NewBlockFromFrame, block.go:100-110) */
  uint8_t *blk_fhash;
  int8_t *blk_has_fhash;
  /* the Store's Roots (inmem_store.go:221-227): base roots (root.go:98-106)
   * unless hgo_reset installed a Frame's roots (Hashgraph.Reset,
   * hashgraph.go:1324-1369).  Per participant slot: NextRound and the
   * SelfParent RootEvent's Index / LamportTimestamp / Round; chain positions
   * start at base = SelfParent.Index + 1 (the first event's Index) */
  int is_reset;
  int32_t *r_next, *r_sp_index, *r_sp_lt, *r_sp_round;
  uint8_t *r_sp_hash; /* [n][32] SelfParent.Hash of a Reset root (Index >= 0; "Root<id>" otherwise) */
  /* Root.Others: entry k belongs to the root of slot oth_root[k], keyed by
   * the hash of the event whose other-parent it describes (oth_key) */
  int32_t n_oth;
  int32_t *oth_root, *oth_creator, *oth_index, *oth_lt, *oth_round;
  uint8_t *oth_key, *oth_hash;
  /* per event: the Others entry its other-parent resolved to (op == -2) */
  int32_t *ext;
  int64_t blk_index0; /* LastBlockIndex()+1 of the first block (Reset: block.Index()+1) */
};

/* Root (root.go:88-96) of one participant in one frame: NextRound, the
 * SelfParent RootEvent (an event id, or -1 for the participant's Root
 * SelfParent: the base root event "Root<id>", root.go:75-84, or after a
 * Reset the installed Root's) and Others: key -> RootEvent, sorted by key
 * hash (Go's encoding/json sorts map keys).  A key or value >= 0 is an
 * event; OTH(k) = -2 - k is entry k of the Store Root's Others (after a
 * Reset: createOtherParentRootEvent returns it, hashgraph.go:568-578, and a
 * Root taken whole from the Store carries its map) */
#define OTH(k) (-2 - (k))
typedef struct {
  int32_t next_round, sp;
  int32_t n_others, cap_others;
  int32_t *oth_key, *oth_val;
} root_t;

struct frame_roots {
  root_t *r; /* [n] in participant order (Participants.ToPeerSlice) */
};

static void *xcalloc(size_t n, size_t s) {
  void *p = calloc(n ? n : 1, s);
  if (!p) abort();
  return p;
}
static void *xrealloc(void *p, size_t s) {
  void *q = realloc(p, s ? s : 1);
  if (!q) abort();
  return q;
}

hgo *hgo_create(int32_t n, const int64_t *participant_ids, int64_t capacity) {
  hgo *h = (hgo *)xcalloc(1, sizeof(hgo));
  h->n = n;
  h->sm = 2 * n / 3 + 1; /* hashgraph.go:54 */
  h->pids = (int64_t *)xcalloc(n, 8);
  memcpy(h->pids, participant_ids, (size_t)n * 8);
  h->cap = capacity;
  size_t C = (size_t)capacity;
  h->creator = (int32_t *)xcalloc(C, 4);
  h->index = (int32_t *)xcalloc(C, 4);
  h->sp = (int32_t *)xcalloc(C, 4);
  h->op = (int32_t *)xcalloc(C, 4);
  h->ntx = (int32_t *)xcalloc(C, 4);
  h->hash = (uint8_t *)xcalloc(C, 32);
  h->sigr = (uint8_t *)xcalloc(C, 32);
  h->la = (coord_t *)xcalloc(C * (size_t)n, sizeof(coord_t));
  h->fd = (coord_t *)xcalloc(C * (size_t)n, sizeof(coord_t));
  h->round_memo = (int32_t *)xcalloc(C, 4);
  h->lt_memo = (int32_t *)xcalloc(C, 4);
  h->ev_round = (int32_t *)xcalloc(C, 4);
  h->ev_lt = (int32_t *)xcalloc(C, 4);
  h->ev_rr = (int32_t *)xcalloc(C, 4);
  h->cons_pos = (int64_t *)xcalloc(C, 8);
  for (int k = 0; k < 2; k++) {
    h->ent_round[k] = (int32_t *)xcalloc(C, 4);
    h->ent_slot[k] = (int32_t *)xcalloc(C, 4);
  }
  h->und = (int32_t *)xcalloc(C, 4);
  h->cons = (int32_t *)xcalloc(C, 4);
  h->frame_ev = (int32_t *)xcalloc(C, 4);
  h->chain = (int32_t **)xcalloc(n, sizeof(int32_t *));
  h->chain_len = (int32_t *)xcalloc(n, 4);
  h->chain_cap = (int32_t *)xcalloc(n, 4);
  h->last_cons = (int32_t *)xcalloc(n, 4);
  for (int32_t i = 0; i < n; i++) h->last_cons[i] = -1;
  h->body = (uint8_t **)xcalloc(C, sizeof(uint8_t *));
  h->sig = (uint8_t **)xcalloc(C, sizeof(uint8_t *));
  h->body_len = (int32_t *)xcalloc(C, 4);
  h->sig_len = (int32_t *)xcalloc(C, 4);
  h->last_round = -1; /* inmem_store.go:45 */
  h->lcr = -1;
  h->ext = (int32_t *)xcalloc(C, 4);
  h->r_next = (int32_t *)xcalloc(n, 4);
  h->r_sp_index = (int32_t *)xcalloc(n, 4);
  h->r_sp_lt = (int32_t *)xcalloc(n, 4);
  h->r_sp_round = (int32_t *)xcalloc(n, 4);
  for (int32_t i = 0; i < n; i++) { /* NewBaseRoot (root.go:75-106) */
    h->r_next[i] = 0;
    h->r_sp_index[i] = h->r_sp_lt[i] = h->r_sp_round[i] = -1;
  }
  return h;
}

void hgo_destroy(hgo *h) {
  if (!h) return;
  free(h->pids);
  free(h->creator); free(h->index); free(h->sp); free(h->op); free(h->ntx);
  free(h->hash); free(h->sigr); free(h->la); free(h->fd);
  free(h->round_memo); free(h->lt_memo);
  free(h->ev_round); free(h->ev_lt); free(h->ev_rr); free(h->cons_pos);
  for (int k = 0; k < 2; k++) { free(h->ent_round[k]); free(h->ent_slot[k]); }
  free(h->und); free(h->cons); free(h->frame_ev);
  for (int i = 0; i < h->n; i++) free(h->chain[i]);
  free(h->chain); free(h->chain_len); free(h->chain_cap);
  free(h->pend);
  for (int32_t r = 0; r < h->rounds_cap; r++) free(h->rounds[r].ev);
  free(h->rounds);
  free(h->blk_rr); free(h->blk_first); free(h->blk_count); free(h->blk_ntx);
  free(h->frame_done); free(h->frame_first); free(h->frame_len);
  for (int32_t r = 0; r < h->rounds_cap; r++) {
    if (!h->roots || !h->roots[r]) continue;
    for (int32_t i = 0; i < h->n; i++) { free(h->roots[r]->r[i].oth_key); free(h->roots[r]->r[i].oth_val); }
    free(h->roots[r]->r);
    free(h->roots[r]);
  }
  free(h->roots);
  free(h->r_sp_hash);
  free(h->last_cons);
  for (int64_t e = 0; e < h->cap; e++) { free(h->body[e]); free(h->sig[e]); }
  free(h->body); free(h->sig); free(h->body_len); free(h->sig_len);
  free(h->blk_fhash); free(h->blk_has_fhash);
  free(h->ext); free(h->r_next); free(h->r_sp_index); free(h->r_sp_lt); free(h->r_sp_round);
  free(h->oth_root); free(h->oth_creator); free(h->oth_index); free(h->oth_lt); free(h->oth_round);
  free(h->oth_key); free(h->oth_hash);
  free(h);
}

/* ------------------------------------------------------------------------ */
/* InmemStore rounds (inmem_store.go:185-211)                               */

static void ensure_round_cap(hgo *h, int32_t r) {
  if (r < h->rounds_cap) return;
  int32_t nc = h->rounds_cap ? h->rounds_cap : 64;
  while (nc <= r) nc *= 2;
  h->rounds = (round_info *)xrealloc(h->rounds, (size_t)nc * sizeof(round_info));
  memset(h->rounds + h->rounds_cap, 0, (size_t)(nc - h->rounds_cap) * sizeof(round_info));
  h->frame_done = (int8_t *)xrealloc(h->frame_done, (size_t)nc);
  memset(h->frame_done + h->rounds_cap, 0, (size_t)(nc - h->rounds_cap));
  h->frame_first = (int64_t *)xrealloc(h->frame_first, (size_t)nc * 8);
  h->frame_len = (int64_t *)xrealloc(h->frame_len, (size_t)nc * 8);
  h->roots = (struct frame_roots **)xrealloc(h->roots, (size_t)nc * sizeof(struct frame_roots *));
  memset(h->roots + h->rounds_cap, 0, (size_t)(nc - h->rounds_cap) * sizeof(struct frame_roots *));
  h->rounds_cap = nc;
}

/* GetRound: KeyNotFound for missing rounds (inmem_store.go:185-191) */
static round_info *get_round(hgo *h, int32_t r) {
  if (r < 0 || r >= h->rounds_cap || !h->rounds[r].exists) return NULL;
  return &h->rounds[r];
}

/* SetRound tracks LastRound (inmem_store.go:193-199) */
static round_info *set_round(hgo *h, int32_t r) {
  ensure_round_cap(h, r);
  h->rounds[r].exists = 1;
  if (r > h->last_round) h->last_round = r;
  return &h->rounds[r];
}

static round_event *ri_find(hgo *h, int32_t r, int32_t x) {
  for (int k = 0; k < 2; k++)
    if (h->ent_round[k][x] == r) return &h->rounds[r].ev[h->ent_slot[k][x]];
  return NULL;
}

static round_event *ri_append(hgo *h, int32_t r, int32_t x) {
  round_info *ri = &h->rounds[r];
  if (ri->len == ri->cap) {
    ri->cap = ri->cap ? 2 * ri->cap : 8;
    ri->ev = (round_event *)xrealloc(ri->ev, (size_t)ri->cap * sizeof(round_event));
  }
  int k = h->ent_round[0][x] == INT32_MIN ? 0 : 1;
  h->ent_round[k][x] = r;
  h->ent_slot[k][x] = ri->len;
  round_event *e = &ri->ev[ri->len++];
  e->id = x; e->witness = 0; e->famous = TRI_UNDEFINED; e->consensus = 0;
  return e;
}

/* RoundInfo.AddEvent (roundInfo.go:44-51) */
static void ri_add_event(hgo *h, int32_t r, int32_t x, int witness) {
  if (!ri_find(h, r, x)) ri_append(h, r, x)->witness = (uint8_t)witness;
}

/* RoundInfo.Witnesses (roundInfo.go:88-96) into buf; returns count */
static int32_t ri_witnesses(const round_info *ri, int32_t **buf, int32_t *bcap) {
  int32_t k = 0;
  if (!ri) return 0;
  for (int32_t i = 0; i < ri->len; i++) {
    if (!ri->ev[i].witness) continue;
    if (k == *bcap) {
      *bcap = *bcap ? 2 * *bcap : 64;
      *buf = (int32_t *)xrealloc(*buf, (size_t)*bcap * 4);
    }
    (*buf)[k++] = ri->ev[i].id;
  }
  return k;
}

/* RoundInfo.WitnessesDecided (roundInfo.go:78-85) */
static int ri_witnesses_decided(const round_info *ri) {
  for (int32_t i = 0; i < ri->len; i++)
    if (ri->ev[i].witness && ri->ev[i].famous == TRI_UNDEFINED) return 0;
  return 1;
}

/* ------------------------------------------------------------------------ */
/* ancestry primitives                                                       */

static inline coord_t *LA(const hgo *h, int32_t e) { return h->la + (size_t)e * h->n; }
static inline coord_t *FD(const hgo *h, int32_t e) { return h->fd + (size_t)e * h->n; }

/* _ancestor / see (hashgraph.go:92-117, 152-157) */
static int see(const hgo *h, int32_t x, int32_t y) {
  if (x == y) return 1;
  return la_get(LA(h, x), h->creator[y]) >= h->index[y];
}

/* _stronglySee (hashgraph.go:172-191) */
static int strongly_see(const hgo *h, int32_t x, int32_t y) {
  const coord_t *lx = LA(h, x), *fy = FD(h, y);
  int c = 0;
  for (int32_t i = 0; i < h->n; i++) c += la_get(lx, i) >= fd_get(fy, i);
  return c >= h->sm;
}

/* round / _round (hashgraph.go:193-278) with the Store's Roots (root.go):
 * sp < 0 is the creator's Root SelfParent (rootsBySelfParent, :211-214);
 * op == -2 is an other-parent known only through Root.Others. */
static int32_t round_of(hgo *h, int32_t x);

static int32_t *g_wbuf;
static int32_t g_wcap;

/* Root.Others[ev.Hex()] of ev's creator's Root: the entry index, or -1 */
static int32_t others_key(const hgo *h, int32_t x) {
  for (int32_t k = 0; k < h->n_oth; k++)
    if (h->oth_root[k] == h->creator[x] && !memcmp(h->oth_key + (size_t)k * 32, h->hash + (size_t)x * 32, 32))
      return k;
  return -1;
}

/* the hash of x's other-parent (a store event, or the Root.Others entry it
 * resolved to at insert) */
static const uint8_t *op_hash(const hgo *h, int32_t x) {
  return h->op[x] >= 0 ? h->hash + (size_t)h->op[x] * 32 : h->oth_hash + (size_t)h->ext[x] * 32;
}

/* `other, ok := root.Others[ex.Hex()]; ok && other.Hash == ex.OtherParent()` */
static int32_t others_match(const hgo *h, int32_t x) {
  if (h->op[x] == -1) return -1;
  const int32_t k = others_key(h, x);
  return k >= 0 && !memcmp(h->oth_hash + (size_t)k * 32, op_hash(h, x), 32) ? k : -1;
}

/* round of x's self-parent: the Root's SelfParent.Round for a first event */
static int32_t sp_round_of(hgo *h, int32_t x) {
  return h->sp[x] < 0 ? h->r_sp_round[h->creator[x]] : round_of(h, h->sp[x]);
}

static int32_t round_impl(hgo *h, int32_t x) {
  int32_t sp = h->sp[x], op = h->op[x];
  const int32_t cr = h->creator[x];
  /* directly attached to the Root: authoritative unless the other-parent is
   * a real event outside Root.Others (:229-236) */
  if (sp < 0 && (op == -1 || others_match(h, x) >= 0)) return h->r_next[cr];
  int32_t pr = sp_round_of(h, x);
  if (op != -1) {
    /* an other-parent in Root.Others takes Root.NextRound (:246-256) */
    int32_t opr = others_match(h, x) >= 0 ? h->r_next[cr] : round_of(h, op);
    if (opr > pr) pr = opr;
  }
  /* count the parentRound witnesses that x strongly sees */
  int32_t nw = ri_witnesses(get_round(h, pr), &g_wbuf, &g_wcap);
  int c = 0;
  for (int32_t i = 0; i < nw; i++) c += strongly_see(h, x, g_wbuf[i]);
  if (c >= h->sm) pr++;
  return pr;
}

static int32_t round_of(hgo *h, int32_t x) {
  if (h->round_memo[x] != UNSET) return h->round_memo[x];
  int32_t r = round_impl(h, x);
  h->round_memo[x] = r;
  return r;
}

/* witness (hashgraph.go:281-296) */
static int witness_of(hgo *h, int32_t x) { return round_of(h, x) > sp_round_of(h, x); }

/* lamportTimestamp / _lamportTimestamp (hashgraph.go:313-379): a first
 * event's self-parent is the Root's SelfParent (:347-349); an other-parent
 * not in the Store takes the LamportTimestamp of its Root.Others entry
 * (:358-375) */
static int32_t lamport_of(hgo *h, int32_t x) {
  if (h->lt_memo[x] != UNSET) return h->lt_memo[x];
  int32_t plt = h->sp[x] < 0 ? h->r_sp_lt[h->creator[x]] : lamport_of(h, h->sp[x]);
  if (h->op[x] != -1) {
    int32_t o = INT32_MIN;
    if (h->op[x] >= 0) {
      o = lamport_of(h, h->op[x]);
    } else {
      const int32_t k = others_match(h, x);
      if (k >= 0) o = h->oth_lt[k];
    }
    if (o > plt) plt = o;
  }
  h->lt_memo[x] = plt + 1;
  return plt + 1;
}

/* ------------------------------------------------------------------------ */
/* InsertEvent (hashgraph.go:714-761)                                        */

static void chain_push(hgo *h, int32_t c, int32_t id) {
  if (h->chain_len[c] == h->chain_cap[c]) {
    h->chain_cap[c] = h->chain_cap[c] ? 2 * h->chain_cap[c] : 64;
    h->chain[c] = (int32_t *)xrealloc(h->chain[c], (size_t)h->chain_cap[c] * 4);
  }
  h->chain[c][h->chain_len[c]++] = id;
}

int hgo_insert(hgo *h, int32_t creator, int32_t index, int32_t sp, int32_t op,
               const uint8_t *hash32, const uint8_t *sig_r32, int32_t ntx) {
  return hgo_insert_ext(h, creator, index, sp, op, -1, -1, hash32, sig_r32, ntx);
}

int hgo_insert_ext(hgo *h, int32_t creator, int32_t index, int32_t sp, int32_t op, int32_t op_creator,
                   int32_t op_index, const uint8_t *hash32, const uint8_t *sig_r32, int32_t ntx) {
  if (creator < 0 || creator >= h->n) return HGO_ERR_BAD_CREATOR;
  if (h->N >= h->cap) return HGO_ERR_CAPACITY;
  /* checkSelfParent: self-parent must be the creator's last known event,
   * or its Root when it has none (hashgraph.go:398-414, inmem_store.go:118-134) */
  int32_t clen = h->chain_len[creator];
  int32_t last = clen ? h->chain[creator][clen - 1] : -1;
  if (sp != last) return HGO_ERR_SELF_PARENT;
  /* checkOtherParent (hashgraph.go:417-436); an other-parent the Store does
   * not hold is looked up in the creator's Root.Others: by (creator, index)
   * as ReadWireInfo resolves it (:1431-1457), then keyed by the event's own
   * hash with the same Hash (:424-431) */
  int32_t ext = -1;
  if (op == -2) {
    int32_t k = -1;
    for (int32_t q = 0; q < h->n_oth && k < 0; q++)
      if (h->oth_root[q] == creator && h->oth_creator[q] == op_creator && h->oth_index[q] == op_index) k = q;
    if (k < 0) return HGO_ERR_OTHER_PARENT;
    int32_t k2 = -1;
    for (int32_t q = 0; q < h->n_oth && k2 < 0; q++)
      if (h->oth_root[q] == creator && !memcmp(h->oth_key + (size_t)q * 32, hash32, 32)) k2 = q;
    if (k2 < 0 || memcmp(h->oth_hash + (size_t)k2 * 32, h->oth_hash + (size_t)k * 32, 32)) return HGO_ERR_OTHER_PARENT;
    ext = k2;
  } else if (op >= h->N || op < -1) {
    return HGO_ERR_OTHER_PARENT;
  }
  /* Index continuity: ParticipantEventsCache.Set rejects skipped/passed
   * indexes (caches.go / common/rolling_index.go:58-96); chains start at the
   * Root's SelfParent.Index + 1 */
  if (index != h->r_sp_index[creator] + 1 + clen) return HGO_ERR_SELF_PARENT;
  if (index > COORD_MAX_INDEX) {
    fprintf(stderr, "hg_oracle: index %d exceeds this build's coordinate storage\n", index);
    abort();
  }

  int32_t x = (int32_t)h->N++;
  h->creator[x] = creator; h->index[x] = index; h->sp[x] = sp; h->op[x] = op;
  h->ext[x] = ext;
  h->ntx[x] = ntx;
  memcpy(h->hash + (size_t)x * 32, hash32, 32);
  memcpy(h->sigr + (size_t)x * 32, sig_r32, 32);
  h->round_memo[x] = UNSET; h->lt_memo[x] = UNSET;
  h->ev_round[x] = UNSET; h->ev_lt[x] = UNSET; h->ev_rr[x] = UNSET;
  h->cons_pos[x] = -1;
  h->ent_round[0][x] = h->ent_round[1][x] = INT32_MIN;

  /* initEventCoordinates (hashgraph.go:439-507) */
  int32_t n = h->n;
  coord_t *la = LA(h, x), *fd = FD(h, x);
  for (int32_t i = 0; i < n; i++) fd_put(fd, i, FD_NONE);
  /* parents the Store does not hold (Roots, Root.Others) contribute nothing */
  if (sp < 0 && op < 0) {
    for (int32_t i = 0; i < n; i++) la_put(la, i, -1);
  } else if (sp < 0) {
    memcpy(la, LA(h, op), (size_t)n * sizeof(coord_t));
  } else if (op < 0) {
    memcpy(la, LA(h, sp), (size_t)n * sizeof(coord_t));
  } else {
    const coord_t *a = LA(h, sp), *b = LA(h, op);
    for (int32_t i = 0; i < n; i++) {
      const int32_t u = la_get(a, i), v = la_get(b, i);
      la_put(la, i, u < v ? v : u);
    }
  }
  fd_put(fd, creator, index);
  la_put(la, creator, index);
  chain_push(h, creator, x); /* Store.SetEvent -> addParticipantEvent */

  /* updateAncestorFirstDescendant (hashgraph.go:510-544): walk each last
   * ancestor's self-parent chain while its firstDescendant is unset */
  for (int32_t i = 0; i < n; i++) {
    const int32_t base = h->r_sp_index[i] + 1; /* Index of chain i's first event */
    int32_t k = la_get(la, i);
    while (k >= base) {
      int32_t a = h->chain[i][k - base];
      coord_t *fa = FD(h, a);
      if (fd_get(fa, creator) != FD_NONE) break;
      fd_put(fa, creator, index);
      k--; /* a.SelfParent(); the Root is not an event -> GetEvent fails -> break */
    }
  }

  h->und[h->und_len++] = x; /* UndeterminedEvents */
  if (index == 0 || ntx > 0) h->pending_loaded++; /* IsLoaded, event.go:169-178 */
  return HGO_OK;
}

int64_t hgo_insert_batch(hgo *h, int64_t count, const int32_t *creator, const int32_t *index,
                         const int32_t *sp, const int32_t *op, const uint8_t *hash32,
                         const uint8_t *sig_r32, const int32_t *ntx) {
  int64_t bad = 0;
  for (int64_t e = 0; e < count; e++)
    bad += hgo_insert(h, creator[e], index[e], sp[e], op[e], hash32 + (size_t)e * 32,
                      sig_r32 + (size_t)e * 32, ntx[e]) != HGO_OK;
  return bad;
}

int64_t hgo_insert_batch_ext(hgo *h, int64_t count, const int32_t *creator, const int32_t *index,
                             const int32_t *sp, const int32_t *op, const int32_t *op_creator,
                             const int32_t *op_index, const uint8_t *hash32, const uint8_t *sig_r32,
                             const int32_t *ntx, int32_t *status) {
  int64_t bad = 0;
  for (int64_t e = 0; e < count; e++) {
    const int rc = hgo_insert_ext(h, creator[e], index[e], sp[e], op[e], op_creator[e], op_index[e],
                                  hash32 + (size_t)e * 32, sig_r32 + (size_t)e * 32, ntx[e]);
    if (status) status[e] = rc;
    bad += rc != HGO_OK;
  }
  return bad;
}

/* Hashgraph.Reset(block, frame) (hashgraph.go:1324-1369) minus the frame's
 * events (the caller inserts them next, as Reset does): Store.Reset(roots)
 * (inmem_store.go:272-282), SetBlock(block) (LastBlockIndex = its Index),
 * setLastConsensusRound(block.RoundReceived()).  Fresh hashgraphs only. */
int hgo_reset(hgo *h, int32_t round_received, int64_t block_index, const int32_t *next_round,
              const int32_t *sp_index, const int32_t *sp_lt, const int32_t *sp_round, int32_t n_others,
              const int32_t *oth_root, const uint8_t *oth_key32, const int32_t *oth_creator,
              const int32_t *oth_index, const int32_t *oth_lt, const int32_t *oth_round,
              const uint8_t *oth_hash32, const uint8_t *sp_hash32) {
  if (h->N || h->is_reset || n_others < 0) return HGO_ERR_STATE;
  for (int32_t i = 0; i < h->n; i++) {
    h->r_next[i] = next_round[i];
    h->r_sp_index[i] = sp_index[i];
    h->r_sp_lt[i] = sp_lt[i];
    h->r_sp_round[i] = sp_round[i];
  }
  if (sp_hash32) {
    h->r_sp_hash = (uint8_t *)xcalloc((size_t)h->n, 32);
    memcpy(h->r_sp_hash, sp_hash32, (size_t)h->n * 32);
  }
  const size_t K = (size_t)n_others;
  h->n_oth = n_others;
  h->oth_root = (int32_t *)xcalloc(K, 4);
  h->oth_creator = (int32_t *)xcalloc(K, 4);
  h->oth_index = (int32_t *)xcalloc(K, 4);
  h->oth_lt = (int32_t *)xcalloc(K, 4);
  h->oth_round = (int32_t *)xcalloc(K, 4);
  h->oth_key = (uint8_t *)xcalloc(K, 32);
  h->oth_hash = (uint8_t *)xcalloc(K, 32);
  if (K) {
    memcpy(h->oth_root, oth_root, K * 4);
    memcpy(h->oth_creator, oth_creator, K * 4);
    memcpy(h->oth_index, oth_index, K * 4);
    memcpy(h->oth_lt, oth_lt, K * 4);
    memcpy(h->oth_round, oth_round, K * 4);
    memcpy(h->oth_key, oth_key32, K * 32);
    memcpy(h->oth_hash, oth_hash32, K * 32);
  }
  h->is_reset = 1;
  h->blk_index0 = block_index + 1;
  h->has_lcr = 1;
  h->lcr = round_received;
  return HGO_OK;
}

void hgo_known(const hgo *h, int32_t *known) { /* InmemStore.KnownEvents (inmem_store.go:152-163) */
  for (int32_t i = 0; i < h->n; i++) known[i] = h->r_sp_index[i] + h->chain_len[i];
}

/* ------------------------------------------------------------------------ */
/* DivideRounds (hashgraph.go:767-849)                                       */

int hgo_divide_rounds(hgo *h) {
  for (int64_t u = 0; u < h->und_len; u++) {
    int32_t x = h->und[u];
    if (h->ev_round[x] == UNSET) {
      int32_t r = round_of(h, x);
      h->ev_round[x] = r;
      round_info *ri = get_round(h, r);
      int fresh = ri == NULL; /* GetRound KeyNotFound -> NewRoundInfo */
      if (fresh) { ensure_round_cap(h, r); ri = &h->rounds[r]; }
      if (!ri->queued && (!h->has_lcr || r >= h->lcr)) {
        if (h->pend_len == h->pend_cap) {
          h->pend_cap = h->pend_cap ? 2 * h->pend_cap : 64;
          h->pend = (pending_round *)xrealloc(h->pend, (size_t)h->pend_cap * sizeof(pending_round));
        }
        h->pend[h->pend_len].index = r;
        h->pend[h->pend_len].decided = 0;
        h->pend_len++;
        ri->queued = 1;
      }
      int w = witness_of(h, x);
      ri_add_event(h, r, x, w);
      set_round(h, r);
    }
    if (h->ev_lt[x] == UNSET) h->ev_lt[x] = lamport_of(h, x);
  }
  return HGO_OK;
}

/* ------------------------------------------------------------------------ */
/* DecideFame (hashgraph.go:852-947)                                         */

static int middle_bit(const hgo *h, int32_t y) { /* hashgraph.go:1526-1535 */
  return h->hash[(size_t)y * 32 + 16] != 0;
}

int hgo_decide_fame(hgo *h) {
  int32_t *W = NULL, wcap = 0;      /* Witnesses of round r */
  int32_t *Wj = NULL, wjcap = 0;    /* RoundWitnesses(j) */
  int32_t *Wp = NULL, wpcap = 0;    /* RoundWitnesses(j-1) */
  /* The Go votes map is keyed [y][x]; for a fixed x the j iteration only
   * reads the votes cast in round j-1, so two arrays indexed by witness
   * position carry exactly the same data flow. */
  int8_t *vprev = NULL, *vcur = NULL;
  int32_t vcap = 0;
  int8_t *decided = (int8_t *)xcalloc((size_t)h->pend_len, 1);

  for (int32_t pos = 0; pos < h->pend_len; pos++) {
    int32_t r = h->pend[pos].index;
    round_info *ri = get_round(h, r);
    if (!ri) { free(W); free(Wj); free(Wp); free(vprev); free(vcur); free(decided); return HGO_ERR_STATE; }
    int32_t nw = ri_witnesses(ri, &W, &wcap);
    for (int32_t xi = 0; xi < nw; xi++) {
      int32_t x = W[xi];
      round_event *rex = ri_find(h, r, x);
      if (rex && rex->witness && rex->famous != TRI_UNDEFINED) continue; /* IsDecided */
      int32_t nprev = 0;
      for (int32_t j = r + 1; j <= h->last_round; j++) {
        int32_t nj = ri_witnesses(get_round(h, j), &Wj, &wjcap);
        if (nj > vcap) {
          vcap = nj * 2;
          vprev = (int8_t *)xrealloc(vprev, (size_t)vcap);
          vcur = (int8_t *)xrealloc(vcur, (size_t)vcap);
        }
        int32_t diff = j - r;
        int decided_x = 0;
        for (int32_t yi = 0; yi < nj; yi++) {
          int32_t y = Wj[yi];
          if (diff == 1) {
            vcur[yi] = (int8_t)see(h, y, x);
          } else {
            int32_t np = ri_witnesses(get_round(h, j - 1), &Wp, &wpcap);
            int yays = 0, nays = 0;
            for (int32_t wi = 0; wi < np; wi++) {
              if (!strongly_see(h, y, Wp[wi])) continue;
              if (wi < nprev && vprev[wi]) yays++;
              else nays++;
            }
            int v = 0, t = nays;
            if (yays >= nays) { v = 1; t = yays; }
            if (diff % h->n > 0) { /* normal round: math.Mod(diff, n) > 0 */
              if (t >= h->sm) {
                rex->famous = v ? TRI_TRUE : TRI_FALSE; /* SetFame */
                vcur[yi] = (int8_t)v;
                decided_x = 1;
                break; /* break VOTE_LOOP */
              }
              vcur[yi] = (int8_t)v;
            } else { /* coin round */
              vcur[yi] = (int8_t)(t >= h->sm ? v : middle_bit(h, y));
            }
          }
        }
        if (decided_x) break;
        int8_t *tmp = vprev; vprev = vcur; vcur = tmp;
        nprev = nj;
      }
    }
    set_round(h, r);
    if (ri_witnesses_decided(ri)) decided[pos] = 1;
  }
  /* updatePendingRounds (hashgraph.go:689-695) */
  for (int32_t pos = 0; pos < h->pend_len; pos++)
    if (decided[pos]) h->pend[pos].decided = 1;
  free(W); free(Wj); free(Wp); free(vprev); free(vcur); free(decided);
  return HGO_OK;
}

/* ------------------------------------------------------------------------ */
/* DecideRoundReceived (hashgraph.go:951-1036)                               */

int hgo_decide_round_received(hgo *h) {
  int32_t *FW = NULL;
  int32_t fcap = 0;
  int64_t keep = 0;
  for (int64_t u = 0; u < h->und_len; u++) {
    int32_t x = h->und[u];
    int received = 0;
    int32_t r = round_of(h, x);
    for (int32_t i = r + 1; i <= h->last_round; i++) {
      round_info *tr = get_round(h, i);
      if (!tr) {
        if (h->has_lcr && r < h->lcr) { received = 1; break; }
        free(FW);
        return HGO_ERR_STATE;
      }
      if (!ri_witnesses_decided(tr)) break;
      /* FamousWitnesses (roundInfo.go:120-128) */
      int32_t nf = 0;
      for (int32_t k = 0; k < tr->len; k++) {
        if (!(tr->ev[k].witness && tr->ev[k].famous == TRI_TRUE)) continue;
        if (nf == fcap) { fcap = fcap ? 2 * fcap : 64; FW = (int32_t *)xrealloc(FW, (size_t)fcap * 4); }
        FW[nf++] = tr->ev[k].id;
      }
      int32_t s = 0;
      for (int32_t k = 0; k < nf; k++) s += see(h, FW[k], x);
      if (s == nf && s > 0) {
        received = 1;
        h->ev_rr[x] = i;
        /* RoundInfo.SetConsensusEvent (roundInfo.go:53-60) */
        round_event *e = ri_find(h, i, x);
        if (!e) e = ri_append(h, i, x);
        e->consensus = 1;
        set_round(h, i);
        break;
      }
    }
    if (!received) h->und[keep++] = x;
  }
  h->und_len = keep;
  free(FW);
  return HGO_OK;
}

/* ------------------------------------------------------------------------ */
/* GetFrame + ProcessDecidedRounds (hashgraph.go:1041-1231)                  */

static const hgo *g_sort_h;
/* ByLamportTimestamp.Less (event.go:332-347): LT, then the ECDSA r parsed
 * as a big.Int.  r is held as 32 big-endian bytes, so memcmp == Cmp. */
static int cmp_lamport(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  int32_t tx = g_sort_h->ev_lt[x] == UNSET ? -1 : g_sort_h->ev_lt[x];
  int32_t ty = g_sort_h->ev_lt[y] == UNSET ? -1 : g_sort_h->ev_lt[y];
  if (tx != ty) return tx < ty ? -1 : 1;
  return memcmp(g_sort_h->sigr + (size_t)x * 32, g_sort_h->sigr + (size_t)y * 32, 32);
}

static int get_frame(hgo *h, int32_t rr, int64_t *first, int64_t *len) {
  ensure_round_cap(h, rr);
  if (h->frame_done[rr]) { *first = h->frame_first[rr]; *len = h->frame_len[rr]; return HGO_OK; }
  round_info *ri = get_round(h, rr);
  if (!ri) return HGO_ERR_STATE;
  int64_t f = h->frame_ev_len;
  for (int32_t k = 0; k < ri->len; k++)
    if (ri->ev[k].consensus) h->frame_ev[h->frame_ev_len++] = ri->ev[k].id;
  int64_t l = h->frame_ev_len - f;
  g_sort_h = h;
  qsort(h->frame_ev + f, (size_t)l, 4, cmp_lamport); /* sort.Sort(ByLamportTimestamp) */
  h->frame_done[rr] = 1; h->frame_first[rr] = f; h->frame_len[rr] = l;
  *first = f; *len = l;
  return HGO_OK;
}

/* ------------------------------------------------------------------------ */
/* Frame roots (GetFrame hashgraph.go:1150-1218, createRoot :546-640)         */

static void root_add_other(root_t *r, int32_t key, int32_t val) {
  if (r->n_others == r->cap_others) {
    r->cap_others = r->cap_others ? 2 * r->cap_others : 4;
    r->oth_key = (int32_t *)xrealloc(r->oth_key, (size_t)r->cap_others * 4);
    r->oth_val = (int32_t *)xrealloc(r->oth_val, (size_t)r->cap_others * 4);
  }
  r->oth_key[r->n_others] = key;
  r->oth_val[r->n_others] = val;
  r->n_others++;
}

/* createRoot(ev) (hashgraph.go:602-640): NextRound = round(ev); SelfParent =
 * the RootEvent of ev's self-parent (for a first event, its creator's base
 * Root event "Root<id>" with Index / LamportTimestamp / Round -1:
 * createSelfParentRootEvent :546-566 reads them from the Root, root.go:73-84);
 * Others[ev] = the RootEvent of its other-parent (createOtherParentRootEvent
 * :568-600 -- a base Root has no Others to take it from) */
static int32_t others_match(const hgo *h, int32_t x);

/* createOtherParentRootEvent(ev) (hashgraph.go:568-600): the creator's Root
 * entry keyed by ev when it names ev's other-parent, else the other-parent */
static int32_t other_root_event(const hgo *h, int32_t ev) {
  const int32_t k = others_match(h, ev);
  return k >= 0 ? OTH(k) : h->op[ev];
}

static void create_root(hgo *h, int32_t ev, root_t *r) {
  r->next_round = round_of(h, ev);
  r->sp = h->sp[ev] >= 0 ? h->sp[ev] : -1;
  if (h->op[ev] != -1) root_add_other(r, ev, other_root_event(h, ev));
}

/* the hash a key stands for: an event's, or Others entry k's key */
static const uint8_t *key_hash(const hgo *h, int32_t key) {
  return key >= 0 ? h->hash + (size_t)key * 32 : h->oth_key + (size_t)(-2 - key) * 32;
}

static int cmp_hash_of(const hgo *hh, int32_t a, int32_t b) { return memcmp(key_hash(hh, a), key_hash(hh, b), 32); }

/* the roots of frame rr, whose sorted events are frame_ev[f .. f + l);
 * lastConsensusEvents as they stand before the frame's events are added */
static void frame_roots(hgo *h, int32_t rr, int64_t f, int64_t l) {
  ensure_round_cap(h, rr);
  if (h->roots[rr]) return; /* GetFrame is cached by the Store (inmem_store.go:254-270) */
  const int32_t n = h->n;
  struct frame_roots *fr = (struct frame_roots *)xcalloc(1, sizeof *fr);
  fr->r = (root_t *)xcalloc((size_t)n, sizeof(root_t));
  int8_t *has = (int8_t *)xcalloc((size_t)n, 1);
  /* "Each time we run into the first Event of a participant, we create a
   * Root for it" (:1161-1172) */
  for (int64_t k = 0; k < l; k++) {
    const int32_t ev = h->frame_ev[f + k], p = h->creator[ev];
    if (!has[p]) { has[p] = 1; create_root(h, ev, &fr->r[p]); }
  }
  /* participants with no event in the frame: createRoot(last consensus
   * event) or, with none, their Root from the Store (:1174-1197): a base
   * Root, or the Root a Reset installed, whole, Others included */
  for (int32_t p = 0; p < n; p++) {
    if (has[p]) continue;
    if (h->last_cons[p] >= 0) {
      create_root(h, h->last_cons[p], &fr->r[p]);
    } else {
      fr->r[p].next_round = h->r_next[p];
      fr->r[p].sp = -1;
      for (int32_t k = 0; k < h->n_oth; k++) {
        if (h->oth_root[k] != p) continue;
        int dup = 0; /* a Go map holds one entry per key (the first here, as the engine) */
        for (int32_t q = 0; q < k && !dup; q++)
          dup = h->oth_root[q] == p && !memcmp(h->oth_key + (size_t)q * 32, h->oth_key + (size_t)k * 32, 32);
        if (!dup) root_add_other(&fr->r[p], OTH(k), OTH(k));
      }
    }
  }
  /* other-parents outside the frame (:1199-1218): `treated` holds the
   * frame's events met so far in sorted order; an event whose other-parent
   * is not among them, and which is not the event its creator's root was
   * made from (same self-parent), adds its other-parent to that root */
  int8_t *treated = (int8_t *)xcalloc((size_t)(h->N ? h->N : 1), 1);
  for (int64_t k = 0; k < l; k++) {
    const int32_t ev = h->frame_ev[f + k];
    treated[ev] = 1;
    const int32_t op = h->op[ev];
    const int32_t spr = h->sp[ev] >= 0 ? h->sp[ev] : -1;
    if (op != -1 && !(op >= 0 && treated[op]) && spr != fr->r[h->creator[ev]].sp)
      root_add_other(&fr->r[h->creator[ev]], ev, other_root_event(h, ev));
  }
  free(treated);
  free(has);
  /* Go's encoding/json writes map keys sorted ("0x" + uppercase hex: the
   * string order is the hash byte order) */
  for (int32_t p = 0; p < n; p++) {
    root_t *r = &fr->r[p];
    for (int32_t a = 1; a < r->n_others; a++) {
      const int32_t kk = r->oth_key[a], vv = r->oth_val[a];
      int32_t b = a - 1;
      while (b >= 0 && cmp_hash_of(h, kk, r->oth_key[b]) < 0) {
        r->oth_key[b + 1] = r->oth_key[b];
        r->oth_val[b + 1] = r->oth_val[b];
        b--;
      }
      r->oth_key[b + 1] = kk;
      r->oth_val[b + 1] = vv;
    }
  }
  h->roots[rr] = fr;
}

/* ---- Go encoding/json (json.NewEncoder(..).Encode) of Frame / Block ---- */
typedef struct { uint8_t *p; int64_t len, cap; } jbuf;
static void jput(jbuf *b, const void *src, int64_t n) {
  if (b->len + n > b->cap) {
    while (b->len + n > b->cap) b->cap = b->cap ? 2 * b->cap : 4096;
    b->p = (uint8_t *)xrealloc(b->p, (size_t)b->cap);
  }
  memcpy(b->p + b->len, src, (size_t)n);
  b->len += n;
}
static void jstr(jbuf *b, const char *s) { jput(b, s, (int64_t)strlen(s)); }
static void jint(jbuf *b, long long v) {
  char t[32];
  jput(b, t, snprintf(t, sizeof t, "%lld", v));
}
/* Event.Hex() = fmt.Sprintf("0x%X", hash) (event.go:239-245) */
static void jhexb(jbuf *b, const uint8_t *x) {
  static const char HX[] = "0123456789ABCDEF";
  char t[66];
  t[0] = '0'; t[1] = 'x';
  for (int i = 0; i < 32; i++) { t[2 + 2 * i] = HX[x[i] >> 4]; t[3 + 2 * i] = HX[x[i] & 15]; }
  jput(b, t, 66);
}
static void jhex(jbuf *b, const hgo *h, int32_t key) { jhexb(b, key_hash(h, key)); }
/* []byte encodes as a base64 (StdEncoding, padded) string */
static void jb64(jbuf *b, const uint8_t *x, int n) {
  static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  char t[4];
  for (int i = 0; i < n; i += 3) {
    const uint32_t v = (uint32_t)x[i] << 16 | (i + 1 < n ? (uint32_t)x[i + 1] << 8 : 0) | (i + 2 < n ? x[i + 2] : 0);
    t[0] = A[v >> 18]; t[1] = A[(v >> 12) & 63];
    t[2] = i + 1 < n ? A[(v >> 6) & 63] : '=';
    t[3] = i + 2 < n ? A[v & 63] : '=';
    jput(b, t, 4);
  }
}
/* RootEvent (root.go:65-71): an event; -1: slot p's Root SelfParent (the
 * base root event "Root<id>" with Index / LamportTimestamp / Round -1, or a
 * Reset root's); OTH(k): Others entry k */
static void jroot_event(jbuf *b, hgo *h, int32_t ev, int32_t p) {
  jstr(b, "{\"Hash\":\"");
  if (ev == -1 && h->r_sp_index[p] >= 0 && h->r_sp_hash) jhexb(b, h->r_sp_hash + (size_t)p * 32);
  else if (ev == -1) { jstr(b, "Root"); jint(b, h->pids[p]); }
  else if (ev < -1) jhexb(b, h->oth_hash + (size_t)(-2 - ev) * 32);
  else jhex(b, h, ev);
  jstr(b, "\",\"CreatorID\":");
  jint(b, h->pids[ev == -1 ? p : ev < -1 ? h->oth_creator[-2 - ev] : h->creator[ev]]);
  jstr(b, ",\"Index\":");
  jint(b, ev == -1 ? h->r_sp_index[p] : ev < -1 ? h->oth_index[-2 - ev] : h->index[ev]);
  jstr(b, ",\"LamportTimestamp\":");
  jint(b, ev == -1 ? h->r_sp_lt[p] : ev < -1 ? h->oth_lt[-2 - ev] : lamport_of(h, ev));
  jstr(b, ",\"Round\":");
  jint(b, ev == -1 ? h->r_sp_round[p] : ev < -1 ? h->oth_round[-2 - ev] : round_of(h, ev));
  jstr(b, "}");
}

static int frame_has_bytes(const hgo *h, int64_t f, int64_t l) {
  for (int64_t k = 0; k < l; k++)
    if (!h->body[h->frame_ev[f + k]] || !h->sig[h->frame_ev[f + k]]) return 0;
  return 1;
}

/* Frame.Marshal (frame.go:17-26): {"Round":..,"Roots":[..],"Events":[..]}
 * + "\n"; an Event encodes its exported fields Body and Signature
 * (event.go:102-106).  Returns 0, or -1 if unavailable. */
static int frame_json(hgo *h, int32_t rr, jbuf *b) {
  if (rr < 0 || rr >= h->rounds_cap || !h->roots[rr] || !h->frame_done[rr]) return -1;
  const int64_t f = h->frame_first[rr], l = h->frame_len[rr];
  if (!frame_has_bytes(h, f, l)) return -1;
  b->len = 0;
  jstr(b, "{\"Round\":");
  jint(b, rr);
  jstr(b, ",\"Roots\":[");
  for (int32_t p = 0; p < h->n; p++) {
    const root_t *r = &h->roots[rr]->r[p];
    if (p) jstr(b, ",");
    jstr(b, "{\"NextRound\":");
    jint(b, r->next_round);
    jstr(b, ",\"SelfParent\":");
    jroot_event(b, h, r->sp, p);
    jstr(b, ",\"Others\":{");
    for (int32_t k = 0; k < r->n_others; k++) {
      if (k) jstr(b, ",");
      jstr(b, "\"");
      jhex(b, h, r->oth_key[k]);
      jstr(b, "\":");
      jroot_event(b, h, r->oth_val[k], p);
    }
    jstr(b, "}}");
  }
  jstr(b, "],\"Events\":[");
  for (int64_t k = 0; k < l; k++) {
    const int32_t ev = h->frame_ev[f + k];
    if (k) jstr(b, ",");
    jstr(b, "{\"Body\":");
    jput(b, h->body[ev], h->body_len[ev]);
    jstr(b, ",\"Signature\":\"");
    jput(b, h->sig[ev], h->sig_len[ev]);
    jstr(b, "\"}");
  }
  jstr(b, "]}\n");
  return 0;
}

/* the base64 transaction strings of an event body's JSON: the text between
 * the brackets of its leading "Transactions" array (EventBody field order,
 * event.go:16-21; null when nil); *len 0 when there are none */
static const uint8_t *body_txs(const hgo *h, int32_t ev, int32_t *len) {
  static const char P[] = "{\"Transactions\":[";
  const uint8_t *x = h->body[ev];
  *len = 0;
  if (h->body_len[ev] < (int32_t)sizeof P || memcmp(x, P, sizeof P - 1)) return NULL;
  int32_t k = sizeof P - 1;
  while (k < h->body_len[ev] && x[k] != ']') k++;
  *len = k - (int32_t)(sizeof P - 1);
  return x + sizeof P - 1;
}

/* Block.Marshal with no signatures yet (block.go:92-97, 178-185):
 * {"Body":{"Index":..,"RoundReceived":..,"StateHash":null,"FrameHash":"b64",
 * "Transactions":[..]},"Signatures":{}} + "\n"; the Body alone (with its own
 * newline) when body_only */
static void block_json(hgo *h, int64_t blk, int body_only, jbuf *b) {
  const int32_t rr = h->blk_rr[blk];
  b->len = 0;
  if (!body_only) jstr(b, "{\"Body\":");
  jstr(b, "{\"Index\":");
  jint(b, h->blk_index0 + blk); /* LastBlockIndex()+1 (block.go:100-110): after a Reset, block.Index()+1 on */
  jstr(b, ",\"RoundReceived\":");
  jint(b, rr);
  jstr(b, ",\"StateHash\":null,\"FrameHash\":\"");
  jb64(b, h->blk_fhash + (size_t)blk * 32, 32);
  jstr(b, "\",\"Transactions\":[");
  int first = 1;
  for (int64_t k = 0; k < h->blk_count[blk]; k++) {
    int32_t tl;
    const uint8_t *t = body_txs(h, h->cons[h->blk_first[blk] + k], &tl);
    if (!tl) continue;
    if (!first) jstr(b, ",");
    jput(b, t, tl);
    first = 0;
  }
  jstr(b, body_only ? "]}\n" : "]},\"Signatures\":{}}\n");
}

int hgo_set_event_bytes(hgo *h, int32_t e, const uint8_t *body, int32_t body_len, const uint8_t *sig,
                        int32_t sig_len) {
  if (e < 0 || e >= h->N || body_len < 0 || sig_len < 0) return HGO_ERR_STATE;
  if (body_len > 0 && body[body_len - 1] == '\n') body_len--; /* the Encoder's newline is not part of the Event's JSON */
  free(h->body[e]);
  free(h->sig[e]);
  h->body[e] = (uint8_t *)xcalloc((size_t)body_len + 1, 1);
  memcpy(h->body[e], body, (size_t)body_len);
  h->body_len[e] = body_len;
  h->sig[e] = (uint8_t *)xcalloc((size_t)sig_len + 1, 1);
  memcpy(h->sig[e], sig, (size_t)sig_len);
  h->sig_len[e] = sig_len;
  return HGO_OK;
}

int hgo_process_decided_rounds(hgo *h) {
  int32_t processed = 0;
  for (int32_t p = 0; p < h->pend_len; p++) {
    pending_round *pr = &h->pend[p];
    if (!pr->decided) break;
    if (h->has_lcr && pr->index == h->lcr) continue;
    int64_t f, l;
    if (get_frame(h, pr->index, &f, &l) != HGO_OK) return HGO_ERR_STATE;
    /* roots before the frame's events become consensus events (not restated
     * for a Reset hashgraph, whose roots would start from the Reset roots) */
    frame_roots(h, pr->index, f, l);
    if (l > 0) {
      int64_t first = h->ncons, txs = 0;
      for (int64_t k = 0; k < l; k++) {
        int32_t e = h->frame_ev[f + k];
        h->cons_pos[e] = h->ncons;
        h->cons[h->ncons++] = e; /* Store.AddConsensusEvent */
        h->consensus_txs += h->ntx[e];
        txs += h->ntx[e];
        if (h->index[e] == 0 || h->ntx[e] > 0) h->pending_loaded--;
        h->last_cons[h->creator[e]] = e; /* InmemStore.AddConsensusEvent (inmem_store.go:178-183) */
      }
      /* NewBlockFromFrame(LastBlockIndex()+1, frame) (block.go:100-110) */
      if (h->nblocks == h->blk_cap) {
        h->blk_cap = h->blk_cap ? 2 * h->blk_cap : 64;
        h->blk_rr = (int32_t *)xrealloc(h->blk_rr, (size_t)h->blk_cap * 4);
        h->blk_first = (int64_t *)xrealloc(h->blk_first, (size_t)h->blk_cap * 8);
        h->blk_count = (int64_t *)xrealloc(h->blk_count, (size_t)h->blk_cap * 8);
        h->blk_ntx = (int64_t *)xrealloc(h->blk_ntx, (size_t)h->blk_cap * 8);
        h->blk_fhash = (uint8_t *)xrealloc(h->blk_fhash, (size_t)h->blk_cap * 32);
        h->blk_has_fhash = (int8_t *)xrealloc(h->blk_has_fhash, (size_t)h->blk_cap);
      }
      { /* FrameHash = SHA-256 of the frame's JSON (frame.go:35-41), when the event bytes are known */
        jbuf b = {0};
        h->blk_has_fhash[h->nblocks] = frame_json(h, pr->index, &b) == 0;
        if (h->blk_has_fhash[h->nblocks]) SHA256(b.p, (size_t)b.len, h->blk_fhash + (size_t)h->nblocks * 32);
        free(b.p);
      }
      h->blk_rr[h->nblocks] = pr->index;
      h->blk_first[h->nblocks] = first;
      h->blk_count[h->nblocks] = l;
      h->blk_ntx[h->nblocks] = txs;
      h->nblocks++;
    }
    processed++;
    if (!h->has_lcr || pr->index > h->lcr) { h->has_lcr = 1; h->lcr = pr->index; }
  }
  /* defer: h.PendingRounds = h.PendingRounds[processedIndex:] */
  if (h->pend_len > processed) /* (an empty queue may have no buffer: memmove(NULL, ...) is UB) */
    memmove(h->pend, h->pend + processed, (size_t)(h->pend_len - processed) * sizeof(pending_round));
  h->pend_len -= processed;
  return HGO_OK;
}

int hgo_run_consensus(hgo *h) {
  int rc;
  if ((rc = hgo_divide_rounds(h))) return rc;
  if ((rc = hgo_decide_fame(h))) return rc;
  if ((rc = hgo_decide_round_received(h))) return rc;
  return hgo_process_decided_rounds(h);
}

/* ------------------------------------------------------------------------ */
/* queries                                                                   */

int64_t hgo_num_events(const hgo *h) { return h->N; }
int32_t hgo_last_round(const hgo *h) { return h->last_round; }
int32_t hgo_last_consensus_round(const hgo *h) { return h->has_lcr ? h->lcr : -1; }
int64_t hgo_consensus_transactions(const hgo *h) { return h->consensus_txs; }
int64_t hgo_pending_loaded_events(const hgo *h) { return h->pending_loaded; }
int64_t hgo_num_consensus_events(const hgo *h) { return h->ncons; }
int64_t hgo_num_undetermined(const hgo *h) { return h->und_len; }
int64_t hgo_num_blocks(const hgo *h) { return h->nblocks; }

void hgo_event_results(const hgo *h, int32_t *round, int8_t *witness, int32_t *lt,
                       int32_t *rr, int8_t *fame, int64_t *cons_pos) {
  for (int64_t x = 0; x < h->N; x++) {
    int32_t r = h->ev_round[x];
    if (round) round[x] = r;
    if (lt) lt[x] = h->ev_lt[x];
    if (rr) rr[x] = h->ev_rr[x];
    if (cons_pos) cons_pos[x] = h->cons_pos[x];
    int8_t w = 0, f = -1;
    if (r != UNSET && r >= 0 && r < h->rounds_cap && h->rounds[r].exists) {
      const round_event *e = ri_find((hgo *)h, r, (int32_t)x);
      if (e) {
        w = (int8_t)e->witness;
        if (w) f = (int8_t)e->famous;
      }
    }
    if (witness) witness[x] = w;
    if (fame) fame[x] = f;
  }
}

void hgo_consensus_order(const hgo *h, int32_t *ids) {
  memcpy(ids, h->cons, (size_t)h->ncons * 4);
}

void hgo_blocks(const hgo *h, int32_t *round_received, int64_t *first, int64_t *count,
                int64_t *ntx) {
  for (int64_t b = 0; b < h->nblocks; b++) {
    if (round_received) round_received[b] = h->blk_rr[b];
    if (first) first[b] = h->blk_first[b];
    if (count) count[b] = h->blk_count[b];
    if (ntx) ntx[b] = h->blk_ntx[b];
  }
}

int32_t hgo_pending_rounds(const hgo *h, int32_t *index, int8_t *decided, int32_t cap) {
  for (int32_t p = 0; p < h->pend_len && p < cap; p++) {
    if (index) index[p] = h->pend[p].index;
    if (decided) decided[p] = h->pend[p].decided;
  }
  return h->pend_len;
}

void hgo_coordinates(const hgo *h, int32_t id, int32_t *la, int32_t *fd) {
  for (int32_t i = 0; i < h->n; i++) {
    if (la) la[i] = la_get(LA(h, id), i);
    if (fd) fd[i] = fd_get(FD(h, id), i);
  }
}

int64_t hgo_undetermined(const hgo *h, int32_t *ids, int64_t cap) {
  int64_t k = h->und_len < cap ? h->und_len : cap;
  if (ids) memcpy(ids, h->und, (size_t)k * 4);
  return h->und_len;
}

int32_t hgo_frame_roots(const hgo *h, int32_t rr, int32_t *next_round, int32_t *sp, int32_t *n_others,
                        int32_t *oth_key, int32_t *oth_val, int32_t cap) {
  if (rr < 0 || rr >= h->rounds_cap || !h->roots[rr]) return -1;
  int32_t k = 0;
  for (int32_t p = 0; p < h->n; p++) {
    const root_t *r = &h->roots[rr]->r[p];
    if (next_round) next_round[p] = r->next_round;
    if (sp) sp[p] = r->sp;
    if (n_others) n_others[p] = r->n_others;
    for (int32_t q = 0; q < r->n_others; q++, k++)
      if (k < cap) {
        if (oth_key) oth_key[k] = r->oth_key[q];
        if (oth_val) oth_val[k] = r->oth_val[q];
      }
  }
  return k;
}

static int64_t jbuf_out(jbuf *b, uint8_t *buf, int64_t cap) {
  if (buf) memcpy(buf, b->p, (size_t)(b->len < cap ? b->len : cap));
  const int64_t len = b->len;
  free(b->p);
  return len;
}

int64_t hgo_frame_json(hgo *h, int32_t rr, uint8_t *buf, int64_t cap) {
  jbuf b = {0};
  if (frame_json(h, rr, &b) != 0) { free(b.p); return -1; }
  return jbuf_out(&b, buf, cap);
}

int hgo_block_frame_hash(const hgo *h, int64_t blk, uint8_t *out32) {
  if (blk < 0 || blk >= h->nblocks || !h->blk_has_fhash[blk]) return -1;
  memcpy(out32, h->blk_fhash + (size_t)blk * 32, 32);
  return 0;
}

int64_t hgo_block_json(hgo *h, int64_t blk, int body_only, uint8_t *buf, int64_t cap) {
  if (blk < 0 || blk >= h->nblocks || !h->blk_has_fhash[blk]) return -1;
  jbuf b = {0};
  block_json(h, blk, body_only, &b);
  return jbuf_out(&b, buf, cap);
}

int hgo_see(hgo *h, int32_t x, int32_t y) { return see(h, x, y); }
int hgo_strongly_see(hgo *h, int32_t x, int32_t y) { return strongly_see(h, x, y); }
int32_t hgo_round_of(hgo *h, int32_t x) { return round_of(h, x); }
int32_t hgo_lamport_of(hgo *h, int32_t x) { return lamport_of(h, x); }
int hgo_witness_of(hgo *h, int32_t x) { return witness_of(h, x); }
