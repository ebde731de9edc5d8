// handle.h -- host state of a libbabble_hip handle (internal; shared by
// api.cpp, the passes and queries, and frames.cpp, the block projection).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <unordered_map>
#include <vector>

#include "babble_hip.h"
#include "engine.h"

using bh::Dev;

namespace bh {

constexpr int ITER_BATCH = 32;  // round-loop iterations per graph replay
constexpr int ITER_FIRST = 4;   // ... for the first two replays of a loop (an incremental call needs a few rounds)
constexpr int NSTAGE = 5;

struct Block {
  int32_t rr;
  int64_t first, count, ntx;
};

// a multi-process group's exchange (comm.cpp): RCCL or the caller's host
// transport; device buffers, ordered on stream s
struct Comm {
  virtual ~Comm() = default;
  virtual int bcast(bh_handle *h, void *buf, size_t bytes, int32_t root, hipStream_t s) = 0;
  virtual int send(bh_handle *h, const void *buf, size_t bytes, int32_t peer, hipStream_t s) = 0;
  virtual int recv(bh_handle *h, void *buf, size_t bytes, int32_t peer, hipStream_t s) = 0;
  virtual int group_start(bh_handle *) { return 0; }  // (RCCL: receives from several peers at once)
  virtual int group_end(bh_handle *) { return 0; }
  // true: the calls wait on the host (the host transport); false: they are
  // enqueued on s and return (RCCL)
  virtual bool blocking() const { return false; }
};
Comm *make_rccl_comm(bh_handle *h, int32_t rank, int32_t world, const uint8_t *id);  // nullptr on failure (h->err)
Comm *make_host_comm(const bh_transport &t, int32_t rank);

}  // namespace bh

using bh::Block;
using bh::ITER_BATCH;
using bh::ITER_FIRST;
using bh::NSTAGE;

struct bh_handle {
  Dev d{};
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  int64_t cap = 0;
  // host mirrors (insert bookkeeping: ParticipantEventsCache + checks)
  std::vector<int64_t> pids;
  // participant ID -> slot: open addressing, power-of-two table >= 4n,
  // linear probing (one or two probes per lookup on the insert loop)
  std::vector<int64_t> slot_key;
  std::vector<int32_t> slot_val;
  uint64_t slot_mask = 0;
  int32_t slot_find(int64_t id) const {
    for (uint64_t i = ((uint64_t)id * 0x9E3779B97F4A7C15ull) >> 32 & slot_mask;; i = (i + 1) & slot_mask) {
      if (slot_val[i] < 0) return -1;
      if (slot_key[i] == id) return slot_val[i];
    }
  }
  std::vector<std::vector<int32_t>> chain;  // ids by creator, by index
  // per-chain prefix lengths at an insertion-order bound (chain_lens_at):
  // chains only grow by appends, so a bound's lengths never change once
  // every event below it is inserted -- kept, since each is n binary searches
  // over cold multi-MB id vectors (~250 us at C3 before the first loop)
  mutable std::unordered_map<int64_t, std::vector<int32_t>> lens_memo;
  std::vector<int32_t> h_creator, h_index, h_sp, h_op, h_ntx;
  std::vector<uint8_t> h_coin;
  std::vector<uint32_t> h_sigw;
  int64_t uploaded = 0;  // events already on the device
  int64_t loaded_total = 0;
  // The Go Hashgraph's state persists across calls: InsertEvent appends to
  // UndeterminedEvents and changes nothing else; each pass updates its own
  // part (hashgraph.go:714-1122).  The engine keeps the same split.
  //   n_div   events covered by the last DivideRounds (round / witness / LT)
  //   n_rr    events covered by the last DecideRoundReceived
  //   R       rounds (Store.LastRound() + 1)
  //   P       processed prefix: LastConsensusRound + 1
  //   pend_dec  PendingRounds' decided flags for rounds [P, R): sticky, as
  //             updatePendingRounds only ever sets them (hashgraph.go:689-695)
  int stage = 0;  // last pass run: 0 none, 1 rounds, 2 fame, 3 rr, 4 processed
  int coords_for = -1;  // N the device coordinates were computed for
  int64_t n_div = 0, n_rr = 0;
  int32_t R = 0, P = 0;
  std::vector<int8_t> pend_dec;     // indexed by round, meaningful for [P, R)
  std::vector<int8_t> decided_h;    // last fame pass: round r's witnesses all decided
  int64_t nundet = 0;               // undetermined among [0, n_rr) after the last rr pass
  int32_t R_rr = 0;                 // R at the last rr pass (frame_cnt covers [0, R_rr))
  int64_t ncons = 0, cons_txs = 0, cons_loaded = 0;
  std::vector<Block> blocks;
  // round-loop graph
  hipGraphExec_t graph = nullptr, graph_s = nullptr;  // ITER_BATCH / ITER_FIRST iterations
  Dev graph_dev{}, graph_dev_s{};
  int32_t *pinned_state = nullptr;
  // pinned staging for a pass's device-to-host reads (rd_async / rd_wait):
  // a pageable destination makes every hipMemcpyAsync a blocking staged copy
  uint8_t *pin_rd = nullptr;
  size_t pin_rd_cap = 0, pin_rd_used = 0;
  struct PinRead {
    void *dst;
    size_t off, bytes;
  };
  std::vector<PinRead> pin_rd_list;
  uint8_t *sha_buf = nullptr;  // bh_hash_bodies scratch
  uint8_t *q_buf = nullptr;    // bh_query_events scratch
  int32_t *pack_buf = nullptr;  // order_finish's read-back (k_pack_frames)
  size_t pack_cap = 0;          // (int32 words)
  size_t q_cap = 0;
  size_t sha_cap = 0;
  hipEvent_t ev[NSTAGE + 1]{};
  hipEvent_t ev_sweep[2]{};  // around k_la_sweep alone (roofline timing)
  hipEvent_t ev_loop[2]{};
  hipEvent_t ev_st = nullptr;  // behind the loop state's read-back (rounds_pipelined: the witness tables run after it)
  bool fuse_fame = false;      // bh_run_consensus: DecideFame follows DivideRounds at once (rounds_tail)   // around each round loop (run_round_loop): its device time, summed per run
  float loop_ms = 0, loop_ms_acc = 0;
  float sweep_ms = 0;
  const char *sweep_kernel = "";
  float stage_ms[NSTAGE]{};
  // timings of the last run not yet read from its events (settle_timings)
  bool tm_seg = false, tm_stages = false, tm_seg_loops = false, tm_seg_sp = false;
  int tm_seg_K = 0;
  int64_t iters = 0;
  int64_t *d_counters_host = nullptr;
  // segment pipeline: coordinates of prefix s + 1 on
  // stream2 while the round loop runs prefix s on `stream`
  hipStream_t stream2 = nullptr;
  std::vector<hipEvent_t> loop_evs;            // around each segment's loop launch (rounds_pipelined, async)
  int ncu = 256;                               // compute units of the device
  int32_t *seg_zero = nullptr;   // [n] zeros: seg_lo of a one-segment view
  int32_t *segbuf = nullptr;     // [2 parities][lo, len][n]
  int32_t *seg_stage = nullptr;  // pinned staging of the segments' [lo, len] rows, one per segment (<= 64)
  hipGraphExec_t seg_graph[2] = {nullptr, nullptr}, seg_graph_s[2] = {nullptr, nullptr};
  Dev seg_graph_dev[2]{}, seg_graph_dev_s[2]{};
  std::vector<hipEvent_t> seg_ev;  // per segment: coordinates done, k_flow32 start / end
  int32_t segments_used = 1;
  int32_t *tlist = nullptr, *tlist_stage = nullptr;  // [2 parities][tlist_cap] segment tile lists
  int64_t tlist_cap = 0;
  std::vector<int32_t> cstart_h;  // chain_start as uploaded
  std::vector<int32_t> cap_h;     // rows of each chain's region
  std::vector<int32_t> lens_h;    // chain lengths as uploaded
  int64_t layout_rows = 0;        // rows of the layout (regions included)
  bool layout_changed = true;
  // incremental calls (a call that only appended events runs them as one
  // more segment): coordinates and round loop hold the first n_coord events
  // of the current layout; lens_coord their chain lengths
  bool inc_valid = false;
  bool fdt_lost = false;  // the wide LT fallback's sweep overwrote FDT (no resume from it)
  bool rows_stale = false;  // n <= 128 segments built la_col only: row-major LA / FDT wait for a query
  // the row-major LA / FDT built (build_rows) for these chain lengths of the
  // current layout: a later build transposes only the rows past them
  bool rows_built = false;
  std::vector<int32_t> rows_lens;
  int64_t n_coord = 0;
  int64_t inc_calls = 0;  // DivideRounds calls that resumed (statistics)
  int64_t persist_loops = 0, persist_fallbacks = 0;  // k_round2p loops run / given up (bh_get_loop_stats)
  std::vector<int32_t> lens_coord;
  // sharding
  int32_t rank = 0, world = 1;
  std::vector<bh_handle *> group;  // in-process group: every shard (group[rank] == this); empty otherwise
  bh::Comm *xport = nullptr;       // multi-process group (bh_comm_init / bh_comm_init_transport)
  bool shard_cols = false;         // split the coordinate dataflow's LA columns (else every shard computes all)
  // the coordinate split (kernels_split.hip): shards
  // 1 .. G-1 run the dataflow for a range of LA columns each and ship every
  // segment's rows of them.  n <= 128 (split_all): the blocks are
  // all-gathered and EVERY shard runs the round loop on the full columns, so
  // fame rounds and frame sorts split between all shards as in the
  // replicated mode; 128 < n <= 512 (the wide split): shard 0 alone receives
  // them and runs the loop, fame and order
  bool split = false;
  bool split_all() const { return split && d.fd_cols; }
  uint8_t *xbuf = nullptr;        // every segment's blocks of every coordinate shard, at SplitPlan::boff
  size_t xcap = 0;
  int32_t *xseg = nullptr;        // [K][lo, hi][n] segment views, then [K][P, Q][n + 1] packing tables
  int32_t xseg_k = 0;             // segments xseg has room for
  std::vector<hipEvent_t> pack_ev;  // coordinate shard: segment k's own block packed (stream2)
  hipStream_t stream3 = nullptr;    // the split's receives and unpacks, beside the dataflow (stream2)
  hipEvent_t xprep = nullptr;       // the call's chain tables prepared (stream2), before any unpack
  int32_t *xbase = nullptr;       // multi-process: rank 0's base for the call (broadcast)
  float xchg_ms = 0;               // exchange time of the last pass sequence (host wall, incl. waits)
  std::vector<int32_t> wofs_h;     // [R + 1] witness offsets (fame exchange ranges; launch size)
  std::vector<int32_t> fofs_h;     // [P + 1] frame offsets (order exchange ranges)
  // block projection (bh_config.frames; frames.cpp)
  bool frames_on = false;
  bh::Frames fr{};
  std::vector<uint8_t> h_hash;     // hashes of events inserted but not yet uploaded
  int64_t arena_cap = 0, arena_len = 0;
  int64_t others_total = 0;        // Others of the processed frames (oofs[P * n])
  size_t json_cap = 0, bjson_cap = 0;
  uint8_t *host_json = nullptr;  // pinned host copy of the JSON a call hashes on the host (frames.cpp)
  size_t host_json_cap = 0;
  int64_t hash_host_frames = 0;  // frames whose FrameHash the host computed (statistics)
  hipEvent_t ev_fr[2]{};           // around the last projection
  float frames_ms = 0;

  // Reset / FastSync roots (bh_reset; hashgraph.go:1324-1369).  Chains
  // start at base_h[c] = Root.SelfParent.Index + 1; Root.Others entries are
  // found by (root slot, key hash) and by (root slot, creator slot, Index)
  bool reset_on = false;
  int32_t reset_lcr = -1;      // block.RoundReceived(): LastConsensusRound after Reset
  int64_t reset_block = -1;    // block.Index(): LastBlockIndex after Reset
  int32_t reset_F = -1;        // highest NextRound / SelfParent.Round of a root
  std::vector<int32_t> base_h, next_h, sp_round_h, sp_lt_h;
  struct Other {
    int32_t root, creator, index, lt, round;
    uint8_t key[32], hash[32];
  };
  std::vector<Other> others;
  std::unordered_map<std::string, int32_t> oth_by_key;  // root slot bytes + key hash -> entry
  std::unordered_map<uint64_t, int32_t> oth_by_index;   // (root slot, creator slot, Index) -> entry
  std::vector<uint8_t> h_hashes;                        // every event's hash (Others matching)
  std::vector<int8_t> h_rflag;                          // Dev::rflag
  std::vector<int32_t> h_ext_lt;                        // Dev::ext_lt
  std::vector<int32_t> h_oth;                           // Frames::oth_of (frames on)
  int64_t E0 = 0;  // events [0, E0) hold every other-parent only Root.Others knows
  int32_t fiat_max = -1;

  // test hook: BH_TEST_FAIL_ALLOC=k makes the k-th device allocation of a
  // bh_reset call fail (tests check that a failed call leaves the handle as
  // it was); -1 otherwise
  int fail_alloc_in = -1;

  // a coordinate rank of a multi-process WIDE split group: it ran no
  // consensus pass, so it holds no results (rank 0 does)
  bool no_results() const { return split && !split_all() && rank > 0 && xport != nullptr; }
  int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
};

#define HIPCHK(h, call)                                                              \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess)                                                            \
      return (h)->fail(BH_ERR_DEVICE, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), \
                       __FILE__, __LINE__);                                          \
  } while (0)

template <class T>
inline int dalloc(bh_handle *h, T **p, size_t count) {
  if (h->fail_alloc_in >= 0 && h->fail_alloc_in-- == 0) {  // test hook (bh_reset, BH_TEST_FAIL_ALLOC)
    *p = nullptr;
    return h->fail(BH_ERR_DEVICE, "injected allocation failure");
  }
  HIPCHK(h, hipMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T)));
  return BH_OK;
}

// frames.cpp
int frames_alloc(bh_handle *h);
void frames_free(bh_handle *h);
// the projection's device tables for R1 rounds into fr (with a Reset's K
// installed Others entries: reset); frames_init gives them their initial
// contents once they are the handle's
int frames_alloc_tables(bh_handle *h, bh::Frames &fr, int64_t R1, int64_t K, bool reset);
void frames_free_tables(bh::Frames &fr);
int frames_init(bh_handle *h);
int frames_prepare(bh_handle *h, bh::Frames &fr, int64_t R1, size_t *json_cap, size_t *bjson_cap);
void frames_reset(bh_handle *h);
// roots, FrameHash and block hashes of the frames [P0, P1) just processed
// (consensus positions [i0, i1))
int frames_project(bh_handle *h, int32_t P0, int32_t P1, int64_t i0, int64_t i1);
