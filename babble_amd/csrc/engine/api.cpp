// api.cpp -- C ABI of libbabble_hip (include/babble_hip.h): host state of the
// drop-in Hashgraph, insert validation, stage orchestration on one HIP
// stream per shard, result queries.  No CPU fallback: every consensus stage
// runs as HIP kernels on the device; without a device bh_create fails.
//
// Sharding.  A handle may be one shard of a group of
// `world` shards, each holding the whole DAG on its own device (or sharing
// one): an in-process group (bh_config.device_ids, shard 0 is the handle the
// caller holds and owns the others) or one shard per process joined by an
// RCCL communicator (bh_comm_init).  Each pass runs the same kernels on
// every shard; the split parts -- LA columns of the coordinate dataflow,
// DecideFame rounds, frame sorts -- cover the shard's range only and are
// then exchanged (peer copies over xGMI in-process, ncclBroadcast per range
// across processes), so every shard ends each pass with identical arrays.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "babble_hip.h"
#include "engine.h"
#include "handle.h"

namespace {

void free_all(bh_handle *h) {
  frames_free(h);
  Dev &d = h->d;
  void *ptrs[] = {d.creator, d.index, d.sp, d.op, d.ntx, d.coin, d.sigw, d.chain_start,
                  d.chain_len, d.chain_ids, d.epos, d.la, d.lt, d.depth, d.chunk_maxd, d.desc, d.B,
                  d.wofs, d.wcnt, d.wids, d.wrow, d.state, d.round, d.witness, d.fame,
                  d.decided, d.nfam, d.minla, d.rr, d.frame_cnt, d.frame_ofs, d.frame_cur,
                  d.blk_of_frame, d.order, d.cons_pos, d.frame_ntx, d.counters, d.diag, d.trapped, d.blocked,
                  d.wfame, d.frame_loaded, d.Bp, d.fd, d.fdt, d.cla, d.last_la, d.rq, d.candfd, d.cand8, d.c8tag, d.Bq, d.opdesc, d.lt_row, d.ssm, d.ssw, d.pbar, d.psnap,
                  d.la_col != d.fdt ? d.la_col : nullptr,  // la_ev aliases fdt
                  d.chain_base, d.lt_seed, d.root_next, d.root_sp_round, d.rflag, d.ext_lt, d.fw, d.rexists};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  if (h->pinned_state) (void)hipHostFree(h->pinned_state);
  if (h->pin_rd) (void)hipHostFree(h->pin_rd);
  if (h->sha_buf) (void)hipFree(h->sha_buf);
  if (h->q_buf) (void)hipFree(h->q_buf);
  if (h->pack_buf) (void)hipFree(h->pack_buf);
  if (h->graph) (void)hipGraphExecDestroy(h->graph);
  if (h->graph_s) (void)hipGraphExecDestroy(h->graph_s);
  for (auto &e : h->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto &e : h->ev_sweep)
    if (e) (void)hipEventDestroy(e);
  for (auto &e : h->ev_loop)
    if (e) (void)hipEventDestroy(e);
  if (h->ev_st) (void)hipEventDestroy(h->ev_st);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  if (h->stream2) (void)hipStreamDestroy(h->stream2);
  for (auto &e : h->loop_evs)
    if (e) (void)hipEventDestroy(e);
  for (auto &g : h->seg_graph)
    if (g) (void)hipGraphExecDestroy(g);
  for (auto &g : h->seg_graph_s)
    if (g) (void)hipGraphExecDestroy(g);
  for (auto &e : h->seg_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->seg_zero) (void)hipFree(h->seg_zero);
  if (h->segbuf) (void)hipFree(h->segbuf);
  if (h->seg_stage) (void)hipHostFree(h->seg_stage);
  if (h->tlist) (void)hipFree(h->tlist);
  if (h->tlist_stage) (void)hipHostFree(h->tlist_stage);
  delete h->xport;
  h->xport = nullptr;
  if (h->xbuf) (void)hipFree(h->xbuf);
  if (h->xseg) (void)hipFree(h->xseg);
  for (auto &e : h->pack_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->xprep) (void)hipEventDestroy(h->xprep);
  if (h->stream3) (void)hipStreamDestroy(h->stream3);
  if (h->xbase) (void)hipFree(h->xbase);
}

// upload events inserted since the last upload
hipError_t wait_stream(hipStream_t s);

int upload(bh_handle *h) {
  const int64_t a = h->uploaded, b = (int64_t)h->h_creator.size();
  if (b == a) return BH_OK;
  const size_t k = (size_t)(b - a);
  Dev &d = h->d;
  hipStream_t s = h->stream;
  HIPCHK(h, hipMemcpyAsync(d.creator + a, h->h_creator.data() + a, k * 4, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(d.index + a, h->h_index.data() + a, k * 4, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(d.sp + a, h->h_sp.data() + a, k * 4, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(d.op + a, h->h_op.data() + a, k * 4, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(d.ntx + a, h->h_ntx.data() + a, k * 4, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(d.coin + a, h->h_coin.data() + a, k, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(d.sigw + a * 8, h->h_sigw.data() + a * 8, k * 32, hipMemcpyHostToDevice, s));
  if (h->frames_on)  // h_hash holds the events [a, b)
    HIPCHK(h, hipMemcpyAsync(h->fr.hash + a * 32, h->h_hash.data(), k * 32, hipMemcpyHostToDevice, s));
  if (h->reset_on) {
    HIPCHK(h, hipMemcpyAsync(d.rflag + a, h->h_rflag.data() + a, k, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipMemcpyAsync(d.ext_lt + a, h->h_ext_lt.data() + a, k * 4, hipMemcpyHostToDevice, s));
    if (h->fr.oth_of)
      HIPCHK(h, hipMemcpyAsync(h->fr.oth_of + a, h->h_oth.data() + a, k * 4, hipMemcpyHostToDevice, s));
  }
  HIPCHK(h, wait_stream(s));
  h->h_hash.clear();
  h->uploaded = b;
  return BH_OK;
}

// A host wait for stream s.  (Spinning on hipStreamQuery instead woke the
// host ~50 us sooner after the round loop, but measured no faster per C3
// step on one box, same-box A/B: profiles/r5_ab_spin.txt -- so the host
// sleeps in hipStreamSynchronize)
hipError_t wait_stream(hipStream_t s) { return hipStreamSynchronize(s); }

// A blocking copy ordered on stream s.  The passes never touch the legacy
// stream: the shards of an in-process group run on threads of their own, and
// a legacy-stream operation while another shard captures a graph on the same
// device fails ("would make the legacy stream depend on a capturing stream")
hipError_t copy_sync(hipStream_t s, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
  hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, s);
  return e == hipSuccess ? wait_stream(s) : e;
}

// A pass's device-to-host reads behind one synchronisation: rd_async
// enqueues each into pinned staging on s, rd_wait synchronises s once and
// copies them out (~20 us per pageable read otherwise: each is a blocking
// staged copy of its own)
int rd_wait(bh_handle *h, hipStream_t s) {
  HIPCHK(h, wait_stream(s));
  for (const auto &r : h->pin_rd_list) memcpy(r.dst, h->pin_rd + r.off, r.bytes);
  h->pin_rd_list.clear();
  h->pin_rd_used = 0;
  return BH_OK;
}

// rd_wait up to an event recorded after the reads (work queued behind it
// keeps running)
int rd_wait_event(bh_handle *h, hipEvent_t e) {
  HIPCHK(h, hipEventSynchronize(e));
  for (const auto &r : h->pin_rd_list) memcpy(r.dst, h->pin_rd + r.off, r.bytes);
  h->pin_rd_list.clear();
  h->pin_rd_used = 0;
  return BH_OK;
}

int rd_async(bh_handle *h, hipStream_t s, void *dst, const void *src, size_t bytes) {
  if (!bytes) return BH_OK;
  const size_t need = ((h->pin_rd_used + 63) & ~(size_t)63) + bytes;
  if (need > h->pin_rd_cap) {
    int rc;
    if (!h->pin_rd_list.empty() && (rc = rd_wait(h, s))) return rc;  // (drain before the buffer moves)
    const size_t cap = std::max<size_t>(need + need / 2, 1 << 16);
    if (h->pin_rd) (void)hipHostFree(h->pin_rd);
    h->pin_rd = nullptr;
    h->pin_rd_cap = 0;
    HIPCHK(h, hipHostMalloc((void **)&h->pin_rd, cap, hipHostMallocDefault));
    h->pin_rd_cap = cap;
  }
  const size_t off = (h->pin_rd_used + 63) & ~(size_t)63;
  HIPCHK(h, hipMemcpyAsync(h->pin_rd + off, src, bytes, hipMemcpyDeviceToHost, s));
  h->pin_rd_list.push_back({dst, off, bytes});
  h->pin_rd_used = off + bytes;
  return BH_OK;
}

// The last run's device timings, read from its events when asked (stage
// table, profile) rather than where the device would wait for the host's
// queries: the segment pipeline's coordinate windows and loop launches
// (rounds_pipelined), then the stage events (order_finish)
void settle_timings(bh_handle *h) {
  if (h->tm_seg) {
    h->tm_seg = false;
    const int K = h->tm_seg_K;
    float ms = 0;
    if (h->tm_seg_loops)
      for (int k = 0; k < K; ++k)
        if (hipEventElapsedTime(&ms, h->loop_evs[(size_t)2 * k], h->loop_evs[(size_t)2 * k + 1]) == hipSuccess)
          h->loop_ms_acc += ms;
    h->sweep_ms = 0;
    for (int k = 0; k < K; ++k)
      if (hipEventElapsedTime(&ms, h->seg_ev[(size_t)3 * k + 1], h->seg_ev[(size_t)3 * k + 2]) == hipSuccess)
        h->sweep_ms += ms;
    if (h->tm_seg_sp) {  // the coordinate time is the coordinate shards'; the receive windows are the exchange
      h->xchg_ms = h->sweep_ms;
      h->sweep_ms = 0;
    }
  }
  if (h->tm_stages) {
    h->tm_stages = false;
    for (int i = 0; i < NSTAGE; ++i) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, h->ev[i], h->ev[i + 1]) == hipSuccess) h->stage_ms[i] = ms;
    }
    float sms = 0;
    if (hipEventElapsedTime(&sms, h->ev_sweep[0], h->ev_sweep[1]) == hipSuccess) h->sweep_ms = sms;
  }
  (void)hipGetLastError();  // (an unrecorded event must not stay sticky)
}

// Chain-major layout: chain c's events occupy rows [chain_start[c],
// chain_start[c] + len_c) of a region of cap_c rows.  The regions are kept
// while every chain fits (appended events extend a region in place, so the
// rows already computed stay valid); when one outgrows its region they are
// laid out again with fresh slack (max(BH_LAYOUT_SLACK or 1024, len / 8)
// rows each, if the allocation has room; none otherwise) and layout_changed
// is set.  Rows past a chain's events are gaps (chain_ids -1).
int set_chain_tables(bh_handle *h, bool wait = true) {
  const int n = h->d.n;
  std::vector<int32_t> len((size_t)n);
  int32_t mx = 0;
  int64_t tot = 0;
  for (int c = 0; c < n; ++c) {
    len[(size_t)c] = (int32_t)h->chain[(size_t)c].size();
    mx = std::max(mx, len[(size_t)c]);
    tot += len[(size_t)c];
  }
  bool fits = (int)h->cap_h.size() == n;
  for (int c = 0; fits && c < n; ++c) fits = len[(size_t)c] <= h->cap_h[(size_t)c];
  h->layout_changed = !fits;
  if (!fits) {
    h->rows_built = false;  // (rows built for the old layout)
    const int64_t min_slack = getenv("BH_LAYOUT_SLACK") ? atoll(getenv("BH_LAYOUT_SLACK")) : 1024;
    const bool slack = h->d.la_rows > h->cap;  // the allocation reserved room for it
    int64_t need = 0;
    for (int c = 0; c < n; ++c) need += len[(size_t)c] + std::max<int64_t>(min_slack, len[(size_t)c] / 8);
    const bool use = slack && need <= h->d.la_rows;
    h->cap_h.resize((size_t)n);
    h->cstart_h.resize((size_t)n);
    int64_t acc = 0;
    for (int c = 0; c < n; ++c) {
      h->cstart_h[(size_t)c] = (int32_t)acc;
      h->cap_h[(size_t)c] = (int32_t)(len[(size_t)c] + (use ? std::max<int64_t>(min_slack, len[(size_t)c] / 8) : 0));
      acc += h->cap_h[(size_t)c];
    }
    h->layout_rows = acc;
    HIPCHK(h, hipMemcpyAsync(h->d.chain_start, h->cstart_h.data(), n * 4, hipMemcpyHostToDevice, h->stream));
  }
  (void)tot;
  h->d.max_chain_len = mx;
  h->lens_h = len;
  HIPCHK(h, hipMemcpyAsync(h->d.chain_len, h->lens_h.data(), n * 4, hipMemcpyHostToDevice, h->stream));
  // (!wait: the caller orders every later reader after h->stream -- the
  // segment pipeline's coordinate stream waits for an event recorded on it
  // -- and lens_h / cstart_h change only in the next call, after its
  // stages' synchronisations)
  if (wait) HIPCHK(h, wait_stream(h->stream));
  return BH_OK;
}

// the round loop's iterations as one graph of `iters` (even) launches for
// the view v, cached per slot (kernel arguments are captured by value)
int build_graph(bh_handle *h, const Dev &v, hipGraphExec_t *graph, Dev *graph_dev, int iters) {
  if (*graph && memcmp(graph_dev, &v, sizeof(Dev)) == 0) return BH_OK;
  if (*graph) {
    (void)hipGraphExecDestroy(*graph);
    *graph = nullptr;
  }
  hipGraph_t g;
  HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < iters; ++i) bh::launch_round_iteration(v, i & 1, h->stream);
  HIPCHK(h, hipStreamEndCapture(h->stream, &g));
  HIPCHK(h, hipGraphInstantiate(graph, g, nullptr, nullptr, 0));
  (void)hipGraphDestroy(g);
  *graph_dev = v;
  return BH_OK;
}

// the round loop on h->stream for view v, its inputs set up already:
// replays batches of iterations, checking completion one batch behind so
// the device never idles on the host round trip.  The first two batches
// are ITER_FIRST iterations (graph_s), the rest ITER_BATCH: a loop that ends
// within a few rounds -- an incremental call's -- runs 8 launches rather
// than 64, most of them no-ops behind the done flag.  Returns the loop state.
int run_round_loop(bh_handle *h, const Dev &v, hipGraphExec_t *graph, Dev *graph_dev, hipGraphExec_t *graph_s,
                   Dev *graph_dev_s, int32_t *st) {
  int rc;
  hipStream_t s = h->stream;
  // BH_NO_GRAPH=1: launch the iterations directly instead of replaying a
  // captured graph (profiling / A-B; results are identical)
  const bool no_graph = getenv("BH_NO_GRAPH") && atoi(getenv("BH_NO_GRAPH"));
  const bool loop_timing = !(getenv("BH_LOOP_TIMING") && !atoi(getenv("BH_LOOP_TIMING")));
  if (bh::round_solo_eligible(v)) {  // one launch runs every round (k_round_solo)
    if (loop_timing) HIPCHK(h, hipEventRecord(h->ev_loop[0], s));
    bh::launch_round_solo(v, s);
    HIPCHK(h, hipGetLastError());
    if (loop_timing) HIPCHK(h, hipEventRecord(h->ev_loop[1], s));
    HIPCHK(h, copy_sync(s, st, v.state, bh::ST_COUNT * 4, hipMemcpyDeviceToHost));
    float lms = 0;
    if (loop_timing && hipEventElapsedTime(&lms, h->ev_loop[0], h->ev_loop[1]) == hipSuccess) h->loop_ms_acc += lms;
    if (!st[bh::ST_DONE]) return h->fail(BH_ERR_STATE, "round loop did not terminate");
    if (st[bh::ST_ERR]) return h->fail(BH_ERR_CAPACITY, "round table capacity exceeded");
    return BH_OK;
  }
  const bool pers = bh::round_persist_eligible(v), wpers = !pers && bh::round_wide_persist_eligible(v);
  if (pers || wpers) {  // one launch, a grid barrier per iteration (k_round2p / k_round_wide<..., true>)
    // the loop's inputs, kept: a barrier that gives up (ST_ERR = 3) leaves
    // them overwritten, and the per-iteration launches below start again
    // from them -- parity 0's boundaries and candidate rows (candfd, which
    // the wide loop's cand16 aliases; cand8 and its tags), the state block
    const int n = v.n;
    const size_t w8 = v.cand8 ? (size_t)n * ((v.npad + 15) / 16 * 16) : 0;
    struct Piece { void *dev; size_t bytes; } pieces[] = {
        {v.Bp, (size_t)n * 4}, {v.candfd, (size_t)n * v.npad * 4}, {v.state, bh::ST_COUNT * 4},
        {v.cand8, wpers ? w8 : 0}, {v.c8tag, wpers && v.c8tag ? (size_t)n * 4 : 0}};
    auto snapshot = [&](bool restore) -> int {
      char *sp = reinterpret_cast<char *>(v.psnap);
      for (const Piece &pc : pieces) {
        if (!pc.bytes) continue;
        HIPCHK(h, hipMemcpyAsync(restore ? pc.dev : sp, restore ? sp : pc.dev, pc.bytes, hipMemcpyDeviceToDevice, s));
        sp += (pc.bytes + 15) & ~(size_t)15;
      }
      return BH_OK;
    };
    if ((rc = snapshot(false))) return rc;
    if (loop_timing) HIPCHK(h, hipEventRecord(h->ev_loop[0], s));
    ++h->persist_loops;
    if (pers) bh::launch_round_persist(v, s);
    else bh::launch_round_wide_persist(v, s);
    HIPCHK(h, hipGetLastError());
    if (loop_timing) HIPCHK(h, hipEventRecord(h->ev_loop[1], s));
    HIPCHK(h, copy_sync(s, st, v.state, bh::ST_COUNT * 4, hipMemcpyDeviceToHost));
    float lms = 0;
    if (loop_timing && hipEventElapsedTime(&lms, h->ev_loop[0], h->ev_loop[1]) == hipSuccess) h->loop_ms_acc += lms;
    if (st[bh::ST_DONE] && st[bh::ST_ERR] != 3) {
      if (st[bh::ST_ERR]) return h->fail(BH_ERR_CAPACITY, "round table capacity exceeded");
      return BH_OK;
    }
    // the grid barrier gave up (some workgroup was never placed): restore and
    // take the per-iteration launches (counted in stats.persist_fallbacks)
    ++h->persist_fallbacks;
    if ((rc = snapshot(true))) return rc;
    if (pers && bh::cand_fe(v)) bh::launch_cand_defe(v, s);  // (k_round2 reads plain entries)
  }
  if (!no_graph && (rc = build_graph(h, v, graph, graph_dev, ITER_BATCH))) return rc;
  if (!no_graph && (rc = build_graph(h, v, graph_s, graph_dev_s, ITER_FIRST))) return rc;
  hipEvent_t done_ev[2];
  HIPCHK(h, hipEventCreateWithFlags(&done_ev[0], hipEventDisableTiming));
  HIPCHK(h, hipEventCreateWithFlags(&done_ev[1], hipEventDisableTiming));
  // the round kernels store 1 into the mapped word pin[0] when the loop ends
  volatile int32_t *pin = h->pinned_state;
  pin[0] = 0;
  bool done = false;
  // the loop's own device time (bh_get_stage_ms entry 7; BH_LOOP_TIMING=0: off, A/B)
  if (loop_timing) HIPCHK(h, hipEventRecord(h->ev_loop[0], s));  // (after any wait queued on s: loop time only)
  const int64_t max_batches = (int64_t)v.R_cap / ITER_BATCH + 4;
  for (int64_t b = 0; b < max_batches && !done; ++b) {
    const bool first = b < 2;
    if (no_graph) {
      for (int i = 0; i < (first ? ITER_FIRST : ITER_BATCH); ++i) bh::launch_round_iteration(v, i & 1, s);
      HIPCHK(h, hipGetLastError());
    } else {
      HIPCHK(h, hipGraphLaunch(first ? *graph_s : *graph, s));
    }
    HIPCHK(h, hipEventRecord(done_ev[b & 1], s));
    if (b > 0) {
      HIPCHK(h, hipEventSynchronize(done_ev[(b - 1) & 1]));
      if (pin[0]) done = true;
    }
  }
  if (loop_timing) HIPCHK(h, hipEventRecord(h->ev_loop[1], s));
  HIPCHK(h, copy_sync(s, st, v.state, bh::ST_COUNT * 4, hipMemcpyDeviceToHost));  // (one synchronisation)
  float lms = 0;
  if (loop_timing && hipEventElapsedTime(&lms, h->ev_loop[0], h->ev_loop[1]) == hipSuccess) h->loop_ms_acc += lms;
  (void)hipEventDestroy(done_ev[0]);
  (void)hipEventDestroy(done_ev[1]);
  if (!st[bh::ST_DONE]) return h->fail(BH_ERR_STATE, "round loop did not terminate");
  if (st[bh::ST_ERR]) return h->fail(BH_ERR_CAPACITY, "round table capacity exceeded");
  return BH_OK;
}

// the chain dataflow sweep where eligible; BH_SWEEP=chunk forces the chunked
// sweep (A/B and parity of both paths)
static bool use_flow(const bh::Dev &d) {
  const char *e = getenv("BH_SWEEP");
  return bh::flow_eligible(d) && !(e && !strcmp(e, "chunk"));
}

// the 32-bit chain-major FD rows (n > 128), allocated the first time a path
// that writes them runs (d.fd_rows): the default wide path never does
int ensure_fd(bh_handle *h) {
  Dev &d = h->d;
  if (d.fd_cols || !d.fd_rows || d.fd) return BH_OK;
  HIPCHK(h, hipMalloc((void **)&d.fd, (size_t)(d.la_rows + 64) * d.npad * 4));
  return BH_OK;
}

// ---------------------------------------------------------------------------
// shards: ranges, local execution, exchanges

// [lo, hi) of `items` owned by shard `rank` of `world`: contiguous, sizes
// differ by at most one (bh_shard_range exposes it to the tests)
inline void shard_range(int64_t items, int32_t world, int32_t rank, int64_t *lo, int64_t *hi) {
  *lo = items * rank / world;
  *hi = items * (rank + 1) / world;
}

// the shards this process drives for handle h
inline std::vector<bh_handle *> local_shards(bh_handle *h) {
  return h->group.empty() ? std::vector<bh_handle *>{h} : h->group;
}

// run fn on every local shard: one host thread per shard of an in-process
// group (each on its own device and stream; the round loop polls its device
// from the host), inline otherwise.  The first failure is reported on h.
template <class F>
int run_local(bh_handle *h, F fn) {
  if (h->group.size() <= 1) return fn(h);
  const size_t G = h->group.size();
  std::vector<int> rc(G, BH_OK);
  std::vector<std::thread> th;
  for (size_t i = 0; i < G; ++i)
    th.emplace_back([&, i] {
      bh_handle *s = h->group[i];
      if (hipSetDevice(s->device) != hipSuccess) { rc[i] = s->fail(BH_ERR_DEVICE, "hipSetDevice"); return; }
      rc[i] = fn(s);
    });
  for (auto &t : th) t.join();
  for (size_t i = 0; i < G; ++i)
    if (rc[i] != BH_OK) {
      if (h->group[i] != h) h->err = "shard " + std::to_string(i) + ": " + h->group[i]->err;
      (void)hipSetDevice(h->device);
      return rc[i];
    }
  (void)hipSetDevice(h->device);
  return BH_OK;
}

// All-gather of per-shard byte ranges of one device buffer (same layout on
// every shard): shard r owns [off[r], off[r] + len[r]) of the buffer `sel`
// selects; afterwards every shard holds every range.  In-process: each
// shard's stream waits for the owner's work, then peer-copies the range
// (xGMI between devices, a device copy on a shared one).  Across processes:
// one ncclBroadcast per owner, in place, grouped.
template <class Sel>
int exchange(bh_handle *h, Sel sel, const std::vector<size_t> &off, const std::vector<size_t> &len) {
  if (h->world <= 1) return BH_OK;
  const auto t0 = std::chrono::steady_clock::now();
  if (h->xport) {
    uint8_t *base = reinterpret_cast<uint8_t *>(sel(h));
    int rc;
    if ((rc = h->xport->group_start(h))) return rc;
    for (int r = 0; r < h->world; ++r)
      if (len[r] && (rc = h->xport->bcast(h, base + off[r], len[r], r, h->stream))) {
        (void)h->xport->group_end(h);
        return rc;
      }
    if ((rc = h->xport->group_end(h))) return rc;
    HIPCHK(h, wait_stream(h->stream));
  } else {
    const size_t G = h->group.size();
    std::vector<hipEvent_t> ready(G);
    for (size_t r = 0; r < G; ++r) {
      bh_handle *o = h->group[r];
      HIPCHK(h, hipSetDevice(o->device));
      HIPCHK(h, hipEventCreateWithFlags(&ready[r], hipEventDisableTiming));
      HIPCHK(h, hipEventRecord(ready[r], o->stream));
    }
    for (size_t t = 0; t < G; ++t) {
      bh_handle *dst = h->group[t];
      HIPCHK(h, hipSetDevice(dst->device));
      uint8_t *db = reinterpret_cast<uint8_t *>(sel(dst));
      for (size_t r = 0; r < G; ++r) {
        if (r == t || !len[r]) continue;
        bh_handle *src = h->group[r];
        HIPCHK(h, hipStreamWaitEvent(dst->stream, ready[r], 0));
        HIPCHK(h, hipMemcpyPeerAsync(db + off[r], dst->device, reinterpret_cast<uint8_t *>(sel(src)) + off[r],
                                     src->device, len[r], dst->stream));
      }
    }
    for (size_t t = 0; t < G; ++t) {
      HIPCHK(h, hipSetDevice(h->group[t]->device));
      HIPCHK(h, wait_stream(h->group[t]->stream));
      (void)hipEventDestroy(ready[t]);
    }
    HIPCHK(h, hipSetDevice(h->device));
  }
  h->xchg_ms += std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return BH_OK;
}

// per-shard ranges of items [base, base + items) of a table of `esz`-byte
// entries (with ofs: item i spans entries [ofs[i], ofs[i + 1]))
std::vector<size_t> range_bytes(const bh_handle *h, int64_t items, size_t esz, bool lengths,
                                const std::vector<int32_t> *ofs = nullptr, int64_t base = 0) {
  std::vector<size_t> v((size_t)h->world);
  for (int r = 0; r < h->world; ++r) {
    int64_t lo, hi;
    shard_range(items, h->world, r, &lo, &hi);
    lo += base;
    hi += base;
    if (ofs) { lo = (*ofs)[(size_t)lo]; hi = (*ofs)[(size_t)hi]; }  // item ranges -> entry ranges
    v[(size_t)r] = lengths ? (size_t)(hi - lo) * esz : (size_t)lo * esz;
  }
  return v;
}

// ---------------------------------------------------------------------------
// stage 1: coordinates, Lamport timestamps, rounds, witnesses

// A Reset hashgraph's coordinates (kernels_reset.hip): the events [0, E0)
// -- every event whose other-parent only Root.Others knows lies in it --
// one at a time, then the chain dataflow resumes every chain after them as
// a segment does (Root LamportTimestamps seed the chains, lt_seed); each
// part is transposed and walked for firstDescendants like a segment
int reset_coords(bh_handle *h, hipStream_t s) {
  Dev &d = h->d;
  const int n = d.n;
  if (!(bh::flow32_eligible(d) && use_flow(d)) && !bh::floww_eligible(d))
    return h->fail(BH_ERR_STATE, "Reset hashgraphs need the chain dataflow (n <= 512, chains within its limits)");
  const int64_t N = d.N, E0 = std::min<int64_t>(h->E0, N);
  int32_t *stg = h->seg_stage;  // [lo, len] of part A, then of part B
  for (int c = 0; c < n; ++c) {
    const auto &ch = h->chain[(size_t)c];
    const int32_t a = (int32_t)(std::lower_bound(ch.begin(), ch.end(), (int32_t)E0) - ch.begin());
    stg[c] = 0;
    stg[n + c] = a;
    stg[2 * n + c] = a;
    stg[3 * n + c] = (int32_t)ch.size();
  }
  HIPCHK(h, hipMemcpyAsync(h->segbuf, stg, (size_t)4 * n * 4, hipMemcpyHostToDevice, s));
  Dev va = d, vb = d;
  va.seg_lo = h->segbuf;
  va.chain_len = h->segbuf + n;
  va.N = E0;
  va.e0 = 0;
  va.tile_list = nullptr;
  vb.seg_lo = h->segbuf + 2 * n;
  vb.chain_len = h->segbuf + 3 * n;
  vb.e0 = E0;
  vb.tile_list = nullptr;
  if (E0 > 0) {
    bh::launch_reset_coords(va, s);
    bh::launch_flow_transpose(va, s);
    bh::launch_fd_idle(va, s);
  }
  HIPCHK(h, hipMemsetAsync(d.state + bh::ST_FLOWOVF, 0, 4, s));
  if (N > E0) {
    if (bh::flow32_eligible(d) && use_flow(d)) {
      bh::launch_flow_desc(vb, s);
      bh::launch_flow(vb, s);
      h->sweep_kernel = bh::flow_kernel(d);
    } else {
      bh::launch_floww(vb, s);
      h->sweep_kernel = bh::floww_kernel(d);
    }
    bh::launch_flow_transpose(vb, s);
    bh::launch_fd_idle(vb, s);
  }
  HIPCHK(h, hipGetLastError());
  return BH_OK;
}

// The segments left only the column-major LA (rounds_pipelined, n <= 128):
// the row-major LA and the complete FDT of the layout's rows up to the
// chain lengths `upto` -- a query's, or an eager call resuming a prefix --
// as the segment pipeline's eager transpose builds them: only the tiles of
// rows past the ones an earlier build covered (their FD entries of older
// rows are completed by the new rows' walk and k_fd_idle), or every row the
// first time and after a relayout.  Synchronous (its staging is reused).
int build_rows(bh_handle *h, const std::vector<int32_t> &upto, hipStream_t s) {
  const int n = h->d.n;
  Dev v = h->d;
  v.e0 = 0;
  v.rows = h->layout_rows;
  v.col0 = 0;
  v.ncol = n;
  v.xpose_fd = 1;
  const bool inc = h->rows_built && (int)h->rows_lens.size() == n;
  int32_t *stg = h->seg_stage;  // [lo | len] per chain
  for (int c = 0; c < n; ++c) {
    stg[c] = inc ? std::min(h->rows_lens[(size_t)c], upto[(size_t)c]) : 0;
    stg[n + c] = upto[(size_t)c];
  }
  HIPCHK(h, hipMemcpyAsync(h->segbuf, stg, (size_t)2 * n * 4, hipMemcpyHostToDevice, s));
  v.seg_lo = h->segbuf;
  v.chain_len = h->segbuf + n;
  v.tile_list = nullptr;
  v.ntiles = 0;
  if (inc) {  // the 64-row tiles holding the new rows, shared boundary tiles once
    int32_t *tl = h->tlist_stage;
    int64_t nt = 0;
    for (int c = 0; c < n; ++c) {
      if (stg[n + c] <= stg[c]) continue;
      const int64_t a = ((int64_t)h->cstart_h[(size_t)c] + stg[c]) >> 6,
                    b = ((int64_t)h->cstart_h[(size_t)c] + stg[n + c] - 1) >> 6;
      for (int64_t t = (nt && tl[nt - 1] >= a) ? tl[nt - 1] + 1 : a; t <= b; ++t) tl[nt++] = (int32_t)t;
    }
    if (nt) HIPCHK(h, hipMemcpyAsync(h->tlist, tl, (size_t)nt * 4, hipMemcpyHostToDevice, s));
    v.tile_list = h->tlist;
    v.ntiles = nt;
  }
  if (!inc || v.ntiles > 0) bh::launch_flow_transpose(v, s);
  bh::launch_fd_idle(v, s);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, wait_stream(s));
  h->rows_lens = upto;
  h->rows_built = true;
  h->rows_stale = false;
  return BH_OK;
}

// coordinates up to the dataflow kernel (this shard's LA columns when split)
int rounds_coords(bh_handle *h) {
  int rc;
  if ((rc = upload(h))) return rc;
  Dev &d = h->d;
  d.N = (int64_t)h->h_creator.size();
  d.e0 = 0;
  d.seg_lo = h->seg_zero;
  h->xchg_ms = 0;
  h->segments_used = 1;
  h->inc_valid = false;
  h->fdt_lost = false;
  h->rows_stale = false;  // (rounds_loop transposes)
  h->rows_built = false;
  if ((rc = set_chain_tables(h))) return rc;
  d.rows = h->layout_rows;
  hipStream_t s = h->stream;
  HIPCHK(h, hipEventRecord(h->ev[0], s));
  bh::launch_prep(d, s);
  if (h->reset_on) {
    int rc2 = reset_coords(h, s);
    if (rc2) return rc2;
  } else if (use_flow(d)) {
    bh::launch_flow_desc(d, s);
    HIPCHK(h, hipEventRecord(h->ev_sweep[0], s));
    bh::launch_flow(d, s);
    HIPCHK(h, hipEventRecord(h->ev_sweep[1], s));
    h->sweep_kernel = bh::flow_kernel(d);
  } else if (bh::floww_eligible(d)) {
    HIPCHK(h, hipEventRecord(h->ev_sweep[0], s));
    bh::launch_floww(d, s);
    HIPCHK(h, hipEventRecord(h->ev_sweep[1], s));
    h->sweep_kernel = bh::floww_kernel(d);
  } else {
    bh::launch_chunk_depth(d, s);
    HIPCHK(h, hipEventRecord(h->ev_sweep[0], s));
    bh::launch_la_sweep(d, s);
    HIPCHK(h, hipEventRecord(h->ev_sweep[1], s));
    bh::launch_permute(d, s);
    h->sweep_kernel = "k_la_sweep";
  }
  HIPCHK(h, hipGetLastError());
  return BH_OK;
}

// the rest: LA rows + firstDescendants, the round loop, witness tables
int rounds_tail(bh_handle *h, const int32_t *st, int64_t e_begin, bool tables_done = false);

int rounds_loop(bh_handle *h) {
  int rc;
  Dev &d = h->d;
  hipStream_t s = h->stream;
  const bool walked = use_flow(d);
  bool wide_flow = bh::floww_eligible(d);
  if (wide_flow) {  // k_floww's watchdog (ST_FLOWOVF = 2): the chunked sweep instead
    int32_t ovf = 0;
    HIPCHK(h, hipMemcpyAsync(&ovf, d.state + bh::ST_FLOWOVF, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(h, wait_stream(s));
    if (ovf == 2 && h->reset_on) {
      // the watchdog counts stalled headers, not a proven deadlock (other
      // work sharing the compute units can starve a wave): the Reset
      // coordinates have no sweep fallback (it knows no Root seeds), so the
      // dataflow runs once more before the call fails
      HIPCHK(h, hipMemsetAsync(d.state + bh::ST_FLOWOVF, 0, 4, s));
      int rc2 = reset_coords(h, s);
      if (rc2) return rc2;
      HIPCHK(h, hipMemcpyAsync(&ovf, d.state + bh::ST_FLOWOVF, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(h, wait_stream(s));
    }
    if (ovf && h->reset_on)
      return h->fail(BH_ERR_CAPACITY, ovf == 2 ? "the wide dataflow gave up twice on a Reset hashgraph"
                                               : "Lamport timestamps beyond the wide dataflow's range after Reset");
    if (ovf == 2) {
      HIPCHK(h, hipMemsetAsync(d.state + bh::ST_FLOWOVF, 0, 4, s));
      bh::launch_chunk_depth(d, s);
      bh::launch_la_sweep(d, s);
      bh::launch_permute(d, s);
      h->sweep_kernel = "k_la_sweep";
      wide_flow = false;
    }
  }
  // LA rows and the firstDescendants walk (FDT) from the dataflow's
  // column-major LA; n > 128 then transposes FDT into chain-major FD rows
  if ((walked || wide_flow) && !h->reset_on) bh::launch_flow_transpose(d, s);  // (reset_coords transposed already)
  d.fd_rows = !((walked || wide_flow) && bh::round_p16(d));  // 32-bit fd rows only where read
  if ((rc = ensure_fd(h))) return rc;
  bh::launch_first_descendants(d, s, walked || wide_flow);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev[1], s));
  h->coords_for = (int)d.N;
  if (d.N == 0) {
    HIPCHK(h, hipEventRecord(h->ev[2], s));
    h->R = 0;
    h->n_div = 0;
    h->wofs_h.assign(1, 0);
    h->stage = 1;
    return BH_OK;
  }
  int32_t st[bh::ST_COUNT];
  d.wide_cols = 0;  // (the wide loop over FDT: rows were transposed above)
  d.use_cla = d.fd_cols && !bh::round_solo_eligible(d);
  if (h->reset_on) {
    // rounds below r0 event by event, then the loop from B[r0]
    HIPCHK(h, hipMemsetAsync(d.rexists, 0, (size_t)d.R_cap + 1, s));
    HIPCHK(h, hipMemsetAsync(d.fw, 0xFF, (size_t)(d.r0 - d.rlo) * d.n * 4, s));
    HIPCHK(h, hipMemsetAsync(d.state + bh::ST_FIATMAX, 0xFF, 4, s));
    bh::launch_fiat(d, s);
    bh::launch_round_resume(d, s);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemcpyAsync(&h->fiat_max, d.state + bh::ST_FIATMAX, 4, hipMemcpyDeviceToHost, s));
    if (getenv("BH_FIAT_DEBUG")) {
      int32_t fs[4] = {0, 0, 0, 0};
      HIPCHK(h, hipMemcpyAsync(fs, d.state + bh::ST_FIATMAX, 16, hipMemcpyDeviceToHost, s));
      HIPCHK(h, wait_stream(s));
      fprintf(stderr, "[k_fiat] max round %d, chains done %d of %d, events visited %d, chunks %d (r0 %d)\n", fs[0], fs[1],
              d.n, fs[2], fs[3], d.r0);
      if (d.diag) {
        unsigned long long g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        HIPCHK(h, copy_sync(s, g, d.diag + 24, sizeof g, hipMemcpyDeviceToHost));
        const double e = (double)(g[4] ? g[4] : 1);
        fprintf(stderr, "[k_fiat] cycles per event (BH_FIAT=serial: finalize + pr, witness rows, counts) or per step "
                "(level-synchronous: parents, counts, rounds): %.0f, %.0f, %.0f (%llu); round stagings %llu\n",
                g[0] / e, g[1] / e, g[2] / e, g[4], g[7]);
        HIPCHK(h, hipMemsetAsync(d.diag + 24, 0, sizeof g, s));
      }
    }
  } else {
    bh::launch_round_init(d, s);
  }
  if ((rc = run_round_loop(h, d, &h->graph, &h->graph_dev, &h->graph_s, &h->graph_dev_s, st))) return rc;
  bh::launch_resume_point(d, st[bh::ST_ROUNDS], nullptr, s);  // each chain's resume round (rq) for the next call
  if ((rc = rounds_tail(h, st, 0))) return rc;
  if (h->reset_on && !h->fdt_lost) {
    // a Reset hashgraph's later calls resume from here (rounds_segmented):
    // the chain dataflow left every LA row and a complete FDT
    h->n_coord = d.N;
    h->lens_coord = h->lens_h;
    h->inc_valid = true;
  }
  return BH_OK;
}

// after the loop: witness tables, per-event rounds, PendingRounds.  Rounds
// and witness flags of events [0, e_begin) are unchanged (an incremental
// call appended events only)
int rounds_tail(bh_handle *h, const int32_t *st, int64_t e_begin, bool tables_done) {
  Dev &d = h->d;
  hipStream_t s = h->stream;
  h->R = st[bh::ST_ROUNDS];
  h->iters = st[bh::ST_ITERS];
  // a Reset hashgraph with no event at round r0 yet: the last round is the fiat pass's
  if (h->reset_on && h->R <= d.r0) h->R = h->fiat_max + 1;
  if (h->reset_on && st[bh::ST_FLOWOVF])  // the fallbacks know no Root LamportTimestamps
    return h->fail(BH_ERR_CAPACITY, "Lamport timestamps beyond the dataflow kernel's range after Reset");
  if (st[bh::ST_FLOWOVF]) {  // LT reached the one-dword limit; LT only feeds the frame order
    if (bh::floww_eligible(d)) {  // the chunked sweep recomputes LA (same values) and LT
      bh::launch_chunk_depth(d, s);
      bh::launch_la_sweep(d, s);
      bh::launch_permute(d, s);
      // its slabs share FDT's memory: the next query recomputes the
      // coordinates, the next pass starts from scratch
      h->coords_for = -1;
      h->fdt_lost = true;
      h->rows_built = false;
    } else {
      bh::launch_flow_lt_fallback(d, s);
    }
  }
  // (tables_done: rounds_pipelined launched them from the device's round
  // count, ahead of its synchronisation)
  if (!tables_done) bh::launch_witness_tables(d, h->R, s);
  bh::launch_assign_rounds(d, e_begin, h->n_div, h->P, s);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev[2], s));
  if (!(h->fuse_fame && h->world == 1)) {
    // the witness offsets (the split's fame exchange reads them), behind the
    // stage's synchronisation.  bh_run_consensus on one shard goes on to
    // DecideFame at once instead: its scatter reads the bounds on the device
    h->wofs_h.resize((size_t)h->R + 1);
    int rc;
    if ((rc = rd_async(h, s, h->wofs_h.data(), d.wofs, ((size_t)h->R + 1) * 4)) || (rc = rd_wait(h, s))) return rc;
  }
  h->n_div = d.N;
  // rounds new to this call join PendingRounds undecided (hashgraph.go:809-815;
  // every round >= LastConsensusRound is queued when it first appears)
  h->pend_dec.resize((size_t)h->R, 0);
  h->stage = 1;
  return BH_OK;
}

// Coordinates and rounds as a pipeline over K insertion-order prefixes
// (segments): the coordinate kernels of prefix s + 1 run on stream2 while
// the round loop runs prefix s on `stream`, resuming at the last round the
// previous prefix fixed (k_resume_point).  Chain dataflow paths only:
// n <= 128 (k_flow32 + k_round2) and 128 < n <= 512 (k_floww2 + the 16-bit
// k_round_wide over the complete FDT); every shard of a group whose
// coordinates are replicated (the default) runs it on its own device.
bool segments_eligible(const bh_handle *h) {
  const Dev &d = h->d;
  if (h->shard_cols) return false;
  if (d.fd_cols) return use_flow(d) && bh::flow32_eligible(d);
  return bh::floww_eligible(d) && bh::round_p16(d);
}

// segments for `events` new events: measured at C3 (10M events): 4
// segments 73.4 ms, 8 segments 72.4 ms, one 84.3 ms (profiles/r2_segments.log).
// The wide path (n > 128) takes one: k_floww2 (145 KiB of LDS) and the
// wide transpose leave no compute unit room for a k_round_wide workgroup,
// so its segments run one after the other and only cost more (C4: 284 ->
// 316 ms with 8, profiles/r3_c4_segments.log); its incremental calls still
// run as one more segment of the same machinery
int segments_for(const Dev &d, int64_t events) {
  // (round 3: C5, 2M events, 79.0M events/s at 4 segments, 87.0M at 8,
  // 88.1M at 12; C2, 1M events, 48.6M at 4, 48.3M at 8; C3 equal at 8 and 12)
  // (round 4, persistent loop, C3: with each segment's LT after the next
  // one's columns, 8 segments 188.8M events/s, 16 187.6M, 24 184.1M)
  // (round 5, C3 10M events, segment k holding a 1.38^k share: 38.1-38.4 ms
  // per step at 10-14 segments against 40.1 at 8 segments of 1.5^k)
  // (round 6: at n <= 96 the dataflow and the loop take about as long, so
  // more, flatter segments shorten the loop left after the dataflow's end;
  // at n = 128 the lean loop is only ~1.14x the dataflow: 16 of 1.15x)
  int K = !d.fd_cols ? 1
          : d.n <= 96 ? (events >= 1000000 ? 12 : 1)
                      : (events >= 4000000 ? 16 : events >= 1500000 ? 8 : events >= 1000000 ? 4 : 1);
  if (const char *e = getenv("BH_SEGMENTS")) K = atoi(e);
  return (int)std::max<int64_t>(1, std::min<int64_t>({K, events / 4096 + 1, 64}));
}

// ---------------------------------------------------------------------------
// the coordinate split (kernels_split.hip): shard 0 of
// a group runs the round loop, fame and order and computes no coordinates;
// shards 1 .. G-1 run the chain dataflow for a range of LA columns each
// (rank 1 also the Lamport timestamps) and ship every segment's rows of
// them to shard 0, packed as 16-bit offsets, over xGMI (peer copies in
// process, ncclSend / ncclRecv across processes)

// segment boundaries of a K-segment pipeline over events [base, N):
// sizes grow geometrically, s_k proportional to 1.5^k.  The loop waits for
// the first segment's coordinates only if every later segment's
// coordinates finish before the loop's previous segment does: segment k + 1's
// dataflow starts when the loop starts segment k (the segment views are
// double-buffered), so s_(k+1) <= (loop time / dataflow time per event) s_k
// suffices -- 1.8 at C3 with k_flow32x2 (5.65 against 3.1 ms per 1.25M
// events), and 1.5 leaves margin.  The pipeline's fill is then the first
// segment's dataflow, 1/49 of the events at K = 8 (round 4: a first segment
// of 1/(4K) and K - 1 equal ones after it, which at C3 left the loop waiting
// ~2 ms for the second segment)
// The growth ratio: segment k + 1's dataflow runs beside segment k's loop,
// so it can grow by (loop time / dataflow time) per event and still be ready
// when the loop reaches it; grown faster, the loop waits for it between
// segments.  That ratio depends on n: at C3 (n = 128) the loop is ~1.14x
// the dataflow (29.4 against 25.9 ms per step with k_round_lean; 1.32 with
// k_round2p left 3.35 ms of waits between the loop's launches,
// profiles/r6_seg_sweep_lean.txt: 34.5 -> 32.0 ms at 1.15 x 16 segments);
// at C5 (n = 64) and C2 (n = 32) the two take about the same time, where
// growing segments only leave a long last loop after the dataflow's end:
// equal segments.  BH_SEG_RATIO overrides it (A/B)
// (round 6, profiles/r6_seg_sweep.txt, r6_seg_sweep_lean.txt: C5 16.89 ->
// 14.3 ms with 12 equal segments, C2 11.63 -> 9.6 ms with 12 equal segments)
constexpr double SEG_RATIO_WIDE = 1.15, SEG_RATIO_NARROW = 1.0;
static double seg_ratio(const Dev &d) {
  if (const char *e = getenv("BH_SEG_RATIO")) return std::max(1.0, atof(e));
  return d.n > 96 ? SEG_RATIO_WIDE : SEG_RATIO_NARROW;
}

static void segment_bounds(int64_t base, int64_t N, int K, double ratio, int64_t *Ns) {
  Ns[0] = base;
  if (K <= 1) { Ns[1] = N; return; }
  double w[64], tot = 0;
  K = std::min(K, 64);
  // segment k holds a ratio^k share: a short first segment (the loop waits
  // for its coordinates) and segments growing about as fast as the loop
  // outruns the dataflow (seg_ratio)
  for (int k = 0; k < K; ++k) tot += (w[k] = std::pow(ratio, k));
  double acc = 0;
  for (int k = 1; k < K; ++k) {
    acc += w[k - 1];
    // at least one event per segment (segments_for keeps >= 4096 per segment on average)
    Ns[k] = std::max(Ns[k - 1] + 1, base + (int64_t)((double)(N - base) * acc / tot));
  }
  Ns[K] = N;
}

// the LA columns of coordinate shard `rank` (>= 1) of a split group
inline void split_cols(const bh_handle *h, int32_t rank, int64_t *c0, int64_t *c1) {
  shard_range(h->d.n, h->world - 1, rank - 1, c0, c1);
}

// the split runs on the chain dataflows: n <= 128 (k_flow32 + k_round2p)
// and 128 < n <= 512 (k_floww2 on the coordinate shards; shard 0 transposes
// each segment for the 16-bit k_round_wide); every shard decides it alike
// from its (identical) host tables
bool split_active(const bh_handle *h) {
  const Dev &d = h->d;
  const bool narrow = bh::flow_eligible(d) && bh::flow32_eligible(d);
  const bool wide = !d.fd_cols && bh::floww_eligible(d) && bh::round_p16(d);
  return h->split && !h->reset_on && d.N > 0 && (narrow || wide) &&
         !(getenv("BH_SWEEP") && !strcmp(getenv("BH_SWEEP"), "chunk"));
}

// per-chain prefix lengths at an insertion-order boundary (ids of a chain
// ascend with its index); bounds at or below the events inserted so far
// are kept (lens_memo)
void chain_lens_at(const bh_handle *h, int64_t bound, int32_t *out) {
  const int n = h->d.n;
  const bool keep = bound <= (int64_t)h->h_creator.size();
  if (keep) {
    const auto it = h->lens_memo.find(bound);
    if (it != h->lens_memo.end() && (int)it->second.size() == n) {
      std::copy(it->second.begin(), it->second.end(), out);
      return;
    }
  }
  for (int c = 0; c < n; ++c) {
    const auto &ch = h->chain[(size_t)c];
    out[c] = (int32_t)(std::lower_bound(ch.begin(), ch.end(), (int32_t)std::min<int64_t>(bound, INT32_MAX)) - ch.begin());
  }
  if (keep) {
    if (h->lens_memo.size() >= 1024) h->lens_memo.clear();
    h->lens_memo[bound].assign(out, out + n);
  }
}

// one call's segments, alike on every shard: boundaries, each segment's
// chain ranges [lo, hi) and packing tables P (rows before chain c) and Q
// (64-row chunks before chain c), the blocks' sizes
struct SplitPlan {
  int K = 0;
  int64_t base = 0;
  std::vector<int64_t> Ns, S, NQ;
  std::vector<int32_t> tab;  // [K][lo, hi][n], then [K][P, Q][n + 1]
  // block (k, r) at byte offset off[k * world + r] of every shard's xbuf
  // (segment-major, then coordinate rank): one layout everywhere, so a
  // block is broadcast in place and peer-copied offset to offset
  std::vector<size_t> off;
  size_t total = 0;
  size_t boff(const bh_handle *h, int k, int32_t rank) const { return off[(size_t)k * h->world + rank]; }
  const int32_t *dview(const bh_handle *h, int k) const { return h->xseg + (size_t)k * 2 * h->d.n; }
  const int32_t *dpq(const bh_handle *h, int k) const {
    return h->xseg + (size_t)K * 2 * h->d.n + (size_t)k * 2 * (h->d.n + 1);
  }
  size_t block_bytes(const bh_handle *h, int k, int32_t rank) const {
    int64_t c0, c1;
    split_cols(h, rank, &c0, &c1);
    return bh::split_layout((int)(c1 - c0), S[(size_t)k], NQ[(size_t)k], rank == 1, nullptr, nullptr);
  }
  bh::SplitBlock block(const bh_handle *h, int k, int32_t rank, uint8_t *at) const {
    int64_t c0, c1;
    split_cols(h, rank, &c0, &c1);
    bh::SplitBlock b;
    bh::split_layout((int)(c1 - c0), S[(size_t)k], NQ[(size_t)k], rank == 1, &b, at);
    b.c0 = (int32_t)c0;
    // (test knobs, read per block: the tests switch them) BH_SPLIT_RANGE
    // lowers the 16-bit range so gossip DAGs fill the overflow slots, from
    // segment BH_SPLIT_RANGE_SEG on (0: every segment) -- a LATER segment's
    // overflow while earlier loops run
    const char *e = getenv("BH_SPLIT_RANGE");
    const char *es = getenv("BH_SPLIT_RANGE_SEG");
    b.range = e && k >= (es ? atoi(es) : 0) ? std::clamp(atoi(e), 0, 65535) : 65535;
    return b;
  }
};

SplitPlan split_plan(const bh_handle *h, int K, int64_t base) {
  const int n = h->d.n;
  const int64_t N = h->d.N;
  SplitPlan p;
  p.K = K;
  p.base = base;
  p.Ns.assign((size_t)K + 1, base);
  segment_bounds(base, N, K, seg_ratio(h->d), p.Ns.data());
  p.tab.assign((size_t)K * 2 * n + (size_t)K * 2 * (n + 1), 0);
  p.S.assign((size_t)K, 0);
  p.NQ.assign((size_t)K, 0);
  for (int k = 0; k < K; ++k) {
    int32_t *lo = p.tab.data() + (size_t)k * 2 * n, *hi = lo + n;
    chain_lens_at(h, p.Ns[(size_t)k], lo);
    chain_lens_at(h, p.Ns[(size_t)k + 1], hi);
    int32_t *P = p.tab.data() + (size_t)K * 2 * n + (size_t)k * 2 * (n + 1), *Q = P + n + 1;
    P[0] = Q[0] = 0;
    for (int c = 0; c < n; ++c) {
      P[c + 1] = P[c] + (hi[c] - lo[c]);
      Q[c + 1] = Q[c] + (hi[c] - lo[c] + 63) / 64;
    }
    p.S[(size_t)k] = P[n];
    p.NQ[(size_t)k] = Q[n];
  }
  p.off.assign((size_t)K * h->world, 0);
  for (int k = 0; k < K; ++k)
    for (int r = 1; r < h->world; ++r) {
      p.off[(size_t)k * h->world + r] = p.total;
      p.total += p.block_bytes(h, k, r);
    }
  return p;
}

// the plan's tables on x's device (one upload), its segment events, and
// `bytes` of block buffer
int split_prepare(bh_handle *x, const SplitPlan &p, size_t bytes) {
  if (p.K > x->xseg_k) {
    if (x->xseg) (void)hipFree(x->xseg);
    x->xseg = nullptr;
    x->xseg_k = 0;
    HIPCHK(x, hipMalloc((void **)&x->xseg, p.tab.size() * 4));
    x->xseg_k = p.K;
  }
  HIPCHK(x, copy_sync(x->stream, x->xseg, p.tab.data(), p.tab.size() * 4, hipMemcpyHostToDevice));
  if (bytes > x->xcap) {
    HIPCHK(x, wait_stream(x->stream2));
    if (x->xbuf) (void)hipFree(x->xbuf);
    x->xbuf = nullptr;
    x->xcap = 0;
    const size_t cap = bytes + bytes / 4;
    HIPCHK(x, hipMalloc((void **)&x->xbuf, cap));
    x->xcap = cap;
  }
  while ((int)x->seg_ev.size() < 4 * p.K) {
    hipEvent_t e;
    HIPCHK(x, hipEventCreate(&e));
    x->seg_ev.push_back(e);
  }
  while ((int)x->pack_ev.size() < p.K) {
    hipEvent_t e;
    HIPCHK(x, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    x->pack_ev.push_back(e);
  }
  if (!x->xprep) HIPCHK(x, hipEventCreateWithFlags(&x->xprep, hipEventDisableTiming));
  if (!x->stream3) {  // (the coordinate stream's priority: the loop stream keeps the higher one)
    int lo_pri = 0, hi_pri = 0;
    HIPCHK(x, hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri));
    HIPCHK(x, hipStreamCreateWithPriority(&x->stream3, hipStreamNonBlocking, lo_pri));
  }
  return BH_OK;
}

// a coordinate shard's part of the call, enqueued on its stream2: per
// segment the descriptors, k_flow32 over its columns (+ LT on rank 1) and
// the packed block (pack_ev[k]).  The narrow split all-gathers the blocks
// from rounds_pipelined (every shard runs the loop); the wide split sends
// each to rank 0 here (ncclSend, or rank 0's peer copy waits for pack_ev)
int split_coords(bh_handle *x, const SplitPlan &p) {
  Dev dv = x->d;
  const int n = dv.n;
  int64_t c0, c1;
  split_cols(x, x->rank, &c0, &c1);
  dv.col0 = (int32_t)c0;
  dv.ncol = (int32_t)(c1 - c0);
  dv.flow_lt = x->rank == 1;
  const bool wide = !dv.fd_cols;  // 128 < n <= 512: k_floww2
  int rc;
  if ((rc = split_prepare(x, p, p.total))) return rc;
  hipStream_t sc = x->stream2;
  x->segments_used = p.K;
  if (p.base == 0) bh::launch_prep(dv, sc);
  else bh::launch_chain_scatter(dv, p.base, sc);
  HIPCHK(x, hipMemsetAsync(dv.state + bh::ST_FLOWOVF, 0, 4, sc));
  for (int k = 0; k < p.K; ++k) {
    Dev v = dv;
    v.seg_lo = const_cast<int32_t *>(p.dview(x, k));
    v.chain_len = v.seg_lo + n;
    v.N = p.Ns[(size_t)k + 1];
    v.e0 = p.Ns[(size_t)k];
    v.rows = x->layout_rows;
    v.tile_list = nullptr;
    if (wide) {
      // k_floww2 over the shard's columns (its LT value as well: every
      // workgroup set carries one; only rank 1's travels)
      if (dv.ncol > 0) bh::launch_floww(v, sc);
    } else {
      bh::launch_flow_desc(v, sc);
      if (dv.ncol > 0 || dv.flow_lt) bh::launch_flow(v, sc);
    }
    uint8_t *at = x->xbuf + p.boff(x, k, x->rank);
    const bh::SplitBlock b = p.block(x, k, x->rank, at);
    bh::launch_split_pack(v, p.dpq(x, k), b, sc);
    HIPCHK(x, hipEventRecord(x->pack_ev[(size_t)k], sc));
    if (wide && x->xport && (rc = x->xport->send(x, at, p.block_bytes(x, k, x->rank), 0, sc))) return rc;
  }
  HIPCHK(x, hipGetLastError());
  // bookkeeping alike on every shard (the next call's base is rank 0's anyway)
  x->coords_for = (int)dv.N;
  x->n_coord = dv.N;
  x->lens_coord = x->lens_h;
  x->inc_valid = true;
  x->rows_stale = true;
  x->sweep_kernel = wide ? bh::floww_kernel(dv) : bh::flow_kernel(dv);
  return BH_OK;
}

// base > 0: an incremental call -- events [0, base) hold coordinates and
// the round loop left its resume point (ST_RESUME) for that prefix.  sp: the
// coordinate split -- the segments' columns arrive from the coordinate
// shards (grp: the in-process group, else over h->xport) instead of being
// computed here; on a coordinate shard of the narrow split (split_all) its
// own columns come from its dataflow (split_coords, stream2) and the
// others' arrive beside it
int rounds_pipelined(bh_handle *h, int K, int64_t base, const SplitPlan *sp = nullptr,
                     const std::vector<bh_handle *> *grp = nullptr) {
  int rc;
  Dev &d = h->d;  // the whole prefix: every segment's view derives from it
  const int n = d.n;
  const bool cshard = sp && h->rank > 0;  // (split_all: a coordinate shard that runs the loop too)
  const bool wide = !d.fd_cols;  // k_floww2 + k_round_wide (cand16 from FDT)
  if (wide) d.fd_rows = 0;
  // n <= 128: k_round2 and fame read only the dataflow's column-major LA, so
  // the segments skip the row-major LA and FDT (the transpose; 21 GB of the
  // C3 step's HBM traffic) -- queries build them on demand (ensure_coords).
  // A Reset hashgraph's fiat pass and the resident loop (BH_ROUND_SOLO) read
  // them; BH_EAGER_ROWS=1 builds them anyway (A/B)
  // 128 < n <= 512: the 16-bit wide loop reads la_col as well (window,
  // candidates' FD rows, fame's LA rows; k_round_wide<*, true, true>) --
  // BH_WIDE_ROWS=1 keeps the FDT / row-major LA loop (A/B)
  const bool eager_env = getenv("BH_EAGER_ROWS") && atoi(getenv("BH_EAGER_ROWS"));
  const bool wide_rows_env = !getenv("BH_WIDE_COLS") || !atoi(getenv("BH_WIDE_COLS")) ||
                             (getenv("BH_WIDE_ROWS") && atoi(getenv("BH_WIDE_ROWS")));  // (off until verified; read per call: the tests switch it)
  d.wide_cols = wide && !sp && !h->reset_on && !wide_rows_env && !eager_env && bh::round_p16(d) && d.cla && d.n <= 512;
  // BH_WIDE_COLS=2 (A/B): the window from the transposed row-major LA, the hand-off from la_col
  if (d.wide_cols && atoi(getenv("BH_WIDE_COLS")) == 2) d.wide_cols = 2;
  // (the wide split: shard 0 transposes each received segment for the
  // row-major loop)
  const bool eager = sp ? wide
                        : ((wide && d.wide_cols != 1) || h->reset_on || eager_env || bh::round_solo_eligible(d) ||
                           d.round_src_rows);
  d.use_cla = (d.fd_cols || d.wide_cols) && !bh::round_solo_eligible(d);
  if (sp) d.round_src_rows = 0;  // the split ships the column-major LA only
  if (base > 0 && eager && h->rows_stale) {
    // the previous call left the prefix's rows unbuilt (a lazy-rows path)
    // and this one resumes on a path that reads them: build them first
    if ((rc = build_rows(h, h->lens_coord, h->stream))) return rc;
  }
  hipStream_t sr = h->stream, sc = h->stream2;
  if (sp && !cshard) {  // (a coordinate shard's split_coords prepared the plan already)
    if ((rc = split_prepare(h, *sp, sp->total))) return rc;
  }
  // the split's receives and unpacks: a stream of their own, beside a
  // coordinate shard's dataflow on stream2
  hipStream_t sx = sp ? h->stream3 : sc;
  h->segments_used = K;
  h->fdt_lost = false;
  if ((int)h->seg_ev.size() < 4 * K) {
    for (int i = (int)h->seg_ev.size(); i < 4 * K; ++i) {
      hipEvent_t e;
      HIPCHK(h, hipEventCreate(&e));
      h->seg_ev.push_back(e);
    }
  }
  // an incremental call resumes at the last round whose boundaries lie
  // inside the previous prefix on every chain this call extends
  // (k_resume_point left each chain's first outside round in rq)
  int32_t host_resume = d.r0;
  if (base > 0) {
    std::vector<int32_t> rq((size_t)n);
    HIPCHK(h, copy_sync(h->stream, rq.data(), d.rq, (size_t)n * 4, hipMemcpyDeviceToHost));
    int32_t m = INT32_MAX;
    for (int c = 0; c < n; ++c)
      if (h->chain[(size_t)c].size() > (size_t)h->lens_coord[(size_t)c]) m = std::min(m, rq[(size_t)c]);
    host_resume = std::max(d.r0, m == INT32_MAX ? d.r0 : m - 1);
  }
  // the coordinate stream starts after everything queued on the main one
  HIPCHK(h, hipEventRecord(h->ev[0], sr));
  HIPCHK(h, hipStreamWaitEvent(sc, h->ev[0], 0));
  if (!cshard) {  // (a coordinate shard's split_coords queued them ahead of its dataflow)
    if (base == 0) {
      bh::launch_prep(d, sc);
    } else {  // only the new events' chain-table entries; loop state kept
      bh::launch_chain_scatter(d, base, sc);
    }
    HIPCHK(h, hipMemsetAsync(d.state + bh::ST_FLOWOVF, 0, 4, sc));
  }
  if (sp && !cshard) {  // the unpacks wait for the chain tables and the cleared flag
    HIPCHK(h, hipEventRecord(h->xprep, sc));
    HIPCHK(h, hipStreamWaitEvent(sx, h->xprep, 0));
  }
  const int64_t N = d.N;
  std::vector<int64_t> Ns((size_t)K + 1, base);
  segment_bounds(base, N, K, seg_ratio(d), Ns.data());
  // per-chain prefix lengths at a boundary: ids of a chain ascend with its index
  auto lens_at = [&](int64_t bound, int32_t *out) { chain_lens_at(h, bound, out); };
  // segment lengths on the device: three buffers round robin, so that
  // segment k + 1's dataflow waits only for loop k - 2 (long finished) and
  // runs beside loop k - 1 -- with two, its launches (the lengths' copy,
  // k_flow_desc32x2) waited for loop k - 1 and landed on the compute units
  // in the gap between two loops, beside k_seg_resume (15 -> 35 us, C3).
  // The eager rows' tile lists keep two
  const int npar = sp || eager ? 2 : 3;
  auto view = [&](int k) {  // segment k: events [Ns[k], Ns[k + 1])
    Dev v = d;
    v.seg_lo = sp ? const_cast<int32_t *>(sp->dview(h, k)) : h->segbuf + (size_t)(k % npar) * 2 * n;
    v.chain_len = v.seg_lo + n;
    v.N = Ns[(size_t)k + 1];
    v.e0 = Ns[(size_t)k];
    v.rows = h->layout_rows;
    return v;
  };
  // the 64-row tiles holding segment k's rows (the transpose's work list):
  // each chain's run [start + lo, start + hi), in layout order, shared
  // boundary tiles once (eager runs wait for each loop: the staging's two
  // halves cannot be overtaken)
  auto tiles = [&](int k, const int32_t *lo, const int32_t *hi, Dev &v, hipStream_t ts) -> int {
    int32_t *tl = h->tlist_stage + (size_t)(k & 1) * h->tlist_cap;
    int64_t nt = 0;
    for (int c = 0; c < n; ++c) {
      if (hi[c] <= lo[c]) continue;
      const int64_t a = ((int64_t)h->cstart_h[(size_t)c] + lo[c]) >> 6, b = ((int64_t)h->cstart_h[(size_t)c] + hi[c] - 1) >> 6;
      for (int64_t t = (nt && tl[nt - 1] >= a) ? tl[nt - 1] + 1 : a; t <= b; ++t) tl[nt++] = (int32_t)t;
    }
    int32_t *dtl = h->tlist + (size_t)(k & 1) * h->tlist_cap;
    if (nt) HIPCHK(h, hipMemcpyAsync(dtl, tl, (size_t)nt * 4, hipMemcpyHostToDevice, ts));
    v.tile_list = dtl;
    v.ntiles = nt;
    return BH_OK;
  };
  // the split: segment k's columns from the coordinate shards (every other
  // one: a coordinate shard of the narrow split computed its own), into the
  // common block layout -- the narrow split all-gathers them (a broadcast
  // per coordinate rank, in place; in process, peer copies), the wide one
  // receives them on shard 0 only
  auto receive = [&](int k) -> int {
    Dev v = view(k);
    HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * K + k], sx));
    if (cshard) HIPCHK(h, hipStreamWaitEvent(sx, h->pack_ev[(size_t)k], 0));  // its own block (its dataflow) done
    if (grp) {
      for (int r = 1; r < h->world; ++r)
        if (r != h->rank) HIPCHK(h, hipStreamWaitEvent(sx, (*grp)[(size_t)r]->pack_ev[(size_t)k], 0));
    }
    HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * k + 1], sx));
    std::vector<bh::SplitBlock> blk((size_t)h->world);
    for (int r = 1; r < h->world; ++r) blk[(size_t)r] = sp->block(h, k, r, h->xbuf + sp->boff(h, k, r));
    if (grp) {  // peer copies (xGMI between devices, a device copy on a shared one)
      for (int r = 1; r < h->world; ++r) {
        if (r == h->rank) continue;
        const bh_handle *x = (*grp)[(size_t)r];
        const size_t o = sp->boff(h, k, r);
        HIPCHK(h, hipMemcpyPeerAsync(h->xbuf + o, h->device, x->xbuf + o, x->device, sp->block_bytes(h, k, r), sx));
      }
    } else {
      int rc2;
      if ((rc2 = h->xport->group_start(h))) return rc2;
      for (int r = 1; r < h->world; ++r) {
        uint8_t *at = h->xbuf + sp->boff(h, k, r);
        const size_t bb = sp->block_bytes(h, k, r);
        rc2 = h->split_all() ? h->xport->bcast(h, at, bb, r, sx) : h->xport->recv(h, at, bb, r, sx);
        if (rc2) {
          (void)h->xport->group_end(h);
          return rc2;
        }
      }
      if ((rc2 = h->xport->group_end(h))) return rc2;
    }
    HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * k + 2], sx));
    for (int r = 1; r < h->world; ++r)
      if (r != h->rank) bh::launch_split_unpack(v, sp->dpq(h, k), blk[(size_t)r], sx);
    bh::launch_lt_rows(v, sx);
    if (eager) {
      // the wide loop reads the row-major LA and FDT: the segment's rows
      // transposed here, from the columns just unpacked
      const int32_t *lo = sp->tab.data() + (size_t)k * 2 * n;
      if ((rc = tiles(k, lo, lo + n, v, sx))) return rc;
      bh::launch_flow_transpose(v, sx);
      bh::launch_fd_idle(v, sx);
    }
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * k], sx));
    if (k == K - 1) HIPCHK(h, hipEventRecord(h->ev[1], sx));
    return BH_OK;
  };
  // where a segment's Lamport timestamps run: k_flow32x2 (the default)
  // carries them in its first workgroup, (n + 1) / 2 workgroups in all.  The
  // one-value k_flow32 (chains past X2_MAXLEN; BH_FLOW1) needs a workgroup of
  // its own for them: inside the column launch while 2n + 1 workgroups fit
  // the compute units beside the loop's n (C5: 82 -> 101M events/s in round
  // 4), else after the next segment's columns on the coordinate stream (at
  // n = 128 a 129th column workgroup would share a unit with a loop
  // workgroup, which every barrier then waits for; profiles/r4_ab_lt.txt)
  const bool lt_combined = wide || bh::flow32x2_eligible(d) || 2 * n + 1 <= h->ncu;
  auto lt_after = [&](int kk) {  // (!lt_combined) segment kk's LT workgroup and per-event LT, on the coordinate stream
    const Dev vk = view(kk);
    Dev vl = vk;
    vl.ncol = 0;
    vl.flow_lt = 1;
    bh::launch_flow(vl, sc);
    bh::launch_lt_rows(vk, sc);
  };
  auto coords = [&](int k) -> int {
    if (sp) return receive(k);
    Dev v = view(k);
    // pinned staging of its own per segment: with the loops enqueued without
    // host waits (async below) the host runs ahead of these copies
    int32_t *stg = h->seg_stage + (size_t)k * 2 * n;
    lens_at(Ns[(size_t)k], stg);
    lens_at(Ns[(size_t)k + 1], stg + n);
    HIPCHK(h, hipMemcpyAsync(v.seg_lo, stg, (size_t)2 * n * 4, hipMemcpyHostToDevice, sc));
    HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * K + k], sc));  // the segment's lengths are on the device
    if (eager) {
      if ((rc = tiles(k, stg, stg + n, v, sc))) return rc;
    } else {
      v.tile_list = nullptr;
      v.ntiles = 0;
    }
    // a whole-DAG wide run takes the whole-layout transpose (32-row tiles,
    // several workgroups per compute unit) instead of 64-row tile lists
    if (wide && K == 1 && base == 0) v.tile_list = nullptr;
    if (wide) {
      HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * k + 1], sc));
      bh::launch_floww(v, sc);  // the segment's descriptors, then k_floww2
    } else {
      bh::launch_flow_desc(v, sc);
      HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * k + 1], sc));
      // the LA columns only: n workgroups.  With the Lamport timestamps'
      // workgroup beside them (n + 1 = 129 at n = 128) one compute unit of
      // the 256 hosts a column workgroup and a round-loop workgroup at once,
      // and every loop iteration waits for that slower one (C3: 10.8 against
      // 9.7 us per iteration); LT, which the loop does not read, follows
      // once the segment's columns are handed to the loop
      Dev vc = v;
      vc.flow_lt = lt_combined ? 1 : 0;
      bh::launch_flow(vc, sc);
    }
    HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * k + 2], sc));
    if (eager) {
      // (wide_cols 2: the loop's windows need the row-major LA, its hand-off
      // no FDT -- the transpose writes LA rows only)
      Dev vt = v;
      vt.xpose_fd = d.wide_cols == 2 ? 0 : 1;
      bh::launch_flow_transpose(vt, sc);  // (its LT copy is redone by k_lt_rows below)
      if (vt.xpose_fd) bh::launch_fd_idle(v, sc);
    }
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->seg_ev[(size_t)3 * k], sc));  // the segment's LA is ready for the loop
    if (!wide && lt_combined) {
      bh::launch_lt_rows(v, sc);
    } else if (!wide) {
      // the Lamport timestamps of the segment before this one, after this
      // segment's columns: the loop's next segment waits only for columns
      // (the last segment's follow its own columns)
      if (k > 0) lt_after(k - 1);
      if (k == K - 1) lt_after(k);
    } else if (!eager) {  // wide: k_floww2 wrote lt_row; per-event LT (the transpose copies it otherwise)
      bh::launch_lt_rows(v, sc);
      HIPCHK(h, hipGetLastError());
    }
    if (k == K - 1) HIPCHK(h, hipEventRecord(h->ev[1], sc));  // the coordinate pipeline's end
    return BH_OK;
  };
  // n <= 128 with the persistent loop: every segment's loop is enqueued
  // without a host round trip (each used to wait for its loop's state: ~0.2
  // ms of idle device per segment at C3, profiles/r5_gaps_c3.txt).  The
  // resume point reads the round count on the device, a failed loop makes
  // the later ones leave at once (ST_PFAIL), and the host reads the state
  // once, after the last loop.  Other loops (wide, one launch per round,
  // BH_SEG_DEBUG) wait for each segment as before
  const bool dbg = getenv("BH_SEG_DEBUG") && atoi(getenv("BH_SEG_DEBUG"));  // per-segment timings to stderr
  const bool async = !wide && !eager && !dbg && bh::round_persist_eligible(d);
  HIPCHK(h, hipMemsetAsync(d.state + bh::ST_PFAIL, 0, 4, sr));
  if (async && (int)h->loop_evs.size() < 2 * K) {
    for (int i = (int)h->loop_evs.size(); i < 2 * K; ++i) {
      hipEvent_t e;
      HIPCHK(h, hipEventCreate(&e));
      h->loop_evs.push_back(e);
    }
  }
  if ((rc = coords(0))) return rc;
  int32_t st[bh::ST_COUNT];
  hipEvent_t sr_mark;  // the loop stream's progress, for segbuf reuse by stream2
  HIPCHK(h, hipEventCreateWithFlags(&sr_mark, hipEventDisableTiming));
  hipEvent_t lt0 = nullptr, lt1 = nullptr;
  if (dbg) {
    HIPCHK(h, hipEventCreate(&lt0));
    HIPCHK(h, hipEventCreate(&lt1));
  }
  bool wd_fired = false;
  for (int k = 0; k < K; ++k) {
    HIPCHK(h, hipStreamWaitEvent(sr, h->seg_ev[(size_t)3 * k], 0));
    if ((wide || sp) && !async) {
      // k_floww2's watchdog (ST_FLOWOVF = 2; the split: a block that ran out
      // of overflow slots) is read before a loop runs on the segment: a loop
      // over unfinished coordinates could fail ("did not terminate",
      // capacity) before the fallback below is reached.  One host
      // synchronisation per segment; a wide batch runs one segment.  (The
      // persistent n <= 128 loop leaves at once on the flag itself.)  Every
      // segment's receive is still posted, so no coordinate rank's send is
      // left unmatched
      int32_t *ovf = h->pinned_state + bh::ST_COUNT + 4;
      HIPCHK(h, hipMemcpyAsync(ovf, d.state + bh::ST_FLOWOVF, 4, hipMemcpyDeviceToHost, sr));
      HIPCHK(h, wait_stream(sr));
      if (*ovf == 2) wd_fired = true;
    }
    // segment k + 1's coordinates (or receive).  A blocking transport (the
    // host transport's receives and broadcasts wait on the host) takes them
    // after loop k is enqueued, so loop k runs while the host waits for
    // segment k + 1; stream-ordered exchanges go first, as the
    // dataflow's launches do
    const bool late = sp && h->xport && h->xport->blocking();
    auto next = [&]() -> int {
      if (k + 1 >= K) return BH_OK;
      // segment k + 1 reuses the segbuf (and tile-list) slot of k + 1 - npar,
      // last read by its loop (async: the loop's own stop event -- no marker
      // packet on the loop stream) or its resume point
      if (async && npar == 3) {
        if (k >= 2) HIPCHK(h, hipStreamWaitEvent(sx, h->loop_evs[(size_t)2 * (k - 2) + 1], 0));
      } else if (async && k > 0) {
        HIPCHK(h, hipStreamWaitEvent(sx, h->loop_evs[(size_t)2 * k - 1], 0));
      } else {
        HIPCHK(h, hipEventRecord(sr_mark, sr));
        HIPCHK(h, hipStreamWaitEvent(sx, sr_mark, 0));
      }
      return coords(k + 1);
    };
    if (!late && (rc = next())) { (void)hipEventDestroy(sr_mark); return rc; }
    if (wd_fired) {  // (every segment's receive is still posted)
      if (late && (rc = next())) { (void)hipEventDestroy(sr_mark); return rc; }
      continue;
    }
    Dev rv = d;  // the loop's view: only the prefix lengths differ from d
    rv.chain_len = view(k).chain_len;
    if (dbg) HIPCHK(h, hipEventRecord(lt0, sr));
    if (k == 0 && base == 0) {
      bh::launch_round_init(rv, sr);
    } else if (async && k > 0) {
      // the previous loop's resume point and this segment's first
      // candidates in one launch (k_seg_resume: k_resume_point +
      // k_round_resume + k_cand_rows)
      Dev rs = rv;
      rs.seg_lo = view(k).seg_lo;  // (the previous prefix's lengths)
      bh::launch_seg_resume(rs, sr);
    } else {
      if (k == 0) {
        if (h->reset_on) {
          // a Reset hashgraph: the rounds below r0 again, event by event
          // (k_fiat_ls, the fiat region only), which also re-derives B[r0]
          HIPCHK(h, hipMemsetAsync(d.rexists, 0, (size_t)d.R_cap + 1, sr));
          HIPCHK(h, hipMemsetAsync(d.fw, 0xFF, (size_t)(d.r0 - d.rlo) * n * 4, sr));
          HIPCHK(h, hipMemsetAsync(d.state + bh::ST_FIATMAX, 0xFF, 4, sr));
          bh::launch_fiat(rv, sr);
          HIPCHK(h, hipGetLastError());
          HIPCHK(h, hipMemcpyAsync(h->pinned_state + bh::ST_COUNT + 2, d.state + bh::ST_FIATMAX, 4,
                                   hipMemcpyDeviceToHost, sr));
        }
        h->pinned_state[bh::ST_COUNT + 1] = host_resume;
        HIPCHK(h, hipMemcpyAsync(d.state + bh::ST_RESUME, h->pinned_state + bh::ST_COUNT + 1, 4, hipMemcpyHostToDevice, sr));
      }
      bh::launch_round_resume(rv, sr);
    }
    if (async) {
      ++h->persist_loops;
      bh::launch_round_persist(rv, sr, h->loop_evs[(size_t)2 * k], h->loop_evs[(size_t)2 * k + 1]);
      HIPCHK(h, hipGetLastError());
    } else if ((rc = run_round_loop(h, rv, &h->seg_graph[k & 1], &h->seg_graph_dev[k & 1], &h->seg_graph_s[k & 1],
                                    &h->seg_graph_dev_s[k & 1], st))) {
      (void)hipEventDestroy(sr_mark);
      return rc;
    }
    if (late && (rc = next())) { (void)hipEventDestroy(sr_mark); return rc; }
    // where the next segment -- or the next call's new events -- resume
    const int32_t *next_len = nullptr;
    if (k + 1 < K) {
      // (async: the next iteration's wait for segment k + 1's columns, recorded
      // after its lengths on the same stream, covers k_seg_resume -- one
      // barrier packet less between two loops)
      if (!async) HIPCHK(h, hipStreamWaitEvent(sr, h->seg_ev[(size_t)3 * K + k + 1], 0));
      next_len = view(k + 1).chain_len;
    }
    // (async: the next segment's k_seg_resume finds it)
    if (!(async && k + 1 < K)) bh::launch_resume_point(rv, async ? -1 : st[bh::ST_ROUNDS], next_len, sr);
    if (dbg) {
      HIPCHK(h, hipEventRecord(lt1, sr));
      HIPCHK(h, wait_stream(sr));
      float lms = 0, cms = 0, fms = 0;
      (void)hipEventElapsedTime(&lms, lt0, lt1);
      (void)hipEventElapsedTime(&fms, h->seg_ev[(size_t)3 * k + 1], h->seg_ev[(size_t)3 * k + 2]);
      (void)hipEventElapsedTime(&cms, h->seg_ev[(size_t)3 * k + 1], h->seg_ev[(size_t)3 * k]);
      int32_t r0 = 0;
      (void)copy_sync(sr, &r0, rv.state + bh::ST_RESUME, 4, hipMemcpyDeviceToHost);
      fprintf(stderr, "[seg %d] coords %.2f ms (%s %.2f) | loop %.2f ms, rounds %d, iters %d, next resume at %d\n", k,
              cms, wide ? "k_floww2" : bh::flow_kernel(d), fms, lms, st[bh::ST_ROUNDS], st[bh::ST_ITERS], r0);
    }
  }
  if (lt0) (void)hipEventDestroy(lt0);
  if (lt1) (void)hipEventDestroy(lt1);
  (void)hipEventDestroy(sr_mark);
  // the witness tables from the device's round count, launched behind the
  // state's read-back so that they run while the host wakes up (the host
  // checks the state before anything reads them: a failed loop's fallback
  // builds them again)
  const bool tables_early = async && !h->reset_on;
  if (async) {  // every loop's end: one host synchronisation for the call
    if ((rc = rd_async(h, sr, st, d.state, bh::ST_COUNT * 4))) return rc;
    if (tables_early) {
      HIPCHK(h, hipEventRecord(h->ev_st, sr));
      bh::launch_witness_tables(d, -1, sr);
      if ((rc = rd_wait_event(h, h->ev_st))) return rc;
    } else if ((rc = rd_wait(h, sr))) {
      return rc;
    }
    const int32_t fail = std::max(st[bh::ST_PFAIL], st[bh::ST_ERR]);
    if (fail == 1 || (fail == 0 && st[bh::ST_FLOWOVF] != 2 && !st[bh::ST_DONE]))
      return h->fail(fail == 1 ? BH_ERR_CAPACITY : BH_ERR_STATE,
                     fail == 1 ? "round table capacity exceeded" : "round loop did not terminate");
    if (fail == 3) {
      // a grid barrier gave up (some workgroup was never placed): the whole
      // call again through the unpipelined passes, one loop launch per
      // iteration (counted in persist_fallbacks)
      ++h->persist_fallbacks;
      h->inc_valid = false;
      h->segments_used = 1;
      HIPCHK(h, wait_stream(sc));
      HIPCHK(h, wait_stream(sx));
      const int32_t keep = d.round_persist;
      d.round_persist = 0;
      if (!(rc = rounds_coords(h))) rc = rounds_loop(h);
      d.round_persist = keep;
      return rc;
    }
  }
  if ((wide || sp) && (wd_fired || st[bh::ST_FLOWOVF] == 2)) {
    // k_floww2's watchdog left a segment's coordinates unfinished (or a
    // split block could not carry its columns): the whole DAG again through
    // the unpipelined passes on this shard (they fall back to the chunked
    // sweep)
    h->inc_valid = false;
    h->segments_used = 1;
    HIPCHK(h, wait_stream(sc));
    HIPCHK(h, wait_stream(sx));
    if ((rc = rounds_coords(h))) return rc;
    return rounds_loop(h);
  }
  // the last segment's Lamport timestamps run after its LA columns were
  // handed to the loop (coords): the passes after DivideRounds (the frame
  // order reads LT) wait for the coordinate stream's end
  HIPCHK(h, hipStreamWaitEvent(sr, h->ev[1], 0));
  h->coords_for = (int)N;
  h->rows_stale = !eager || d.wide_cols == 2;  // (wide_cols 2 built no FDT)
  if (!h->rows_stale) {  // (the segments' eager transposes built every row so far)
    h->rows_lens = h->lens_h;
    h->rows_built = true;
  }
  h->sweep_kernel = wide ? bh::floww_kernel(d) : bh::flow_kernel(d);
  if (h->reset_on && base > 0) h->fiat_max = h->pinned_state[bh::ST_COUNT + 2];
  if ((rc = rounds_tail(h, st, base, tables_early))) return rc;
  // the timings: every event completed before rounds_tail's synchronisation.
  // Read when asked (settle_timings): ~2K event queries here would hold the
  // device idle between DivideRounds and DecideFame
  h->tm_seg_K = K;
  h->tm_seg_loops = async && !(getenv("BH_LOOP_TIMING") && !atoi(getenv("BH_LOOP_TIMING")));
  h->tm_seg_sp = sp != nullptr;
  h->tm_seg = true;
  if (sp) settle_timings(h);  // (the exchange time feeds the split's stage table now)
  h->n_coord = N;
  h->lens_coord = h->lens_h;
  h->inc_valid = !h->fdt_lost;
  return BH_OK;
}

// DivideRounds of one shard through the segment pipeline where it applies
// (*used = false otherwise, with nothing launched).  A call that only
// appended events resumes from the last one (the cost
// follows the new events)
int rounds_segmented(bh_handle *h, bool *used) {
  int rc;
  *used = false;
  Dev &d = h->d;
  d.N = (int64_t)h->h_creator.size();
  if (d.N == 0) return BH_OK;
  if ((rc = upload(h))) return rc;
  if ((rc = set_chain_tables(h, false))) return rc;
  const bool eligible = segments_eligible(h);
  const int64_t base = (!h->layout_changed && h->inc_valid && d.N >= h->n_coord) ? h->n_coord : 0;
  if (getenv("BH_SEG_DEBUG") && atoi(getenv("BH_SEG_DEBUG")))
    fprintf(stderr, "[segments] N %lld eligible %d layout_changed %d inc_valid %d n_coord %lld reset %d E0 %lld\n",
            (long long)d.N, (int)eligible, (int)h->layout_changed, (int)h->inc_valid, (long long)h->n_coord,
            (int)h->reset_on, (long long)h->E0);
  if (!eligible) return BH_OK;
  // a Reset hashgraph's first call (and any call that brings events whose
  // other-parent only Root.Others knows) computes the whole DAG
  // (rounds_coords / rounds_loop: k_reset_coords, the fiat pass); the calls
  // after it append a segment like any other handle
  if (h->reset_on && (base == 0 || h->E0 > base)) return BH_OK;
  *used = true;
  d.rows = h->layout_rows;
  d.e0 = 0;
  d.seg_lo = h->seg_zero;
  if (base == d.N) {  // nothing new to divide: DivideRounds changes nothing
    h->stage = std::max(h->stage, 1);
    return BH_OK;
  }
  h->inc_calls += base > 0;
  return rounds_pipelined(h, h->reset_on ? 1 : segments_for(d, d.N - base), base);
}

// DivideRounds of a split group: this process's
// shards -- the whole group in process, or this rank -- each in its role.
// Rank 0 decides the call's base (its own resume state; broadcast across
// processes), so every shard cuts the same segments.  The narrow split
// (split_all): the coordinate shards' dataflow first (stream2), then every
// shard's pipeline, which all-gathers the blocks and runs the loop; the
// wide split: the same dataflow and sends, then shard 0's pipeline alone
int rounds_split_stage(bh_handle *h) {
  int rc;
  std::vector<bh_handle *> sh = local_shards(h);
  for (bh_handle *x : sh) {
    HIPCHK(x, hipSetDevice(x->device));
    x->d.N = (int64_t)x->h_creator.size();
    x->xchg_ms = 0;
    if ((rc = upload(x))) return rc;
    if ((rc = set_chain_tables(x))) return rc;
  }
  (void)hipSetDevice(h->device);
  const bool all = h->split_all();
  bh_handle *h0 = sh[0]->rank == 0 ? sh[0] : nullptr;  // the loop shard, if this process drives it
  const int64_t N = sh[0]->d.N;
  int64_t base = 0;
  if (h0) base = (!h0->layout_changed && h0->inc_valid && N >= h0->n_coord) ? h0->n_coord : 0;
  if (h->xport) {  // across processes: rank 0's base
    if (!h->xbase) HIPCHK(h, hipMalloc((void **)&h->xbase, 8));
    int64_t *pin = reinterpret_cast<int64_t *>(h->pinned_state + bh::ST_COUNT + 6);  // (8-B aligned pinned words)
    *pin = base;
    HIPCHK(h, hipMemcpyAsync(h->xbase, pin, 8, hipMemcpyHostToDevice, h->stream));
    if ((rc = h->xport->bcast(h, h->xbase, 8, 0, h->stream))) return rc;
    HIPCHK(h, copy_sync(h->stream, pin, h->xbase, 8, hipMemcpyDeviceToHost));
    base = *pin;
  }
  // the shards that run the loop, fame and order
  std::vector<bh_handle *> loopers;
  for (bh_handle *x : sh)
    if (all || x->rank == 0) loopers.push_back(x);
  auto on_loopers = [&](auto fn) -> int {  // (one host thread per shard in process: their host waits overlap)
    if (loopers.empty()) return BH_OK;
    if (loopers.size() == 1) {
      HIPCHK(loopers[0], hipSetDevice(loopers[0]->device));
      const int r = fn(loopers[0]);
      if (r && loopers[0] != h) h->err = "shard " + std::to_string(loopers[0]->rank) + ": " + loopers[0]->err;
      (void)hipSetDevice(h->device);
      return r;
    }
    return run_local(h, fn);
  };
  if (!split_active(sh[0])) {
    // n > 128 beyond the wide dataflow's limits, chains beyond k_flow32's,
    // a Reset hashgraph, or nothing inserted: the unsplit path on every
    // shard that runs the loop (no exchange); the others start over when
    // the split applies again
    for (bh_handle *x : sh)
      if (!all && x->rank > 0) x->inc_valid = false;
    return on_loopers([](bh_handle *x) {
      bool used = false;
      int r;
      if ((r = rounds_segmented(x, &used)) || used) return r;
      if ((r = rounds_coords(x))) return r;
      return rounds_loop(x);
    });
  }
  if (base == N) {  // nothing new to divide
    for (bh_handle *x : loopers) x->stage = std::max(x->stage, 1);
    return BH_OK;
  }
  // the wide split pipelines as well: k_floww2 runs on the coordinate
  // shards, so shard 0's loop over segment k no longer shares its compute
  // units with the dataflow of segment k + 1 (segments_for keeps the
  // unsplit wide path at one segment for that reason)
  int K = segments_for(sh[0]->d, N - base);
  if (!sh[0]->d.fd_cols && !getenv("BH_SEGMENTS")) K = N - base >= 1000000 ? 4 : 1;
  const SplitPlan plan = split_plan(sh[0], K, base);
  // the coordinate shards' dataflow first: the receives wait on it
  for (bh_handle *x : sh) {
    if (x->rank == 0) continue;
    HIPCHK(x, hipSetDevice(x->device));
    if ((rc = split_coords(x, plan))) {
      if (x != h) h->err = "shard " + std::to_string(x->rank) + ": " + x->err;
      (void)hipSetDevice(h->device);
      return rc;
    }
  }
  (void)hipSetDevice(h->device);
  const std::vector<bh_handle *> *grp = h->xport ? nullptr : &h->group;
  rc = on_loopers([&](bh_handle *x) {
    x->d.rows = x->layout_rows;
    x->d.e0 = 0;
    x->d.seg_lo = x->seg_zero;
    x->inc_calls += base > 0;
    return rounds_pipelined(x, plan.K, base, &plan, grp);
  });
  for (bh_handle *x : sh) {  // the sends / copies of this call are done
    if (x->rank == 0) continue;
    HIPCHK(x, hipSetDevice(x->device));
    HIPCHK(x, wait_stream(x->stream2));
    if (x->stream3) HIPCHK(x, wait_stream(x->stream3));
  }
  (void)hipSetDevice(h->device);
  return rc;
}

int stage_rounds(bh_handle *h) {
  int rc;
  h->xchg_ms = 0;
  for (bh_handle *x : local_shards(h)) {
    x->loop_ms_acc = 0;
    x->tm_seg = x->tm_stages = false;  // (the last run's events are about to be reused: unread timings go)
  }
  if (h->split) return rounds_split_stage(h);
  if (!h->shard_cols) {
    // every shard holds the whole DAG and computes the same coordinates and
    // rounds: each runs the segment pipeline on its own device (one host
    // thread per shard of an in-process group), so a group is never slower
    // than one shard
    int nused = 0;
    std::vector<bh_handle *> sh = local_shards(h);
    std::vector<char> used(sh.size(), 0);
    rc = run_local(h, [&](bh_handle *x) {
      bool u = false;
      const int r = rounds_segmented(x, &u);
      for (size_t i = 0; i < sh.size(); ++i)
        if (sh[i] == x) used[i] = u;
      return r;
    });
    if (rc) return rc;
    for (char u : used) nused += u;
    if (nused == (int)sh.size()) return BH_OK;
    if (nused) return h->fail(BH_ERR_STATE, "shards disagree on the segment pipeline");
  }
  if ((rc = run_local(h, rounds_coords))) return rc;
  if (h->world > 1 && h->shard_cols && use_flow(h->d)) {
    // LA columns: shard r computed columns [col0, col0 + ncol), each a
    // contiguous (la_rows + 64)-int32 run of la_col
    const size_t colb = (size_t)(h->d.la_rows + 64) * 4;
    std::vector<size_t> off = range_bytes(h, h->d.n, colb, false), len = range_bytes(h, h->d.n, colb, true);
    if ((rc = exchange(h, [](bh_handle *x) -> void * { return x->d.la_col; }, off, len))) return rc;
  }
  return run_local(h, rounds_loop);
}

// ---------------------------------------------------------------------------
// stage 2: DecideFame -- this shard's rounds, then exchanged

// the shards the passes after DivideRounds split between: every shard
// (replicated coordinates, or the narrow split, where every shard ran the
// loop), or with the wide split shard 0 alone (it holds the rounds)
inline bool pass_solo(const bh_handle *h) { return h->split && !h->split_all(); }
inline int32_t pass_world(const bh_handle *h) { return pass_solo(h) ? 1 : h->world; }
inline int32_t pass_rank(const bh_handle *h) { return pass_solo(h) ? 0 : h->rank; }

template <class F>
int run_pass(bh_handle *h, F fn) {
  if (!pass_solo(h)) return run_local(h, fn);
  return h->rank == 0 ? fn(h) : BH_OK;  // (in process, h is shard 0)
}

// DecideRoundReceived's launch and its undetermined-count read-back (done
// by the caller's rd_wait), then the host state once that has landed
int32_t last_consensus_round(const bh_handle *h);
int rr_launch(bh_handle *h, int64_t *und) {
  bh::launch_round_received(h->d, h->R, h->P, last_consensus_round(h), h->stream);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev[4], h->stream));
  return rd_async(h, h->stream, und, h->d.counters + 3, 8);
}

void rr_done(bh_handle *h, int64_t und) {
  h->nundet = und;
  h->n_rr = h->n_div;
  h->R_rr = h->R;
  h->stage = 3;
}

// only PendingRounds' rounds [P, R): a processed round's witnesses are
// decided for good (or trapped), DecideFame never visits it again
int fame_local(bh_handle *h) {
  if (h->stage < 1) return h->fail(BH_ERR_STATE, "DecideFame before DivideRounds");
  int64_t r0, r1;
  shard_range(std::max(0, h->R - h->P), pass_world(h), pass_rank(h), &r0, &r1);
  if (r1 > r0) bh::launch_fame(h->d, h->R, (int32_t)(h->P + r0), (int32_t)(h->P + r1), h->stream);
  HIPCHK(h, hipGetLastError());
  return BH_OK;
}

int fame_finish(bh_handle *h) {
  if (h->R > h->P) {  // (a Reset hashgraph starts with P = LastConsensusRound, possibly above R)
    if (h->world == 1) bh::launch_fame_scatter_rounds(h->d, h->P, h->R, h->stream);  // (bounds on the device)
    else bh::launch_fame_scatter_range(h->d, h->wofs_h[(size_t)h->P], h->wofs_h[(size_t)h->R], h->stream);
  }
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev[3], h->stream));
  // the decided flags of PendingRounds' rounds [P, R) only (the rest are
  // final) and the error word, behind one synchronisation
  h->decided_h.assign((size_t)h->R, 0);
  int rc;
  if (h->R > h->P && (rc = rd_async(h, h->stream, h->decided_h.data() + h->P, h->d.decided + h->P, (size_t)(h->R - h->P))))
    return rc;
  int32_t err = 0;
  if ((rc = rd_async(h, h->stream, &err, h->d.state + bh::ST_ERR, 4))) return rc;
  // bh_run_consensus on one shard: DecideRoundReceived, which reads nothing
  // the host learns here, is queued behind fame before the synchronisation
  // (one host round trip less; its stage completes below, after fame's)
  const bool with_rr = h->fuse_fame && h->world == 1;
  int64_t und = 0;
  if (with_rr && (rc = rr_launch(h, &und))) return rc;
  if ((rc = rd_wait(h, h->stream))) return rc;
  if (err) return h->fail(BH_ERR_STATE, "inconsistent fame decision (forked DAG?)");
  // updatePendingRounds (hashgraph.go:689-695): set, never cleared
  for (int32_t r = h->P; r < h->R; ++r)
    if (h->decided_h[(size_t)r]) h->pend_dec[(size_t)r] = 1;
  h->stage = 2;
  if (with_rr) rr_done(h, und);
  return BH_OK;
}

int stage_fame(bh_handle *h) {
  int rc;
  if ((rc = run_pass(h, fame_local))) return rc;
  if (pass_world(h) > 1) {
    const int64_t R = h->R - h->P, P = h->P;
    const int npad = h->d.npad;
    struct {
      void *(*sel)(bh_handle *);
      size_t esz;
      bool by_witness;
    } parts[] = {
        {[](bh_handle *x) -> void * { return x->d.wfame; }, 1, true},
        {[](bh_handle *x) -> void * { return x->d.decided; }, 1, false},
        {[](bh_handle *x) -> void * { return x->d.nfam; }, 4, false},
        {[](bh_handle *x) -> void * { return x->d.minla; }, (size_t)npad * 4, false},
    };
    for (auto &pt : parts) {
      const std::vector<int32_t> *ofs = pt.by_witness ? &h->wofs_h : nullptr;
      if ((rc = exchange(h, pt.sel, range_bytes(h, R, pt.esz, false, ofs, P), range_bytes(h, R, pt.esz, true, ofs, P))))
        return rc;
    }
  }
  return run_pass(h, fame_finish);
}

// ---------------------------------------------------------------------------
// stage 3: DecideRoundReceived (every shard, every event)

// Hashgraph.LastConsensusRound (-1 = nil): the last processed round, or the
// Reset block's round until a later one is processed
int32_t last_consensus_round(const bh_handle *h) {
  return h->reset_on ? std::max(h->P - 1, h->reset_lcr) : h->P - 1;
}

// PendingRounds: after a Reset, the entry of LastConsensusRound stays at the
// head of the queue once processed -- ProcessDecidedRounds skips it without
// counting it (hashgraph.go:1063-1065, 1043-1047) -- then rounds [P, R)
int32_t stale_head(const bh_handle *h) { return h->reset_on && h->P > h->reset_lcr ? 1 : 0; }

int stage_rr_local(bh_handle *h) {
  if (h->stage < 2) return h->fail(BH_ERR_STATE, "DecideRoundReceived before DecideFame");
  int64_t und = 0;
  int rc;
  if ((rc = rr_launch(h, &und)) || (rc = rd_wait(h, h->stream))) return rc;
  rr_done(h, und);
  return BH_OK;
}

int stage_rr(bh_handle *h) { return run_pass(h, stage_rr_local); }

// ---------------------------------------------------------------------------
// stage 4: ProcessDecidedRounds -- frames sorted by range, then exchanged

// P after this call: PendingRounds walked in order while their (sticky)
// decided flag is set (hashgraph.go:1041-1122)
int32_t next_prefix(const bh_handle *h) {
  int32_t P1 = h->P;
  while (P1 < h->R && h->pend_dec[(size_t)P1]) ++P1;
  return P1;
}

int order_local(bh_handle *h) {
  if (h->stage < 3) return h->fail(BH_ERR_STATE, "ProcessDecidedRounds before DecideRoundReceived");
  Dev &d = h->d;
  hipStream_t s = h->stream;
  const int32_t P1 = next_prefix(h);
  h->pinned_state[bh::ST_COUNT] = P1;  // pinned staging word (the first ST_COUNT hold the loop's done flag)
  HIPCHK(h, hipMemcpyAsync(d.state + bh::ST_P, h->pinned_state + bh::ST_COUNT, 4, hipMemcpyHostToDevice, s));
  // frames [P, P1): rounds this call processes (earlier frames are final)
  bh::launch_order_buckets(d, h->R, h->P, s);
  int64_t f0, f1;
  shard_range(P1 - h->P, pass_world(h), pass_rank(h), &f0, &f1);
  bh::launch_order_sort(d, (int32_t)(h->P + f0), (int32_t)(h->P + f1), s);
  HIPCHK(h, hipGetLastError());
  if (pass_world(h) > 1) {  // frame offsets: the order exchange's ranges
    h->fofs_h.resize((size_t)P1 + 1);
    int rc;
    if ((rc = rd_async(h, s, h->fofs_h.data(), d.frame_ofs, (size_t)P1 * 4)) ||
        (rc = rd_async(h, s, h->fofs_h.data() + P1, d.state + bh::ST_NCONS, 4)) || (rc = rd_wait(h, s)))
      return rc;
  }
  return BH_OK;
}

int order_finish(bh_handle *h) {
  Dev &d = h->d;
  hipStream_t s = h->stream;
  const int32_t P1 = next_prefix(h);
  if (pass_world(h) > 1)  // frames sorted by other shards arrived
    bh::launch_cons_pos(d, h->fofs_h[(size_t)h->P], h->fofs_h[(size_t)P1], s);
  bh::launch_trap_processed(d, h->P, P1, s);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev[5], s));
  // the state and the frames this call processed, [P0, P1), behind one
  // synchronisation: earlier frames, their blocks and their counts are
  // final, so a call reads back only its own (O(new frames), not O(every
  // frame so far) -- a long-running node's calls stay flat)
  const int32_t P0 = h->P;
  const size_t k = (size_t)std::max(0, P1 - P0);
  int32_t st[bh::ST_COUNT];
  std::vector<int32_t> cnt(k), ofs(k), ld(k);
  std::vector<int64_t> ntx(k);
  int rc;
  // packed on the device first: one copy (k_pack_frames)
  const size_t words = bh::pack_words((int32_t)k);
  if (words > h->pack_cap) {
    if (h->pack_buf) (void)hipFree(h->pack_buf);
    h->pack_buf = nullptr;
    h->pack_cap = 0;
    if ((rc = dalloc(h, &h->pack_buf, words + words / 2))) return rc;
    h->pack_cap = words + words / 2;
  }
  bh::launch_pack_frames(d, P0, (int32_t)k, h->pack_buf, s);
  HIPCHK(h, hipGetLastError());
  std::vector<int32_t> pk(words);
  if ((rc = rd_async(h, s, pk.data(), h->pack_buf, words * 4)) || (rc = rd_wait(h, s))) return rc;
  memcpy(st, pk.data(), sizeof st);
  if (k) {
    memcpy(cnt.data(), pk.data() + bh::ST_COUNT, k * 4);
    memcpy(ofs.data(), pk.data() + bh::ST_COUNT + k, k * 4);
    memcpy(ld.data(), pk.data() + bh::ST_COUNT + 2 * k, k * 4);
    memcpy(ntx.data(), pk.data() + bh::pack_ntx_at((int32_t)k), k * 8);
  }
  const int64_t ncons0 = h->ncons;
  h->P = P1;
  h->ncons = st[bh::ST_NCONS];
  if (k) {
    for (size_t i = 0; i < k; ++i) {
      if (cnt[i] > 0) h->blocks.push_back(Block{P0 + (int32_t)i, ofs[i], cnt[i], ntx[i]});
      h->cons_txs += ntx[i];
      h->cons_loaded += ld[i];
    }
  }
  if (h->frames_on && P1 > P0) {
    const int rc = frames_project(h, P0, P1, ncons0, h->ncons);
    if (rc != BH_OK) return rc;
  }
  h->stage = 4;
  h->tm_stages = true;  // (the stage events are read when asked: settle_timings)
  if (d.diag) {  // diagnostic run only: phase counters to stderr, then reset
    std::vector<unsigned long long> gv(bh::DG_COUNT);
    unsigned long long *g = gv.data();
    if (copy_sync(h->stream, g, d.diag, bh::DG_COUNT * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      if (const char *tp = getenv("BH_TIMELINE")) {  // k_round2 stamps for offline analysis
        if (FILE *f = fopen(tp, "wb")) {
          fwrite(g + bh::DG_TL, 8, bh::DG_COUNT - bh::DG_TL, f);
          fclose(f);
        }
      }
      fprintf(stderr, "[bh diag] sweep: total %llu cyc, wait_desc %llu, wait_ring %llu, substeps %llu, far %llu, chunks %llu | mem: pref %llu store %llu idle %llu\n",
              g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8]);
      fprintf(stderr, "[bh diag] k_flow wave0: steps %llu, cycles %llu (%.1f/step)\n",
              g[16], g[17], g[17] / (double)(g[16] ? g[16] : 1));
      const double nc = (double)(g[14] ? g[14] : 1);
      fprintf(stderr, "[bh diag] k_round: calls %llu, avg total %.0f cyc: loads %.0f, (unused) %.0f, search %.0f\n",
              g[14], g[13] / nc, g[10] / nc, g[11] / nc, g[12] / nc);
      fprintf(stderr, "[bh diag] k_round2: hand-off waves past the 64 rows %llu, windows without SM %llu\n", g[21], g[22]);
    }
    (void)hipMemsetAsync(d.diag, 0, bh::DG_COUNT * 8, h->stream);
  }
  (void)hipGetLastError();  // an unrecorded stage event (empty DAG) must not stay sticky
  return BH_OK;
}

int stage_order(bh_handle *h) {
  int rc;
  if ((rc = run_pass(h, order_local))) return rc;
  if (pass_world(h) > 1) {
    const int32_t P0 = h->P, F = next_prefix(h) - h->P;
    // order: frame f's sorted events at [frame_ofs[f], frame_ofs[f + 1])
    if ((rc = exchange(h, [](bh_handle *x) -> void * { return x->d.order; },
                       range_bytes(h, F, 4, false, &h->fofs_h, P0), range_bytes(h, F, 4, true, &h->fofs_h, P0))))
      return rc;
    if ((rc = exchange(h, [](bh_handle *x) -> void * { return x->d.frame_ntx; }, range_bytes(h, F, 8, false, nullptr, P0),
                       range_bytes(h, F, 8, true, nullptr, P0))))
      return rc;
    if ((rc = exchange(h, [](bh_handle *x) -> void * { return x->d.frame_loaded; },
                       range_bytes(h, F, 4, false, nullptr, P0), range_bytes(h, F, 4, true, nullptr, P0))))
      return rc;
  }
  return run_pass(h, order_finish);
}

}  // namespace

// ===========================================================================
extern "C" {

static int create_one(const bh_config *cfg, int device, bh_handle **out);

void bh_destroy(bh_handle *h);

// How a group shares the coordinates (BH_SHARD_COORDS):
//   split (2) -- the coordinate shards 1 .. G-1 compute LA column ranges and
//     ship them per segment (kernels_split.hip).  n <= 128: all-gathered,
//     every shard runs the round loop, fame rounds and frame sorts split
//     between all shards.  128 < n <= 512 (the wide split): shard 0 alone
//     receives them and runs the loop, fame and order.  The default where
//     the coordinate shards' links carry a step's columns in less than the
//     step (DESIGN.md section 7's table, 2.06 B per column and event): from
//     G = 3 at n <= 128 (C3: 2.7 GB per step, 42 ms over G = 2's one link
//     against a 35-ms step), from G = 4 up to n = 512 (C4: 21 GB);
//   columns (1) -- every shard computes a range of LA columns, all-gathered;
//   replicate (0, the default otherwise) -- every shard computes all of it;
//     fame rounds and frame sorts are split.
static int shard_mode(int n, int world) {
  const char *e = getenv("BH_SHARD_COORDS");
  if (e && !strcmp(e, "columns")) return 1;
  if (e && !strcmp(e, "replicate")) return 0;
  if (e && !strcmp(e, "split")) return 2;
  return (n <= bh::FL_MAXN && world >= 3) || (n <= bh::FW_MAXN && world >= 4) ? 2 : 0;
}

int bh_create(const bh_config *cfg, bh_handle **out) {
  if (!cfg || !out || cfg->n_participants < 1 || cfg->max_events < 0 || !cfg->participant_ids)
    return BH_ERR_INVALID;
  *out = nullptr;
  if (cfg->n_devices <= 1) return create_one(cfg, cfg->n_devices == 1 && cfg->device_ids ? cfg->device_ids[0] : cfg->device, out);
  if (!cfg->device_ids) return BH_ERR_INVALID;
  // in-process shard group: shard 0 is the handle returned, it owns the rest
  const int G = cfg->n_devices;
  std::vector<bh_handle *> g((size_t)G, nullptr);
  for (int r = 0; r < G; ++r) {
    const int rc = create_one(cfg, cfg->device_ids[r], &g[(size_t)r]);
    if (rc != BH_OK) {
      for (bh_handle *x : g) bh_destroy(x);
      return rc;
    }
  }
  const int mode = shard_mode(cfg->n_participants, G);
  for (int r = 0; r < G; ++r) {
    bh_handle *x = g[(size_t)r];
    x->rank = r;
    x->world = G;
    x->shard_cols = mode == 1;
    x->split = mode == 2;
    int64_t c0 = 0, c1 = x->d.n;
    if (x->shard_cols) shard_range(x->d.n, G, r, &c0, &c1);
    x->d.col0 = (int32_t)c0;
    x->d.ncol = (int32_t)(c1 - c0);
    // peer access between the group's devices (xGMI); same-device pairs need none
    (void)hipSetDevice(x->device);
    for (int q = 0; q < G; ++q)
      if (cfg->device_ids[q] != x->device) {
        const hipError_t e = hipDeviceEnablePeerAccess(cfg->device_ids[q], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      }
  }
  g[0]->group = g;
  (void)hipSetDevice(g[0]->device);
  *out = g[0];
  return BH_OK;
}

static int create_one(const bh_config *cfg, int device, bh_handle **out) {
  bh_handle *h = new bh_handle();
  const int n = cfg->n_participants;
  for (int i = 1; i < n; ++i)
    if (cfg->participant_ids[i] <= cfg->participant_ids[i - 1]) {
      delete h;
      return BH_ERR_INVALID;  // peers must be ID-sorted (peers.go:63-73)
    }
  int ndev = 0;
  if (device < 0 || hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device) {
    delete h;
    return BH_ERR_DEVICE;
  }
  if (hipSetDevice(device) != hipSuccess) {
    delete h;
    return BH_ERR_DEVICE;
  }
  h->device = device;
  h->pids.assign(cfg->participant_ids, cfg->participant_ids + n);
  {
    size_t sz = 8;
    while (sz < (size_t)n * 4) sz <<= 1;
    h->slot_key.assign(sz, 0);
    h->slot_val.assign(sz, -1);
    h->slot_mask = sz - 1;
    for (int i = 0; i < n; ++i) {
      uint64_t j = ((uint64_t)h->pids[i] * 0x9E3779B97F4A7C15ull) >> 32 & h->slot_mask;
      while (h->slot_val[j] >= 0) j = (j + 1) & h->slot_mask;
      h->slot_key[j] = h->pids[i];
      h->slot_val[j] = i;
    }
  }
  h->chain.resize(n);
  h->cap = cfg->max_events;
  Dev &d = h->d;
  d.n = n;
  d.npad = (n + 3) & ~3;
  d.sm = 2 * n / 3 + 1;  // hashgraph.go:54
  d.ring_log2 = n < 256 ? 14 : 12;  // sweep LDS: one workgroup per CU below 256 columns
  d.flow_ltclamp = getenv("BH_FLOW_LTCLAMP") ? atoi(getenv("BH_FLOW_LTCLAMP")) : INT32_MAX;
  d.flow_wd = getenv("BH_FLOWW_WATCHDOG") ? atoi(getenv("BH_FLOWW_WATCHDOG")) : (1 << 20);
  d.flow_lt = 1;
  d.round_persist = getenv("BH_ROUND_PERSIST") ? atoi(getenv("BH_ROUND_PERSIST")) != 0 : 1;
  d.round_f32 = getenv("BH_ROUND_F32") ? atoi(getenv("BH_ROUND_F32")) != 0 : 1;
  d.pbar_spin = getenv("BH_PBAR_SPIN") ? std::max(0, atoi(getenv("BH_PBAR_SPIN"))) : (1 << 24);
  // the XCD-hierarchical barrier above 64 workgroups (with per-workgroup
  // release words in both forms: C3 7.6 -> 7.05 us per iteration; C5's 64
  // workgroups 6.9 -> 6.6 and C2's 32 4.2 -> 3.9 keep the one counter,
  // profiles/r4_ab_xcd_barrier.txt); BH_PBAR=xcd|flat overrides
  d.pbar_mode = getenv("BH_PBAR") ? (!strcmp(getenv("BH_PBAR"), "xcd") ? 1 : 0) : (n > 64 ? 1 : 0);
  d.prestage = getenv("BH_PRESTAGE") ? atoi(getenv("BH_PRESTAGE")) != 0 : 1;
  d.xpose_fd = 1;
  // the persistent wide loop's priorities: hand-off / barrier / staging at 2,
  // the CU's two workgroups alternating through the search (C4 42.3 -> 40.6 us
  // per round, profiles/r4_ab_wide.txt); BH_WIDE_PRIO=0|1 for A/B
  d.wide_prio = getenv("BH_WIDE_PRIO") ? atoi(getenv("BH_WIDE_PRIO")) : 2;
  d.win_reuse = getenv("BH_WIN_REUSE") ? atoi(getenv("BH_WIN_REUSE")) : 1;
  d.round_src_rows = getenv("BH_ROUND_SRC") && !strcmp(getenv("BH_ROUND_SRC"), "rows");
  d.N = 0;
  d.col0 = 0;
  d.ncol = n;
  const int64_t C = std::max<int64_t>(h->cap, 1);
  d.R_cap = (int32_t)std::min<int64_t>(C / d.sm + 2, INT32_MAX / 2);
  d.W_cap = C + n;
  const size_t R1 = (size_t)d.R_cap + 1;
  int rc = BH_OK;
  auto A = [&](auto **p, size_t cnt) {
    if (rc == BH_OK) rc = dalloc(h, p, cnt);
  };
  A(&d.creator, C); A(&d.index, C); A(&d.sp, C); A(&d.op, C); A(&d.ntx, C);
  A(&d.coin, C); A(&d.sigw, (size_t)C * 8);
  // chain-major rows: on the chain dataflow paths (n <= 512) each chain's
  // region keeps slack rows (set_chain_tables) so appended events extend it
  // in place and a call can resume where the last one stopped; room for
  // C/8 + 1024 per chain of it (a multiple of 64 rows: LA columns start 16-B
  // aligned for k_floww2's 4-row stores)
  const int64_t L = ((n <= 512 ? C + C / 8 + (int64_t)n * 1024 : C) + 63) & ~(int64_t)63;
  A(&d.chain_start, n); A(&d.chain_len, n); A(&d.chain_ids, (size_t)L); A(&d.epos, C);
  d.la_rows = L;
  A(&d.la, (size_t)(L + 64) * d.npad);
  // the chunked sweep's slabs (la_ev) are dead once permuted into la; the
  // firstDescendants walk output (fdt) reuses the same allocation.  The
  // flow path's column-major LA (la_col) is read while FDT is written
  // (k_flow_transpose walks as it transposes): its own allocation
  A(&d.fdt, (size_t)(L + 128) * d.npad);  // whole 64-row tiles (fdt_pos)
  d.la_ev = d.fdt;
  // the dataflow's column-major LA has its own allocation: the transpose
  // reads it while the firstDescendants walk writes FDT (n <= 512; wider
  // groups take the chunked sweep, whose slabs may share FDT's memory)
  if (n <= 512) A(&d.la_col, (size_t)(L + 64) * d.npad);
  else d.la_col = d.fdt;
  A(&d.opdesc, (size_t)2 * (L + 128));  // k_flow32: int2 entries
  A(&d.lt_row, (size_t)L + 64);
  d.fd_cols = d.npad <= 128;
  d.round_p8 = getenv("BH_ROUND_P8") ? std::clamp(atoi(getenv("BH_ROUND_P8")), 0, bh::P8_XMAX) : bh::P8_XMAX;
  // ballot tables: every round from 0 (bh_reset moves the base up)
  d.rbase = 0;
  d.rspan = (int32_t)R1;
  d.cla_span = (int32_t)std::min<size_t>(R1, std::max<size_t>(64, bh::CLA_BYTES / ((size_t)n * d.npad * 4)));
  if (d.fd_cols) {
    A(&d.ssm, R1 * n * 16);
    A(&d.cla, (size_t)d.cla_span * n * d.npad);
    d.round_lpc = 8;  // k_round2: 8 lanes per candidate at every n <= 128
  } else {
    // chain-major 32-bit FD rows (fd) are allocated on first use (ensure_fd):
    // only the 32-bit wide loop, n > 512 fame and the chunked sweep's
    // queries read them; the 16-bit loop reads the complete FDT
    d.fd = nullptr;
    if (n <= 512) A(&d.ssw, R1 * n * 8);  // k_round_wide's masks for k_fame_masks<16>
    if (n <= 512) A(&d.cla, (size_t)d.cla_span * n * d.npad);  // and its candidates' LA rows (wide_cols)
  }
  A(&d.last_la, (size_t)(n + 1) * d.npad);
  A(&d.rq, (size_t)n);
  A(&d.candfd, (size_t)2 * n * d.npad);
  d.cand16 = !d.fd_cols && n <= 512 ? reinterpret_cast<uint32_t *>(d.candfd) : nullptr;  // (npad + 7) / 8 * 4 <= npad dwords a row
  d.round_ilp2 = getenv("BH_ROUND_ILP2") ? atoi(getenv("BH_ROUND_ILP2")) != 0 : 1;
  d.round_p8g = getenv("BH_ROUND_P8G") ? std::clamp(atoi(getenv("BH_ROUND_P8G")), 0, 64) : bh::P8G_DELTA;
  if (d.cand16) {  // k_round_wide<*, true>
    A(&d.cand8, (size_t)2 * n * ((d.npad + 15) / 16 * 16));
    A(&d.c8tag, (size_t)2 * n);
    A(&d.Bq, (size_t)2 * d.npad);
    if (rc == BH_OK && hipMemset(d.c8tag, 0xFF, (size_t)2 * n * 4) != hipSuccess) rc = BH_ERR_DEVICE;
    if (rc == BH_OK && hipMemset(d.Bq, 0, (size_t)2 * d.npad * 4) != hipSuccess) rc = BH_ERR_DEVICE;
  }
  A(&d.lt, C + 64); A(&d.depth, C); A(&d.chunk_maxd, C / 64 + 1); A(&d.desc, (size_t)C + 64);
  A(&d.B, R1 * n); A(&d.wofs, R1); A(&d.wcnt, R1); A(&d.wids, (size_t)d.W_cap);
  A(&d.wrow, (size_t)d.W_cap);
  A(&d.Bp, (size_t)2 * n); A(&d.state, bh::ST_COUNT); A(&d.pbar, 1024 + 32 * 512);  // (kernels_rounds.hip PBAR_INTS)
  // the persistent loops' input snapshot (run_round_loop): Bp, candfd, the
  // state block, cand8 and its tags, each rounded to 16 B
  A(&d.psnap, (size_t)n + 4 + (size_t)n * d.npad + bh::ST_COUNT + (size_t)n * ((d.npad + 15) / 16 * 4) + n + 4);
  A(&d.round, C); A(&d.witness, C); A(&d.fame, C); A(&d.trapped, C); A(&d.blocked, R1);
  A(&d.wfame, (size_t)d.W_cap); A(&d.frame_loaded, R1);
  A(&d.decided, R1); A(&d.nfam, R1); A(&d.minla, R1 * d.npad); A(&d.rr, C);
  A(&d.frame_cnt, R1); A(&d.frame_ofs, R1); A(&d.frame_cur, R1); A(&d.blk_of_frame, R1);
  A(&d.order, C); A(&d.cons_pos, C); A(&d.frame_ntx, R1); A(&d.counters, 4);
  if (rc == BH_OK) {
    bh::configure_coord_kernels();
    bh::configure_flow_kernels();
    bh::configure_round_kernels();
    bh::configure_fd_kernels();
    bh::configure_fame_kernels();
    bh::configure_order_kernels();
  }
  {  // the round loop's stream gets the higher priority: its kernels sit on
     // the critical path while the coordinate pipeline streams beside it
    int lo_pri = 0, hi_pri = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri);
    if (rc == BH_OK && hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, hi_pri) != hipSuccess)
      rc = BH_ERR_DEVICE;
    if (rc == BH_OK && hipStreamCreateWithPriority(&h->stream2, hipStreamNonBlocking, lo_pri) != hipSuccess)
      rc = BH_ERR_DEVICE;
    hipDeviceProp_t prop;
    if (rc == BH_OK && hipGetDeviceProperties(&prop, device) == hipSuccess) h->ncu = prop.multiProcessorCount;
  }
  if (rc == BH_OK) rc = dalloc(h, &h->seg_zero, (size_t)n);
  if (rc == BH_OK) rc = dalloc(h, &h->segbuf, (size_t)6 * n);  // (three segments' [lo | len], rounds_pipelined)
  if (rc == BH_OK && hipMemset(h->seg_zero, 0, (size_t)n * 4) != hipSuccess) rc = BH_ERR_DEVICE;
  if (rc == BH_OK && hipHostMalloc((void **)&h->seg_stage, (size_t)2 * 64 * n * 4, hipHostMallocDefault) != hipSuccess)
    rc = BH_ERR_DEVICE;
  d.seg_lo = h->seg_zero;
  d.e0 = 0;
  d.rows = 0;
  d.tile_list = nullptr;
  d.ntiles = 0;
  h->tlist_cap = L / 64 + n + 64;
  if (rc == BH_OK) rc = dalloc(h, &h->tlist, (size_t)2 * h->tlist_cap);
  if (rc == BH_OK && hipHostMalloc((void **)&h->tlist_stage, (size_t)2 * h->tlist_cap * 4, hipHostMallocDefault) != hipSuccess)
    rc = BH_ERR_DEVICE;
  if (rc == BH_OK && hipHostMalloc((void **)&h->pinned_state, 2 * bh::ST_COUNT * 4, hipHostMallocMapped) != hipSuccess)
    rc = BH_ERR_DEVICE;
  if (rc == BH_OK && hipHostGetDevicePointer((void **)&d.hdone, h->pinned_state, 0) != hipSuccess)
    rc = BH_ERR_DEVICE;
  for (auto &e : h->ev)
    if (rc == BH_OK && hipEventCreate(&e) != hipSuccess) rc = BH_ERR_DEVICE;
  for (auto &e : h->ev_sweep)
    if (rc == BH_OK && hipEventCreate(&e) != hipSuccess) rc = BH_ERR_DEVICE;
  for (auto &e : h->ev_loop)
    if (rc == BH_OK && hipEventCreate(&e) != hipSuccess) rc = BH_ERR_DEVICE;
  if (rc == BH_OK && hipEventCreateWithFlags(&h->ev_st, hipEventDisableTiming) != hipSuccess) rc = BH_ERR_DEVICE;
  if (rc == BH_OK && hipMemset(d.state, 0, bh::ST_COUNT * 4) != hipSuccess) rc = BH_ERR_DEVICE;
  if (rc == BH_OK && hipMemset(d.counters, 0, 4 * 8) != hipSuccess) rc = BH_ERR_DEVICE;
  if (rc == BH_OK && hipMemset(d.blocked, 0, R1 * 4) != hipSuccess) rc = BH_ERR_DEVICE;
  if (rc == BH_OK && cfg->frames) {
    h->frames_on = true;
    rc = frames_alloc(h);
  }
  if (rc == BH_OK && getenv("BH_DIAG") && atoi(getenv("BH_DIAG"))) {
    rc = dalloc(h, &d.diag, bh::DG_COUNT);
    if (rc == BH_OK && hipMemset(d.diag, 0, bh::DG_COUNT * 8) != hipSuccess) rc = BH_ERR_DEVICE;
  }
  if (rc != BH_OK) {
    free_all(h);
    delete h;
    return rc;
  }
  *out = h;
  return BH_OK;
}

void bh_destroy(bh_handle *h) {
  if (!h) return;
  if (!h->group.empty() && h->group[0] == h)  // an in-process group's owner
    for (size_t r = 1; r < h->group.size(); ++r) {
      bh_handle *x = h->group[r];
      (void)hipSetDevice(x->device);
      free_all(x);
      delete x;
    }
  (void)hipSetDevice(h->device);
  free_all(h);
  delete h;
}

const char *bh_last_error(const bh_handle *h) { return h ? h->err.c_str() : "null handle"; }

static int insert_one(bh_handle *h, const bh_events *ev, int32_t *status, int64_t *n_accepted);
static inline uint64_t others_key(int32_t root, int32_t creator, int32_t index);

int bh_insert_events(bh_handle *h, const bh_events *ev, int32_t *status, int64_t *n_accepted) {
  if (!h || !ev) return BH_ERR_INVALID;
  if (h->group.size() <= 1) return insert_one(h, ev, status, n_accepted);
  // every shard holds the whole DAG: the same batch, validated the same way
  int rc = BH_OK;
  for (size_t r = 0; r < h->group.size(); ++r) {
    bh_handle *x = h->group[r];
    (void)hipSetDevice(x->device);
    const int q = r == 0 ? insert_one(x, ev, status, n_accepted) : insert_one(x, ev, nullptr, nullptr);
    if (r == 0) rc = q;
    else if (q == BH_ERR_DEVICE) rc = h->fail(q, "shard %zu: %s", r, x->err.c_str());
  }
  (void)hipSetDevice(h->device);
  return rc;
}

static int insert_one(bh_handle *h, const bh_events *ev, int32_t *status, int64_t *n_accepted) {
  if (!ev->creator_id || !ev->index || !ev->self_parent_index || !ev->other_parent_creator_id ||
      !ev->other_parent_index || !ev->hash || !ev->sig_r || !ev->n_transactions)
    return h->fail(BH_ERR_INVALID, "null field in bh_events");
  int first = BH_OK;
  int64_t acc = 0;
  {  // geometric growth, sized for the whole batch up front
    const size_t need = h->h_creator.size() + (size_t)std::max<int64_t>(ev->count, 0);
    if (need > h->h_creator.capacity()) {
      const size_t to = std::max(need, 2 * h->h_creator.capacity());
      for (auto *v : {&h->h_creator, &h->h_index, &h->h_sp, &h->h_op, &h->h_ntx}) v->reserve(to);
      h->h_coin.reserve(to);
      h->h_sigw.reserve(to * 8);
    }
  }
  for (int64_t i = 0; i < ev->count; ++i) {
    int code = BH_OK;
    int32_t c = h->slot_find(ev->creator_id[i]), op = -1;
    int32_t oth = -1;    // the Root.Others entry keyed by this event that names its other-parent
    bool ext = false;    // ... and the Store does not hold that other-parent
    if (c < 0) {
      code = BH_ERR_UNKNOWN_PARTICIPANT;
    } else {
      const auto &ch = h->chain[c];
      // chains start after their Root's SelfParent (Index -1 for a base Root)
      const int32_t base = h->reset_on ? h->base_h[(size_t)c] : 0;
      const int32_t last = base + (int32_t)ch.size() - 1;
      // checkSelfParent (hashgraph.go:398-414): self-parent must be the
      // creator's last known event (its Root when it has none)
      if (ev->self_parent_index[i] != last) code = BH_ERR_SELF_PARENT;
      // ParticipantEventsCache continuity (rolling_index.go: SkippedIndex)
      else if (ev->index[i] != last + 1) code = BH_ERR_SKIPPED_INDEX;
      else if (ev->other_parent_index[i] >= 0 || ev->other_parent_creator_id[i] >= 0) {
        // checkOtherParent (hashgraph.go:417-436) via ReadWireInfo's lookup
        const int32_t oslot = h->slot_find(ev->other_parent_creator_id[i]);
        if (oslot < 0) code = BH_ERR_OTHER_PARENT;
        else {
          const auto &oc = h->chain[oslot];
          const int32_t k = ev->other_parent_index[i] - (h->reset_on ? h->base_h[(size_t)oslot] : 0);
          if (k >= 0 && k < (int32_t)oc.size()) op = oc[k];
          if (h->reset_on) {
            // Root.Others[ev.Hex()] (hashgraph.go:229-256, 358-375, 424-431)
            std::string key((const char *)&c, 4);
            key.append((const char *)ev->hash + i * 32, 32);
            const auto it = h->oth_by_key.find(key);
            const int32_t e2 = it == h->oth_by_key.end() ? -1 : it->second;
            if (op >= 0) {  // held by the Store; Others may still name the same event
              if (e2 >= 0 && !memcmp(h->others[(size_t)e2].hash, h->h_hashes.data() + (size_t)op * 32, 32)) oth = e2;
            } else {
              // ReadWireInfo: the creator's Root.Others entry with this
              // (CreatorID, Index) (:1435-1456), then checkOtherParent: the
              // entry keyed by the event's own hash must name the same hash
              const auto i1 = h->oth_by_index.find(others_key(c, oslot, ev->other_parent_index[i]));
              const int32_t e1 = i1 == h->oth_by_index.end() ? -1 : i1->second;
              if (e1 >= 0 && e2 >= 0 && !memcmp(h->others[(size_t)e1].hash, h->others[(size_t)e2].hash, 32)) {
                oth = e2;
                ext = true;
              } else {
                code = BH_ERR_OTHER_PARENT;
              }
            }
          } else if (op < 0) {
            code = BH_ERR_OTHER_PARENT;
          }
        }
      }
      if (code == BH_OK && (int64_t)h->h_creator.size() >= h->cap) code = BH_ERR_CAPACITY;
    }
    if (status) status[i] = code;
    if (code != BH_OK) {
      if (first == BH_OK) {
        first = code;
        const char *msg = code == BH_ERR_SELF_PARENT ? "CheckSelfParent: Self-parent not last known event by creator"
                        : code == BH_ERR_OTHER_PARENT ? "CheckOtherParent: Other-parent not known"
                        : code == BH_ERR_SKIPPED_INDEX ? "SetEvent: ParticipantEvents, Skipped Index"
                        : code == BH_ERR_CAPACITY ? "capacity exceeded"
                        : "ParticipantEvents, Unknown Participant";
        h->fail(code, "event %lld: %s", (long long)i, msg);
      }
      continue;
    }
    const int32_t id = (int32_t)h->h_creator.size();
    auto &ch = h->chain[c];
    h->h_creator.push_back(c);
    h->h_index.push_back((int32_t)ch.size());  // chain position (Index - the chain's base)
    if (h->reset_on) {
      h->h_hashes.insert(h->h_hashes.end(), ev->hash + i * 32, ev->hash + i * 32 + 32);
      h->h_rflag.push_back((int8_t)((oth >= 0 ? 1 : 0) | (ext ? 2 : 0)));
      h->h_ext_lt.push_back(ext ? h->others[(size_t)oth].lt : bh::UNSET);
      h->h_oth.push_back(oth);
      if (ext) h->E0 = id + 1;
    }
    h->h_sp.push_back(ch.empty() ? -1 : ch.back());
    h->h_op.push_back(op);
    h->h_ntx.push_back(ev->n_transactions[i]);
    h->h_coin.push_back(ev->hash[i * 32 + 16] != 0 ? 1 : 0);
    if (h->frames_on) h->h_hash.insert(h->h_hash.end(), ev->hash + i * 32, ev->hash + i * 32 + 32);
    const uint8_t *rb = ev->sig_r + i * 32;
    uint32_t w[8];  // big-endian words of r
    memcpy(w, rb, 32);
    for (int q = 0; q < 8; ++q) h->h_sigw.push_back(__builtin_bswap32(w[q]));
    ch.push_back(id);
    if (ev->index[i] == 0 || ev->n_transactions[i] > 0) h->loaded_total++;
    ++acc;
  }
  if (n_accepted) *n_accepted = acc;
  if (acc) {  // InsertEvent touches no pass's results (hashgraph.go:714-761)
    (void)hipSetDevice(h->device);
    int rc = upload(h);
    if (rc) return rc;
  }
  return first;
}

int bh_divide_rounds(bh_handle *h) {
  if (!h) return BH_ERR_INVALID;
  (void)hipSetDevice(h->device);
  return stage_rounds(h);
}
int bh_decide_fame(bh_handle *h) {
  if (!h) return BH_ERR_INVALID;
  (void)hipSetDevice(h->device);
  return stage_fame(h);
}
int bh_decide_round_received(bh_handle *h) {
  if (!h) return BH_ERR_INVALID;
  (void)hipSetDevice(h->device);
  return stage_rr(h);
}
int bh_process_decided_rounds(bh_handle *h) {
  if (!h) return BH_ERR_INVALID;
  (void)hipSetDevice(h->device);
  return stage_order(h);
}
int bh_run_consensus(bh_handle *h) {
  int rc;
  if (!h) return BH_ERR_INVALID;
  (void)hipSetDevice(h->device);
  // fuse_fame: DecideFame follows DivideRounds at once (rounds_tail reads no
  // witness offsets back) and, on one shard, DecideRoundReceived rides on
  // DecideFame's synchronisation (fame_finish)
  h->fuse_fame = true;
  rc = stage_rounds(h);
  if (!rc) rc = stage_fame(h);
  h->fuse_fame = false;
  if (rc) return rc;
  if (h->stage < 3 && (rc = stage_rr(h))) return rc;
  return stage_order(h);
}
int bh_synchronize(bh_handle *h) {
  if (!h) return BH_ERR_INVALID;
  for (bh_handle *x : local_shards(h)) {
    HIPCHK(h, hipSetDevice(x->device));
    HIPCHK(h, wait_stream(x->stream));
  }
  HIPCHK(h, hipSetDevice(h->device));
  return BH_OK;
}

int bh_reset_consensus(bh_handle *h) {
  if (!h) return BH_ERR_INVALID;
  for (bh_handle *x : local_shards(h)) {
    HIPCHK(h, hipSetDevice(x->device));
    HIPCHK(h, wait_stream(x->stream));
    // (on the handle's stream, ahead of the next pass: no blocking
    // legacy-stream memset between two bench steps)
    HIPCHK(h, hipMemsetAsync(x->d.blocked, 0, ((size_t)x->d.R_cap + 1) * 4, x->stream));
    x->stage = 0;
    x->coords_for = -1;
    x->n_div = x->n_rr = 0;
    x->R = x->R_rr = 0;
    x->P = x->reset_on ? x->reset_lcr : 0;
    x->pend_dec.clear();
    x->decided_h.clear();
    x->nundet = 0;
    x->ncons = x->cons_txs = x->cons_loaded = 0;
    x->blocks.clear();
    x->inc_valid = false;
    x->n_coord = 0;
    if (x->frames_on) frames_reset(x);
  }
  HIPCHK(h, hipSetDevice(h->device));
  return BH_OK;
}

// The per-round tables for R_cap rounds (a Reset hashgraph starts at the
// frame's round, so its tables must reach past it), allocated into `t`'s
// fields (contents zeroed); the ballot tables hold only rounds [rbase,
// R_cap].  On failure everything allocated here is freed and `t` keeps no
// pointer of it.
struct RoundTables {
  unsigned long long *ssm = nullptr, *ssw = nullptr;
  int32_t *cla = nullptr;
  int32_t cla_span = 0;
  int32_t *B = nullptr, *wofs = nullptr, *wcnt = nullptr, *blocked = nullptr, *frame_loaded = nullptr, *nfam = nullptr,
          *minla = nullptr, *frame_cnt = nullptr, *frame_ofs = nullptr, *frame_cur = nullptr, *blk_of_frame = nullptr;
  int8_t *decided = nullptr, *rexists = nullptr;
  int64_t *frame_ntx = nullptr;
  void *all(int i) {
    void *p[] = {ssm, ssw, B, wofs, wcnt, blocked, frame_loaded, nfam, minla, frame_cnt, frame_ofs, frame_cur,
                 blk_of_frame, decided, rexists, frame_ntx};
    return i < 16 ? p[i] : nullptr;
  }
  void free_all() {
    for (int i = 0; i < 16; ++i)
      if (void *p = all(i)) (void)hipFree(p);
    if (cla) (void)hipFree(cla);
    *this = RoundTables{};
  }
};

static int alloc_round_tables(bh_handle *h, RoundTables &t, int32_t R_cap, int32_t rbase, bool ssm, bool ssw) {
  const size_t R1 = (size_t)R_cap + 1, span = R1 - (size_t)rbase;
  const int n = h->d.n;
  int rc = BH_OK;
  auto A = [&](auto **p, size_t cnt) {
    if (rc == BH_OK) rc = dalloc(h, p, cnt);
    if (rc == BH_OK && hipMemset(*p, 0, std::max<size_t>(cnt, 1) * sizeof(**p)) != hipSuccess) rc = BH_ERR_DEVICE;
  };
  if (ssm) A(&t.ssm, span * n * 16);
  if (ssm || ssw) {
    t.cla_span = (int32_t)std::min<size_t>(span, std::max<size_t>(64, bh::CLA_BYTES / ((size_t)n * h->d.npad * 4)));
    A(&t.cla, (size_t)t.cla_span * n * h->d.npad);
  }
  if (ssw) A(&t.ssw, span * n * 8);
  A(&t.B, R1 * n); A(&t.wofs, R1); A(&t.wcnt, R1); A(&t.blocked, R1); A(&t.frame_loaded, R1);
  A(&t.decided, R1); A(&t.nfam, R1); A(&t.minla, R1 * h->d.npad); A(&t.frame_cnt, R1);
  A(&t.frame_ofs, R1); A(&t.frame_cur, R1); A(&t.blk_of_frame, R1); A(&t.frame_ntx, R1);
  A(&t.rexists, R1);
  if (rc != BH_OK) {
    t.free_all();
    return h->fail(rc, "round tables for %d rounds: %s", R_cap, h->err.c_str());
  }
  return BH_OK;
}

// the handle's round tables become t's (the old ones are freed)
static void commit_round_tables(bh_handle *h, RoundTables &t, int32_t R_cap, int32_t rbase) {
  Dev &d = h->d;
  void *old[] = {d.ssm, d.ssw, d.B, d.wofs, d.wcnt, d.blocked, d.frame_loaded, d.nfam, d.minla, d.frame_cnt,
                 d.frame_ofs, d.frame_cur, d.blk_of_frame, d.decided, d.rexists, d.frame_ntx, d.cla};
  for (void *p : old)
    if (p) (void)hipFree(p);
  d.ssm = t.ssm; d.ssw = t.ssw; d.cla = t.cla; d.cla_span = t.cla_span; d.B = t.B; d.wofs = t.wofs; d.wcnt = t.wcnt; d.blocked = t.blocked;
  d.frame_loaded = t.frame_loaded; d.nfam = t.nfam; d.minla = t.minla; d.frame_cnt = t.frame_cnt;
  d.frame_ofs = t.frame_ofs; d.frame_cur = t.frame_cur; d.blk_of_frame = t.blk_of_frame; d.decided = t.decided;
  d.rexists = t.rexists; d.frame_ntx = t.frame_ntx;
  d.R_cap = R_cap;
  d.rbase = rbase;
  d.rspan = R_cap + 1 - rbase;
  t = RoundTables{};
}

// Root.Others lookup by (root slot, creator slot, Index): ReadWireInfo's
// search for an other-parent the Store does not hold (hashgraph.go:1435-1456)
static inline uint64_t others_key(int32_t root, int32_t creator, int32_t index) {
  return ((uint64_t)(uint32_t)root << 48) ^ ((uint64_t)(uint32_t)creator << 32) ^ (uint64_t)(uint32_t)index;
}

int bh_reset(bh_handle *h, const bh_roots *rt) {
  if (!h || !rt || !rt->next_round || !rt->self_parent_index || !rt->self_parent_lamport || !rt->self_parent_round ||
      rt->n_others < 0 || (rt->n_others > 0 && (!rt->other_root || !rt->other_key || !rt->other_creator_id ||
                                                 !rt->other_index || !rt->other_lamport || !rt->other_round ||
                                                 !rt->other_hash)))
    return BH_ERR_INVALID;
  if (!h->h_creator.empty() || h->reset_on || h->stage != 0)
    return h->fail(BH_ERR_STATE, "bh_reset: a fresh handle only (no events inserted, no pass run)");
  if (!h->group.empty() || h->world > 1) return h->fail(BH_ERR_STATE, "bh_reset: one shard");
  if (h->frames_on && !rt->self_parent_hash)
    return h->fail(BH_ERR_INVALID, "bh_reset: the block projection needs each Root's SelfParent hash");
  if (rt->round_received < 0 || rt->block_index < -1) return h->fail(BH_ERR_INVALID, "bh_reset: bad block");
  (void)hipSetDevice(h->device);
  struct FailHook {  // the test hook covers this call only
    bh_handle *h;
    explicit FailHook(bh_handle *x) : h(x) {
      const char *e = getenv("BH_TEST_FAIL_ALLOC");
      h->fail_alloc_in = e && atoi(e) > 0 ? atoi(e) - 1 : -1;
    }
    ~FailHook() { h->fail_alloc_in = -1; }
  } hook(h);
  Dev &d = h->d;
  const int n = d.n;
  int32_t F = -1, lo = INT32_MAX;
  for (int c = 0; c < n; ++c) {
    if (rt->self_parent_index[c] < -1 || rt->next_round[c] < 0)
      return h->fail(BH_ERR_INVALID, "bh_reset: root %d: bad SelfParent index / NextRound", c);
    F = std::max(F, std::max(rt->next_round[c], rt->self_parent_round[c]));
    lo = std::min(lo, std::min(rt->next_round[c], rt->self_parent_round[c]));
  }
  // rounds >= F + 1 follow the closed form; every
  // pending round must be among them, as GetFrame's roots guarantee
  if (F >= rt->round_received)
    return h->fail(BH_ERR_INVALID, "bh_reset: a root's round %d is not below the block's round %d", F,
                   rt->round_received);
  std::vector<bh_handle::Other> others;
  std::unordered_map<std::string, int32_t> by_key;
  std::unordered_map<uint64_t, int32_t> by_index;
  for (int32_t k = 0; k < rt->n_others; ++k) {
    bh_handle::Other o{};
    o.root = rt->other_root[k];
    o.creator = h->slot_find(rt->other_creator_id[k]);
    if (o.root < 0 || o.root >= n || o.creator < 0)
      return h->fail(BH_ERR_INVALID, "bh_reset: Others entry %d: bad root / creator", k);
    o.index = rt->other_index[k];
    o.lt = rt->other_lamport[k];
    o.round = rt->other_round[k];
    memcpy(o.key, rt->other_key + (size_t)k * 32, 32);
    memcpy(o.hash, rt->other_hash + (size_t)k * 32, 32);
    std::string key((const char *)&o.root, 4);
    key.append((const char *)o.key, 32);
    by_key.emplace(key, (int32_t)others.size());  // a Go map holds one entry per key
    by_index.emplace(others_key(o.root, o.creator, o.index), (int32_t)others.size());  // the first match, as the scan
    others.push_back(o);
  }
  const int64_t C = std::max<int64_t>(h->cap, 1);
  const int64_t need = (int64_t)rt->round_received + C / d.sm + 2;
  if (need > INT32_MAX / 2) return h->fail(BH_ERR_CAPACITY, "bh_reset: round %d too large", rt->round_received);
  const int32_t r0 = F + 1, rlo = std::max(0, lo);
  const int32_t R_cap = (int32_t)std::max<int64_t>(d.R_cap, need);
  // every allocation first; the handle changes only once all of them succeeded
  RoundTables t;
  int rc;
  if ((rc = alloc_round_tables(h, t, R_cap, r0, d.ssm != nullptr, d.ssw != nullptr))) return rc;
  // the block projection's tables for the new round range, with the
  // installed Roots (each Root's entries: unique keys sorted by key hash,
  // Go's encoding/json map order; a Go map holds one entry per key)
  bh::Frames nf{};
  size_t json_cap = 0, bjson_cap = 0;
  if (h->frames_on) {
    const int32_t K = rt->n_others;
    std::vector<int32_t> ord((size_t)K), ofs((size_t)n + 1, 0);
    for (int32_t k = 0; k < K; ++k) ord[(size_t)k] = k;
    std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) {
      if (others[(size_t)a].root != others[(size_t)b].root) return others[(size_t)a].root < others[(size_t)b].root;
      return memcmp(others[(size_t)a].key, others[(size_t)b].key, 32) < 0;
    });
    ord.erase(std::unique(ord.begin(), ord.end(),
                          [&](int32_t a, int32_t b) {
                            return others[(size_t)a].root == others[(size_t)b].root &&
                                   !memcmp(others[(size_t)a].key, others[(size_t)b].key, 32);
                          }),
              ord.end());
    for (int32_t k : ord) ofs[(size_t)others[(size_t)k].root + 1]++;
    for (int c = 0; c < n; ++c) ofs[(size_t)c + 1] += ofs[(size_t)c];
    std::vector<uint8_t> kb((size_t)K * 32 + 1), hb((size_t)K * 32 + 1);
    std::vector<int32_t> cr((size_t)K + 1), ix((size_t)K + 1), lt((size_t)K + 1), rd((size_t)K + 1);
    for (int32_t k = 0; k < K; ++k) {
      const auto &o = others[(size_t)k];
      memcpy(&kb[(size_t)k * 32], o.key, 32);
      memcpy(&hb[(size_t)k * 32], o.hash, 32);
      cr[(size_t)k] = o.creator;
      ix[(size_t)k] = o.index;
      lt[(size_t)k] = o.lt;
      rd[(size_t)k] = o.round;
    }
    int rcf = frames_alloc_tables(h, nf, (int64_t)R_cap + 1, K, true);
    auto up = [&](void *dst, const void *src, size_t bytes) {
      if (rcf == BH_OK && bytes && hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess) rcf = BH_ERR_DEVICE;
    };
    up(nf.rsp_hash, rt->self_parent_hash, (size_t)n * 32);
    up(nf.ro_key, kb.data(), (size_t)K * 32);
    up(nf.ro_hash, hb.data(), (size_t)K * 32);
    up(nf.ro_creator, cr.data(), (size_t)K * 4);
    up(nf.ro_index, ix.data(), (size_t)K * 4);
    up(nf.ro_lt, lt.data(), (size_t)K * 4);
    up(nf.ro_round, rd.data(), (size_t)K * 4);
    up(nf.ro_ofs, ofs.data(), ((size_t)n + 1) * 4);
    up(nf.ro_list, ord.data(), ord.size() * 4);
    // the initial contents and the JSON buffers too: nothing of the
    // projection can fail after the commit below
    if (rcf == BH_OK) rcf = frames_prepare(h, nf, (int64_t)R_cap + 1, &json_cap, &bjson_cap);
    if (rcf != BH_OK) {
      frames_free_tables(nf);
      t.free_all();
      return h->fail(rcf, "bh_reset: block projection tables");
    }
  }
  int32_t *cb = nullptr, *ls = nullptr, *rn = nullptr, *rs = nullptr, *elt = nullptr, *fw = nullptr;
  int8_t *rf = nullptr;
  std::vector<int32_t> base_h((size_t)n);
  for (int c = 0; c < n; ++c) base_h[(size_t)c] = rt->self_parent_index[c] + 1;
  auto up = [&](int32_t **p, const int32_t *v) -> int {
    if (dalloc(h, p, (size_t)n)) return BH_ERR_DEVICE;
    HIPCHK(h, hipMemcpy(*p, v, (size_t)n * 4, hipMemcpyHostToDevice));
    return BH_OK;
  };
  if ((rc = up(&cb, base_h.data())) || (rc = up(&ls, rt->self_parent_lamport)) || (rc = up(&rn, rt->next_round)) ||
      (rc = up(&rs, rt->self_parent_round)) || (rc = dalloc(h, &rf, (size_t)C)) || (rc = dalloc(h, &elt, (size_t)C)) ||
      (rc = dalloc(h, &fw, (size_t)(r0 - rlo) * n))) {
    for (void *p : {(void *)cb, (void *)ls, (void *)rn, (void *)rs, (void *)rf, (void *)elt, (void *)fw})
      if (p) (void)hipFree(p);
    t.free_all();
    frames_free_tables(nf);
    return rc;
  }
  // commit
  commit_round_tables(h, t, R_cap, r0);
  if (h->frames_on) {
    frames_free_tables(h->fr);
    h->fr = nf;
    h->json_cap = json_cap;
    h->bjson_cap = bjson_cap;
    h->arena_cap = h->arena_len = 0;
    h->others_total = 0;
  }
  for (void *p : {(void *)d.chain_base, (void *)d.lt_seed, (void *)d.root_next, (void *)d.root_sp_round, (void *)d.rflag,
                  (void *)d.ext_lt, (void *)d.fw})
    if (p) (void)hipFree(p);
  d.chain_base = cb; d.lt_seed = ls; d.root_next = rn; d.root_sp_round = rs; d.rflag = rf; d.ext_lt = elt; d.fw = fw;
  d.r0 = r0;
  d.rlo = rlo;
  d.frame_lo = rt->round_received + 1;  // round_received's frame is the block itself (hashgraph.go:1063-1065)
  d.blk_base = (int32_t)(rt->block_index + 1);  // NewBlockFromFrame(LastBlockIndex()+1, ...) (hashgraph.go:1096-1097)
  h->base_h = std::move(base_h);
  h->next_h.assign(rt->next_round, rt->next_round + n);
  h->sp_round_h.assign(rt->self_parent_round, rt->self_parent_round + n);
  h->sp_lt_h.assign(rt->self_parent_lamport, rt->self_parent_lamport + n);
  h->others = std::move(others);
  h->oth_by_key = std::move(by_key);
  h->oth_by_index = std::move(by_index);
  h->reset_on = true;
  h->reset_lcr = rt->round_received;
  h->reset_block = rt->block_index;
  h->reset_F = F;
  h->P = rt->round_received;  // rounds below LastConsensusRound are never queued (hashgraph.go:809-815)
  h->inc_valid = false;
  return BH_OK;
}

int bh_comm_unique_id(uint8_t *id) {
  if (!id) return BH_ERR_INVALID;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return BH_ERR_DEVICE;
  memcpy(id, u.internal, sizeof u.internal);
  return BH_OK;
}

// a process's shard of a multi-process group: its transport, rank and role
static int comm_join(bh_handle *h, int32_t rank, int32_t world, bh::Comm *x) {
  h->xport = x;
  h->rank = rank;
  h->world = world;
  const int mode = world > 1 ? shard_mode(h->d.n, world) : 0;  // see bh_create
  h->shard_cols = mode == 1;
  h->split = mode == 2;
  int64_t c0 = 0, c1 = h->d.n;
  if (h->shard_cols) shard_range(h->d.n, world, rank, &c0, &c1);
  h->d.col0 = (int32_t)c0;
  h->d.ncol = (int32_t)(c1 - c0);
  return BH_OK;
}

int bh_comm_init(bh_handle *h, int32_t rank, int32_t world, const uint8_t *id) {
  if (!h || !id || world < 1 || rank < 0 || rank >= world || !h->group.empty() || h->xport)
    return BH_ERR_INVALID;
  if (h->n_div || !h->h_creator.empty()) return h->fail(BH_ERR_STATE, "bh_comm_init after events were inserted");
  (void)hipSetDevice(h->device);
  bh::Comm *x = nullptr;
  if (world > 1 && !(x = bh::make_rccl_comm(h, rank, world, id))) return BH_ERR_DEVICE;
  return comm_join(h, rank, world, x);
}

int bh_comm_init_transport(bh_handle *h, int32_t rank, int32_t world, const bh_transport *t) {
  if (!h || !t || !t->send || !t->recv || !t->broadcast || world < 1 || rank < 0 || rank >= world ||
      !h->group.empty() || h->xport)
    return BH_ERR_INVALID;
  if (h->n_div || !h->h_creator.empty())
    return h->fail(BH_ERR_STATE, "bh_comm_init_transport after events were inserted");
  return comm_join(h, rank, world, world > 1 ? bh::make_host_comm(*t, rank) : nullptr);
}

void bh_shard_range(int64_t items, int32_t world, int32_t rank, int64_t *lo, int64_t *hi) {
  int64_t a = 0, b = 0;
  if (world >= 1 && rank >= 0 && rank < world && items >= 0) shard_range(items, world, rank, &a, &b);
  if (lo) *lo = a;
  if (hi) *hi = b;
}

int bh_get_stats(bh_handle *h, bh_stats *o) {
  if (!h || !o) return BH_ERR_INVALID;
  if (h->no_results()) return h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  memset(o, 0, sizeof *o);
  o->n_events = (int64_t)h->h_creator.size();
  o->last_round = h->R - 1;
  o->last_consensus_round = last_consensus_round(h);
  o->consensus_events = h->ncons;
  o->consensus_transactions = h->cons_txs;
  o->pending_loaded_events = h->loaded_total - h->cons_loaded;
  // received by the last DecideRoundReceived, plus everything inserted since
  o->undetermined_events = h->nundet + (o->n_events - h->n_rr);
  o->blocks = (int64_t)h->blocks.size() + (h->reset_on ? h->reset_block + 1 : 0);
  o->pending_rounds = std::max(0, h->R - h->P) + stale_head(h);
  o->first_block = h->reset_on ? h->reset_block + 1 : 0;
  return BH_OK;
}

int bh_get_event_meta(bh_handle *h, int64_t first, int64_t count, int32_t *round, int8_t *witness,
                      int32_t *lamport, int32_t *round_received, int8_t *fame, int64_t *consensus_pos) {
  if (!h || first < 0 || count < 0 || first + count > (int64_t)h->h_creator.size()) return BH_ERR_INVALID;
  if (h->no_results()) return h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  if (count == 0) return BH_OK;
  (void)hipSetDevice(h->device);
  HIPCHK(h, wait_stream(h->stream));
  const Dev &d = h->d;
  // events [first, first + k) were divided; the rest are not (Go: nil fields)
  const int64_t k = std::max<int64_t>(0, std::min<int64_t>(count, h->n_div - first));
  const size_t rest = (size_t)(count - k);
  auto get = [&](void *dst, const void *src, size_t esz) -> hipError_t {
    return k > 0 ? hipMemcpy(dst, (const char *)src + (size_t)first * esz, (size_t)k * esz, hipMemcpyDeviceToHost)
                 : hipSuccess;
  };
  if (round) { HIPCHK(h, get(round, d.round, 4)); std::fill(round + k, round + k + rest, INT32_MIN); }
  if (lamport) { HIPCHK(h, get(lamport, d.lt, 4)); std::fill(lamport + k, lamport + k + rest, INT32_MIN); }
  if (witness) { HIPCHK(h, get(witness, d.witness, 1)); std::fill(witness + k, witness + k + rest, 0); }
  if (fame) { HIPCHK(h, get(fame, d.fame, 1)); std::fill(fame + k, fame + k + rest, -1); }
  if (round_received) {
    HIPCHK(h, get(round_received, d.rr, 4));
    for (int64_t i = 0; i < k; ++i)  // left UndeterminedEvents without one (Reset): nil
      if (round_received[i] == bh::RR_DROP) round_received[i] = INT32_MIN;
    std::fill(round_received + k, round_received + k + rest, INT32_MIN);
  }
  if (consensus_pos) {
    HIPCHK(h, get(consensus_pos, d.cons_pos, 8));
    std::fill(consensus_pos + k, consensus_pos + k + rest, -1);
  }
  return BH_OK;
}

int bh_get_consensus_order(bh_handle *h, int64_t first, int64_t count, int32_t *ids) {
  if (!h || !ids || first < 0 || count < 0) return BH_ERR_INVALID;
  if (h->no_results()) return h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  if (first + count > h->ncons) return h->fail(BH_ERR_INVALID, "range beyond consensus");
  (void)hipSetDevice(h->device);
  HIPCHK(h, wait_stream(h->stream));
  if (count) HIPCHK(h, hipMemcpy(ids, h->d.order + first, (size_t)count * 4, hipMemcpyDeviceToHost));
  return BH_OK;
}

int bh_get_blocks(bh_handle *h, int64_t first, int64_t count, int32_t *round_received,
                  int64_t *first_event, int64_t *n_events, int64_t *n_transactions) {
  if (!h || first < 0 || count < 0 || first + count > (int64_t)h->blocks.size()) return BH_ERR_INVALID;
  if (h->no_results()) return h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  for (int64_t i = 0; i < count; ++i) {
    const Block &b = h->blocks[(size_t)(first + i)];
    if (round_received) round_received[i] = b.rr;
    if (first_event) first_event[i] = b.first;
    if (n_events) n_events[i] = b.count;
    if (n_transactions) n_transactions[i] = b.ntx;
  }
  return BH_OK;
}

int32_t bh_get_pending_rounds(bh_handle *h, int32_t *index, int8_t *decided, int32_t cap) {
  if (!h) return 0;
  if (h->no_results()) return -h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  const int32_t head = stale_head(h), cnt = std::max(0, h->R - h->P) + head;
  for (int32_t i = 0; i < cnt && i < cap; ++i) {
    if (index) index[i] = h->P - head + i;
    if (decided) decided[i] = i < head ? 1 : h->pend_dec[(size_t)(h->P - head + i)];
  }
  return cnt;
}

int64_t bh_get_undetermined(bh_handle *h, int32_t *ids, int64_t cap) {
  if (!h) return 0;
  if (h->no_results()) return -h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  const int64_t N = (int64_t)h->h_creator.size();
  const int64_t total = h->nundet + (N - h->n_rr);
  if (!ids || cap <= 0) return total;
  std::vector<int32_t> rr((size_t)h->n_rr);
  (void)hipSetDevice(h->device);
  if (wait_stream(h->stream) != hipSuccess) return -1;
  if (h->n_rr && hipMemcpy(rr.data(), h->d.rr, (size_t)h->n_rr * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  int64_t k = 0;
  for (int64_t i = 0; i < h->n_rr && k < cap; ++i)
    if (rr[(size_t)i] == INT32_MIN) ids[k++] = (int32_t)i;
  for (int64_t i = h->n_rr; i < N && k < cap; ++i) ids[k++] = (int32_t)i;
  return total;
}

int bh_get_round_info(bh_handle *h, int32_t r, bh_round_info *info, int32_t *witness_ids, int8_t *fame,
                      int32_t cap) {
  if (!h || !info) return BH_ERR_INVALID;
  if (h->no_results()) return h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  if (r < 0 || r >= h->R) return h->fail(BH_ERR_KEY_NOT_FOUND, "GetRound %d: Not Found", r);
  (void)hipSetDevice(h->device);
  HIPCHK(h, wait_stream(h->stream));
  const Dev &d = h->d;
  const int n = d.n;
  memset(info, 0, sizeof *info);
  info->round = r;
  if (r < d.r0) {  // below a Reset's closed form: k_fiat's rounds, which may be missing
    int8_t ex = 0;
    HIPCHK(h, hipMemcpy(&ex, d.rexists + r, 1, hipMemcpyDeviceToHost));
    if (!ex) return h->fail(BH_ERR_KEY_NOT_FOUND, "GetRound %d: Not Found", r);
    std::vector<int32_t> rd((size_t)h->n_div);
    if (h->n_div) HIPCHK(h, hipMemcpy(rd.data(), d.round, (size_t)h->n_div * 4, hipMemcpyDeviceToHost));
    info->n_events = (int32_t)std::count(rd.begin(), rd.end(), r);
  } else {
    // round r on chain c = indexes [B[r][c], B[r+1][c]) (B[R][c] = chain length)
    std::vector<int32_t> b((size_t)2 * n), len((size_t)n);
    HIPCHK(h, hipMemcpy(b.data(), d.B + (int64_t)r * n, (size_t)2 * n * 4, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemcpy(len.data(), d.chain_len, (size_t)n * 4, hipMemcpyDeviceToHost));
    int64_t ne = 0;
    for (int c = 0; c < n; ++c) ne += std::min(b[(size_t)(n + c)], len[(size_t)c]) - std::min(b[(size_t)c], len[(size_t)c]);
    info->n_events = (int32_t)ne;
  }
  int32_t wofs = 0, wcnt = 0;
  HIPCHK(h, hipMemcpy(&wofs, d.wofs + r, 4, hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemcpy(&wcnt, d.wcnt + r, 4, hipMemcpyDeviceToHost));
  std::vector<int32_t> w((size_t)wcnt);
  std::vector<int8_t> f((size_t)wcnt);
  if (wcnt) HIPCHK(h, hipMemcpy(w.data(), d.wids + wofs, (size_t)wcnt * 4, hipMemcpyDeviceToHost));
  bool all = true;
  for (int32_t i = 0; i < wcnt; ++i) {
    HIPCHK(h, hipMemcpy(&f[(size_t)i], d.fame + w[(size_t)i], 1, hipMemcpyDeviceToHost));
    all = all && f[(size_t)i] != 0;
    if (i < cap) {
      if (witness_ids) witness_ids[i] = w[(size_t)i];
      if (fame) fame[i] = f[(size_t)i];
    }
  }
  info->n_witnesses = wcnt;
  info->witnesses_decided = all ? 1 : 0;
  if (r < h->R_rr && r >= d.frame_lo) {
    HIPCHK(h, hipMemcpy(&info->n_consensus, d.frame_cnt + r, 4, hipMemcpyDeviceToHost));
  } else if (r < h->R_rr && h->n_rr) {  // a frame never emitted (Reset): count the events received in r
    std::vector<int32_t> rr((size_t)h->n_rr);
    HIPCHK(h, hipMemcpy(rr.data(), d.rr, (size_t)h->n_rr * 4, hipMemcpyDeviceToHost));
    info->n_consensus = (int32_t)std::count(rr.begin(), rr.end(), r);
  }
  // every round >= LastConsensusRound is queued when it first appears; after
  // a Reset the rounds below the block's are never queued
  info->queued = !h->reset_on || r >= h->reset_lcr ? 1 : 0;
  const bool head = stale_head(h) && r == h->P - 1;
  info->pending = r >= h->P || head ? 1 : 0;
  info->pending_decided = r >= h->P ? h->pend_dec[(size_t)r] : head ? 1 : 0;
  return BH_OK;
}

// the coordinates of every inserted event on the device (they are produced
// lazily by the first pass; a query between an insert and the next
// DivideRounds computes them here).  Go's ancestor / see / stronglySee read
// the Store and change no pass state, so neither does this: the stage and
// the round loop's resume point stay, and on the chain dataflow paths (FDT
// complete, the same values the next segment would write) the next
// DivideRounds still resumes incrementally.
static int ensure_coords(bh_handle *h) {
  Dev &d = h->d;
  const int64_t N = (int64_t)h->h_creator.size();
  if (h->coords_for == N && h->rows_stale) {
    int rc;
    if ((rc = build_rows(h, h->lens_coord, h->stream))) return rc;
  }
  if (h->coords_for != N) {
    int rc;
    hipStream_t s = h->stream;
    if ((rc = upload(h))) return rc;
    d.N = N;
    d.e0 = 0;
    d.seg_lo = h->seg_zero;
    if ((rc = set_chain_tables(h))) return rc;
    d.rows = h->layout_rows;
    // the chain table only (launch_prep would also reset the loop state)
    if (d.rows > 0) HIPCHK(h, hipMemsetAsync(d.chain_ids, 0xFF, (size_t)d.rows * 4, s));
    bh::launch_chain_scatter(d, 0, s);
    HIPCHK(h, hipMemsetAsync(d.state + bh::ST_FLOWOVF, 0, 4, s));
    const bool walked = use_flow(d);
    bool wide = !walked && bh::floww_eligible(d) && !h->reset_on;
    bool keep = walked && !h->layout_changed && !h->reset_on;
    if (h->reset_on) {
      if ((rc = reset_coords(h, s))) return rc;
      d.fd_rows = !bh::round_p16(d);
    } else if (walked) {
      d.fd_rows = 1;
    } else if (wide) {
      d.fd_rows = !bh::round_p16(d);
      Dev full = d;
      full.col0 = 0;
      full.ncol = d.n;
      bh::launch_floww(full, s);
      int32_t ovf = 0;
      HIPCHK(h, hipMemcpyAsync(&ovf, d.state + bh::ST_FLOWOVF, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(h, wait_stream(s));
      if (ovf) {  // the watchdog or the LT clamp: the chunked sweep below
        HIPCHK(h, hipMemsetAsync(d.state + bh::ST_FLOWOVF, 0, 4, s));
        wide = false;
      } else {
        keep = !h->layout_changed && bh::round_p16(d);
      }
    }
    if (!walked && !wide && !h->reset_on) d.fd_rows = 1;  // (the chunked sweep's FDT is not complete)
    if ((rc = ensure_fd(h))) return rc;
    Dev full = d;  // every LA column, whatever this shard's share of the dataflow
    full.col0 = 0;
    full.ncol = d.n;
    if (h->reset_on) {
      bh::launch_first_descendants(full, s, true);
    } else if (walked) {
      bh::launch_flow_coordinates(full, s);
      bh::launch_first_descendants(full, s, true);
    } else if (wide) {
      bh::launch_flow_transpose(full, s);
      bh::launch_first_descendants(full, s, true);
    } else {
      bh::launch_coordinates(full, s);
      bh::launch_first_descendants(full, s, false);
    }
    if (!keep) h->inc_valid = false;
    HIPCHK(h, hipGetLastError());
    h->coords_for = (int)N;
    h->rows_stale = false;
    if (h->n_div < N) {
      // the passes that follow (DecideFame, DecideRoundReceived,
      // ProcessDecidedRounds) see the events DivideRounds covered, as Go's
      // do -- its rounds' Store entries: the divided prefix's chain lengths
      // and event count go back to the device view
      std::vector<int32_t> lens((size_t)d.n);
      for (int c = 0; c < d.n; ++c) {
        const auto &ch = h->chain[(size_t)c];
        lens[(size_t)c] = (int32_t)(std::lower_bound(ch.begin(), ch.end(), (int32_t)h->n_div) - ch.begin());
      }
      HIPCHK(h, hipMemcpyAsync(d.chain_len, lens.data(), (size_t)d.n * 4, hipMemcpyHostToDevice, s));
      HIPCHK(h, wait_stream(s));
      d.N = h->n_div;
      h->lens_h = lens;
    }
    if (h->layout_changed && h->R > 0)  // the witness tables' LA / FD rows moved with the layout
      bh::launch_witness_tables(d, h->R, s);
  }
  HIPCHK(h, wait_stream(h->stream));
  return BH_OK;
}

int bh_get_coordinates(bh_handle *h, int64_t id, int32_t *last_ancestors, int32_t *first_descendants) {
  if (!h || id < 0 || id >= (int64_t)h->h_creator.size()) return BH_ERR_INVALID;
  if (h->no_results()) return h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  (void)hipSetDevice(h->device);
  Dev &d = h->d;
  if (int rc = ensure_coords(h)) return rc;
  const int32_t c = h->h_creator[(size_t)id];
  const int64_t row = (int64_t)h->cstart_h[(size_t)c] + h->h_index[(size_t)id];  // chain-major layout
  HIPCHK(h, wait_stream(h->stream));
  if (last_ancestors)
    HIPCHK(h, hipMemcpy(last_ancestors, d.la + row * d.npad, (size_t)d.n * 4, hipMemcpyDeviceToHost));
  if (first_descendants && (d.fd_cols || !d.fd_rows)) {  // one column of FDT
    HIPCHK(h, hipMemcpy2D(first_descendants, 4, d.fdt + bh::fdt_pos(row, 0, d.npad), 64 * 4, 4, (size_t)d.n,
                          hipMemcpyDeviceToHost));
  } else if (first_descendants) {
    HIPCHK(h, hipMemcpy(first_descendants, d.fd + row * d.npad, (size_t)d.n * 4, hipMemcpyDeviceToHost));
  }
  if (h->reset_on)  // chain positions -> Index (chains start after their Root's SelfParent)
    for (int i = 0; i < d.n; ++i) {
      if (last_ancestors && last_ancestors[i] >= 0) last_ancestors[i] += h->base_h[(size_t)i];
      if (first_descendants && first_descendants[i] != bh::FD_NONE) first_descendants[i] += h->base_h[(size_t)i];
    }
  return BH_OK;
}

int bh_query_events(bh_handle *h, int32_t kind, int64_t count, const int64_t *x, const int64_t *y, int32_t *out) {
  if (!h) return BH_ERR_INVALID;
  if (h->no_results()) return h->fail(BH_ERR_STATE, "results live on rank 0 of a split group (this is rank %d)", h->rank);
  if (kind < BH_Q_ANCESTOR || kind > BH_Q_ROUND_DIFF || count < 0 || (count > 0 && (!x || !y || !out)))
    return h->fail(BH_ERR_INVALID, "bh_query_events: bad kind or buffers");
  const int64_t N = (int64_t)h->h_creator.size();
  for (int64_t i = 0; i < count; ++i)
    if (x[i] < 0 || x[i] >= N || y[i] < 0 || y[i] >= N)
      return h->fail(BH_ERR_KEY_NOT_FOUND, "bh_query_events: event %lld / %lld not inserted", (long long)x[i],
                     (long long)y[i]);
  if (count == 0) return BH_OK;
  if (kind == BH_Q_ROUND_DIFF && h->n_div < N)
    return h->fail(BH_ERR_STATE, "roundDiff before DivideRounds covered every event");
  (void)hipSetDevice(h->device);
  if (int rc = ensure_coords(h)) return rc;
  const size_t need = (size_t)count * 20;
  if (need > h->q_cap) {
    if (h->q_buf) (void)hipFree(h->q_buf);
    h->q_buf = nullptr;
    h->q_cap = 0;
    HIPCHK(h, hipMalloc((void **)&h->q_buf, need));
    h->q_cap = need;
  }
  int64_t *dx = reinterpret_cast<int64_t *>(h->q_buf), *dy = dx + count;
  int32_t *dout = reinterpret_cast<int32_t *>(dy + count);
  hipStream_t s = h->stream;
  HIPCHK(h, hipMemcpyAsync(dx, x, (size_t)count * 8, hipMemcpyHostToDevice, s));
  HIPCHK(h, hipMemcpyAsync(dy, y, (size_t)count * 8, hipMemcpyHostToDevice, s));
  bh::launch_query(h->d, kind, count, dx, dy, dout, s);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipMemcpyAsync(out, dout, (size_t)count * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(h, wait_stream(s));
  return BH_OK;
}

int32_t bh_get_stage_ms(bh_handle *h, float *ms, int32_t cap) {
  if (!h) return 0;
  settle_timings(h);
  for (int i = 0; i < NSTAGE && i < cap; ++i) ms[i] = h->stage_ms[i];
  if (cap > NSTAGE) ms[NSTAGE] = h->xchg_ms;
  if (cap > NSTAGE + 1) ms[NSTAGE + 1] = h->frames_ms;
  if (cap > NSTAGE + 2) ms[NSTAGE + 2] = h->loop_ms_acc;
  return NSTAGE + 3;
}

int bh_get_profile(bh_handle *h, int64_t *rounds_iterated, float *sweep_ms) {
  if (!h) return BH_ERR_INVALID;
  settle_timings(h);
  if (rounds_iterated) *rounds_iterated = h->iters;
  if (sweep_ms) *sweep_ms = h->sweep_ms;
  return BH_OK;
}

const char *bh_get_profile_kernel(const bh_handle *h) { return h ? h->sweep_kernel : ""; }

int bh_get_pipeline(bh_handle *h, int32_t *segments, int64_t *incremental_calls) {
  if (!h) return BH_ERR_INVALID;
  if (segments) *segments = h->segments_used;
  if (incremental_calls) *incremental_calls = h->inc_calls;
  return BH_OK;
}

int bh_get_loop_stats(bh_handle *h, int64_t *persistent_loops, int64_t *persist_fallbacks) {
  if (!h) return BH_ERR_INVALID;
  if (persistent_loops) *persistent_loops = h->persist_loops;
  if (persist_fallbacks) *persist_fallbacks = h->persist_fallbacks;
  return BH_OK;
}

int bh_hash_bodies(bh_handle *h, const uint8_t *bytes, const int64_t *offsets, int64_t count,
                   uint8_t *digests) {
  if (!h) return BH_ERR_INVALID;
  if (count < 0 || (count > 0 && (!bytes || !offsets || !digests)))
    return h->fail(BH_ERR_INVALID, "bh_hash_bodies: null buffer or negative count");
  if (count == 0) return BH_OK;
  (void)hipSetDevice(h->device);
  const int64_t base = offsets[0], total = offsets[count] - base;
  std::vector<int64_t> off((size_t)count);
  std::vector<int32_t> len((size_t)count);
  for (int64_t i = 0; i < count; ++i) {
    const int64_t l = offsets[i + 1] - offsets[i];
    if (l < 0 || l > INT32_MAX / 8) return h->fail(BH_ERR_INVALID, "bh_hash_bodies: offsets not ascending");
    off[(size_t)i] = offsets[i] - base;
    len[(size_t)i] = (int32_t)l;
  }
  // one device buffer: bytes (+128 B of read slack for the block loads),
  // offsets, lengths, digests; kept for the next call
  const size_t nb = ((size_t)total + 128 + 15) & ~(size_t)15;
  const size_t need = nb + (size_t)count * (8 + 4 + 32);
  if (need > h->sha_cap) {
    if (h->sha_buf) (void)hipFree(h->sha_buf);
    h->sha_buf = nullptr;
    h->sha_cap = 0;
    HIPCHK(h, hipMalloc((void **)&h->sha_buf, need));
    h->sha_cap = need;
  }
  uint8_t *db = h->sha_buf;
  int64_t *doff = reinterpret_cast<int64_t *>(db + nb);
  int32_t *dlen = reinterpret_cast<int32_t *>(doff + count);
  uint8_t *dout = reinterpret_cast<uint8_t *>(dlen + count);
  HIPCHK(h, hipMemcpyAsync(db, bytes + base, (size_t)total, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(doff, off.data(), (size_t)count * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(dlen, len.data(), (size_t)count * 4, hipMemcpyHostToDevice, h->stream));
  bh::launch_sha256(db, doff, dlen, count, dout, h->stream);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipMemcpyAsync(digests, dout, (size_t)count * 32, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, wait_stream(h->stream));
  return BH_OK;
}

int bh_verify_signatures(bh_handle *h, const uint8_t *hashes, const uint8_t *sig_r, const uint8_t *sig_s,
                         const int32_t *keys, int64_t count, const uint8_t *pubkeys, int32_t n_keys,
                         uint8_t *ok) {
  if (!h) return BH_ERR_INVALID;
  if (count < 0 || n_keys <= 0 || (count > 0 && (!hashes || !sig_r || !sig_s || !keys || !pubkeys || !ok)))
    return h->fail(BH_ERR_INVALID, "bh_verify_signatures: null buffer or bad count");
  if (count == 0) return BH_OK;
  for (int64_t i = 0; i < count; ++i)
    if (keys[i] < 0 || keys[i] >= n_keys) return h->fail(BH_ERR_INVALID, "bh_verify_signatures: key index out of range");
  (void)hipSetDevice(h->device);
  const size_t need = (size_t)count * (3 * 32 + 4 + 1) + (size_t)n_keys * 64 + 64;
  if (need > h->sha_cap) {  // shares the hashing scratch buffer
    if (h->sha_buf) (void)hipFree(h->sha_buf);
    h->sha_buf = nullptr;
    h->sha_cap = 0;
    HIPCHK(h, hipMalloc((void **)&h->sha_buf, need));
    h->sha_cap = need;
  }
  uint8_t *dh = h->sha_buf, *dr = dh + count * 32, *ds = dr + count * 32;
  int32_t *dk = reinterpret_cast<int32_t *>(ds + count * 32);
  uint8_t *dp = reinterpret_cast<uint8_t *>(dk + count), *dok = dp + (size_t)n_keys * 64;
  HIPCHK(h, hipMemcpyAsync(dh, hashes, (size_t)count * 32, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(dr, sig_r, (size_t)count * 32, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(ds, sig_s, (size_t)count * 32, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(dk, keys, (size_t)count * 4, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(dp, pubkeys, (size_t)n_keys * 64, hipMemcpyHostToDevice, h->stream));
  bh::launch_ecdsa_verify(dh, dr, ds, dk, dp, count, dok, h->stream);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipMemcpyAsync(ok, dok, (size_t)count, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, wait_stream(h->stream));
  return BH_OK;
}

}  // extern "C"
