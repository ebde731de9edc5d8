// kernels_frames.hip -- the block projection.
//
// GetFrame (hashgraph.go:1125-1231) gives every processed round-received f
// one Root per participant, in peer order:
//   * a creator with events in the frame: createRoot of its first event in
//     frame order (:1161-1172) -- NextRound = its round, SelfParent = the
//     RootEvent of its self-parent (the base root event "Root<id>" with
//     Index / LamportTimestamp / Round -1 for a first event, root.go:73-84),
//     Others[it] = the RootEvent of its other-parent (createRoot :602-640);
//   * any other participant: createRoot of its last consensus event
//     (InmemStore.lastConsensusEvents, inmem_store.go:178-183), or its base
//     Root when it has none (:1174-1197);
//   * every later event of the frame whose other-parent is not an earlier
//     event of the frame adds Others[event] = RootEvent(other-parent) to its
//     creator's root (:1199-1218).
// Frame.Marshal (frame.go:17-26) is Go encoding/json of {Round, Roots,
// Events}: struct fields in order, map keys sorted (the "0x"+uppercase-hex
// keys sort as the hash bytes), an Event as {"Body":..,"Signature":".."}.
// FrameHash = SHA-256 of it (frame.go:35-41); the block
// (NewBlockFromFrame, block.go:100-123) carries it with the frame's
// transactions, and the block's hash is SHA-256 of Block.Marshal
// (block.go:178-205) with no signatures yet.
//
// Device plan for the frames [f0, f0 + F) one ProcessDecidedRounds call
// emits (consensus positions [i0, i1), frames sorted):
//   roots:  min / max position of each creator per frame (atomics) ->
//           per-participant max-scan over frames carries the last consensus
//           event -> root_src; Others counted per root, scanned, filled,
//           and sorted by key hash (a root has a handful);
//   JSON:   every piece (root, event) measured by the same writer that
//           later emits it (JW with a null destination), exclusive scans
//           give every piece its offset, roots are written by one thread
//           each, events by one wave each (coalesced byte copies of the
//           stored body / signature), then one SHA-256 lane per frame.
// Integer and byte work, HBM / latency bound.
#include "engine.h"

namespace bh {

void launch_sha256(const uint8_t *data, const int64_t *off, const int32_t *len, int64_t count, uint8_t *out,
                   hipStream_t s);

// ---------------------------------------------------------------------------
// exclusive scan of int64 x[0, m) in place, x[m] = total
constexpr int SCAN_T = 1024, SCAN_V = 4, SCAN_TILE = SCAN_T * SCAN_V;

__device__ int64_t block_excl_scan(int64_t v, int64_t *sh, int64_t *total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {
    const int64_t a = t >= off ? sh[t - off] : 0;
    __syncthreads();
    sh[t] += a;
    __syncthreads();
  }
  const int64_t incl = sh[t];
  *total = sh[SCAN_T - 1];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_tile(int64_t *x, int64_t m, int64_t *part) {
  __shared__ int64_t sh[SCAN_T];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_V;
  int64_t v[SCAN_V], s = 0;
#pragma unroll
  for (int u = 0; u < SCAN_V; ++u) {
    v[u] = base + u < m ? x[base + u] : 0;
    s += v[u];
  }
  int64_t tot;
  int64_t run = block_excl_scan(s, sh, &tot);
#pragma unroll
  for (int u = 0; u < SCAN_V; ++u)
    if (base + u < m) {
      x[base + u] = run;
      run += v[u];
    }
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_part(int64_t *part, int64_t nb, int64_t *x, int64_t m) {
  __shared__ int64_t sh[SCAN_T];
  const int64_t per = (nb + SCAN_T - 1) / SCAN_T;
  const int64_t lo = min(nb, (int64_t)threadIdx.x * per), hi = min(nb, lo + per);
  int64_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += part[i];
  int64_t tot;
  int64_t run = block_excl_scan(s, sh, &tot);
  for (int64_t i = lo; i < hi; ++i) {
    const int64_t v = part[i];
    part[i] = run;
    run += v;
  }
  if (threadIdx.x == 0) x[m] = tot;
}

__global__ __launch_bounds__(256) void k_scan_add(int64_t *x, int64_t m, const int64_t *part) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < m) x[i] += part[i / SCAN_TILE];
}

static void scan_excl(int64_t *x, int64_t m, int64_t *part, hipStream_t s) {
  const int64_t nb = (m + SCAN_TILE - 1) / SCAN_TILE;
  if (nb > 0) k_scan_tile<<<(unsigned)nb, SCAN_T, 0, s>>>(x, m, part);
  k_scan_part<<<1, SCAN_T, 0, s>>>(part, nb, x, m);
  if (nb > 1) k_scan_add<<<(unsigned)((m + 255) / 256), 256, 0, s>>>(x, m, part);
}

// ---------------------------------------------------------------------------
// roots

__global__ __launch_bounds__(256) void k_root_minmax(Dev d, Frames fr, int32_t f0, int64_t i0, int64_t i1) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= i1) return;
  const int32_t e = d.order[i];
  const int64_t g = (int64_t)(d.rr[e] - f0) * d.n + d.creator[e];
  atomicMin(&fr.first_pos[g], (int32_t)i);
  atomicMax(&fr.last_in[g], (int32_t)i);
}

// one workgroup per participant: the last consensus event before each frame
// is a running max of positions over the frames (a later frame's positions
// are all larger), seeded with the previous calls' last_pos
__global__ __launch_bounds__(SCAN_T) void k_root_carry(Dev d, Frames fr, int32_t f0, int32_t F) {
  __shared__ int64_t sh[SCAN_T];
  const int32_t p = blockIdx.x, n = d.n;
  const int32_t per = (F + SCAN_T - 1) / SCAN_T;
  const int32_t lo = min(F, (int32_t)threadIdx.x * per), hi = min(F, lo + per);
  int32_t mx = -1;
  for (int32_t j = lo; j < hi; ++j) mx = max(mx, fr.last_in[(int64_t)j * n + p]);
  // inclusive max-scan of the chunk maxima: thread t's carry-in is the
  // largest position among the earlier chunks (or the earlier calls')
  sh[threadIdx.x] = mx;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {
    const int64_t a = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : -1;
    __syncthreads();
    sh[threadIdx.x] = max(sh[threadIdx.x], a);
    __syncthreads();
  }
  int32_t carry = max(fr.last_pos[p], threadIdx.x > 0 ? (int32_t)sh[threadIdx.x - 1] : -1);
  for (int32_t j = lo; j < hi; ++j) {
    const int64_t g = (int64_t)j * n + p;
    const int32_t fp = fr.first_pos[g];
    fr.root_src[(int64_t)(f0 + j) * n + p] = fp != NO_FIRST ? d.order[fp] : (carry >= 0 ? d.order[carry] : -1);
    carry = max(carry, fr.last_in[g]);
  }
  if (threadIdx.x == SCAN_T - 1) fr.last_pos[p] = carry;
}

// the installed Root entry naming e's other-parent (a Reset hashgraph), -1
__device__ __forceinline__ int32_t root_other_of(const Frames &fr, int32_t e) { return fr.oth_of ? fr.oth_of[e] : -1; }

// createOtherParentRootEvent(e) (hashgraph.go:568-600): the installed Root's
// entry when it names e's other-parent, else the other-parent event
__device__ __forceinline__ int32_t other_root_event(const Dev &d, const Frames &fr, int32_t e) {
  const int32_t k = root_other_of(fr, e);
  return k >= 0 ? -2 - k : d.op[e];
}

// Others of an event of the frame that is not its creator's first in it:
// its other-parent, unless that is an earlier event of the same frame (an
// other-parent only a Reset Root knows never is)
__device__ __forceinline__ bool other_entry(const Dev &d, const Frames &fr, int32_t f0, int64_t i, int32_t e,
                                            int64_t *g) {
  const int32_t op = d.op[e];
  if (op < 0 && root_other_of(fr, e) < 0) return false;
  const int32_t f = d.rr[e];
  *g = (int64_t)(f - f0) * d.n + d.creator[e];
  if (fr.first_pos[*g] == (int32_t)i) return false;
  if (op < 0) return true;
  const int64_t opp = d.cons_pos[op];
  return !(opp >= d.frame_ofs[f] && opp < i);
}

// Others of each root: createRoot's entry (the source event's other-parent),
// or, for a Reset Root kept whole, all its installed entries
__global__ __launch_bounds__(256) void k_others_roots(Dev d, Frames fr, int32_t f0, int64_t G, bool fill) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= G) return;
  const int32_t s = fr.root_src[(int64_t)f0 * d.n + g];
  const int32_t p = (int32_t)(g % d.n);
  int32_t cnt = 0;
  if (s >= 0) cnt = d.op[s] >= 0 || root_other_of(fr, s) >= 0;
  else if (fr.ro_ofs) cnt = fr.ro_ofs[p + 1] - fr.ro_ofs[p];
  if (!fill) {
    fr.sz[g] = cnt;
  } else if (cnt) {
    const int64_t k = fr.oofs[(int64_t)f0 * d.n + g] + atomicAdd(&fr.ocur[g], cnt);
    if (s >= 0) {
      fr.okey[k] = s;
      fr.oval[k] = other_root_event(d, fr, s);
    } else {
      for (int32_t q = 0; q < cnt; ++q) {
        const int32_t ent = fr.ro_list[fr.ro_ofs[p] + q];
        fr.okey[k + q] = -2 - ent;
        fr.oval[k + q] = -2 - ent;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_others_events(Dev d, Frames fr, int32_t f0, int64_t i0, int64_t i1,
                                                       bool fill) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= i1) return;
  const int32_t e = d.order[i];
  int64_t g;
  if (!other_entry(d, fr, f0, i, e, &g)) return;
  if (!fill) {
    atomicAdd(reinterpret_cast<unsigned long long *>(&fr.sz[g]), 1ull);
  } else {
    const int64_t k = fr.oofs[(int64_t)f0 * d.n + g] + atomicAdd(&fr.ocur[g], 1);
    fr.okey[k] = e;
    fr.oval[k] = other_root_event(d, fr, e);
  }
}

__global__ __launch_bounds__(256) void k_others_base(Frames fr, int64_t at, int64_t G, int64_t obase) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g <= G) fr.oofs[at + g] = obase + fr.sz[g];
}

// the hash an Others key stands for: an event's, or installed entry k's key
__device__ __forceinline__ const uint8_t *key_ptr(const Frames &fr, int32_t key) {
  return key >= 0 ? fr.hash + (int64_t)key * 32 : fr.ro_key + (int64_t)(-2 - key) * 32;
}

__device__ __forceinline__ bool hash_less(const Frames &fr, int32_t a, int32_t b) {
  const uint32_t *x = reinterpret_cast<const uint32_t *>(key_ptr(fr, a));
  const uint32_t *y = reinterpret_cast<const uint32_t *>(key_ptr(fr, b));
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t u = __builtin_bswap32(x[q]), v = __builtin_bswap32(y[q]);
    if (u != v) return u < v;
  }
  return false;
}

__global__ __launch_bounds__(256) void k_others_sort(Frames fr, int64_t at, int64_t G) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= G) return;
  const int64_t lo = fr.oofs[at + g], hi = fr.oofs[at + g + 1];
  for (int64_t a = lo + 1; a < hi; ++a) {
    const int32_t k = fr.okey[a], v = fr.oval[a];
    int64_t b = a - 1;
    while (b >= lo && hash_less(fr, k, fr.okey[b])) {
      fr.okey[b + 1] = fr.okey[b];
      fr.oval[b + 1] = fr.oval[b];
      --b;
    }
    fr.okey[b + 1] = k;
    fr.oval[b + 1] = v;
  }
}

void launch_frame_roots(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                        int64_t obase, hipStream_t s) {
  if (F <= 0) return;
  const int64_t G = (int64_t)F * d.n;
  (void)hipMemsetAsync(fr.first_pos, 0x7f, (size_t)G * 4, s);
  (void)hipMemsetAsync(fr.last_in, 0xff, (size_t)G * 4, s);
  (void)hipMemsetAsync(fr.ocur, 0, (size_t)G * 4, s);
  const unsigned ge = (unsigned)((i1 - i0 + 255) / 256), gg = (unsigned)((G + 255) / 256);
  if (i1 > i0) k_root_minmax<<<ge, 256, 0, s>>>(d, fr, f0, i0, i1);
  k_root_carry<<<d.n, SCAN_T, 0, s>>>(d, fr, f0, F);
  k_others_roots<<<gg, 256, 0, s>>>(d, fr, f0, G, false);
  if (i1 > i0) k_others_events<<<ge, 256, 0, s>>>(d, fr, f0, i0, i1, false);
  scan_excl(fr.sz, G, fr.part, s);
  k_others_base<<<(unsigned)((G + 256) / 256), 256, 0, s>>>(fr, (int64_t)f0 * d.n, G, obase);
  k_others_roots<<<gg, 256, 0, s>>>(d, fr, f0, G, true);
  if (i1 > i0) k_others_events<<<ge, 256, 0, s>>>(d, fr, f0, i0, i1, true);
  k_others_sort<<<gg, 256, 0, s>>>(fr, (int64_t)f0 * d.n, G);
}

// ---------------------------------------------------------------------------
// Go encoding/json pieces.  JW measures (p == nullptr) or writes; sizes and
// bytes come from the same code, so offsets always match what is written.
struct JW {
  uint8_t *p;
  int64_t n;
  __device__ void put(const char *s, int len) {
    if (p)
      for (int k = 0; k < len; ++k) p[n + k] = (uint8_t)s[k];
    n += len;
  }
  template <int L>
  __device__ void lit(const char (&s)[L]) { put(s, L - 1); }
  __device__ void num(int64_t v) {
    char t[20];
    int k = 20;
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    do {
      t[--k] = (char)('0' + u % 10);
      u /= 10;
    } while (u);
    if (v < 0) t[--k] = '-';
    put(t + k, 20 - k);
  }
  // Event.Hex(): "0x" + uppercase hex (event.go:239-245)
  __device__ void hex(const uint8_t *h) {
    if (p) {
      p[n] = '0';
      p[n + 1] = 'x';
      for (int i = 0; i < 32; ++i) {
        const int hi = h[i] >> 4, lo = h[i] & 15;
        p[n + 2 + 2 * i] = (uint8_t)(hi < 10 ? '0' + hi : 'A' + hi - 10);
        p[n + 3 + 2 * i] = (uint8_t)(lo < 10 ? '0' + lo : 'A' + lo - 10);
      }
    }
    n += 66;
  }
  // []byte: padded base64 (StdEncoding)
  __device__ void b64(const uint8_t *x, int len) {
    const char *A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < len; i += 3) {
      if (p) {
        const uint32_t v = (uint32_t)x[i] << 16 | (i + 1 < len ? (uint32_t)x[i + 1] << 8 : 0u) |
                           (i + 2 < len ? (uint32_t)x[i + 2] : 0u);
        p[n] = (uint8_t)A[v >> 18];
        p[n + 1] = (uint8_t)A[(v >> 12) & 63];
        p[n + 2] = (uint8_t)(i + 1 < len ? A[(v >> 6) & 63] : '=');
        p[n + 3] = (uint8_t)(i + 2 < len ? A[v & 63] : '=');
      }
      n += 4;
    }
  }
  __device__ void raw(const uint8_t *src, int64_t len) {
    if (p)
      for (int64_t k = 0; k < len; ++k) p[n + k] = src[k];
    n += len;
  }
};

// RootEvent (root.go:65-71): an event; -1: slot's Root SelfParent (the
// base root event "Root<id>" with Index / LamportTimestamp / Round -1, or a
// Reset Root's, root.go:75-84); -2 - k: installed Others entry k
__device__ void root_event(JW &w, const Dev &d, const Frames &fr, int32_t ev, int32_t slot) {
  const bool rst = d.chain_base != nullptr;
  const int32_t spi = ev == -1 && rst ? d.chain_base[slot] - 1 : -1;  // Root.SelfParent.Index
  const int32_t k = -2 - ev;
  w.lit("{\"Hash\":\"");
  if (ev == -1 && spi >= 0) {
    w.hex(fr.rsp_hash + (int64_t)slot * 32);
  } else if (ev == -1) {
    w.lit("Root");
    w.num(fr.pids[slot]);
  } else if (ev < -1) {
    w.hex(fr.ro_hash + (int64_t)k * 32);
  } else {
    w.hex(fr.hash + (int64_t)ev * 32);
  }
  w.lit("\",\"CreatorID\":");
  w.num(fr.pids[ev == -1 ? slot : ev < -1 ? fr.ro_creator[k] : d.creator[ev]]);
  w.lit(",\"Index\":");
  w.num(ev == -1 ? spi : ev < -1 ? fr.ro_index[k] : d.index[ev] + (rst ? d.chain_base[d.creator[ev]] : 0));
  w.lit(",\"LamportTimestamp\":");
  w.num(ev == -1 ? (rst ? d.lt_seed[slot] : -1) : ev < -1 ? fr.ro_lt[k] : d.lt[ev]);
  w.lit(",\"Round\":");
  w.num(ev == -1 ? (rst ? d.root_sp_round[slot] : -1) : ev < -1 ? fr.ro_round[k] : d.round[ev]);
  w.lit("}");
}

// Root (root.go:88-96) of slot p in frame f, with its separating comma
__device__ void root_json(JW &w, const Dev &d, const Frames &fr, int32_t f, int32_t p) {
  const int64_t g = (int64_t)f * d.n + p;
  const int32_t src = fr.root_src[g];
  if (p) w.lit(",");
  w.lit("{\"NextRound\":");
  w.num(src >= 0 ? d.round[src] : d.chain_base ? d.root_next[p] : 0);
  w.lit(",\"SelfParent\":");
  root_event(w, d, fr, src < 0 ? -1 : max(d.sp[src], -1), p);
  w.lit(",\"Others\":{");
  const int64_t lo = fr.oofs[g], hi = fr.oofs[g + 1];
  for (int64_t k = lo; k < hi; ++k) {
    if (k > lo) w.lit(",");
    w.lit("\"");
    w.hex(key_ptr(fr, fr.okey[k]));
    w.lit("\":");
    root_event(w, d, fr, fr.oval[k], 0);
  }
  w.lit("}}");
}

__device__ __forceinline__ int64_t frame_head_len(int32_t f) {
  JW w{nullptr, 0};
  w.lit("{\"Round\":");
  w.num(f);
  w.lit(",\"Roots\":[");
  return w.n;
}
constexpr int64_t FRAME_MID = sizeof("],\"Events\":[") - 1;
constexpr int64_t FRAME_TAIL = sizeof("]}\n") - 1;
constexpr int64_t EV_HEAD = sizeof("{\"Body\":") - 1;
constexpr int64_t EV_SIG = sizeof(",\"Signature\":\"") - 1;
constexpr int64_t EV_TAIL = sizeof("\"}") - 1;

__global__ __launch_bounds__(256) void k_frame_missing(Dev d, Frames fr, int32_t f0, int64_t i0, int64_t i1) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= i1) return;
  const int32_t e = d.order[i];
  if (fr.body_len[e] < 0 || fr.sig_len[e] < 0) fr.missing[d.rr[e] - f0] = 1;
}

__global__ __launch_bounds__(256) void k_root_sizes(Dev d, Frames fr, int32_t f0, int64_t G) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= G) return;
  JW w{nullptr, 0};
  root_json(w, d, fr, f0 + (int32_t)(g / d.n), (int32_t)(g % d.n));
  fr.sz[g] = w.n;
}

__global__ __launch_bounds__(256) void k_event_sizes(Dev d, Frames fr, int64_t i0, int64_t i1) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= i1) return;
  const int32_t e = d.order[i];
  const int32_t f = d.rr[e];
  fr.sz2[i - i0] = (i > d.frame_ofs[f]) + EV_HEAD + max(fr.body_len[e], 0) + EV_SIG + max(fr.sig_len[e], 0) + EV_TAIL;
}

// frame j's bytes: head, roots, middle, events, tail (0 when bytes are missing)
__global__ __launch_bounds__(256) void k_frame_sizes(Dev d, Frames fr, int32_t f0, int32_t F, int64_t i0) {
  const int32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= F) return;
  const int32_t f = f0 + j;
  const int64_t fs = d.frame_ofs[f] - i0, fe = fs + d.frame_cnt[f];
  const int64_t n = d.n;
  const int64_t len = fr.missing[j] ? 0
                                    : frame_head_len(f) + (fr.sz[(j + 1) * n] - fr.sz[j * n]) + FRAME_MID +
                                          (fr.sz2[fe] - fr.sz2[fs]) + FRAME_TAIL;
  fr.jofs[j] = len;
  fr.jlen[j] = (int32_t)len;
}

void launch_frame_json_size(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                            hipStream_t s) {
  if (F <= 0) return;
  const int64_t G = (int64_t)F * d.n;
  (void)hipMemsetAsync(fr.missing, 0, (size_t)F, s);
  const unsigned ge = (unsigned)((i1 - i0 + 255) / 256);
  if (i1 > i0) {
    k_frame_missing<<<ge, 256, 0, s>>>(d, fr, f0, i0, i1);
    k_event_sizes<<<ge, 256, 0, s>>>(d, fr, i0, i1);
  }
  scan_excl(fr.sz2, i1 - i0, fr.part, s);
  k_root_sizes<<<(unsigned)((G + 255) / 256), 256, 0, s>>>(d, fr, f0, G);
  scan_excl(fr.sz, G, fr.part, s);
  k_frame_sizes<<<(unsigned)((F + 255) / 256), 256, 0, s>>>(d, fr, f0, F, i0);
  scan_excl(fr.jofs, F, fr.part, s);
}

__global__ __launch_bounds__(256) void k_frame_write_frame(Dev d, Frames fr, int32_t f0, int32_t F, int64_t i0) {
  const int32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= F || fr.missing[j]) return;
  const int32_t f = f0 + j;
  const int64_t n = d.n;
  const int64_t fs = d.frame_ofs[f] - i0, fe = fs + d.frame_cnt[f];
  JW w{fr.json, fr.jofs[j]};
  w.lit("{\"Round\":");
  w.num(f);
  w.lit(",\"Roots\":[");
  w.n += fr.sz[(j + 1) * n] - fr.sz[j * n];
  w.lit("],\"Events\":[");
  w.n += fr.sz2[fe] - fr.sz2[fs];
  w.lit("]}\n");
}

__global__ __launch_bounds__(256) void k_frame_write_roots(Dev d, Frames fr, int32_t f0, int64_t G) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= G) return;
  const int32_t j = (int32_t)(g / d.n);
  if (fr.missing[j]) return;
  const int32_t f = f0 + j;
  JW w{fr.json, fr.jofs[j] + frame_head_len(f) + (fr.sz[g] - fr.sz[(int64_t)j * d.n])};
  root_json(w, d, fr, f, (int32_t)(g % d.n));
}

// one wave per event: the piece's bytes copied by 64 lanes, coalesced
__global__ __launch_bounds__(256) void k_frame_write_events(Dev d, Frames fr, int32_t f0, int64_t i0, int64_t i1) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= i1) return;
  const int32_t e = d.order[i];
  const int32_t f = d.rr[e], j = f - f0;
  if (fr.missing[j]) return;
  const int64_t n = d.n;
  const int64_t fs = d.frame_ofs[f];
  const int64_t at = fr.jofs[j] + frame_head_len(f) + (fr.sz[(j + 1) * n] - fr.sz[j * n]) + FRAME_MID +
                     (fr.sz2[i - i0] - fr.sz2[fs - i0]);
  const int comma = i > fs;
  const int64_t bl = fr.body_len[e], sl = fr.sig_len[e];
  const uint8_t *body = fr.arena + fr.body_off[e], *sig = fr.arena + fr.sig_off[e];
  const int64_t b0 = comma + EV_HEAD, s0 = b0 + bl + EV_SIG, t0 = s0 + sl, L = t0 + EV_TAIL;
  const char *H = ",{\"Body\":", *S = ",\"Signature\":\"", *T = "\"}";
  uint8_t *out = fr.json + at;
  for (int64_t k = lane; k < L; k += 64) {
    uint8_t c;
    if (k < b0) c = (uint8_t)H[k + 1 - comma];
    else if (k < b0 + bl) c = body[k - b0];
    else if (k < s0) c = (uint8_t)S[k - b0 - bl];
    else if (k < t0) c = sig[k - s0];
    else c = (uint8_t)T[k - t0];
    out[k] = c;
  }
}

__global__ __launch_bounds__(256) void k_frame_store(Dev d, Frames fr, int32_t f0, int32_t F, const uint8_t *h32) {
  const int32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= F) return;
  const int32_t f = f0 + j;
  const bool ok = !fr.missing[j] && d.frame_cnt[f] > 0;
  fr.fvalid[f] = ok;
  if (ok)
    for (int k = 0; k < 32; ++k) fr.fhash[(int64_t)f * 32 + k] = h32[(int64_t)j * 32 + k];
}

void launch_frame_json_write(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                             bool store, hipStream_t s) {
  if (F <= 0) return;
  const int64_t G = (int64_t)F * d.n;
  k_frame_write_frame<<<(unsigned)((F + 255) / 256), 256, 0, s>>>(d, fr, f0, F, i0);
  k_frame_write_roots<<<(unsigned)((G + 255) / 256), 256, 0, s>>>(d, fr, f0, G);
  if (i1 > i0) k_frame_write_events<<<(unsigned)((i1 - i0 + 3) / 4), 256, 0, s>>>(d, fr, f0, i0, i1);
  if (store) {
    launch_sha256(fr.json, fr.jofs, fr.jlen, F, fr.dig, s);
    launch_frame_store(d, fr, f0, F, fr.dig, s);
  }
}

void launch_frame_store(const Dev &d, const Frames &fr, int32_t f0, int32_t F, const uint8_t *dig, hipStream_t s) {
  if (F > 0) k_frame_store<<<(unsigned)((F + 255) / 256), 256, 0, s>>>(d, fr, f0, F, dig);
}

// ---------------------------------------------------------------------------
// Block.Marshal: {"Body":{"Index":b,"RoundReceived":f,"StateHash":null,
// "FrameHash":"<base64>","Transactions":[..]},"Signatures":{}}\n.  The
// transactions are the frame's events' in order; each body's JSON already
// holds them base64-encoded as its leading "Transactions" array
// (EventBody field order, event.go:16-21), so they are copied from there.
__device__ __forceinline__ int32_t tx_span(const Frames &fr, int32_t e, int64_t *at) {
  const char P[] = "{\"Transactions\":[";
  const int L = sizeof(P) - 1;
  const int32_t bl = fr.body_len[e];
  const uint8_t *b = fr.arena + fr.body_off[e];
  if (bl < L + 1) return 0;
  for (int k = 0; k < L; ++k)
    if (b[k] != (uint8_t)P[k]) return 0;  // "Transactions":null
  int32_t k = L;
  while (k < bl && b[k] != ']') ++k;
  *at = fr.body_off[e] + L;
  return k - L;
}

__global__ __launch_bounds__(256) void k_tx_sizes(Dev d, Frames fr, int64_t i0, int64_t i1) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= i1) return;
  int64_t at;
  const int32_t tl = tx_span(fr, d.order[i], &at);
  fr.sz2[i - i0] = tl > 0 ? tl + 1 : 0;  // with a separating comma
}

__device__ void block_head(JW &w, const Dev &d, const Frames &fr, int32_t f) {
  w.lit("{\"Body\":{\"Index\":");
  w.num(d.blk_of_frame[f]);
  w.lit(",\"RoundReceived\":");
  w.num(f);
  w.lit(",\"StateHash\":null,\"FrameHash\":\"");
  w.b64(fr.fhash + (int64_t)f * 32, 32);
  w.lit("\",\"Transactions\":[");
}
constexpr int64_t BLOCK_TAIL = sizeof("]},\"Signatures\":{}}\n") - 1;

__global__ __launch_bounds__(256) void k_block_sizes(Dev d, Frames fr, int32_t f0, int32_t F, int64_t i0) {
  const int32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= F) return;
  const int32_t f = f0 + j;
  int64_t len = 0;
  if (!fr.missing[j] && d.frame_cnt[f] > 0) {
    const int64_t fs = d.frame_ofs[f] - i0, fe = fs + d.frame_cnt[f];
    const int64_t S = fr.sz2[fe] - fr.sz2[fs];
    JW w{nullptr, 0};
    block_head(w, d, fr, f);
    len = w.n + (S > 0 ? S - 1 : 0) + BLOCK_TAIL;
  }
  fr.bofs[j] = len;
  fr.blen[j] = (int32_t)len;
}

void launch_block_json_size(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                            hipStream_t s) {
  if (F <= 0) return;
  if (i1 > i0) k_tx_sizes<<<(unsigned)((i1 - i0 + 255) / 256), 256, 0, s>>>(d, fr, i0, i1);
  scan_excl(fr.sz2, i1 - i0, fr.part, s);
  k_block_sizes<<<(unsigned)((F + 255) / 256), 256, 0, s>>>(d, fr, f0, F, i0);
  scan_excl(fr.bofs, F, fr.part, s);
}

__global__ __launch_bounds__(256) void k_block_write_frame(Dev d, Frames fr, int32_t f0, int32_t F, int64_t i0) {
  const int32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= F || fr.blen[j] == 0) return;
  const int32_t f = f0 + j;
  const int64_t fs = d.frame_ofs[f] - i0, fe = fs + d.frame_cnt[f];
  const int64_t S = fr.sz2[fe] - fr.sz2[fs];
  JW w{fr.bjson, fr.bofs[j]};
  block_head(w, d, fr, f);
  w.n += S > 0 ? S - 1 : 0;
  w.lit("]},\"Signatures\":{}}\n");
}

__global__ __launch_bounds__(256) void k_block_write_txs(Dev d, Frames fr, int32_t f0, int64_t i0, int64_t i1) {
  const int64_t i = i0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= i1) return;
  const int32_t e = d.order[i];
  const int32_t f = d.rr[e], j = f - f0;
  if (fr.blen[j] == 0) return;
  int64_t at;
  const int32_t tl = tx_span(fr, e, &at);
  if (tl == 0) return;
  JW h{nullptr, 0};
  block_head(h, d, fr, f);
  const int64_t before = fr.sz2[i - i0] - fr.sz2[d.frame_ofs[f] - i0];
  JW w{fr.bjson, fr.bofs[j] + h.n + (before > 0 ? before - 1 : 0)};
  if (before > 0) w.lit(",");
  w.raw(fr.arena + at, tl);
}

__global__ __launch_bounds__(256) void k_block_store(Dev d, Frames fr, int32_t f0, int32_t F, const uint8_t *h32) {
  const int32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j >= F || fr.blen[j] == 0) return;
  for (int k = 0; k < 32; ++k) fr.bhash[(int64_t)(f0 + j) * 32 + k] = h32[(int64_t)j * 32 + k];
}

void launch_block_json_write(const Dev &d, const Frames &fr, int32_t f0, int32_t F, int64_t i0, int64_t i1,
                             bool store, hipStream_t s) {
  if (F <= 0) return;
  k_block_write_frame<<<(unsigned)((F + 255) / 256), 256, 0, s>>>(d, fr, f0, F, i0);
  if (i1 > i0) k_block_write_txs<<<(unsigned)((i1 - i0 + 255) / 256), 256, 0, s>>>(d, fr, f0, i0, i1);
  if (store) {
    launch_sha256(fr.bjson, fr.bofs, fr.blen, F, fr.dig, s);
    launch_block_store(d, fr, f0, F, fr.dig, s);
  }
}

void launch_block_store(const Dev &d, const Frames &fr, int32_t f0, int32_t F, const uint8_t *dig, hipStream_t s) {
  if (F > 0) k_block_store<<<(unsigned)((F + 255) / 256), 256, 0, s>>>(d, fr, f0, F, dig);
}

__global__ void k_root_query(Dev d, Frames fr, int32_t f, int32_t *out) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= d.n) return;
  const int64_t g = (int64_t)f * d.n + p;
  const int32_t src = fr.root_src[g];
  out[3 * p] = src >= 0 ? d.round[src] : d.chain_base ? d.root_next[p] : 0;
  out[3 * p + 1] = src < 0 ? -1 : max(d.sp[src], -1);
  out[3 * p + 2] = (int32_t)(fr.oofs[g + 1] - fr.oofs[g]);
}

void launch_root_query(const Dev &d, const Frames &fr, int32_t f, int32_t *out, hipStream_t s) {
  k_root_query<<<(d.n + 255) / 256, 256, 0, s>>>(d, fr, f, out);
}

}  // namespace bh
