// kernels_rounds.hip -- rounds, witnesses and witness firstDescendants.
//
// Reference: _round (hashgraph.go:205-278): round(x) = pr + [#{w in W(pr):
// stronglySee(x, w)} >= SM], pr = max(round(sp), round(op)); witness
// (hashgraph.go:281-296): round(x) > round(sp(x)); _stronglySee
// (hashgraph.go:172-191); firstDescendants (hashgraph.go:510-544).
//
// Batch closed form (proof in DESIGN.md; the oracle checks it in tests).
// LA is non-decreasing along a creator's chain, so on every chain c the
// events of round >= r are a suffix starting at index B[r][c].  Let C(r) be
// the candidates (c, B[r][c]) -- the first event of each chain with round
// >= r.  Then
//   round(x) >= r+1  <=>  x strongly sees >= SM members of C(r)
// (if x strongly sees a candidate of round > r, that candidate strongly
// sees SM witnesses of round r, and so does x, because stronglySee is
// preserved by descendants), so
//   B[r+1][c] = first k >= B[r][c] whose event strongly sees SM of C(r),
//   W(r)      = { c in C(r) : B[r+1][c] > B[r][c] }   (round exactly r).
// The witness resolution therefore never sits on the serial path.  One
// step per ROUND (not per event or DAG level), two launches, one
// workgroup per chain c in each:
//   k_cand_fd  column c of the firstDescendants rows of every candidate:
//              the first event of chain c seeing it, by binary search in an
//              LDS window of chain c starting at B[r][c] (descendants of a
//              round >= r event have round >= r); also compacts W(r-1) and
//              its FD rows for DecideFame (known now that B[r] exists);
//   k_scan     FD rows of C(r) and the same window staged in LDS; two lanes
//              per candidate binary-search T_q, the first window row that
//              strongly sees it (monotone along the chain); B[r+1][c] = the
//              SM-th smallest T_q.
// B[r] and the candidate FD rows are double-buffered by round parity (a
// launch argument), so a captured graph of iterations replays without host
// involvement and the critical path starts with one independent load; the
// round index itself (device state) is only needed for the history writes.
#include "engine.h"

namespace bh {

constexpr int MAXN = 1024;   // participants supported by the LDS tables
constexpr int WROWS = 32;    // window rows per chain

__device__ __forceinline__ int popc64(unsigned long long x) { return __popcll(x); }

// stage `rows` rows of `q4` int4s (global row stride `gs` ints) into LDS
// (row stride rs ints).  U loads per thread are issued before the first LDS
// write, so a workgroup pays ~one L2 round trip per U*blockDim int4s
// instead of one per blockDim (the loop body would otherwise wait on each).
template <int U>
__device__ __forceinline__ void stage_rows(int32_t *dst, int rs, const int32_t *src, int64_t gs,
                                           int rows, int q4) {
  const int total = rows * q4;
  for (int b = threadIdx.x; b < total; b += U * blockDim.x) {
    int4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = b + u * blockDim.x;
      if (i < total) {
        const int row = i / q4, c4 = i - row * q4;
        v[u] = reinterpret_cast<const int4 *>(src + row * gs)[c4];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = b + u * blockDim.x;
      if (i < total) {
        const int row = i / q4, c4 = i - row * q4;
        reinterpret_cast<int4 *>(dst + row * rs)[c4] = v[u];
      }
    }
  }
}

// load rows [k0, k0+rows) of chain c (global rows cs+k) into LDS, stride rs
template <int U>
__device__ __forceinline__ void load_window(const Dev &d, int32_t *win, int rs, int32_t cs,
                                            int32_t k0, int rows) {
  stage_rows<U>(win, rs, d.la + (int64_t)(cs + k0) * d.npad, d.npad, rows, d.npad / 4);
}

// ---------------------------------------------------------------------------
// k_cand_fd(r): column c of the firstDescendants rows of every candidate of
// round r, written to fdc[r] (kept for every round: the fame stage reads the
// witnesses' rows from there, so nothing is compacted on the serial path).
__global__ __launch_bounds__(512) void k_cand_fd(Dev d, int p) {
  extern __shared__ __attribute__((aligned(16))) int32_t rsm[];
  __shared__ int32_t bcur[MAXN];
  __shared__ int32_t sh_ncand, sh_open;
  __shared__ int8_t open[MAXN];
  if (d.state[ST_DONE]) return;
  const int t = threadIdx.x;
  const int n = d.n, npad = d.npad, rs = npad + 4;
  const int c = blockIdx.x;
  const int r = d.state[ST_CUR];
  const int32_t *Bp = d.Bp + (int64_t)p * n;  // B[r]
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  int32_t k0 = Bp[c];
  int rows = min(WROWS, max(0, len - k0));
  int32_t *win = rsm;  // [WROWS][rs]
  const bool dg = d.diag != nullptr && t == 0;
  const unsigned long long tr0 = dg ? stamp() : 0;
  unsigned long long tr1 = 0, nfdw = 0;
  constexpr int QPT = MAXN / 512;
  int32_t bq[QPT], lq[QPT];
#pragma unroll
  for (int u = 0; u < QPT; ++u) {  // issued before the window, consumed after it
    const int q = t + u * 512;
    bq[u] = q < n ? Bp[q] : 0;
    lq[u] = q < n ? d.chain_len[q] : 0;
  }
  load_window<2>(d, win, rs, cs, k0, rows);
  if (t == 0) sh_ncand = 0;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < QPT; ++u) {
    const int q = t + u * 512;
    if (q < n) {
      const bool has = bq[u] < lq[u];
      bcur[q] = bq[u];
      open[q] = has && q != c;
      if (has) atomicAdd(&sh_ncand, 1);
      // a candidate's own column is its own index
      if (has && q == c) d.fdc[((int64_t)r * n + q) * npad + c] = bq[u];
    }
  }
  __syncthreads();
  if (sh_ncand == 0) {
    if (c == 0 && t == 0) { d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; }
    return;
  }
  if (r + 1 >= d.R_cap) {
    if (c == 0 && t == 0) { d.state[ST_ERR] = 1; d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; }
    return;
  }
  if (dg) tr1 = stamp();
  // ---- binary search per candidate, window by window ----
  int32_t *fcur = d.fdc + (int64_t)r * n * npad;
  for (;;) {
    if (t == 0) sh_open = 0;
    __syncthreads();
    for (int q = t; q < n; q += blockDim.x) {
      if (!open[q]) continue;
      const int32_t kw = bcur[q];
      int32_t res = -1;
      if (rows > 0 && win[(rows - 1) * rs + q] >= kw) {
        int lo = 0, hi = rows - 1;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (win[mid * rs + q] >= kw) hi = mid;
          else lo = mid + 1;
        }
        res = k0 + lo;
      } else if (k0 + rows >= len) {
        res = FD_NONE;
      }
      if (res != -1) {
        fcur[(int64_t)q * npad + c] = res;
        open[q] = 0;
      } else {
        atomicAdd(&sh_open, 1);
      }
    }
    __syncthreads();
    if (sh_open == 0) break;
    if (dg) ++nfdw;
    k0 += rows;
    rows = min(WROWS, len - k0);
    load_window<2>(d, win, rs, cs, k0, rows);
    __syncthreads();
  }
  if (c == 0)  // padding columns never match
    for (int q = t; q < n; q += blockDim.x)
      for (int i = n; i < npad; ++i) fcur[(int64_t)q * npad + i] = FD_NONE;
  if (dg) {
    const unsigned long long te = stamp();
    atomicAdd(&d.diag[DG_RF_P1], tr1 - tr0);
    atomicAdd(&d.diag[DG_RF_FD], te - tr1);
    atomicAdd(&d.diag[DG_RF_TOTAL], te - tr0);
    atomicAdd(&d.diag[DG_RF_CALLS], 1ull);
    atomicAdd(&d.diag[DG_RF_FDWIN], nfdw);
  }
}

// ---------------------------------------------------------------------------
// k_scan(r): B[r+1][c].  Two lanes per candidate, each taking every other
// int4 of the columns (adjacent 16-B pieces: with the npad+8 row pitch the
// 16 lanes of a ds_read_b128 group hit distinct banks), combined with a lane
// swap; T_q by binary search over the window; B[r+1][c] = SM-th smallest T_q.
// All staging loads (the chain's window, the candidates' FD rows, B[r]) are
// issued together, so the workgroup waits for one round trip, not three.
constexpr int SCAN_PAD = 8;

template <bool FD_LDS>
__global__ __launch_bounds__(256) void k_scan(Dev d, int p) {
  extern __shared__ __attribute__((aligned(16))) int32_t ssm[];
  __shared__ int32_t hist[WROWS + 1];
  __shared__ int32_t clist[MAXN];
  __shared__ int8_t has[MAXN];
  __shared__ int32_t sh_res, sh_nc;
  if (d.state[ST_DONE]) return;
  const int r = d.state[ST_CUR];
  const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = d.n, npad = d.npad, sm = d.sm, rs = npad + SCAN_PAD;
  const int32_t *Bp = d.Bp + (int64_t)p * n;
  const int32_t *fcur = d.fdc + (int64_t)r * n * npad;
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  int32_t *win = ssm;                  // [WROWS][rs]
  int32_t *fds = ssm + WROWS * rs;     // [n][rs] when FD_LDS (row q = chain q's candidate)
  int32_t k0 = Bp[c];
  const int q4 = npad / 4;
  const bool dg = d.diag != nullptr && t == 0;
  const unsigned long long ts0 = dg ? stamp() : 0;
  unsigned long long ts_load = 0, ts_comp = 0, nwin = 0;
  constexpr int QPT = MAXN / 256;
  int32_t bq[QPT], lq[QPT];
#pragma unroll
  for (int u = 0; u < QPT; ++u) {
    const int q = t + u * 256;
    bq[u] = q < n ? Bp[q] : 0;
    lq[u] = q < n ? d.chain_len[q] : 0;
  }
  int rows = min(WROWS, max(0, len - k0));
  {
    // one batch: window rows then (FD_LDS) all n candidate rows
    const int totA = rows * q4, tot = totA + (FD_LDS ? n * q4 : 0);
    const int32_t *srcA = d.la + (int64_t)(cs + k0) * npad;
    constexpr int U = 20;
    for (int b0 = t; b0 < tot; b0 += U * 256) {
      int4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = b0 + u * 256;
        if (i < tot) {
          const bool a = i < totA;
          const int j = a ? i : i - totA;
          const int row = j / q4, c4 = j - row * q4;
          const int32_t *src = a ? srcA + (int64_t)row * npad : fcur + (int64_t)row * npad;
          v[u] = reinterpret_cast<const int4 *>(src)[c4];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = b0 + u * 256;
        if (i < tot) {
          const bool a = i < totA;
          const int j = a ? i : i - totA;
          const int row = j / q4, c4 = j - row * q4;
          reinterpret_cast<int4 *>((a ? win : fds) + row * rs)[c4] = v[u];
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < QPT; ++u) {
    const int q = t + u * 256;
    if (q < n) has[q] = bq[u] < lq[u];
  }
  for (int q = t; q <= WROWS; q += blockDim.x) hist[q] = 0;
  __syncthreads();
  if (wave == 0) {  // candidate list in chain order
    int nc = 0;
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int q = c0 + lane;
      const bool h = q < n && has[q];
      const unsigned long long m = __ballot(h);
      if (h) clist[nc + popc64(m & ((1ull << lane) - 1ull))] = q;
      nc += popc64(m);
    }
    if (lane == 0) sh_nc = nc;
  }
  __syncthreads();
  const int nC = sh_nc;
  const int half = t & 1;
  int32_t result = len;
  while (k0 < len) {
    const unsigned long long ts1 = dg ? stamp() : 0;
    if (dg) { ts_load += ts1 - ts0; ++nwin; }
    for (int w0 = 0; w0 < nC; w0 += blockDim.x / 2) {
      const int wi = w0 + (t >> 1);
      const bool act = wi < nC;
      const int q = act ? clist[wi] : 0;
      const int32_t *f = FD_LDS ? fds + q * rs : fcur + (int64_t)q * npad;
      auto ss = [&](int row) -> bool {
        const int4 *x4 = reinterpret_cast<const int4 *>(win + row * rs);
        const int4 *f4 = reinterpret_cast<const int4 *>(f);
        int cnt = 0;
        if (act) {
#pragma unroll 8
          for (int i = half; i < q4; i += 2) {
            const int4 a = x4[i], b = f4[i];
            cnt += (a.x >= b.x) + (a.y >= b.y) + (a.z >= b.z) + (a.w >= b.w);
          }
        }
        cnt += __shfl_xor(cnt, 1);
        return cnt >= sm;
      };
      int tw = WROWS;  // not within the window
      if (ss(rows - 1)) {
        int lo = 0, hi = rows - 1;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (ss(mid)) hi = mid;
          else lo = mid + 1;
        }
        tw = lo;
      }
      if (act && half == 0) atomicAdd(&hist[tw], 1);
    }
    __syncthreads();
    // first window row whose running count of T_q reaches SM: one wave,
    // inclusive prefix sum over the (<= 32) histogram bins
    if (wave == 0) {
      int h = lane < rows ? hist[lane] : 0;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(h, off);
        h += lane >= off ? o : 0;
      }
      const unsigned long long hit = __ballot(lane < rows && h >= sm);
      if (lane == 0) sh_res = hit ? (int)__builtin_ctzll(hit) : -1;
    }
    __syncthreads();
    if (dg) ts_comp = stamp();
    if (sh_res >= 0) { result = k0 + sh_res; break; }
    // T not reached in this window (rare): the next one
    k0 += rows;
    rows = min(WROWS, len - k0);
    if (rows <= 0) break;
    load_window<4>(d, win, rs, cs, k0, rows);
    for (int q = t; q <= WROWS; q += blockDim.x) hist[q] = 0;
    __syncthreads();
  }
  if (dg) {
    const unsigned long long te = stamp();
    atomicAdd(&d.diag[DG_SC_LOAD], ts_load);
    atomicAdd(&d.diag[DG_SC_COMPUTE], ts_comp ? ts_comp - ts0 - ts_load : 0);
    atomicAdd(&d.diag[DG_SC_TOTAL], te - ts0);
    atomicAdd(&d.diag[DG_SC_CALLS], 1ull);
    atomicAdd(&d.diag[DG_SC_WINDOWS], nwin);
  }
  if (t == 0) {
    d.Bp[(int64_t)(p ^ 1) * n + c] = result;
    d.B[(int64_t)(r + 1) * n + c] = result;  // history for the per-event pass
    // the last workgroup to finish advances the round (every workgroup has
    // read ST_CUR before it arrives)
    __threadfence();
    const int prev = atomicAdd(&d.state[ST_ARRIVE], 1);
    if (prev == (int)gridDim.x - 1) {
      d.state[ST_ARRIVE] = 0;
      d.state[ST_CUR] = r + 1;
      d.state[ST_ITERS] += 1;
    }
  }
}

size_t scan_lds_bytes(const Dev &d, bool fd_lds) {
  size_t b = (size_t)WROWS * (d.npad + SCAN_PAD) * 4;
  if (fd_lds) b += (size_t)d.n * (d.npad + SCAN_PAD) * 4;
  return b;
}

void configure_round_kernels() {
  (void)hipFuncSetAttribute((const void *)k_scan<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            140 * 1024);
  (void)hipFuncSetAttribute((const void *)k_scan<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            140 * 1024);
  (void)hipFuncSetAttribute((const void *)k_cand_fd, hipFuncAttributeMaxDynamicSharedMemorySize,
                            140 * 1024);
}

// iteration parity p = round & 1 (ITER_BATCH is even, rounds start at 0)
void launch_round_iteration(const Dev &d, int p, hipStream_t s) {
  const size_t wbytes = (size_t)WROWS * (d.npad + 4) * 4;
  k_cand_fd<<<d.n, 512, wbytes, s>>>(d, p);
  const bool fd_lds = scan_lds_bytes(d, true) <= 128 * 1024;
  if (fd_lds)
    k_scan<true><<<d.n, 256, scan_lds_bytes(d, true), s>>>(d, p);
  else
    k_scan<false><<<d.n, 256, scan_lds_bytes(d, false), s>>>(d, p);
}

// ---------------------------------------------------------------------------
// witness tables for DecideFame, once after the loop: W(r) = the candidates
// of round r whose round is exactly r (B[r+1][q] > B[r][q]), in chain order;
// wrow = the row of their firstDescendants in fdc (r * n + q).
__global__ __launch_bounds__(64) void k_wcount(Dev d) {
  const int r = blockIdx.x, lane = threadIdx.x, n = d.n;
  int cnt = 0;
  for (int q = lane; q < n; q += 64) {
    const int32_t b0 = d.B[(int64_t)r * n + q], b1 = d.B[(int64_t)(r + 1) * n + q];
    cnt += (b0 < d.chain_len[q] && b1 > b0) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if (lane == 0) d.wcnt[r] = cnt;
}

__global__ __launch_bounds__(1024) void k_wscan(Dev d, int R) {
  __shared__ int32_t part[1024];
  const int t = threadIdx.x;
  const int per = (R + 1023) / 1024;
  const int lo = min(R, t * per), hi = min(R, lo + per);
  int32_t s = 0;
  for (int r = lo; r < hi; ++r) s += d.wcnt[r];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int32_t a = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += a;
    __syncthreads();
  }
  int32_t run = part[t] - s;
  for (int r = lo; r < hi; ++r) {
    d.wofs[r] = run;
    run += d.wcnt[r];
  }
  if (t == 1023) d.wofs[R] = part[1023];
}

__global__ __launch_bounds__(64) void k_wfill(Dev d) {
  const int r = blockIdx.x, lane = threadIdx.x, n = d.n;
  int32_t j = d.wofs[r];
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int q = c0 + lane;
    int32_t b0 = 0;
    bool w = false;
    if (q < n) {
      b0 = d.B[(int64_t)r * n + q];
      w = b0 < d.chain_len[q] && d.B[(int64_t)(r + 1) * n + q] > b0;
    }
    const unsigned long long m = __ballot(w);
    if (w) {
      const int32_t k = j + popc64(m & ((1ull << lane) - 1ull));
      d.wids[k] = d.chain_ids[d.chain_start[q] + b0];
      d.wrow[k] = r * n + q;
    }
    j += popc64(m);
  }
}

void launch_witness_tables(const Dev &d, int R, hipStream_t s) {
  if (R <= 0) return;
  k_wcount<<<R, 64, 0, s>>>(d);
  k_wscan<<<1, 1024, 0, s>>>(d, R);
  k_wfill<<<R, 64, 0, s>>>(d);
}

// ---------------------------------------------------------------------------
// per-event round / witness from the boundary table (DivideRounds output,
// hashgraph.go:782-827): round(x) = max r with B[r][c] <= k.
__global__ void k_assign(Dev d) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int32_t R = d.state[ST_ROUNDS];
  const int32_t c = d.creator[e], k = d.index[e];
  const int n = d.n;
  int lo = 0, hi = R - 1;  // B[0][c] = 0 <= k
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d.B[(int64_t)mid * n + c] <= k) lo = mid;
    else hi = mid - 1;
  }
  d.round[e] = lo;
  const bool w = d.B[(int64_t)lo * n + c] == k;
  d.witness[e] = w ? 1 : 0;
  d.fame[e] = w ? 0 : -1;
  d.rr[e] = UNSET;
  d.cons_pos[e] = -1;
}

void launch_assign_rounds(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  k_assign<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d);
}

// firstDescendants row of one event (bh_get_coordinates)
__global__ void k_fd_row(Dev d, int64_t e, int32_t *out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d.n) return;
  const int32_t cw = d.creator[e], kw = d.index[e];
  if (cw == c) { out[c] = kw; return; }
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  int32_t res = FD_NONE;
  for (int32_t k = 0; k < len; ++k)
    if (d.la[(int64_t)(cs + k) * d.npad + cw] >= kw) { res = k; break; }
  out[c] = res;
}

void launch_fd_row(const Dev &d, int64_t e, int32_t *out, hipStream_t s) {
  k_fd_row<<<(d.n + 63) / 64, 64, 0, s>>>(d, e, out);
}

}  // namespace bh
