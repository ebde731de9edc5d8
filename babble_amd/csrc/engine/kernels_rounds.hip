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

// load rows [k0, k0+rows) of chain c (global rows cs+k) into LDS, stride rs
__device__ __forceinline__ void load_window(const Dev &d, int32_t *win, int rs, int32_t cs,
                                            int32_t k0, int rows) {
  const int q4 = d.npad / 4;
  for (int q = threadIdx.x; q < rows * q4; q += blockDim.x) {
    const int row = q / q4, c4 = q - row * q4;
    reinterpret_cast<int4 *>(win + row * rs)[c4] =
        reinterpret_cast<const int4 *>(d.la + (int64_t)(cs + k0 + row) * d.npad)[c4];
  }
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(512) void k_cand_fd(Dev d, int p) {
  extern __shared__ __attribute__((aligned(16))) int32_t rsm[];
  __shared__ int32_t bcur[MAXN], bprev[MAXN], lens[MAXN];
  __shared__ int32_t wsel[MAXN];   // W(r-1) compaction: slot of chain q, -1 if not a witness
  __shared__ int32_t sh_ncand, sh_nw, sh_open;
  __shared__ int8_t open[MAXN];
  if (d.state[ST_DONE]) return;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = d.n, npad = d.npad, rs = npad + 4;
  const int c = blockIdx.x;
  const int32_t *Bp = d.Bp + (int64_t)p * n;          // B[r]
  const int32_t *Bq = d.Bp + (int64_t)(p ^ 1) * n;    // B[r-1] (unused at r = 0)
  const int r = d.state[ST_CUR];
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  int32_t k0 = Bp[c];
  int rows = min(WROWS, max(0, len - k0));
  int32_t *win = rsm;  // [WROWS][rs]
  const bool dg = d.diag != nullptr && t == 0;
  const unsigned long long tr0 = dg ? stamp() : 0;
  unsigned long long tr1 = 0, tr2 = 0, nfdw = 0;
  load_window(d, win, rs, cs, k0, rows);
  if (t == 0) { sh_ncand = 0; sh_nw = 0; }
  for (int q = t; q < n; q += blockDim.x) {
    bcur[q] = Bp[q];
    bprev[q] = Bq[q];
    lens[q] = d.chain_len[q];
  }
  __syncthreads();
  if (dg) tr1 = stamp();
  // ---- W(r-1) = candidates of r-1 whose round is exactly r-1 ----
  if (r > 0) {
    if (wave == 0) {
      int nw = 0;
      for (int c0 = 0; c0 < n; c0 += 64) {
        const int q = c0 + lane;
        const bool isw = q < n && bprev[q] < lens[q] && bcur[q] > bprev[q];
        const unsigned long long m = __ballot(isw);
        if (q < n) wsel[q] = isw ? nw + popc64(m & ((1ull << lane) - 1ull)) : -1;
        nw += popc64(m);
      }
      if (lane == 0) sh_nw = nw;
    }
    __syncthreads();
    const int32_t wb = d.wofs[r - 1];
    const int32_t *fprev = d.fdc + (int64_t)(p ^ 1) * n * npad;
    for (int q = t; q < n; q += blockDim.x) {
      const int j = wsel[q];
      if (j < 0) continue;
      d.fdw[(int64_t)(wb + j) * npad + c] = fprev[(int64_t)q * npad + c];
      if (c == 0) {
        d.wids[wb + j] = d.candp[(p ^ 1) * n + q];
        for (int i = n; i < npad; ++i) d.fdw[(int64_t)(wb + j) * npad + i] = FD_NONE;
      }
    }
    if (c == 0 && t == 0) {
      d.wcnt[r - 1] = sh_nw;
      d.wofs[r] = wb + sh_nw;
    }
  }
  // ---- candidates of round r ----
  for (int q = t; q < n; q += blockDim.x) {
    const bool has = bcur[q] < lens[q];
    open[q] = has ? 1 : 0;
    if (has) atomicAdd(&sh_ncand, 1);
    if (c == 0) d.candp[p * n + q] = has ? d.chain_ids[d.chain_start[q] + bcur[q]] : -1;
  }
  __syncthreads();
  if (sh_ncand == 0) {
    if (c == 0 && t == 0) { d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; }
    return;
  }
  // offset of W(r): block 0 publishes it in this launch, so use the local copy
  const int32_t wofs_r = r > 0 ? d.wofs[r - 1] + sh_nw : 0;
  if (r + 1 >= d.R_cap || (int64_t)wofs_r + n > d.W_cap) {
    if (c == 0 && t == 0) { d.state[ST_ERR] = 1; d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; }
    return;
  }
  if (dg) tr2 = stamp();
  // ---- firstDescendants column c of every candidate, window by window ----
  int32_t *fcur = d.fdc + (int64_t)p * n * npad;
  for (int q = t; q < n; q += blockDim.x)
    if (open[q] && q == c) { fcur[(int64_t)q * npad + c] = bcur[q]; open[q] = 0; }
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
    load_window(d, win, rs, cs, k0, rows);
    __syncthreads();
  }
  if (c == 0)  // padding columns never match
    for (int q = t; q < n; q += blockDim.x)
      for (int i = n; i < npad; ++i) fcur[(int64_t)q * npad + i] = FD_NONE;
  if (dg) {
    const unsigned long long te = stamp();
    atomicAdd(&d.diag[DG_RF_P1], tr1 - tr0);
    atomicAdd(&d.diag[DG_RF_ROWS], tr2 - tr1);
    atomicAdd(&d.diag[DG_RF_FD], te - tr2);
    atomicAdd(&d.diag[DG_RF_TOTAL], te - tr0);
    atomicAdd(&d.diag[DG_RF_CALLS], 1ull);
    atomicAdd(&d.diag[DG_RF_FDWIN], nfdw);
  }
}

// ---------------------------------------------------------------------------
// Two lanes per candidate (each half of the columns, combined with a lane
// swap); T_q by binary search over the window; B[r+1][c] = SM-th smallest T_q.
template <bool FD_LDS>
__global__ __launch_bounds__(256) void k_scan(Dev d, int p) {
  extern __shared__ __attribute__((aligned(16))) int32_t ssm[];
  __shared__ int32_t hist[WROWS + 1];
  __shared__ int32_t clist[MAXN];
  __shared__ int32_t sh_res, sh_nc;
  if (d.state[ST_DONE]) return;
  const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = d.n, npad = d.npad, sm = d.sm, rs = npad + 4;
  const int32_t *Bp = d.Bp + (int64_t)p * n;
  const int32_t *fcur = d.fdc + (int64_t)p * n * npad;
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  int32_t *win = ssm;                  // [WROWS][rs]
  int32_t *fds = ssm + WROWS * rs;     // [n][rs] when FD_LDS (by candidate slot)
  int32_t k0 = Bp[c];
  const int q4 = npad / 4;
  const int h4 = (q4 + 1) / 2;         // int4 columns per half
  const bool dg = d.diag != nullptr && t == 0;
  const unsigned long long ts0 = dg ? stamp() : 0;
  unsigned long long ts_load = 0, ts_comp = 0, nwin = 0;
  // candidate list (chains with B[r][q] < len)
  if (wave == 0) {
    int nc = 0;
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int q = c0 + lane;
      const bool has = q < n && Bp[q] < d.chain_len[q];
      const unsigned long long m = __ballot(has);
      if (has) clist[nc + popc64(m & ((1ull << lane) - 1ull))] = q;
      nc += popc64(m);
    }
    if (lane == 0) sh_nc = nc;
  }
  if (FD_LDS) {  // all n rows: chains without a candidate are never read
    for (int q = t; q < n * q4; q += blockDim.x) {
      const int w = q / q4, c4 = q - w * q4;
      reinterpret_cast<int4 *>(fds + w * rs)[c4] =
          reinterpret_cast<const int4 *>(fcur + (int64_t)w * npad)[c4];
    }
  }
  __syncthreads();
  const int nC = sh_nc;
  const int half = t & 1;
  const int i0 = half * h4, i1 = min(q4, i0 + h4);
  int32_t result = len;
  while (k0 < len) {
    const int rows = min(WROWS, len - k0);
    load_window(d, win, rs, cs, k0, rows);
    for (int q = t; q <= WROWS; q += blockDim.x) hist[q] = 0;
    __syncthreads();
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
          for (int i = i0; i < i1; ++i) {
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
    if (t == 0) {
      int acc = 0, res = -1;
      for (int q = 0; q < rows; ++q) {
        acc += hist[q];
        if (acc >= sm) { res = q; break; }
      }
      sh_res = res;
    }
    __syncthreads();
    if (dg) ts_comp = stamp();
    if (sh_res >= 0) { result = k0 + sh_res; break; }
    k0 += rows;
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
    const int r = d.state[ST_CUR];
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
  size_t b = (size_t)WROWS * (d.npad + 4) * 4;
  if (fd_lds) b += (size_t)d.n * (d.npad + 4) * 4;
  return b;
}

void configure_round_kernels() {
  (void)hipFuncSetAttribute((const void *)k_scan<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            140 * 1024);
  (void)hipFuncSetAttribute((const void *)k_scan<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            140 * 1024);
  (void)hipFuncSetAttribute((const void *)k_cand_fd, hipFuncAttributeMaxDynamicSharedMemorySize,
                            120 * 1024);
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
