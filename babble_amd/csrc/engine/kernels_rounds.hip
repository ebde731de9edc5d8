// kernels_rounds.hip -- rounds, witnesses and witness firstDescendants.
//
// Reference: _round (hashgraph.go:205-278): round(x) = pr + [#{w in W(pr):
// stronglySee(x, w)} >= SM], pr = max(round(sp), round(op)); witness
// (hashgraph.go:281-296): round(x) > round(sp(x)); _stronglySee
// (hashgraph.go:172-191); firstDescendants (hashgraph.go:510-544).
//
// Batch closed form (proof in DESIGN.md; the oracle checks it in tests):
// round(x) >= r+1  <=>  x strongly sees >= SM witnesses of round r.  LA is
// non-decreasing along a creator's chain, so on every chain c the events of
// round >= r are a suffix starting at index B[r][c]:
//   W(r)      = candidates (c, B[r][c]) whose round is exactly r,
//   B[r+1][c] = first k >= B[r][c] whose event strongly sees SM of W(r).
// The serial work is one step per ROUND (not per event or DAG level), two
// launches per step, one workgroup per chain c in each:
//   k_resolve_fd  every workgroup resolves W(r) from B[r] (redundantly --
//                 cheaper than a third launch) and writes column c of the
//                 witnesses' firstDescendants rows: the first event of chain c
//                 seeing w, by binary search in an LDS window of chain c
//                 starting at B[r][c] (descendants of a round-r witness have
//                 round >= r);
//   k_scan        stages the FD rows of W(r) and the same window in LDS; each
//                 thread owns one witness w and binary-searches T_w, the first
//                 window row that strongly sees w (monotone along the chain);
//                 B[r+1][c] = the SM-th smallest T_w.  The last workgroup to
//                 finish advances the round index.
// All kernels read the round index from device state, so a captured graph
// of iterations replays without host involvement; they exit once ST_DONE.
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
__global__ __launch_bounds__(512) void k_resolve_fd(Dev d) {
  extern __shared__ __attribute__((aligned(16))) int32_t rsm[];
  __shared__ int32_t cand[MAXN];   // candidate event id of chain c, -1 if none
  __shared__ int32_t bsh[MAXN];    // B[r][c]
  __shared__ int8_t flag[MAXN];    // 0 none, 1 witness, 2 unresolved, 3 not a witness
  __shared__ int32_t urow[MAXN];   // exact path: row of x's last ancestor on chain i
  __shared__ int32_t wlist[MAXN];  // W(r), chain order
  __shared__ int32_t sh_cnt, sh_x, sh_ncand, sh_nflag, sh_nw;
  if (d.state[ST_DONE]) return;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nwaves = blockDim.x >> 6;
  const int n = d.n, npad = d.npad, rs = npad + 4;
  const int c = blockIdx.x;
  const int r = d.state[ST_CUR];
  const int32_t *Br = d.B + (int64_t)r * n;
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  const int32_t k0 = Br[c];
  const int rows = min(WROWS, max(0, len - k0));
  int32_t *win = rsm;
  // the FD search window does not depend on the resolution: issue it first
  load_window(d, win, rs, cs, k0, rows);
  if (t == 0) { sh_ncand = 0; sh_nflag = 0; }
  __syncthreads();
  for (int q = t; q < n; q += blockDim.x) {
    const int32_t b = Br[q];
    const bool has = b < d.chain_len[q];
    cand[q] = has ? d.chain_ids[d.chain_start[q] + b] : -1;
    bsh[q] = b;
    flag[q] = has ? 1 : 0;
    if (has) atomicAdd(&sh_ncand, 1);
  }
  __syncthreads();
  if (sh_ncand == 0) {
    if (c == 0 && t == 0) { d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; }
    return;
  }
  if (r + 1 >= d.R_cap || (int64_t)d.wofs[r] + n > d.W_cap) {
    if (c == 0 && t == 0) { d.state[ST_ERR] = 1; d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; }
    return;
  }
  // A candidate is surely a witness unless SM other candidates are its
  // ancestors (stronglySee implies ancestry).
  for (int q = wave; q < n; q += nwaves) {
    if (cand[q] < 0) continue;
    const int32_t *row = d.la + (int64_t)d.epos[cand[q]] * npad;
    int cnt = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      const bool ok = i < n && i != q && cand[i] >= 0 && row[i] >= bsh[i];
      cnt += popc64(__ballot(ok));
    }
    if (lane == 0 && cnt >= d.sm) { flag[q] = 2; atomicAdd(&sh_nflag, 1); }
  }
  __syncthreads();
  if (sh_nflag > 0) {
    // exact resolution in topological order: x is not a witness iff it
    // strongly sees SM witnesses of this round; stronglySee(x, w) from LA
    // alone: x's last ancestors on >= SM chains see w.
    for (;;) {
      if (t == 0) {
        int best = -1;
        for (int q = 0; q < n; ++q)
          if (flag[q] == 2 && (best < 0 || cand[q] < cand[best])) best = q;
        sh_x = best;
        sh_cnt = 0;
      }
      __syncthreads();
      const int cx = sh_x;
      if (cx < 0) break;
      const int32_t x = cand[cx];
      const int32_t *xrow = d.la + (int64_t)d.epos[x] * npad;
      for (int i = t; i < n; i += blockDim.x) {
        const int32_t k = xrow[i];
        urow[i] = k >= 0 ? d.chain_start[i] + k : -1;
      }
      __syncthreads();
      for (int q = wave; q < n; q += nwaves) {
        if (q == cx || flag[q] != 1) continue;
        if (xrow[q] < bsh[q]) continue;  // witness cand[q] is not an ancestor of x
        int cnt = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {
          const int i = i0 + lane;
          const bool ok = i < n && urow[i] >= 0 && d.la[(int64_t)urow[i] * npad + q] >= bsh[q];
          cnt += popc64(__ballot(ok));
        }
        if (lane == 0 && cnt >= d.sm) atomicAdd(&sh_cnt, 1);
      }
      __syncthreads();
      if (t == 0) flag[cx] = sh_cnt >= d.sm ? 3 : 1;
      __syncthreads();
    }
  }
  // W(r) in chain order
  if (wave == 0) {
    int nw = 0;
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int q = c0 + lane;
      const bool isw = q < n && flag[q] == 1;
      const unsigned long long m = __ballot(isw);
      const int before = popc64(m & ((1ull << lane) - 1ull));
      if (isw) wlist[nw + before] = cand[q];
      nw += popc64(m);
    }
    if (lane == 0) sh_nw = nw;
  }
  __syncthreads();
  const int nW = sh_nw;
  const int32_t base = d.wofs[r];
  if (c == 0) {
    for (int j = t; j < nW; j += blockDim.x) {
      d.wids[base + j] = wlist[j];
      for (int i = n; i < npad; ++i) d.fdw[(int64_t)(base + j) * npad + i] = FD_NONE;
    }
    if (t == 0) {
      d.wcnt[r] = nW;
      d.wofs[r + 1] = base + nW;
      d.state[ST_FLAGGED] += sh_nflag;
    }
  }
  // firstDescendants column c: first row of chain c with LA[.][cw] >= kw
  for (int j = t; j < nW; j += blockDim.x) {
    const int32_t w = wlist[j];
    const int32_t cw = d.creator[w], kw = d.index[w];
    int32_t res = FD_NONE;
    if (cw == c) {
      res = kw;
    } else if (rows > 0 && win[(rows - 1) * rs + cw] >= kw) {
      int lo = 0, hi = rows - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (win[mid * rs + cw] >= kw) hi = mid;
        else lo = mid + 1;
      }
      res = k0 + lo;
    } else {
      for (int32_t k = k0 + rows; k < len; ++k)  // beyond the window (rare)
        if (d.la[(int64_t)(cs + k) * npad + cw] >= kw) { res = k; break; }
    }
    d.fdw[(int64_t)(base + j) * npad + c] = res;
  }
}

// ---------------------------------------------------------------------------
template <bool FD_LDS>
__global__ __launch_bounds__(256) void k_scan(Dev d) {
  extern __shared__ __attribute__((aligned(16))) int32_t ssm[];
  __shared__ int32_t hist[WROWS + 1];
  __shared__ int32_t sh_res;
  if (d.state[ST_DONE]) return;
  const int r = d.state[ST_CUR];
  const int c = blockIdx.x, t = threadIdx.x;
  const int n = d.n, npad = d.npad, sm = d.sm, rs = npad + 4;
  const int32_t nW = d.wcnt[r], base = d.wofs[r];
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  int32_t *win = ssm;                  // [WROWS][rs]
  int32_t *fds = ssm + WROWS * rs;     // [nW][rs] when FD_LDS
  int32_t k0 = d.B[(int64_t)r * n + c];
  const int q4 = npad / 4;
  if (FD_LDS) {
    for (int q = t; q < nW * q4; q += blockDim.x) {
      const int w = q / q4, c4 = q - w * q4;
      reinterpret_cast<int4 *>(fds + w * rs)[c4] =
          reinterpret_cast<const int4 *>(d.fdw + (int64_t)(base + w) * npad)[c4];
    }
  }
  int32_t result = len;
  while (k0 < len) {
    const int rows = min(WROWS, len - k0);
    load_window(d, win, rs, cs, k0, rows);
    for (int q = t; q <= WROWS; q += blockDim.x) hist[q] = 0;
    __syncthreads();
    // T_w: first window row that strongly sees w (binary search; monotone)
    for (int w = t; w < nW; w += blockDim.x) {
      const int32_t *f = FD_LDS ? fds + w * rs : d.fdw + (int64_t)(base + w) * npad;
      auto ss = [&](int row) {
        const int4 *x4 = reinterpret_cast<const int4 *>(win + row * rs);
        const int4 *f4 = reinterpret_cast<const int4 *>(f);
        int cnt = 0;
        for (int i = 0; i < q4; ++i) {
          const int4 a = x4[i], b = f4[i];
          cnt += (a.x >= b.x) + (a.y >= b.y) + (a.z >= b.z) + (a.w >= b.w);
        }
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
      atomicAdd(&hist[tw], 1);
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
    if (sh_res >= 0) { result = k0 + sh_res; break; }
    k0 += rows;
    __syncthreads();
  }
  if (t == 0) {
    d.B[(int64_t)(r + 1) * n + c] = result;
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
  (void)hipFuncSetAttribute((const void *)k_resolve_fd, hipFuncAttributeMaxDynamicSharedMemorySize,
                            100 * 1024);
}

void launch_round_iteration(const Dev &d, hipStream_t s) {
  k_resolve_fd<<<d.n, 512, (size_t)WROWS * (d.npad + 4) * 4, s>>>(d);
  const bool fd_lds = scan_lds_bytes(d, true) <= 128 * 1024;
  if (fd_lds)
    k_scan<true><<<d.n, 256, scan_lds_bytes(d, true), s>>>(d);
  else
    k_scan<false><<<d.n, 256, scan_lds_bytes(d, false), s>>>(d);
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
