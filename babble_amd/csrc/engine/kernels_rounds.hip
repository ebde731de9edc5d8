// kernels_rounds.hip -- rounds, witnesses and witness firstDescendants.
//
// Reference: _round (hashgraph.go:205-278): round(x) = pr + [#{w in W(pr):
// stronglySee(x, w)} >= SM], pr = max(round(sp), round(op)); witness
// (hashgraph.go:281-296): round(x) > round(sp(x)); _stronglySee
// (hashgraph.go:172-191).
//
// Batch closed form used here (proof in DESIGN.md, checked against the
// oracle by tests): round(x) >= r+1  <=>  x strongly sees >= SM witnesses
// of round r.  LA is non-decreasing along a creator's chain, so for every
// chain c the events of round >= r form a suffix starting at B[r][c], and
//   B[r+1][c] = first k >= B[r][c] whose event strongly sees SM of W(r),
//   W(r)      = the candidates (c, B[r][c]) whose round is exactly r.
// The serial work is therefore one step per ROUND (not per event or per DAG
// level); each step is three launches:
//   k_resolve  (1 workgroup) candidates -> W(r), exact check for the rare
//              candidate that could strongly see SM other candidates;
//   k_fd       (one workgroup per chain c) firstDescendants column c of
//              every witness of W(r): the first event of chain c that sees w;
//   k_scan     (one workgroup per chain c) B[r+1][c] by window + binary
//              search, the FD rows of W(r) staged in LDS.
// Kernels read the round index from device state so a captured graph of
// iterations replays without host involvement; all exit once ST_DONE is set.
#include "engine.h"

namespace bh {

constexpr int MAXN = 1024;  // participants supported by the LDS tables below

__device__ __forceinline__ int popc64(unsigned long long x) { return __popcll(x); }

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_resolve(Dev d) {
  __shared__ int32_t cand[MAXN];   // candidate event id of chain c, -1 if none
  __shared__ int32_t bsh[MAXN];    // B[r][c]
  __shared__ int8_t flag[MAXN];    // 0 none, 1 witness, 2 unresolved, 3 not a witness
  __shared__ int32_t urow[MAXN];   // exact path: row of x's last ancestor on chain i
  __shared__ int32_t sh_cnt, sh_x, sh_ncand, sh_nflag;
  if (d.state[ST_DONE]) return;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nwaves = blockDim.x >> 6;
  const int n = d.n;
  const int r = d.state[ST_NEXT];
  if (t == 0) { sh_ncand = 0; sh_nflag = 0; }
  __syncthreads();
  const int32_t *Br = d.B + (int64_t)r * n;
  for (int c = t; c < n; c += blockDim.x) {
    const int32_t b = Br[c];
    const bool has = b < d.chain_len[c];
    cand[c] = has ? d.chain_ids[d.chain_start[c] + b] : -1;
    bsh[c] = b;
    flag[c] = has ? 1 : 0;
    if (has) atomicAdd(&sh_ncand, 1);
  }
  __syncthreads();
  if (sh_ncand == 0) {
    if (t == 0) { d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; }
    return;
  }
  if (r + 1 >= d.R_cap || (int64_t)d.wofs[r] + n > d.W_cap) {
    if (t == 0) { d.state[ST_ERR] = 1; d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; }
    return;
  }
  // A candidate is surely a witness unless SM other candidates are its
  // ancestors (stronglySee implies ancestry).
  for (int c = wave; c < n; c += nwaves) {
    if (cand[c] < 0) continue;
    const int32_t *row = d.la + (int64_t)d.epos[cand[c]] * d.npad;
    int cnt = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      const bool ok = i < n && i != c && cand[i] >= 0 && row[i] >= bsh[i];
      cnt += popc64(__ballot(ok));
    }
    if (lane == 0 && cnt >= d.sm) { flag[c] = 2; atomicAdd(&sh_nflag, 1); }
  }
  __syncthreads();
  if (sh_nflag > 0) {
    // exact resolution in topological order: x is not a witness iff it
    // strongly sees SM witnesses of this round.  stronglySee(x, w) is
    // evaluated from LA alone: x's last ancestors on >= SM chains see w.
    for (;;) {
      if (t == 0) {
        int best = -1;
        for (int c = 0; c < n; ++c)
          if (flag[c] == 2 && (best < 0 || cand[c] < cand[best])) best = c;
        sh_x = best;
        sh_cnt = 0;
      }
      __syncthreads();
      const int cx = sh_x;
      if (cx < 0) break;
      const int32_t x = cand[cx];
      const int32_t *xrow = d.la + (int64_t)d.epos[x] * d.npad;
      for (int i = t; i < n; i += blockDim.x) {
        const int32_t k = xrow[i];
        urow[i] = k >= 0 ? d.chain_start[i] + k : -1;
      }
      __syncthreads();
      for (int c = wave; c < n; c += nwaves) {
        if (c == cx || flag[c] != 1) continue;
        if (xrow[c] < bsh[c]) continue;  // witness cand[c] is not an ancestor of x
        int cnt = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {
          const int i = i0 + lane;
          const bool ok = i < n && urow[i] >= 0 && d.la[(int64_t)urow[i] * d.npad + c] >= bsh[c];
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
    const int32_t base = d.wofs[r];
    int nw = 0;
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int c = c0 + lane;
      const bool isw = c < n && flag[c] == 1;
      const unsigned long long m = __ballot(isw);
      const int before = popc64(m & ((1ull << lane) - 1ull));
      if (isw) d.wids[base + nw + before] = cand[c];
      nw += popc64(m);
    }
    if (lane == 0) {
      d.wcnt[r] = nw;
      d.wofs[r + 1] = base + nw;
      d.state[ST_CUR] = r;
      d.state[ST_NEXT] = r + 1;
      d.state[ST_ITERS] += 1;
      d.state[ST_FLAGGED] += sh_nflag;
    }
  }
}

// ---------------------------------------------------------------------------
// firstDescendants column c of the witnesses of W(r): the first event of
// chain c whose lastAncestor on the witness's chain reaches the witness
// (the closed form of updateAncestorFirstDescendant, hashgraph.go:510-544).
// Every descendant of a round-r witness has round >= r, so the search starts
// at B[r][c].
__global__ __launch_bounds__(256) void k_fd(Dev d) {
  if (d.state[ST_DONE]) return;
  const int r = d.state[ST_CUR];
  const int c = blockIdx.x;
  const int n = d.n;
  const int32_t nW = d.wcnt[r], base = d.wofs[r];
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  const int32_t start = d.B[(int64_t)r * n + c];
  for (int j = threadIdx.x; j < nW; j += blockDim.x) {
    const int32_t w = d.wids[base + j];
    const int32_t cw = d.creator[w], kw = d.index[w];
    int32_t res = FD_NONE;
    if (cw == c) {
      res = kw;
    } else {
      for (int32_t k = start; k < len; k += 8) {
        int32_t v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
          v[q] = (k + q < len) ? d.la[(int64_t)(cs + k + q) * d.npad + cw] : -1;
        int hit = -1;
#pragma unroll
        for (int q = 7; q >= 0; --q)
          if (v[q] >= kw) hit = q;
        if (hit >= 0) { res = k + hit; break; }
      }
    }
    d.fdw[(int64_t)(base + j) * d.npad + c] = res;
  }
  // padding columns never match
  if (c == 0)
    for (int j = threadIdx.x; j < nW; j += blockDim.x)
      for (int i = n; i < d.npad; ++i) d.fdw[(int64_t)(base + j) * d.npad + i] = FD_NONE;
}

// ---------------------------------------------------------------------------
// B[r+1][c]: first event of chain c (from B[r][c]) that strongly sees SM
// witnesses of W(r).  Window of SCAN_WIN rows in LDS, test the last row,
// then binary search (monotone along the chain).
template <bool FD_LDS>
__global__ __launch_bounds__(256) void k_scan(Dev d) {
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  __shared__ int32_t wss[MAXN];
  __shared__ int32_t sh_total;
  if (d.state[ST_DONE]) return;
  const int r = d.state[ST_CUR];
  const int c = blockIdx.x, t = threadIdx.x;
  const int n = d.n, npad = d.npad, sm = d.sm;
  const int32_t nW = d.wcnt[r], base = d.wofs[r];
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  const int fstride = n + 1;  // padded LDS row stride of the FD rows
  int32_t *win = smem;                                     // [SCAN_WIN][npad]
  int32_t *fds = smem + SCAN_WIN * npad;                   // [nW][n+1] when FD_LDS
  if (FD_LDS) {
    for (int idx = t; idx < nW * n; idx += blockDim.x) {
      const int w = idx / n, i = idx - w * n;
      fds[w * fstride + i] = d.fdw[(int64_t)(base + w) * npad + i];
    }
  }
  // thread -> (witness, column segment) mapping for one probe
  int seg = 256 / (nW > 0 ? nW : 1);
  if (seg < 1) seg = 1;
  if (seg > n) seg = n;
  const int colw = (n + seg - 1) / seg;

  auto probe = [&](int row) -> bool {  // does window row `row` strongly see SM of W(r)?
    for (int w = t; w < nW; w += blockDim.x) wss[w] = 0;
    if (t == 0) sh_total = 0;
    __syncthreads();
    const int32_t *x = win + row * npad;
    for (int p = t; p < nW * seg; p += blockDim.x) {
      const int w = p / seg, s = p - w * seg;
      const int i0 = s * colw, i1 = min(n, i0 + colw);
      int cnt = 0;
      if (FD_LDS) {
        const int32_t *f = fds + w * fstride;
        for (int i = i0; i < i1; ++i) cnt += x[i] >= f[i];
      } else {
        const int32_t *f = d.fdw + (int64_t)(base + w) * npad;
        for (int i = i0; i < i1; ++i) cnt += x[i] >= f[i];
      }
      if (cnt) atomicAdd(&wss[w], cnt);
    }
    __syncthreads();
    int mine = 0;
    for (int w = t; w < nW; w += blockDim.x) mine += wss[w] >= sm;
    if (mine) atomicAdd(&sh_total, mine);
    __syncthreads();
    const bool res = sh_total >= sm;
    __syncthreads();
    return res;
  };

  int32_t k0 = d.B[(int64_t)r * n + c];
  int32_t result = len;
  while (k0 < len) {
    const int rows = min(SCAN_WIN, len - k0);
    __syncthreads();
    const int4 *src = reinterpret_cast<const int4 *>(d.la + (int64_t)(cs + k0) * npad);
    int4 *dst = reinterpret_cast<int4 *>(win);
    for (int q = t; q < rows * npad / 4; q += blockDim.x) dst[q] = src[q];
    __syncthreads();
    if (probe(rows - 1)) {
      int lo = 0, hi = rows - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (probe(mid)) hi = mid;
        else lo = mid + 1;
      }
      result = k0 + lo;
      break;
    }
    k0 += rows;
  }
  if (t == 0) d.B[(int64_t)(r + 1) * n + c] = result;
}

void configure_round_kernels() {
  (void)hipFuncSetAttribute((const void *)k_scan<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            120 * 1024);
  (void)hipFuncSetAttribute((const void *)k_scan<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            120 * 1024);
}

void launch_round_iteration(const Dev &d, hipStream_t s) {
  k_resolve<<<1, 1024, 0, s>>>(d);
  k_fd<<<d.n, 256, 0, s>>>(d);
  const size_t win_bytes = (size_t)SCAN_WIN * d.npad * 4;
  const size_t fd_bytes = (size_t)d.n * (d.n + 1) * 4;
  if (win_bytes + fd_bytes <= 120 * 1024)
    k_scan<true><<<d.n, 256, win_bytes + fd_bytes, s>>>(d);
  else
    k_scan<false><<<d.n, 256, win_bytes, s>>>(d);
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
