// kernels_fame.hip -- DecideFame (hashgraph.go:852-947) for every round at once.
//
// For a witness x of round r the vote of y in W(j) is
//   j = r+1 : see(y, x)                        (hashgraph.go:879-884)
//   j > r+1 : majority of the votes of the W(j-1) witnesses y strongly sees
//             (yays >= nays -> yes, hashgraph.go:886-911); in a normal round
//             (diff % n != 0) t >= SM decides x's fame and ends x's loop;
//             in a coin round t >= SM keeps the vote, else y's middle byte
//             (hashgraph.go:913-928, middleBit :1526-1535).
// Votes depend only on the DAG, not on the order the Go code visits the map
// entries, so every round is decided independently: one workgroup per round
// r keeps the votes of all x in W(r) as bitsets over the voters (n/64 words),
// and tallies with popcount(S_j[y] & V_{j-1}[x]), where S_j[y] is the bitset
// of the W(j-1) witnesses y strongly sees.  For n <= 128 S_j comes from the
// round loop's ballots (k_fame_masks, below), for n <= 512 from the wide
// loop's chain masks (same kernel, 512-bit masks); for larger n it is an
// n x n x n integer compare-and-count, register-tiled 8x8 per thread over
// LA rows (voters) and firstDescendants rows (voted) (k_fame).  The
// workgroup then publishes the round's decided flag, its famous count and
// min over famous witnesses of LA (what DecideRoundReceived needs,
// hashgraph.go:968-1001).
#include "engine.h"

namespace bh {

// DecideFame for n > 128 (the k_round / k_round_wide path, where the round
// loop keeps no ballots): S_j recomputed from LA / FD rows read from HBM
__global__ __launch_bounds__(256) void k_fame(Dev d, int32_t R, int32_t r0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  const int r = r0 + (int)blockIdx.x, t = threadIdx.x, nt = blockDim.x;
  const int n = d.n, npad = d.npad, sm = d.sm;
  const int WW = (n + 63) >> 6;       // words per voter bitset
  // carve
  unsigned long long *Vp = reinterpret_cast<unsigned long long *>(fsm);
  unsigned long long *Vc = Vp + n * WW;
  unsigned long long *S = Vc + n * WW;
  int32_t *xs = reinterpret_cast<int32_t *>(S + n * WW);  // W(r) event ids
  int32_t *xc = xs + n;    // creator of x
  int32_t *xk = xc + n;    // index of x
  int32_t *dec = xk + n;   // 0 undecided, 1 famous, 2 not famous
  int32_t *nd = dec + n;   // decisions of the current j (bit0 yes, bit1 no)
  int32_t *rid = nd + n;   // [3][n] chain-major rows: W(r) (kept), then W(j-1) / W(j) alternating
  int32_t *misc = rid + 3 * n;  // [0] undecided count, [1] error
  const int32_t *fdrows = d.fd;

  const int32_t nx = d.wcnt[r], xb = d.wofs[r];
  for (int i = t; i < nx; i += nt) {
    const int32_t e = d.wids[xb + i];
    xs[i] = e;
    xc[i] = d.creator[e];
    xk[i] = d.index[e];
    dec[i] = 0;
    rid[i] = d.wrow[xb + i];  // rows of W(r), for minLA at the end
  }
  if (t == 0) { misc[0] = nx; misc[1] = 0; }
  __syncthreads();
  int cur = 1;  // rid[cur * n ..] (cur = 1 or 2): rows of the latest W(j)

  if (r + 1 < R) {
    // ---- j = r+1: vote = see(y, x) = LA[y][creator(x)] >= index(x) ----
    int32_t ny = d.wcnt[r + 1], yb = d.wofs[r + 1];
    for (int i = t; i < ny; i += nt) rid[n + i] = d.wrow[yb + i];
    for (int i = t; i < nx * WW; i += nt) Vp[i] = 0ull;
    __syncthreads();
    for (int p = t; p < nx * ny; p += nt) {
      const int x = p / ny, y = p - x * ny;
      const int32_t a = d.la[(int64_t)rid[n + y] * npad + xc[x]];
      if (a >= xk[x]) atomicOr(&Vp[x * WW + (y >> 6)], 1ull << (y & 63));
    }
    __syncthreads();
    // ---- j >= r+2 ----
    for (int j = r + 2; j < R; ++j) {
      if (misc[0] == 0) break;
      const int32_t nw = ny;  // W(j-1): rows rid[cur * n ..]
      ny = d.wcnt[j];
      yb = d.wofs[j];
      int32_t *wr_ = rid + cur * n, *yr_ = rid + (3 - cur) * n;
      for (int i = t; i < ny; i += nt) yr_[i] = d.wrow[yb + i];
      for (int i = t; i < ny * WW; i += nt) S[i] = 0ull;
      for (int i = t; i < nx * WW; i += nt) Vc[i] = 0ull;
      for (int i = t; i < nx; i += nt) nd[i] = 0;
      __syncthreads();
      cur = 3 - cur;
      // S_j: 8x8 (y, w) tiles per thread, count columns with LA[y] >= FD[w]
      // (w rows strided by tw: w = wt + b * tw)
      const int ty = (ny + 7) >> 3, tw = (nw + 7) >> 3;
      for (int tile = t; tile < ty * tw; tile += nt) {
        const int y0 = (tile / tw) * 8, wt = tile % tw;
        const int32_t *yr[8];
        const int32_t *wr[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          const int y = min(y0 + a, ny - 1), w = min(wt + a * tw, nw - 1);
          yr[a] = d.la + (int64_t)yr_[y] * npad;
          wr[a] = fdrows + (int64_t)wr_[w] * npad;
        }
        int cnt[8][8];
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int b = 0; b < 8; ++b) cnt[a][b] = 0;
        for (int i = 0; i < npad; i += 4) {
          int4 yv[8], wv[8];
#pragma unroll
          for (int a = 0; a < 8; ++a) {
            yv[a] = *reinterpret_cast<const int4 *>(yr[a] + i);
            wv[a] = *reinterpret_cast<const int4 *>(wr[a] + i);
          }
#pragma unroll
          for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int b = 0; b < 8; ++b)
              cnt[a][b] += (yv[a].x >= wv[b].x) + (yv[a].y >= wv[b].y) + (yv[a].z >= wv[b].z) +
                           (yv[a].w >= wv[b].w);
        }
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          const int y = y0 + a;
          if (y >= ny) continue;
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            const int w = wt + b * tw;
            if (w < nw && cnt[a][b] >= sm) atomicOr(&S[y * WW + (w >> 6)], 1ull << (w & 63));
          }
        }
      }
      __syncthreads();
      // tallies and votes
      const int diff = j - r;
      const bool normal = (diff % n) != 0;
      for (int p = t; p < nx * ny; p += nt) {
        const int x = p / ny, y = p - x * ny;
        if (dec[x]) continue;
        int yays = 0, tot = 0;
        for (int q = 0; q < WW; ++q) {
          const unsigned long long s = S[y * WW + q];
          yays += __popcll(s & Vp[x * WW + q]);
          tot += __popcll(s);
        }
        const int nays = tot - yays;
        const bool v = yays >= nays;
        const int tt = v ? yays : nays;
        bool vote;
        if (normal) {
          if (tt >= sm) atomicOr(&nd[x], v ? 1 : 2);
          vote = v;
        } else {
          vote = tt >= sm ? v : d.coin[d.wids[yb + y]] != 0;
        }
        if (vote) atomicOr(&Vc[x * WW + (y >> 6)], 1ull << (y & 63));
      }
      __syncthreads();
      for (int x = t; x < nx; x += nt) {
        if (dec[x] == 0 && nd[x]) {
          if (nd[x] == 3) misc[1] = 1;  // conflicting decisions: impossible without forks
          dec[x] = nd[x] == 1 ? 1 : 2;
          atomicSub(&misc[0], 1);
        }
      }
      __syncthreads();
      unsigned long long *tmp = Vp;
      Vp = Vc;
      Vc = tmp;
    }
  }
  // ---- publish ----
  __syncthreads();
  for (int x = t; x < nx; x += nt) d.wfame[xb + x] = (int8_t)dec[x];
  __syncthreads();
  if (t == 0) {
    d.decided[r] = misc[0] == 0 ? 1 : 0;
    if (misc[1]) d.state[ST_ERR] = 2;
  }
  // famous count and min LA over famous witnesses (see(w, x) for all w in FW)
  for (int c = t; c < npad; c += nt) {
    int32_t m = INT32_MAX;
    int cntf = 0;
    for (int x = 0; x < nx; ++x) {
      if (dec[x] != 1) continue;
      ++cntf;
      m = min(m, d.la[(int64_t)rid[x] * npad + c]);
    }
    d.minla[(int64_t)r * npad + c] = m;
    if (c == 0) d.nfam[r] = cntf;
  }
}

// ---------------------------------------------------------------------------
// k_fame_masks (n <= 128, the k_round2 path): DecideFame from the round
// loop's results.  The stronglySee rows fame needs -- S_j[y] over W(j-1)
// for y in W(j) -- are exactly what k_round2 evaluated when its search
// verified y's row against the candidates of round j-1 (ssm); the first
// votes see(y, x) for y in W(r+1) are LA[y][c(x)] >= k(x).  Sets are 128-bit
// masks indexed by CHAIN (a round has at most one witness per chain), so
// voting is AND + popcount: one workgroup per round r, thread (x, half)
// owns the vote word of witness x over 64 chains of W(j).
__device__ __forceinline__ uint32_t fame_wmask_word(const Dev &d, int j, int w) {
  // word w of the W(j) chain mask: B[j][q] < len_q and B[j+1][q] > B[j][q]
  uint32_t m = 0;
  for (int b = 0; b < 32; ++b) {
    const int q = w * 32 + b;
    if (q >= d.n) break;
    const int32_t b0 = d.B[(int64_t)j * d.n + q], b1 = d.B[(int64_t)(j + 1) * d.n + q];
    if (b0 < d.chain_len[q] && b1 > b0) m |= 1u << b;
  }
  return m;
}

// the W(j) chain mask, every thread one chain's bit (a ballot per wave):
// words [0, NW) of dst, written by the waves' first lanes (2 words a wave;
// 64 NW threads cover 32 NW chains twice over)
template <int NW>
__device__ __forceinline__ void fame_wmask_coop(const Dev &d, int j, uint32_t *dst) {
  const int q = threadIdx.x;
  bool bit = false;
  if (q < d.n) {
    const int32_t b0 = d.B[(int64_t)j * d.n + q], b1 = d.B[(int64_t)(j + 1) * d.n + q];
    bit = b0 < d.chain_len[q] && b1 > b0;
  }
  const unsigned long long m = __ballot(bit);
  const int w = 2 * (q >> 6);
  if ((q & 63) == 0 && w < NW) {
    dst[w] = (uint32_t)m;
    if (w + 1 < NW) dst[w + 1] = (uint32_t)(m >> 32);
  }
}

// the k_round2 ballots of (chain c, round j) packed into a 128-bit chain mask
__device__ __forceinline__ uint32_t fame_ballot_word(const unsigned long long *b, int lpc, int w) {
  uint32_t word = 0;
  if (lpc == 8) {  // 8 candidates per wave: bits 0, 8, .., 56
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned long long m = b[w * 4 + k];
      word |= (uint32_t)(((m & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56) << (8 * k);
    }
  } else {  // 16 per wave: bits 0, 4, .., 60
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      unsigned long long m = b[w * 2 + k] & 0x1111111111111111ull;
      m = (m | (m >> 3)) & 0x0303030303030303ull;
      m = (m | (m >> 6)) & 0x000F000F000F000Full;
      m = (m | (m >> 12)) & 0x000000FF000000FFull;
      m = (m | (m >> 24)) & 0xFFFFull;
      word |= (uint32_t)m << (16 * k);
    }
  }
  return word;
}

// Chain masks of NW 32-bit words (MAXN = 32 NW chains): NW = 4 for the
// k_round2 path (ballots in its raw LPC-strided layout, ssm), NW = 16 for
// the k_round_wide path (n <= 512; packed chain masks, ssw).  2 MAXN
// threads: thread (x, h) owns vote words [h NW/2, (h+1) NW/2) of witness x,
// i.e. the voters y of that half of the chains.
template <int NW>
struct FameLds {
  static constexpr int MAXN = 32 * NW;
  uint32_t V[2][NW][MAXN];  // votes: [cur][word over W(j-1) chains][x chain] (lanes = consecutive x)
  uint32_t S[MAXN][NW];     // stronglySee rows of W(j), restricted to W(j-1)
  uint32_t wx[NW], wp[NW], wc[NW];  // W(r), W(j-1), W(j)
  int32_t dec[MAXN], nd[MAXN], yev[MAXN], xev[MAXN], xk[MAXN];
  int32_t frow[MAXN];  // LA rows of famous witnesses
  int32_t misc[2];     // [0] undecided, [1] conflicting decisions
  int32_t nfam_s;
};

// S_j[y] word w: the W(j-1) chains y = (chain, B[j]) strongly sees
template <int NW>
__device__ __forceinline__ uint32_t fame_ss_word(const Dev &d, int y, int j, int w) {
  if (NW == 4) return fame_ballot_word(d.ssm + ballot_row(d, y, j) * 16, d.round_lpc, w);
  const unsigned long long m = d.ssw[ballot_row(d, y, j) * 8 + (w >> 1)];
  return (uint32_t)(m >> (32 * (w & 1)));
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_fame_masks(Dev d, int32_t R, int32_t r0) {
  constexpr int MAXN = 32 * NW, HW_ = NW / 2, HY = MAXN / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm_[];
  FameLds<NW> &L = *reinterpret_cast<FameLds<NW> *>(fsm_);
  const int r = r0 + (int)blockIdx.x, t = threadIdx.x, nt = blockDim.x;
  const int n = d.n, npad = d.npad, sm = d.sm;
  // cla rows of rounds r + 1 (first votes) and r (minLA), unless a later
  // round of this loop reused their ring slot, or the round lies below the
  // loop's first round (a Reset hashgraph's fiat rounds < r0 = rbase, which
  // no loop wrote and the ring does not hold): then la_at
  const bool cy = d.use_cla && r + 1 >= d.r0 && r + 1 > R - d.cla_span;
  const bool cx = d.use_cla && r >= d.r0 && r > R - d.cla_span;
  fame_wmask_coop<NW>(d, r, L.wx);
  for (int q = t; q < MAXN; q += nt) {
    L.dec[q] = 0;
    L.nd[q] = 0;
    L.xev[q] = -1;
    L.xk[q] = 0;
    L.yev[q] = 0;  // j = r+1: LA row of y
    if (q < n) {
      const int32_t b0 = d.B[(int64_t)r * n + q];
      if (b0 < d.chain_len[q]) L.xev[q] = d.chain_ids[d.chain_start[q] + b0];
      L.xk[q] = b0;
      if (r + 1 < R)
        L.yev[q] = cy ? (int32_t)cla_row(d, q, r + 1)
                             : d.chain_start[q] + min(d.B[(int64_t)(r + 1) * n + q], d.chain_len[q] - 1);
    }
  }
  __syncthreads();
  if (t == 0) {
    int u = 0;
    for (int w = 0; w < NW; ++w) u += __popc(L.wx[w]);
    L.misc[0] = u;
    L.misc[1] = 0;
  }
  const int x = t % MAXN, h = t / MAXN;  // vote words h*HW_ .. +HW_ of witness x
  const bool isx = (L.wx[x >> 5] >> (x & 31)) & 1u;
  int cur = 0;
  if (r + 1 < R) {
    // ---- j = r+1: vote(y, x) = see(y, x) ----
    fame_wmask_coop<NW>(d, r + 1, L.wc);
    __syncthreads();
    {
      const int xc = min(x, n - 1);
      for (int k = 0; k < HW_; ++k) {
        // the word's 32 voters' LA entries loaded together (independent
        // gathers in flight), then compared
        const uint32_t wk = (h * HY + k * 32) < n ? L.wc[(h * HY + k * 32) >> 5] : 0u;
        uint32_t v = 0;
        if (cy) {
          int32_t a[32];
#pragma unroll
          for (int b = 0; b < 32; ++b) {
            const int y = min(h * HY + k * 32 + b, n - 1);
            a[b] = (wk >> b & 1u) ? d.cla[(int64_t)L.yev[y] * npad + xc] : INT32_MIN;
          }
#pragma unroll
          for (int b = 0; b < 32; ++b)
            if (a[b] >= L.xk[xc] && (wk >> b & 1u)) v |= 1u << b;
        } else {
          for (int b = 0; b < 32; ++b) {
            const int y = h * HY + k * 32 + b;
            if (y >= n || !(wk >> b & 1u)) continue;
            if (la_at(d, L.yev[y], xc) >= L.xk[xc]) v |= 1u << b;
          }
        }
        L.V[0][h * HW_ + k][x] = v;
      }
    }
    __syncthreads();
    // ---- j >= r+2 ----
    for (int j = r + 2; j < R; ++j) {
      if (L.misc[0] == 0) break;
      if (t < NW) L.wp[t] = L.wc[t];
      __syncthreads();  // (wc read into wp before it is rewritten)
      fame_wmask_coop<NW>(d, j, L.wc);
      __syncthreads();
      for (int y = t; y < n; y += nt) {
        const bool isy = (L.wc[y >> 5] >> (y & 31)) & 1u;
        L.yev[y] = isy ? d.chain_ids[d.chain_start[y] + d.B[(int64_t)j * n + y]] : -1;
#pragma unroll
        for (int w = 0; w < NW; ++w) L.S[y][w] = isy ? fame_ss_word<NW>(d, y, j, w) & L.wp[w] : 0u;
      }
      __syncthreads();
      const int diff = j - r;
      const bool normal = (diff % n) != 0;
      if (isx && !L.dec[x]) {
        int decide = 0;
        // x's votes in registers: they are read for every voter y
        uint32_t vx[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) vx[w] = L.V[cur][w][x];
        for (int k = 0; k < HW_; ++k) {
          uint32_t v = 0;
          for (int b = 0; b < 32; ++b) {
            const int y = h * HY + k * 32 + b;
            if (y >= n || !((L.wc[y >> 5] >> (y & 31)) & 1u)) continue;
            int yays = 0, tot = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
              yays += __popc(L.S[y][w] & vx[w]);
              tot += __popc(L.S[y][w]);
            }
            const int nays = tot - yays;
            const bool vv = yays >= nays;
            const int tt = vv ? yays : nays;
            bool vote;
            if (normal) {
              if (tt >= sm) decide |= vv ? 1 : 2;
              vote = vv;
            } else {
              vote = tt >= sm ? vv : d.coin[L.yev[y]] != 0;
            }
            if (vote) v |= 1u << b;
          }
          L.V[cur ^ 1][h * HW_ + k][x] = v;
        }
        if (decide) atomicOr(&L.nd[x], decide);
      }
      __syncthreads();
      if (t < MAXN && isx && L.dec[x] == 0 && L.nd[x]) {
        if (L.nd[x] == 3) L.misc[1] = 1;  // conflicting decisions: impossible without forks
        L.dec[x] = L.nd[x] == 1 ? 1 : 2;
        atomicSub(&L.misc[0], 1);
      }
      __syncthreads();
      cur ^= 1;
    }
  }
  // ---- publish ----
  __syncthreads();
  if (t < MAXN && isx) {  // witness x's position in W(r): the witnesses of lower chains before it
    int rank = 0;
    for (int w = 0; w < (x >> 5); ++w) rank += __popc(L.wx[w]);
    rank += __popc(L.wx[x >> 5] & ((1u << (x & 31)) - 1u));
    d.wfame[d.wofs[r] + rank] = (int8_t)L.dec[x];
  }
  if (t == 0) {
    d.decided[r] = L.misc[0] == 0 ? 1 : 0;
    if (L.misc[1]) d.state[ST_ERR] = 2;
    int m = 0;
    for (int q = 0; q < n; ++q)
      if (((L.wx[q >> 5] >> (q & 31)) & 1u) && L.dec[q] == 1)
        L.frow[m++] = cx ? (int32_t)cla_row(d, q, r) : d.chain_start[q] + d.B[(int64_t)r * n + q];
    L.nfam_s = m;
  }
  __syncthreads();
  // famous count and min LA over famous witnesses (roundReceived)
  const int nf = L.nfam_s;
  for (int c = t; c < npad; c += nt) {
    int32_t m = INT32_MAX;
    if (cx)
      for (int i = 0; i < nf; ++i) m = min(m, d.cla[(int64_t)L.frow[i] * npad + c]);
    else
      for (int i = 0; i < nf; ++i) m = min(m, c < n ? la_at(d, L.frow[i], c) : -1);
    d.minla[(int64_t)r * npad + c] = m;
    if (c == 0) d.nfam[r] = nf;
  }
}

size_t fame_lds_bytes(int n) {
  const int WW = (n + 63) >> 6;
  return (size_t)3 * n * WW * 8 + (size_t)8 * n * 4 + 16;
}

void configure_fame_kernels() {
  (void)hipFuncSetAttribute((const void *)k_fame, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  (void)hipFuncSetAttribute((const void *)k_fame_masks<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(FameLds<16>));
}

void launch_fame(const Dev &d, int32_t R, int32_t r0, int32_t r1, hipStream_t s) {
  if (r1 <= r0) return;
  if (d.fd_cols) {  // masks from the k_round2 loop
    k_fame_masks<4><<<r1 - r0, 256, sizeof(FameLds<4>), s>>>(d, R, r0);
    return;
  }
  if (d.ssw) {  // masks from the k_round_wide loop (n <= 512)
    k_fame_masks<16><<<r1 - r0, 1024, sizeof(FameLds<16>), s>>>(d, R, r0);
    return;
  }
  k_fame<<<r1 - r0, 256, fame_lds_bytes(d.n), s>>>(d, R, r0);
}

// per-event fame from the witness-ordered results; a trapped witness
//  stays Undefined whatever the votes say
__global__ void k_fame_scatter(Dev d, int32_t w0, int32_t w1) {
  const int32_t i = w0 + (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= w1) return;
  const int32_t e = d.wids[i];
  d.fame[e] = d.trapped[e] ? 0 : d.wfame[i];
}

void launch_fame_scatter(const Dev &d, int32_t W, hipStream_t s) { launch_fame_scatter_range(d, 0, W, s); }

void launch_fame_scatter_range(const Dev &d, int32_t w0, int32_t w1, hipStream_t s) {
  if (w1 <= w0) return;
  k_fame_scatter<<<(unsigned)((w1 - w0 + 255) / 256), 256, 0, s>>>(d, w0, w1);
}

// the witnesses of rounds [P, R), bounded on the device (wofs[P], wofs[R]):
// the host launches it without having read wofs back (fame_finish, one shard)
__global__ void k_fame_scatter_rounds(Dev d, int32_t P, int32_t R) {
  const int32_t w0 = d.wofs[P], w1 = d.wofs[R];
  for (int32_t i = w0 + (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); i < w1; i += (int32_t)(gridDim.x * blockDim.x)) {
    const int32_t e = d.wids[i];
    d.fame[e] = d.trapped[e] ? 0 : d.wfame[i];
  }
}

void launch_fame_scatter_rounds(const Dev &d, int32_t P, int32_t R, hipStream_t s) {
  if (R <= P) return;
  const int64_t most = (int64_t)(R - P) * d.n;  // (at most one witness per chain and round)
  k_fame_scatter_rounds<<<(unsigned)std::min<int64_t>((most + 255) / 256, 4096), 256, 0, s>>>(d, P, R);
}

}  // namespace bh
