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
// step per ROUND (not per event or DAG level), one launch (k_round), one
// workgroup per chain c: the candidates' firstDescendants rows (precomputed
// for every event, kernels_fd.hip) are gathered into registers, the window
// of chain c starting at B[r][c] into LDS; lane groups binary-search T_q,
// the first window row that strongly sees candidate q (monotone along the
// chain); B[r+1][c] = the SM-th smallest T_q.
// B[r] and the round index are double-buffered by round parity (a launch
// argument), so a captured graph of iterations replays without host
// involvement and every load of an iteration depends only on B[r].
#include "engine.h"

#include <hip/hip_ext.h>

#include <algorithm>

namespace bh {

// the round loop's end, told to the host through mapped pinned memory (a
// system-scope store), so the host polls it between graph replays instead of
// copying the state back after every batch
__device__ __forceinline__ void signal_done(const Dev &d) {
  if (d.hdone) __hip_atomic_store(d.hdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}


constexpr int WROWS = 32;    // window rows per chain

__device__ __forceinline__ int popc64(unsigned long long x) { return __popcll(x); }

// ---------------------------------------------------------------------------
// k_round(p): one round-loop iteration, B[r+1][c] for one chain c per
// workgroup.  Candidate q = (q, B[r][q]); its firstDescendants row is row
// chain_start[q] + B[r][q] of FD (kernels_fd.hip), gathered straight into
// registers: LPC lanes per candidate, each holding every LPC-th 16-B piece
// (16 pieces = 64 columns per lane).  The window (rows B[r][c] .. +WROWS of
// chain c) is staged in LDS.  T_q = the first window row strongly seeing q
// (monotone along the chain) by binary search; B[r+1][c] = the SM-th
// smallest T_q (a 32-bin histogram and a wave prefix).  All loads of an
// iteration depend only on B[r] (parity buffer p), so the iteration costs
// one dependent gather; the round index (for the history row B[r+1] and
// the termination record) is double-buffered by parity in the state block.
constexpr int SCAN_PAD = 4;
constexpr int PIECES = 16;  // 16-B pieces of a candidate row per lane

__device__ __forceinline__ int ge4(int4 a, int4 b) {
  return (a.x >= b.x) + (a.y >= b.y) + (a.z >= b.z) + (a.w >= b.w);
}

// #{a < b} over 4 lanes of LA (>= -1) against FD (>= 0 or FD_NONE): a - b
// never overflows, so its sign bit is the comparison
__device__ __forceinline__ int lt4(int4 a, int4 b) {
  const uint32_t dx = (uint32_t)a.x - (uint32_t)b.x, dy = (uint32_t)a.y - (uint32_t)b.y;
  const uint32_t dz = (uint32_t)a.z - (uint32_t)b.z, dw = (uint32_t)a.w - (uint32_t)b.w;
  return (int)((dx >> 31) + (dy >> 31) + (dz >> 31) + (dw >> 31));
}

// sum over an aligned group of LPC lanes, every lane gets the total (DPP for
// groups within a row of 16 lanes)
template <int LPC>
__device__ __forceinline__ int group_total(int v) {
  if (LPC >= 2) v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
  if (LPC >= 4) v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
  if (LPC >= 8) v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, true);  // row_half_mirror
  if (LPC >= 16) v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, true); // row_mirror
  return v;
}

// 16-bit rows (chains <= P16_MAXLEN events): LA + 1 in [0, len] against
// FD + 1 in [1, len] or 0xFFFF (none), two columns per dword.  Per dword:
// saturating f - x (non-zero iff x < f), min 1, accumulate -- three packed
// ops for two columns.  Inline asm: the compiler would split the packed
// compare back into per-half compares.
__device__ __forceinline__ uint32_t lt16x2_acc(uint32_t acc, uint32_t x, uint32_t f, uint32_t one) {
  uint32_t dd;
  asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(dd) : "v"(f), "v"(x));
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(dd) : "v"(dd), "v"(one));
  asm("v_pk_add_u16 %0, %1, %2" : "=v"(dd) : "v"(acc), "v"(dd));
  return dd;
}

__device__ __forceinline__ uint32_t pack_la16(int32_t a, int32_t b) {
  return (uint32_t)(a + 1) | ((uint32_t)(b + 1) << 16);
}

// 8-bit window-relative rows (k_round_wide, P16 windows whose LA spread fits):
// per column i, base_i = max(LA[first window row][i], 0); a window row's LA
// is x = LA + 1 - base in [0, 126] (LA is non-decreasing down the window, so
// the last row bounds it), a candidate's FD f = min(max(FD + 1 - base, 0),
// 127).  Then LA >= FD <=> x >= f: below the window's first row f = 0 <= x
// (LA >= base > FD), past its last row f = 127 > x, exact in between.  Four
// columns per dword, x stored with bit 7 set: ((x | 0x80) - f) & 0x80 is set
// iff x >= f, with no borrow between bytes, counted by v_bcnt.
// the FD row of event `row` (chain-major) from FDT into dst as 16-bit FD + 1
// pairs (cand16); every thread of the workgroup calls it
__device__ __forceinline__ void gather_cand16(const Dev &d, int64_t row, uint32_t *dst) {
  const int npad = d.npad, n = d.n, w = (npad + 7) / 8 * 4;
  auto h16 = [](int32_t v) { return min((uint32_t)v + 1u, 0xFFFFu); };  // FD_NONE + 1 wraps to 2^31
  for (int j = threadIdx.x; j < w; j += blockDim.x) {
    const int i0 = 2 * j, i1 = 2 * j + 1;
    const int32_t v0 = i0 < n ? d.fdt[fdt_pos(row, i0, npad)] : FD_NONE;
    const int32_t v1 = i1 < n ? d.fdt[fdt_pos(row, i1, npad)] : FD_NONE;
    dst[j] = h16(v0) | (h16(v1) << 16);
  }
}

// two 16-bit FD + 1 values (0xFFFF: none) less base (saturating), capped at 127
__device__ __forceinline__ uint32_t fd8x2(uint32_t f, uint32_t b) {
  uint32_t dd;
  asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(dd) : "v"(f), "v"(b));
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(dd) : "v"(dd), "v"(0x007F007Fu));
  return dd;
}
// columns (lo.l, lo.h, hi.l, hi.h) as bytes 0..3
__device__ __forceinline__ uint32_t pack8(uint32_t lo, uint32_t hi) {
  return __builtin_amdgcn_perm(hi, lo, 0x06040200u);
}

// Loads and stores of what other workgroups of the same launch store (the
// persistent loops): sc1, so neither this CU's L1 nor this XCD's L2 can serve
// a stale line (MI355X_MICROARCH.md, the hand-off table); plain otherwise.
template <bool SC1>
__device__ __forceinline__ int32_t ldx(const int32_t *p) {
  if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool SC1, class T>
__device__ __forceinline__ void stx(T *p, T v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
// 16-B element `idx` of a buffer whose descriptor is rs (SC1: buffer load
// with sc1), or of the plain pointer base
template <bool SC1>
__device__ __forceinline__ int4 ld128(__amdgpu_buffer_rsrc_t rs, const int4 *base, int64_t idx) {
  if constexpr (SC1) return __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(idx * 16), 0, 16));
  else return base[idx];
}

// The persistent loops' grid barrier.  pbar layout (ints): [0] the counter
// (flat) / top counter (hierarchical), [32 (1 + x)] XCD x's arrivals,
// [288 + x] XCD x's workgroups, [PBAR_REL + 32 w] workgroup w's release word,
// each on 128-B lines of its own.  pbar_mode 1 (XCD-hierarchical) from the
// second barrier on: a workgroup adds to its XCD's counter; the XCD's last
// arriver (told by the value its add returns) adds to the top counter; the
// workgroup whose top add completes it (told the same way) releases every
// workgroup by storing it + 1 into its release word, which each polls
// alone.  The chain from the last arrival to a release is two returned
// atomics and one store, and no line is polled by more than one workgroup
// (a shared release line polled by 64 workgroups spread the releases over
// 5 us).  Flat (pbar_mode 0, and the first barrier): every workgroup adds to
// [0], and the add that completes it releases everyone the same way.
constexpr int PBAR_REL = 1024;
constexpr int PBAR_INTS = PBAR_REL + 32 * 512;  // (n <= 512 workgroups)

__device__ __forceinline__ int pbar_register(const Dev &d) {  // thread 0, at the start: this workgroup's XCD, counted
  int xcc = 0;
  if (d.pbar_mode == 1) {
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    xcc &= 7;
    // an add whose returned value is used: performed before this workgroup's first arrival
    if (__hip_atomic_fetch_add(d.pbar + 288 + xcc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0) xcc = 0;
  }
  return xcc;
}
// wave 0 of each workgroup (lane 0 holds xcc, gx, nx), after every wave's
// stores have drained and a workgroup barrier.  The arrival that completes
// the barrier -- of the top counter (hierarchical) or of the one counter
// (flat, and the first barrier) -- is told so by its add's returned value
// and releases every workgroup: release word w = it + 1.
__device__ __forceinline__ void pbar_arrive(const Dev &d, int it, int xcc, int32_t gx, int G, int32_t nx) {
  const int lane = threadIdx.x & 63;
  int last = 0;
  if (lane == 0) {
    if (d.pbar_mode == 1 && it > 0) {
      if (__hip_atomic_fetch_add(d.pbar + 32 * (1 + xcc), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == it * gx - 1)
        last = __hip_atomic_fetch_add(d.pbar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G + it * nx - 1;
    } else {  // flat: (it + 1) G arrivals in all; the hierarchical top counter starts from the first barrier's G
      last = __hip_atomic_fetch_add(d.pbar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (it + 1) * G - 1;
    }
  }
  if (__shfl(last, 0))
    for (int w = lane; w < G; w += 64)
      __hip_atomic_store(d.pbar + PBAR_REL + 32 * w, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool pbar_poll(const Dev &d, const int32_t *w, int32_t target) {
  int spins = 0;
  while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > d.pbar_spin) return false;
  }
  return true;
}
// thread 0; false: the barrier gave up (d.pbar_spin polls)
__device__ __forceinline__ bool pbar_wait(const Dev &d, int it, int G) {
  (void)G;
  return pbar_poll(d, d.pbar + PBAR_REL + 32 * blockIdx.x, it + 1);
}
// after the first barrier every workgroup has counted itself
__device__ __forceinline__ void pbar_counts(const Dev &d, int xcc, int32_t &gx, int32_t &nx) {
  if (d.pbar_mode != 1) return;
  gx = __hip_atomic_load(d.pbar + 288 + xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  nx = 0;
  for (int x = 0; x < 8; ++x) nx += __hip_atomic_load(d.pbar + 288 + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0;
}

// k_round_wide's hand-off of the new candidate (c, row) for iteration r + 1:
// its cand16 row (gather_cand16's layout) and, with the shared base on, its
// cand8 row -- byte i = min(max(FD + 1 - base_i, 0), 127) with base_i =
// max(B[r][i] - round_p8g, 0) from Bcur = B[r] (the base iteration r + 1
// reads back from the B history), 127 past column n -- then the row's tag.
// Four columns per thread; every thread of the workgroup calls it.
template <bool SC1 = false>
__device__ __forceinline__ void handoff_wide(const Dev &d, int64_t row, int p1, int c, const int32_t *Bcur,
                                             int32_t rnext) {
  const int npad = d.npad, n = d.n, w16 = (npad + 7) / 8 * 4, w8 = (npad + 15) / 16 * 16;
  uint32_t *dst16 = d.cand16 + ((int64_t)p1 * n + c) * w16;
  const bool g = d.cand8 != nullptr && d.round_p8g > 0 && d.round_p8 > 0;
  uint32_t *dst8 = g ? reinterpret_cast<uint32_t *>(d.cand8 + ((int64_t)p1 * n + c) * w8) : nullptr;
  for (int j = threadIdx.x; j < w8 / 4; j += blockDim.x) {
    uint32_t h[4], b8 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = 4 * j + k;
      const int32_t v = i < n ? d.fdt[fdt_pos(row, i, npad)] : FD_NONE;
      h[k] = min((uint32_t)v + 1u, 0xFFFFu);  // FD_NONE + 1 wraps to 2^31
      if (g) {
        const int32_t base = i < n ? max(ldx<SC1>(Bcur + i) - d.round_p8g, 0) : 0;
        const uint32_t f = i < n ? min((uint32_t)max((int32_t)h[k] - base, 0), 127u) : 127u;
        b8 |= f << (8 * k);
      }
    }
    if (2 * j < w16) stx<SC1>(dst16 + 2 * j, h[0] | (h[1] << 16));
    if (2 * j + 1 < w16) stx<SC1>(dst16 + 2 * j + 1, h[2] | (h[3] << 16));
    if (g) stx<SC1>(dst8 + j, b8);
  }
  // read by the next launch (the kernel boundary orders it after the row),
  // or after the persistent loop's grid barrier (sc1 stores, drained first)
  if (g && threadIdx.x == 0) stx<SC1>(d.c8tag + (int64_t)p1 * n + c, rnext);
}

// The first j in [lo, hi) with col[j] >= k (col non-decreasing), or hi:
// the whole wave searches (lo, hi, k uniform), 64 probes per pass.
__device__ __forceinline__ int32_t first_ge_wave(const int32_t *col, int32_t lo, int32_t hi, int32_t k) {
  const int lane = threadIdx.x & 63;
  while (hi - lo > 64) {
    const int32_t s = (hi - lo + 63) >> 6;
    const unsigned long long m = __ballot(col[min(lo + (lane + 1) * s, hi) - 1] >= k);
    if (!m) return hi;
    const int f = __builtin_ctzll(m);
    hi = min(lo + (f + 1) * s, hi);
    lo += f * s;
  }
  const unsigned long long m = __ballot(lo + lane < hi && col[lo + lane] >= k);
  return m ? lo + __builtin_ctzll(m) : hi;
}

// k_round_wide<*, true, 1 / 2>'s hand-off of the new candidate (c, row) for
// iteration r + 1 from the dataflow's column-major LA (no FDT):
// FD[(c, row)][i] = min{j : LA[(i, j)][c] >= row} is non-decreasing in the
// candidate's row, so chain i's entry starts at the previous candidate's
// (cand16[p][c]); 4 lanes per chain count the rows below `row` among the 48
// from there (rounded down to 4), 64 chains per pass.  An entry beyond them
// (an advance of more than ~45 rows) is searched by the wave
// (first_ge_wave).  Writes cand16 (16-bit FD + 1), cand8 against the shared
// base (as handoff_wide) and the candidate's LA row into cla (fame).
template <int GL>
__device__ __forceinline__ int32_t first_ge_group(const int32_t *col, int32_t lo, int32_t hi, int32_t k, bool on,
                                                  bool near);

template <int NT, bool SC1 = false>
__device__ __forceinline__ void handoff_wide_cols(const Dev &d, int p, int c, int32_t row, const int32_t *Bcur,
                                                  int32_t rnext) {
  constexpr int K = 2048 / NT, HR = 48, KL = 512 / NT;  // chains per thread (n <= 512), rows per chain, LA values per thread
  const int t = threadIdx.x, l4 = t & 3;
  const int n = d.n, npad = d.npad, w16 = (npad + 7) / 8 * 4, w8 = (npad + 15) / 16 * 16;
  const int64_t stride = la_col_stride(d);
  const int32_t *colc = d.la_col + (int64_t)c * stride;
  const uint16_t *prev = reinterpret_cast<const uint16_t *>(d.cand16 + ((int64_t)p * n + c) * w16);
  uint16_t *dst16 = reinterpret_cast<uint16_t *>(d.cand16 + ((int64_t)(p ^ 1) * n + c) * w16);
  const bool g = d.cand8 != nullptr && d.round_p8g > 0 && d.round_p8 > 0;
  uint8_t *dst8 = g ? d.cand8 + ((int64_t)(p ^ 1) * n + c) * w8 : nullptr;
  const int64_t crow = (int64_t)d.chain_start[c] + row;
  int32_t la[KL];
#pragma unroll
  for (int k = 0; k < KL; ++k) {
    const int i = t + NT * k;
    la[k] = i < n ? d.la_col[(int64_t)i * stride + crow] : -1;
  }
  int32_t a[K], cs[K], end[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = (t >> 2) + (NT / 4) * k;
    uint32_t h = 0xFFFFu;
    if (i < n) {  // (SC1: the row this workgroup stored sc1 last round, read the same way)
      if constexpr (SC1) h = (uint32_t)ldx<true>(reinterpret_cast<const int32_t *>(prev) + i / 2) >> (16 * (i & 1)) & 0xFFFFu;
      else h = prev[i];
    }
    cs[k] = i < n ? d.chain_start[i] : 0;
    end[k] = i < n ? cs[k] + d.chain_len[i] : 0;
    a[k] = h == 0xFFFFu ? -1 : cs[k] + (int32_t)h - 1;  // the previous entry (absolute row), -1: none
  }
  int4 v[K][3];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int u = 0; u < 3; ++u)
      v[k][u] = a[k] >= 0 ? *reinterpret_cast<const int4 *>(colc + ((a[k] & ~3) + 12 * l4 + 4 * u)) : make_int4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < KL; ++k)
    if (t + NT * k < npad) d.cla[cla_row(d, c, rnext) * npad + t + NT * k] = la[k];
  int32_t fd[K];
  bool miss[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = (t >> 2) + (NT / 4) * k;
    const int32_t ab = a[k] & ~3, x0 = ab + 12 * l4, elo = a[k] - x0, ehi = end[k] - x0;
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      cnt += (4 * u + 0 >= elo) & (4 * u + 0 < ehi) & (v[k][u].x < row);
      cnt += (4 * u + 1 >= elo) & (4 * u + 1 < ehi) & (v[k][u].y < row);
      cnt += (4 * u + 2 >= elo) & (4 * u + 2 < ehi) & (v[k][u].z < row);
      cnt += (4 * u + 3 >= elo) & (4 * u + 3 < ehi) & (v[k][u].w < row);
    }
    cnt = group_total<4>(cnt);
    const int32_t jn = a[k] + cnt, bend = min(ab + HR, end[k]);
    fd[k] = FD_NONE;
    miss[k] = false;
    if (a[k] >= 0) {
      if (i == c) fd[k] = row;  // an event is its own first descendant
      else if (jn < bend) fd[k] = jn - cs[k];
      else if (bend < end[k]) miss[k] = true;
      // else: no row of chain i in this view sees the candidate
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    // beyond the 48 rows (a candidate that jumped far): each such chain's 4
    // lanes search on at once, the first pass over the next 256 rows
    if (__any(miss[k])) {
      const int32_t lo = min((a[k] & ~3) + HR, end[k]);
      const int32_t j = first_ge_group<4>(colc, lo, end[k], row, miss[k], true);
      if (miss[k]) fd[k] = j < end[k] ? j - cs[k] : FD_NONE;
    }
  }
  // the 16-bit and byte rows, 4 entries per lane into one dword each
  // (SC1: stored sc1, read by the other workgroups after the grid barrier)
  uint32_t *d16 = reinterpret_cast<uint32_t *>(dst16);
  uint32_t *d8 = reinterpret_cast<uint32_t *>(dst8);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = (t >> 2) + (NT / 4) * k;
    const uint32_t h = i < n ? min((uint32_t)fd[k] + 1u, 0xFFFFu) : 0xFFFFu;  // FD_NONE + 1 wraps to 2^31
    uint32_t b = 127u;
    if (g && i < n) {
      const int32_t base = max(ldx<SC1>(Bcur + i) - d.round_p8g, 0);
      b = min((uint32_t)max((int32_t)h - base, 0), 127u);
    }
    // chains i .. i + 3 sit in lanes l4 = 0 of four consecutive lane quads: gather them to the first
    const uint32_t h1 = __shfl_down(h, 4), h2 = __shfl_down(h, 8), h3 = __shfl_down(h, 12);
    const uint32_t b1 = __shfl_down(b, 4), b2 = __shfl_down(b, 8), b3 = __shfl_down(b, 12);
    if (l4 == 0 && (i & 3) == 0 && i < 2 * w16) {
      stx<SC1>(d16 + i / 2, h | (h1 << 16));
      if (i + 2 < 2 * w16) stx<SC1>(d16 + i / 2 + 1, h2 | (h3 << 16));
      if (g && i < w8) stx<SC1>(d8 + i / 4, b | (b1 << 8) | (b2 << 16) | (b3 << 24));
    }
  }
  if (g && t == 0) stx<SC1>(d.c8tag + (int64_t)(p ^ 1) * n + c, rnext);
}

template <int LPC>
__global__ __launch_bounds__(256) void k_round(Dev d, int p) {
  extern __shared__ __attribute__((aligned(16))) int32_t ssm[];
  __shared__ int32_t hist[WROWS + 1];
  __shared__ int32_t sh_res, sh_nc;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c = blockIdx.x;
  const int n = d.n, npad = d.npad, sm = d.sm, rs = npad + SCAN_PAD, q4 = npad / 4;
  const int32_t *Bp = d.Bp + (int64_t)p * n;  // B[r]
  const bool dg = d.diag != nullptr && t == 0;
  const unsigned long long ts0 = dg ? stamp() : 0;
  // ---- loads that depend on nothing: state, B[r], chain tables ----
  const int done = d.state[ST_DONE];
  const int r = d.state[ST_CUR0 + p];
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  const int32_t k0 = Bp[c];
  const int part = t % LPC;
  const int q = t / LPC;
  int32_t bq = 0, lq = 0, sq = 0;
  if (q < n) { bq = Bp[q]; lq = d.chain_len[q]; sq = d.chain_start[q]; }
  if (done) return;
  const bool act = q < n && bq < lq;
  const int qpl = (q4 + LPC - 1) / LPC;  // pieces per lane (<= PIECES)
  const unsigned long long ts1 = dg ? stamp() : 0;
  // ---- the one dependent gather: window rows of chain c and the
  // candidates' firstDescendants rows, all issued before any is consumed ----
  int rows = min(WROWS, max(0, len - k0));
  int32_t *win = ssm;  // [WROWS][rs]
  const int wtot = rows * q4;
  const int4 *wsrc = reinterpret_cast<const int4 *>(d.la + (int64_t)(cs + k0) * npad);
  int4 wv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) wv[u] = wtot > 0 ? wsrc[min(u * 256 + t, wtot - 1)] : make_int4(0, 0, 0, 0);
  int4 f[PIECES];
  {
    const int4 *fr = reinterpret_cast<const int4 *>(d.fd + (int64_t)(act ? sq + bq : 0) * npad);
#pragma unroll
    for (int u = 0; u < PIECES; ++u) {
      const int pc = u * LPC + part;
      f[u] = (u < qpl && pc < q4) ? fr[pc] : make_int4(FD_NONE, FD_NONE, FD_NONE, FD_NONE);
    }
  }
  if (t <= WROWS) hist[t] = 0;
  if (t == 0) sh_nc = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = u * 256 + t;
    if (i < wtot) {
      const int row = i / q4;
      reinterpret_cast<int4 *>(win + row * rs)[i - row * q4] = wv[u];
    }
  }
  for (int i = 4 * 256 + t; i < wtot; i += 256) {  // windows wider than 16 KiB
    const int row = i / q4;
    reinterpret_cast<int4 *>(win + row * rs)[i - row * q4] = wsrc[i];
  }
  __syncthreads();
  const unsigned long long ts2 = dg ? stamp() : 0;
  {
    const unsigned long long m = __ballot(act && part == 0);
    if (lane == 0 && m) atomicAdd(&sh_nc, __popcll(m));
  }
  // strongly-see test of window row `row` against this lane group's candidate
  auto ss = [&](int row) -> bool {
    const int4 *x4 = reinterpret_cast<const int4 *>(win + row * rs);
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < PIECES; ++u)
      if (u < qpl) cnt += ge4(x4[min(u * LPC + part, q4 - 1)], f[u]);
#pragma unroll
    for (int o = 1; o < LPC; o <<= 1) cnt += __shfl_xor(cnt, o);
    return cnt >= sm;
  };
  int32_t result = len, wk0 = k0;
  for (;;) {
    // T_q within the window: first row strongly seeing q (fixed-depth
    // binary search; converged groups re-test their row)
    int tw = WROWS;
    if (rows > 0 && ss(rows - 1)) {
      int lo = 0, hi = rows - 1;
#pragma unroll
      for (int it = 0; it < 5; ++it) {
        const int mid = (lo + hi) >> 1;
        const bool s = ss(mid);
        hi = s ? mid : hi;
        lo = s ? lo : mid + 1;
      }
      tw = lo;
    }
    if (act && part == 0 && tw < WROWS) atomicAdd(&hist[tw], 1);
    __syncthreads();
    if (sh_nc == 0) break;  // no candidates: the round loop is over
    if (wave == 0) {  // first row whose running count reaches SM
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
    const int res = sh_res;
    if (res >= 0) { result = wk0 + res; break; }
    // SM not reached in this window (rare): the next window of chain c
    wk0 += rows;
    rows = min(WROWS, len - wk0);
    if (rows <= 0) break;
    __syncthreads();
    {
      const int tot = rows * q4;
      const int4 *src = reinterpret_cast<const int4 *>(d.la + (int64_t)(cs + wk0) * npad);
      for (int i = t; i < tot; i += 256) {
        const int row = i / q4;
        reinterpret_cast<int4 *>(win + row * rs)[i - row * q4] = src[i];
      }
    }
    if (t <= WROWS) hist[t] = 0;
    __syncthreads();
  }
  if (dg) {
    const unsigned long long te = stamp();
    atomicAdd(&d.diag[DG_RD_B], ts1 - ts0);
    atomicAdd(&d.diag[DG_RD_LOAD], ts2 - ts1);
    atomicAdd(&d.diag[DG_RD_COMP], te - ts2);
    atomicAdd(&d.diag[DG_RD_TOTAL], te - ts0);
    atomicAdd(&d.diag[DG_RD_CALLS], 1ull);
  }
  if (t == 0) {
    if (sh_nc == 0) {  // R = r
      if (c == 0) { d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; signal_done(d); }
      return;
    }
    if (r + 1 >= d.R_cap) {
      if (c == 0) { d.state[ST_ERR] = 1; d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; signal_done(d); }
      return;
    }
    d.Bp[(int64_t)(p ^ 1) * n + c] = result;
    d.B[(int64_t)(r + 1) * n + c] = result;  // history for the per-event pass
    if (c == 0) {
      d.state[ST_CUR0 + (p ^ 1)] = r + 1;
      d.state[ST_ITERS] = r + 1;
    }
  }
}

// n > 256/LPC candidates (wide configurations): T_q per candidate pass
// accumulated in one histogram over the whole window, windows advanced
// until SM is reached.  Lane `part` of a candidate's group owns the PIECES
// consecutive 16-B pieces part*PIECES .. +PIECES of the row: its FD pieces
// sit in registers, its LA pieces of a window row in LDS at a fixed offset
// (row * WRS4 + part * (PIECES + 1), skewed by one piece per lane so the
// group's reads fall in distinct banks), so a probe is PIECES ds_read_b128
// with immediate offsets, issued back to back, and 4 * PIECES compares.
// Pieces past the row (pc >= q4) are -1 in LDS and FD_NONE in registers.
//
// P16: the same search over 16-bit rows (cand16, LA converted while staged):
// lane `part` owns 8 pieces of 8 columns, half the LDS reads and 3/5 of the
// compare work per probe.
// COLS: 0 = window rows from the row-major LA, candidates' FD rows gathered
// from FDT (handoff_wide); 1 = both from the column-major LA (no transpose);
// 2 = window rows from the row-major LA, hand-off from la_col (A/B)
// PERS (k_round_wide<*, true, 0, 256, true>, the default where it fits): the
// whole loop in one launch, every round's iteration followed by a grid
// barrier instead of a kernel boundary (as k_round2p at n <= 128): what the
// workgroups hand each other -- boundaries (Bp, B), candidates' rows (cand16,
// cand8) and tags -- goes through sc1 stores and loads.  512 workgroups, two
// per compute unit, all resident.
template <int LPC, bool P16, int COLS = 0, int NT = 256, bool PERS = false, int ILPK = 2>
__global__ __launch_bounds__(NT, NT / 128) void k_round_wide(Dev d, int p) {  // 2 workgroups per CU (NT / 128 waves per SIMD)
  extern __shared__ __attribute__((aligned(16))) int4 win4[];  // [WROWS][WRS4]
  constexpr int PP = P16 ? 8 : PIECES;  // 16-B pieces per lane
  constexpr int WRS4 = LPC * (PP + 1);
  __shared__ int32_t hist[WROWS + 1];
  __shared__ int32_t sh_res, sh_nc;
  __shared__ int8_t tq_s[512];  // T_q of every candidate in the current window (ssw, n <= 512)
  __shared__ uint32_t wbase2[256];  // P8: base of columns 2j, 2j + 1 as 16-bit pairs (the window's first row)
  __shared__ uint32_t gbase2[256];  // P8: the same from the shared base max(B[r-1][i] - round_p8g, 0)
  __shared__ int32_t sh_wide;       // P8: some column's LA spread exceeds P8_XMAX (16-bit window)
  __shared__ int32_t sh_gbad;       // P8: the window does not fit the shared base

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c = blockIdx.x;
  const int n = d.n, npad = d.npad, sm = d.sm, q4 = npad / 4;
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  if (d.state[ST_DONE]) return;
  if (PERS) p = 0;  // (the loop's first iteration has parity 0)
  int r = d.state[ST_CUR0 + p];
  int32_t own = d.Bp[(int64_t)p * n + c];  // B[r][c]: this workgroup's own boundary
  // (PERS: sc1 buffer loads of the candidates' rows)
  const __amdgpu_buffer_rsrc_t rs8 = __builtin_amdgcn_make_buffer_rsrc(d.cand8, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs16 = __builtin_amdgcn_make_buffer_rsrc(d.cand16, (short)0, 0x7fffffff, 0x00020000);
  int xcc = 0;
  int32_t gx = 0, nx = 0;
  if (PERS && t == 0) xcc = pbar_register(d);
  bool prestaged = false;  // (PERS) the first window of this round is in LDS already
  constexpr int PP8 = PP / 2, WRS8 = LPC * (PP8 + 1);  // P8: 16-B pieces of 16 columns per lane
  // the first window of chain c from row wk0 for round rr (own_: its
  // boundary): the fit check against the window's own and the shared base,
  // then the rows staged in LDS (sets p8, p8g, wb2).  PERS: the next round's
  // is staged while this round's grid barrier is waited for (its rows and
  // B[r] are known before the barrier)
  bool p8 = false, p8g = false;
  const uint32_t *wb2 = wbase2;
  // (PERS, P8) the window last staged: its first row, rows, base; the next
  // window reuses the rows both share -- re-based in LDS by each column's
  // base difference, split into a non-negative add and subtract (dpos, dneg)
  // so no byte carries -- and loads only the rows past them (BH_WIN_REUSE)
  int32_t ws_old = -1, wr_old = 0;
  bool p8_old = false, g_old = false;
  __shared__ uint16_t dpos16[256], dneg16[256];
  auto stage = [&](const int32_t wk0, const int wrows, const int rr, const int32_t own_, unsigned long long *sst = nullptr) {
      // COLS: the window's 36 aligned rows of every column from la_col, issued
      // before the fit check below reads its two rows
      constexpr int CQ = LPC * 16, CT = NT / CQ, CNP = (9 + CT - 1) / CT;  // column quads, threads per quad, pieces per thread
      const int cg = t % CQ, ch = t / CQ;
      const int32_t crb = (cs + wk0) & ~3;
      const int coff = cs + wk0 - crb;
      int4 cpv[COLS == 1 ? CNP : 1][4];
      if constexpr (COLS == 1) {
  #pragma unroll
        for (int u = 0; u < CNP; ++u) {
          const int pc = ch + u * CT;
  #pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int col = 4 * cg + k;
            cpv[u][k] = pc < 9 && col < n ? *reinterpret_cast<const int4 *>(d.la_col + (int64_t)col * la_col_stride(d) + (crb + 4 * pc))
                                          : make_int4(-1, -1, -1, -1);
          }
        }
      }
      p8 = false;
      p8g = false;
      if constexpr (P16) {
        if (d.round_p8) {
          // P8 when every column's spread down the window fits (first row: the
          // base, last row: the largest LA).  The first window of an iteration
          // whose previous round's boundaries are known also tries the shared
          // base (B[r-1][i] - round_p8g): then every candidate whose row its
          // producer already converted (c8tag) needs no conversion here
          const bool tryg = d.cand8 != nullptr && d.round_p8g > 0 && rr > d.r0 && wk0 == own_;
          if (t == 0) { sh_wide = 0; sh_gbad = !tryg; }
          __syncthreads();
          if (sst) sst[0] = __builtin_amdgcn_s_memrealtime();
          const int32_t *r0p = d.la + (int64_t)(cs + wk0) * npad, *r1p = r0p + (int64_t)(wrows - 1) * npad;
          const int32_t *Bprev = d.B + (int64_t)(rr - 1) * n;
          // LA of column i at the window's first / last row (-1 past n, 0 past npad)
          auto la_w = [&](int i, int last) -> int32_t {
            if (i >= npad) return 0;
            if constexpr (COLS == 1)
              return i < n ? d.la_col[(int64_t)i * la_col_stride(d) + cs + wk0 + (last ? wrows - 1 : 0)] : -1;
            else
              return (last ? r1p : r0p)[i];
          };
          bool bad = false, gbad = false;
          const uint32_t ob2 = (g_old ? gbase2 : wbase2)[t & 255];  // (the last window's base, columns 2t, 2t + 1)
          for (int j = t; j < 256; j += 256) {
            const int i0 = 2 * j, i1 = 2 * j + 1;
            const int32_t a0 = la_w(i0, 0), a1 = la_w(i1, 0);
            const int32_t z0 = la_w(i0, 1), z1 = la_w(i1, 1);
            const int32_t b0 = max(a0, 0), b1 = max(a1, 0);
            wbase2[j] = (uint32_t)b0 | ((uint32_t)b1 << 16);
            bad |= z0 + 1 - b0 > d.round_p8 || z1 + 1 - b1 > d.round_p8;
            if (tryg) {
              // columns past n keep the window base (their candidate bytes are 127 either way)
              const int32_t g0 = i0 < n ? max(ldx<PERS>(Bprev + i0) - d.round_p8g, 0) : b0;
              const int32_t g1 = i1 < n ? max(ldx<PERS>(Bprev + i1) - d.round_p8g, 0) : b1;
              gbase2[j] = (uint32_t)g0 | ((uint32_t)g1 << 16);
              gbad |= a0 + 1 < g0 || a1 + 1 < g1 || z0 + 1 - g0 > d.round_p8 || z1 + 1 - g1 > d.round_p8;
            }
          }
          if (__any(bad) && lane == 0) sh_wide = 1;
          if (__any(gbad) && lane == 0) sh_gbad = 1;
          __syncthreads();
          if (sst) sst[1] = __builtin_amdgcn_s_memrealtime();
          p8g = !sh_gbad;
          p8 = p8g || !sh_wide;
          if (PERS && COLS != 1 && d.win_reuse && p8 && p8_old && t < 256) {
            const uint32_t nb2 = (p8g ? gbase2 : wbase2)[t];
            const int32_t e0 = (int32_t)(ob2 & 0xFFFFu) - (int32_t)(nb2 & 0xFFFFu), e1 = (int32_t)(ob2 >> 16) - (int32_t)(nb2 >> 16);
            dpos16[t] = (uint16_t)(max(e0, 0) | (max(e1, 0) << 8));
            dneg16[t] = (uint16_t)(max(-e0, 0) | (max(-e1, 0) << 8));
          }
        }
      }
      wb2 = p8g ? gbase2 : wbase2;
      __syncthreads();
      if constexpr (COLS == 1) {
        // quad cg's 4 columns, 4 rows per piece: P8 one dword per row (bytes
        // x | 0x80, as below), P16 two (16-bit LA + 1 pairs); window row = the
        // piece's row - coff, rows outside [0, wrows) skipped
        uint32_t *w32 = reinterpret_cast<uint32_t *>(win4);
        uint32_t bs[4] = {0, 0, 0, 0};
        if (p8) {
          const uint32_t b01 = wb2[2 * cg], b23 = wb2[2 * cg + 1];
          bs[0] = b01 & 0xFFFFu; bs[1] = b01 >> 16; bs[2] = b23 & 0xFFFFu; bs[3] = b23 >> 16;
        }
        const int pc8 = cg >> 2, pc16 = cg >> 1;
        const int o8 = (pc8 + pc8 / PP8) * 4 + (cg & 3), o16 = (pc16 + pc16 / PP) * 4 + 2 * (cg & 1);
  #pragma unroll
        for (int u = 0; u < CNP; ++u) {
          const int pc = ch + u * CT;
          if (pc >= 9) continue;
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int wr = 4 * pc + e - coff;
            if (wr < 0 || wr >= wrows) continue;
            auto el = [&](int k) -> int32_t {
              const int4 v = cpv[u][k];
              return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
            };
            if (p8) {
              uint32_t x = 0;
  #pragma unroll
              for (int k = 0; k < 4; ++k) x |= ((uint32_t)(el(k) + 1 - (int32_t)bs[k]) & 0xFFu) << (8 * k);
              w32[wr * WRS8 * 4 + o8] = x | 0x80808080u;
            } else {
              w32[wr * WRS4 * 4 + o16] = pack_la16(el(0), el(1));
              w32[wr * WRS4 * 4 + o16 + 1] = pack_la16(el(2), el(3));
            }
          }
        }
      } else if (p8) {
        // columns 16 pc .. 16 pc + 15 as bytes x | 0x80
        constexpr int RP8 = LPC * PP8;
        const int4 *src = reinterpret_cast<const int4 *>(d.la + (int64_t)(cs + wk0) * npad);
        const int lim = wrows * RP8;
        auto ld8 = [&](int i, int4 (&a)[4]) {
  #pragma unroll
          for (int h = 0; h < 4; ++h) {
            const int row = i / RP8, col = 16 * (i - row * RP8) + 4 * h;  // npad is a multiple of 4
            a[h] = i < lim && col < npad ? src[row * q4 + col / 4] : make_int4(0, 0, 0, 0);
          }
        };
        auto put8 = [&](int i, const int4 (&a)[4]) {
          const int row = i / RP8, pc = i - row * RP8;
          uint32_t w[4];
  #pragma unroll
          for (int h = 0; h < 4; ++h) {
            const int col = 16 * pc + 4 * h;
            uint32_t v = 0x80808080u;
            if (col < npad) {
              const uint32_t b01 = wb2[col / 2], b23 = wb2[col / 2 + 1];
              const uint32_t x0 = (uint32_t)(a[h].x + 1 - (int32_t)(b01 & 0xFFFFu)), x1 = (uint32_t)(a[h].y + 1 - (int32_t)(b01 >> 16));
              const uint32_t x2 = (uint32_t)(a[h].z + 1 - (int32_t)(b23 & 0xFFFFu)), x3 = (uint32_t)(a[h].w + 1 - (int32_t)(b23 >> 16));
              v = (x0 | (x1 << 8) | (x2 << 16) | (x3 << 24)) | 0x80808080u;
            }
            w[h] = v;
          }
          win4[row * WRS8 + pc + pc / PP8] = make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
        };
        // rows shared with the last window: new row k = old row k + dl
        const int dl = wk0 - ws_old;
        const int nr = PERS && COLS != 1 && d.win_reuse && p8 && p8_old && ws_old >= 0 && dl >= 0 && dl < wr_old
                           ? min(wr_old - dl, wrows) : 0;
        if (nr > 0) {
          constexpr int NRI = (WROWS * RP8 + NT - 1) / NT;
          int4 o[NRI];
          const uint32_t *dp = reinterpret_cast<const uint32_t *>(dpos16), *dn = reinterpret_cast<const uint32_t *>(dneg16);
#pragma unroll
          for (int u = 0; u < NRI; ++u) {
            const int i = t + u * NT, row = i / RP8, pc = i - row * RP8;
            if (i < nr * RP8) o[u] = win4[(row + dl) * WRS8 + pc + pc / PP8];
          }
          __syncthreads();
#pragma unroll
          for (int u = 0; u < NRI; ++u) {
            const int i = t + u * NT, row = i / RP8, pc = i - row * RP8;
            if (i < nr * RP8) {
              const int m = 4 * pc;  // dwords of columns 16 pc ..
              win4[row * WRS8 + pc + pc / PP8] =
                  make_int4((int)(((uint32_t)o[u].x + dp[m]) - dn[m]), (int)(((uint32_t)o[u].y + dp[m + 1]) - dn[m + 1]),
                            (int)(((uint32_t)o[u].z + dp[m + 2]) - dn[m + 2]), (int)(((uint32_t)o[u].w + dp[m + 3]) - dn[m + 3]));
            }
          }
        }
        for (int i = nr * RP8 + t; i < lim; i += NT) {
          int4 a[4];
          ld8(i, a);
          put8(i, a);
        }
      } else {
        constexpr int RP = LPC * PP;  // pieces per padded row
        const int4 *src = reinterpret_cast<const int4 *>(d.la + (int64_t)(cs + wk0) * npad);
        for (int i = t; i < wrows * RP; i += NT) {
          const int row = i / RP, pc = i - row * RP;
          if constexpr (P16) {  // columns 8pc .. 8pc + 7 (npad is a multiple of 4)
            const int4 a = src[row * q4 + min(2 * pc, q4 - 1)];
            const int4 b = src[row * q4 + min(2 * pc + 1, q4 - 1)];
            const bool va = 8 * pc < npad, vb = 8 * pc + 4 < npad;  // else -1 (packs to 0)
            win4[row * WRS4 + pc + pc / PP] =
                make_int4(va ? (int)pack_la16(a.x, a.y) : 0, va ? (int)pack_la16(a.z, a.w) : 0,
                          vb ? (int)pack_la16(b.x, b.y) : 0, vb ? (int)pack_la16(b.z, b.w) : 0);
          } else {
            win4[row * WRS4 + pc + pc / PP] = pc < q4 ? src[row * q4 + pc] : make_int4(-1, -1, -1, -1);
          }
        }
      }
      if (t <= WROWS) hist[t] = 0;
      ws_old = wk0;
      wr_old = wrows;
      p8_old = p8;
      g_old = p8g;
      __syncthreads();
      if (sst) sst[2] = __builtin_amdgcn_s_memrealtime();
  };
  for (int it = 0;; ++it) {
  const int32_t *Bp = d.Bp + (int64_t)p * n;
  // BH_DIAG timeline (tools/timeline.py): start, first window staged, search
  // done, end -- chains < 128 of rounds TL_R0 .. TL_R0 + TL_NR
  const bool dgt = d.diag != nullptr && t == 0 && c < 128 && r >= TL_R0 && r < TL_R0 + TL_NR;
  const unsigned long long rt0 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
  unsigned long long rt1 = 0, rt2 = 0;
  constexpr int CPP = NT / LPC;
  const int part = t % LPC;
  const int npass = (n + CPP - 1) / CPP;
  if (t == 0) sh_nc = 0;
  __syncthreads();
  {
    // candidates of round r: counted before any window, since a chain whose
    // boundary already reached its end has no window at all and must still
    // write B[r + 1] = len (and not read as "no candidates anywhere")
    int nc = 0;
    for (int q = t; q < n; q += blockDim.x) nc += ldx<PERS>(Bp + q) < d.chain_len[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nc += __shfl_xor(nc, off);
    if (lane == 0 && nc) atomicAdd(&sh_nc, nc);
  }
  __syncthreads();
  int32_t wk0 = own;
  int32_t result = len;
  for (;;) {
    const int wrows = min(WROWS, len - wk0);
    if (wrows <= 0) break;
    if (!(PERS && prestaged && wk0 == own)) stage(wk0, wrows, r, own);  // (PERS: else staged during the barrier)
    prestaged = false;
    if (PERS && d.wide_prio) __builtin_amdgcn_s_setprio(0);
    if (dgt && !rt1) rt1 = __builtin_amdgcn_s_memrealtime();
    if (p8 && d.round_ilp2) {
      // byte rows, ILPK candidates per lane group at once (passes pass ..
      // pass + ILPK - 1): their binary searches interleave, so each probe's
      // LDS reads and compares overlap the others' (two waves per SIMD hide
      // little of a lone search's LDS latency)
      // a candidate's byte row, its tag and its chain's B / length are loaded
      // together, none waiting on another (the tag decides only afterwards
      // whether the bytes are used or the 16-bit row is converted)
      const int w8q = (npad + 15) / 16;
      auto raw_f8 = [&](int q, uint32_t (&f8)[4 * PP8]) {
        const int64_t f0 = ((int64_t)p * n + min(q, n - 1)) * w8q;
#pragma unroll
        for (int u = 0; u < PP8; ++u) {
          const int pc = part * PP8 + u;
          const int4 v = ld128<PERS>(rs8, reinterpret_cast<const int4 *>(d.cand8), f0 + min(pc, w8q - 1));
          const bool ok = pc < w8q;
          f8[4 * u] = ok ? (uint32_t)v.x : 0x7F7F7F7Fu;
          f8[4 * u + 1] = ok ? (uint32_t)v.y : 0x7F7F7F7Fu;
          f8[4 * u + 2] = ok ? (uint32_t)v.z : 0x7F7F7F7Fu;
          f8[4 * u + 3] = ok ? (uint32_t)v.w : 0x7F7F7F7Fu;
        }
      };
      auto load_f8 = [&](int q, bool act, int32_t tag, uint32_t (&f8)[4 * PP8]) {
        if (!(p8g && act && tag == r)) {
          const int f16q = (npad + 7) / 8;
          const int64_t f0 = ((int64_t)p * n + (act ? q : 0)) * f16q + part * PP;
          const int nvalid = f16q - part * PP;
          const uint4 *bb = reinterpret_cast<const uint4 *>(wb2) + part * PP;
#pragma unroll
          for (int u = 0; u < PP; ++u) {
            const int4 v = ld128<PERS>(rs16, reinterpret_cast<const int4 *>(d.cand16), f0 + min(u, max(nvalid - 1, 0)));
            const uint4 b = bb[u];
            const bool ok = u < nvalid;
            const uint32_t e0 = fd8x2(ok ? (uint32_t)v.x : 0xFFFFFFFFu, b.x), e1 = fd8x2(ok ? (uint32_t)v.y : 0xFFFFFFFFu, b.y);
            const uint32_t e2 = fd8x2(ok ? (uint32_t)v.z : 0xFFFFFFFFu, b.z), e3 = fd8x2(ok ? (uint32_t)v.w : 0xFFFFFFFFu, b.w);
            f8[2 * u] = pack8(e0, e1);
            f8[2 * u + 1] = pack8(e2, e3);
          }
        }
      };
      const int4 *xb8 = win4 + part * (PP8 + 1);
      for (int pass = 0; pass < npass; pass += ILPK) {
        // (BH_WIDE_PRIO=2: the two workgroups of a compute unit -- c and c +
        // G/2 in dispatch order -- take turns at the higher priority, pass by
        // pass, instead of the older one issuing first throughout)
        if (PERS && d.wide_prio == 2) {
          if (((pass / ILPK) ^ (2 * c >= (int)gridDim.x)) & 1) __builtin_amdgcn_s_setprio(1);
          else __builtin_amdgcn_s_setprio(0);
        }
        int qv[ILPK];
        bool act[ILPK];
        int32_t tag[ILPK];
        uint32_t f[ILPK][4 * PP8];
#pragma unroll
        for (int k = 0; k < ILPK; ++k) {
          qv[k] = (pass + k) * CPP + t / LPC;
          const int q1 = min(qv[k], n - 1);
          const int32_t bq = ldx<PERS>(Bp + q1), lq = d.chain_len[q1];
          tag[k] = ldx<PERS>(d.c8tag + (int64_t)p * n + q1);
          raw_f8(qv[k], f[k]);
          act[k] = qv[k] < n && bq < lq;
        }
#pragma unroll
        for (int k = 0; k < ILPK; ++k) load_f8(qv[k], act[k], tag[k], f[k]);
        // the ILPK candidates' probes of rows rw[k], all reads issued first
        auto ssk = [&](const int (&rw)[ILPK], bool (&sv)[ILPK]) {
          int4 x[ILPK][PP8];
#pragma unroll
          for (int k = 0; k < ILPK; ++k)
#pragma unroll
            for (int u = 0; u < PP8; ++u) x[k][u] = xb8[rw[k] * WRS8 + u];
          int g[ILPK];
#pragma unroll
          for (int k = 0; k < ILPK; ++k) g[k] = 0;
#pragma unroll
          for (int u = 0; u < PP8; ++u)
#pragma unroll
            for (int k = 0; k < ILPK; ++k) {
              g[k] += __builtin_popcount(((uint32_t)x[k][u].x - f[k][4 * u]) & 0x80808080u);
              g[k] += __builtin_popcount(((uint32_t)x[k][u].y - f[k][4 * u + 1]) & 0x80808080u);
              g[k] += __builtin_popcount(((uint32_t)x[k][u].z - f[k][4 * u + 2]) & 0x80808080u);
              g[k] += __builtin_popcount(((uint32_t)x[k][u].w - f[k][4 * u + 3]) & 0x80808080u);
            }
#pragma unroll
          for (int k = 0; k < ILPK; ++k) sv[k] = group_total<LPC>(g[k]) >= sm;
        };
        // binary search over [0, wrows - 1] without probing the last row
        // first: that row is probed afterwards only where no probe came out
        // true (the candidate is seen at the last row, or not at all -- few);
        // a short window's spare iterations probe lo == hi itself
        int lo[ILPK], hi[ILPK];
        bool vf[ILPK];
#pragma unroll
        for (int k = 0; k < ILPK; ++k) { lo[k] = 0; hi[k] = wrows - 1; vf[k] = false; }
#pragma unroll
        for (int pr = 0; pr < 5; ++pr) {
          int mid[ILPK];
          bool tv[ILPK];
#pragma unroll
          for (int k = 0; k < ILPK; ++k) mid[k] = (lo[k] + hi[k]) >> 1;  // (<= hi, also once lo = hi + 1)
          ssk(mid, tv);
#pragma unroll
          for (int k = 0; k < ILPK; ++k)
            if (lo[k] <= hi[k]) {
              if (tv[k]) { hi[k] = mid[k]; vf[k] = true; } else { lo[k] = mid[k] + 1; }
            }
        }
        bool un[ILPK], anyu = false;  // lo = hi = wrows - 1, unverified
#pragma unroll
        for (int k = 0; k < ILPK; ++k) { un[k] = !vf[k] && lo[k] < wrows; anyu |= un[k]; }
        if (__any(anyu)) {
          int last[ILPK];
          bool tv[ILPK];
#pragma unroll
          for (int k = 0; k < ILPK; ++k) last[k] = wrows - 1;
          ssk(last, tv);
#pragma unroll
          for (int k = 0; k < ILPK; ++k) vf[k] = vf[k] || (un[k] && tv[k]);
        }
#pragma unroll
        for (int k = 0; k < ILPK; ++k) {
          const int tw = vf[k] ? lo[k] : WROWS;
          if (act[k] && part == 0 && tw < WROWS) atomicAdd(&hist[tw], 1);
          if (d.ssw && part == 0 && qv[k] < n) tq_s[qv[k]] = (int8_t)(act[k] ? tw : WROWS);
        }
      }
    } else
    for (int pass = 0; pass < npass; ++pass) {
      const int q = pass * CPP + t / LPC;
      int32_t bq = 0, lq = 0, sq = 0;
      if (q < n) { bq = ldx<PERS>(Bp + q); lq = d.chain_len[q]; sq = d.chain_start[q]; }
      const bool act = q < n && bq < lq;
      int tw = WROWS;
      if (p8) {
        // the candidate's 16-bit FD row, window-relative 8-bit (fd8x2 / pack8)
        uint32_t f8[4 * PP8];
        if (p8g && act && ldx<PERS>(d.c8tag + (int64_t)p * n + q) == r) {
          // converted by its producer against the same shared base (handoff_wide)
          const int w8q = (npad + 15) / 16;  // 16-B pieces per cand8 row
          const int64_t f0 = ((int64_t)p * n + q) * w8q;
#pragma unroll
          for (int u = 0; u < PP8; ++u) {
            const int pc = part * PP8 + u;
            const int4 v = ld128<PERS>(rs8, reinterpret_cast<const int4 *>(d.cand8), f0 + min(pc, w8q - 1));  // (in the row: the pieces past it are 127s)
            const bool ok = pc < w8q;
            f8[4 * u] = ok ? (uint32_t)v.x : 0x7F7F7F7Fu;
            f8[4 * u + 1] = ok ? (uint32_t)v.y : 0x7F7F7F7Fu;
            f8[4 * u + 2] = ok ? (uint32_t)v.z : 0x7F7F7F7Fu;
            f8[4 * u + 3] = ok ? (uint32_t)v.w : 0x7F7F7F7Fu;
          }
        } else {
          const int f16q = (npad + 7) / 8;
          const int64_t f0 = ((int64_t)p * n + (act ? q : 0)) * f16q + part * PP;
          const int nvalid = f16q - part * PP;
          const uint4 *bb = reinterpret_cast<const uint4 *>(wb2) + part * PP;
#pragma unroll
          for (int u = 0; u < PP; ++u) {
            const int4 v = ld128<PERS>(rs16, reinterpret_cast<const int4 *>(d.cand16), f0 + min(u, max(nvalid - 1, 0)));
            const uint4 b = bb[u];
            const bool ok = u < nvalid;
            const uint32_t e0 = fd8x2(ok ? (uint32_t)v.x : 0xFFFFFFFFu, b.x), e1 = fd8x2(ok ? (uint32_t)v.y : 0xFFFFFFFFu, b.y);
            const uint32_t e2 = fd8x2(ok ? (uint32_t)v.z : 0xFFFFFFFFu, b.z), e3 = fd8x2(ok ? (uint32_t)v.w : 0xFFFFFFFFu, b.w);
            f8[2 * u] = pack8(e0, e1);
            f8[2 * u + 1] = pack8(e2, e3);
          }
        }
        const int4 *xb8 = win4 + part * (PP8 + 1);
        auto ss8 = [&](int row) -> bool {
          const int4 *x4 = xb8 + row * WRS8;
          int4 x[PP8];
#pragma unroll
          for (int u = 0; u < PP8; ++u) x[u] = x4[u];
          int ge = 0;
#pragma unroll
          for (int u = 0; u < PP8; ++u) {
            ge += __builtin_popcount(((uint32_t)x[u].x - f8[4 * u]) & 0x80808080u);
            ge += __builtin_popcount(((uint32_t)x[u].y - f8[4 * u + 1]) & 0x80808080u);
            ge += __builtin_popcount(((uint32_t)x[u].z - f8[4 * u + 2]) & 0x80808080u);
            ge += __builtin_popcount(((uint32_t)x[u].w - f8[4 * u + 3]) & 0x80808080u);
          }
          return group_total<LPC>(ge) >= sm;
        };
        if (ss8(wrows - 1)) {
          int lo = 0, hi = wrows - 1;
#pragma unroll
          for (int it = 0; it < 5; ++it) {
            const int mid = (lo + hi) >> 1;
            const bool s = ss8(mid);
            hi = s ? mid : hi;
            lo = s ? lo : mid + 1;
          }
          tw = lo;
        }
      } else {
      int4 f[PP];
      if constexpr (P16) {
        const int f16q = (npad + 7) / 8;  // 16-B pieces per cand16 row
        const int64_t f0 = ((int64_t)p * n + (act ? q : 0)) * f16q + part * PP;
        const int nvalid = f16q - part * PP;
#pragma unroll
        for (int u = 0; u < PP; ++u) {
          const int4 v = ld128<PERS>(rs16, reinterpret_cast<const int4 *>(d.cand16), f0 + min(u, max(nvalid - 1, 0)));
          f[u] = u < nvalid ? v : make_int4(-1, -1, -1, -1);  // 0xFFFF: never reached
        }
      } else {
        // every lane holds PIECES pieces; those past the row (pc >= q4) are
        // FD_NONE, which no LA value reaches, so the probe needs no per-piece
        // branch and its LDS reads issue back to back
        const int4 *fr = reinterpret_cast<const int4 *>(d.fd + (int64_t)(act ? sq + bq : 0) * npad) + part * PP;
        const int nvalid = q4 - part * PP;  // this lane's pieces inside the row
#pragma unroll
        for (int u = 0; u < PP; ++u) {
          const int4 v = fr[min(u, max(nvalid - 1, 0))];
          f[u] = u < nvalid ? v : make_int4(FD_NONE, FD_NONE, FD_NONE, FD_NONE);
        }
      }
      const int4 *xb = win4 + part * (PP + 1);
      auto ss = [&](int row) -> bool {
        const int4 *x4 = xb + row * WRS4;
        int4 x[PP];
#pragma unroll
        for (int u = 0; u < PP; ++u) x[u] = x4[u];
        int lt = 0;
        if constexpr (P16) {
          const uint32_t one = 0x00010001u;
          uint32_t acc = 0;
#pragma unroll
          for (int u = 0; u < PP; ++u) {
            acc = lt16x2_acc(acc, (uint32_t)x[u].x, (uint32_t)f[u].x, one);
            acc = lt16x2_acc(acc, (uint32_t)x[u].y, (uint32_t)f[u].y, one);
            acc = lt16x2_acc(acc, (uint32_t)x[u].z, (uint32_t)f[u].z, one);
            acc = lt16x2_acc(acc, (uint32_t)x[u].w, (uint32_t)f[u].w, one);
          }
          lt = (int)((acc & 0xFFFFu) + (acc >> 16));
        } else {
#pragma unroll
          for (int u = 0; u < PP; ++u) lt += lt4(x[u], f[u]);
        }
        constexpr int NCOL = LPC * PP * (P16 ? 8 : 4);  // columns per group, padding included
        return NCOL - group_total<LPC>(lt) >= sm;
      };
      if (ss(wrows - 1)) {
        int lo = 0, hi = wrows - 1;
#pragma unroll
        for (int it = 0; it < 5; ++it) {
          const int mid = (lo + hi) >> 1;
          const bool s = ss(mid);
          hi = s ? mid : hi;
          lo = s ? lo : mid + 1;
        }
        tw = lo;
      }
      }
      if (act && part == 0 && tw < WROWS) atomicAdd(&hist[tw], 1);
      if (d.ssw && part == 0 && q < n) tq_s[q] = (int8_t)(act ? tw : WROWS);
    }
    __syncthreads();
    if (dgt) rt2 = __builtin_amdgcn_s_memrealtime();
    if (sh_nc == 0) break;
    if (wave == 0) {
      int h = lane < wrows ? hist[lane] : 0;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(h, off);
        h += lane >= off ? o : 0;
      }
      const unsigned long long hit = __ballot(lane < wrows && h >= sm);
      if (lane == 0) sh_res = hit ? (int)__builtin_ctzll(hit) : -1;
    }
    __syncthreads();
    if (sh_res >= 0) { result = wk0 + sh_res; break; }
    wk0 += wrows;
  }
  // BH_WIDE_PRIO: the hand-off, the arrival and the next window's staging at
  // a higher priority -- the workgroup that ends a round last stages its next
  // window after everyone else has been released, beside its compute unit's
  // other workgroup's search, and that staging is the next round's critical
  // path (profiles/r4_ab_wide.txt, barrier phases)
  if (PERS && d.wide_prio) __builtin_amdgcn_s_setprio(2);
  // fame's input for the new candidate y = (c, result): the candidates of
  // round r it strongly sees are those whose T_q in the final window is at
  // most y's row (stronglySee is monotone along the chain)
  constexpr int NSW = 512 / NT;  // ssw words per wave
  unsigned long long swm[NSW];
  if (d.diag != nullptr && d.ssw && r >= TL_R0 && r < TL_R0 + TL_NR && c < 8) {
    // BH_DIAG: the candidates' T_q in the final window, its offset and the
    // result's (tools/tq_stats.py: how spread the searches' answers are)
    uint32_t *tq = reinterpret_cast<uint32_t *>(d.diag + DG_TQ + ((int64_t)(r - TL_R0) * 8 + c) * 66);
    for (int q = t; q < 128; q += NT) tq[q] = reinterpret_cast<const uint32_t *>(tq_s)[q];
    if (t == 0) {
      tq[128] = (uint32_t)(wk0 - own);
      tq[129] = (uint32_t)(result - own);
      tq[130] = (uint32_t)sh_nc;
      tq[131] = (uint32_t)n;
    }
  }
  const bool has_ssw = d.ssw && sh_nc > 0 && result < len && r + 1 < d.R_cap;
  if (has_ssw) {
    const int res = sh_res;
#pragma unroll
    for (int k = 0; k < NSW; ++k) {
      const int q = k * NT + t;
      swm[k] = __ballot(q < n && tq_s[q] <= res);
      if (!PERS && lane == 0) d.ssw[ballot_row(d, c, r + 1) * 8 + ((k * NT) >> 6) + wave] = swm[k];
    }
  }
  // the hand-off: the new candidate's FD row for the next iteration
  if (P16 && sh_nc > 0 && result < len && r + 1 < d.R_cap) {
    if constexpr (COLS != 0) handoff_wide_cols<NT, PERS>(d, p, c, result, Bp, r + 1);
    else handoff_wide<PERS>(d, (int64_t)cs + result, p ^ 1, c, Bp, r + 1);
  }
  if (dgt) {
    unsigned long long *tl = d.diag + DG_TL + ((r - TL_R0) * 128 + c) * 4;
    tl[0] = rt0;
    tl[1] = rt2;
    tl[2] = rt1;
    tl[3] = __builtin_amdgcn_s_memrealtime();
  }
  // the loop's end (the same in every workgroup: the candidate count and
  // the round are), else this iteration's boundary
  const bool stop = sh_nc == 0 || r + 1 >= d.R_cap;
  if (t == 0) {
    if (sh_nc == 0) {
      if (c == 0) { d.state[ST_ROUNDS] = r; d.state[ST_ITERS] = r; d.state[ST_DONE] = 1; signal_done(d); }
    } else if (r + 1 >= d.R_cap) {
      if (c == 0) { d.state[ST_ERR] = 1; d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; signal_done(d); }
    } else {
      stx<PERS>(d.Bp + (int64_t)(p ^ 1) * n + c, result);
      if (!PERS) d.B[(int64_t)(r + 1) * n + c] = result;  // (PERS: after the arrival below)
      if (c == 0) {
        d.state[ST_CUR0 + (p ^ 1)] = r + 1;
        d.state[ST_ITERS] = r + 1;
      }
    }
  }
  if (!PERS || stop) return;
  // ---- grid barrier (PERS) ----
  // BH_DIAG barrier phases (every chain): end, arrived, staged, released
  const bool dgb = d.diag != nullptr && t == 0 && r >= TL_R0 && r < TL_R0 + TL_NR;
  unsigned long long *tlb = dgb ? d.diag + DG_TLB + ((int64_t)(r - TL_R0) * 512 + c) * 4 : nullptr;
  if (dgb) tlb[0] = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have left
  __syncthreads();
  if (t < 64) pbar_arrive(d, it, xcc, gx, gridDim.x, nx);
  if (dgb) tlb[1] = __builtin_amdgcn_s_memrealtime();
  // fame's ballots and the round table: read after the loop, or B[r + 1]
  // two barriers from now (the shared base) -- stored after the arrival, so
  // the drain above waits only for the hand-over
  if (has_ssw && lane == 0)
#pragma unroll
    for (int k = 0; k < NSW; ++k) d.ssw[ballot_row(d, c, r + 1) * 8 + ((k * NT) >> 6) + wave] = swm[k];
  if (t == 0) stx<PERS>(d.B + (int64_t)(r + 1) * n + c, result);
  {
    // the next round's first window, staged while the other workgroups
    // arrive: its rows start at this round's result, its shared base is
    // B[r] (stored before the previous barrier)
    const int wrows_n = min(WROWS, len - result);
    if (wrows_n > 0 && d.prestage) {
      stage(result, wrows_n, r + 1, result, dgb ? d.diag + DG_TLS + ((int64_t)(r - TL_R0) * 512 + c) * 4 : nullptr);
      prestaged = true;
    }
  }
  if (dgb) tlb[2] = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    sh_res = pbar_wait(d, it, gridDim.x) ? 0 : -1;
    if (it == 0) pbar_counts(d, xcc, gx, nx);
  }
  if (dgb) tlb[3] = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  if (sh_res < 0) {  // the barrier gave up: the host restores the inputs and relaunches per iteration
    if (t == 0) {
      d.state[ST_ERR] = 3;
      d.state[ST_ROUNDS] = r;
      d.state[ST_DONE] = 1;
      if (c == 0) signal_done(d);
    }
    return;
  }
  own = result;
  ++r;
  p ^= 1;
  }  // for (it)
}

// ---------------------------------------------------------------------------
// k_round2(p): the round-loop iteration for n <= 128 (npad <= 128), built so
// that every load it starts with is independent of B[r]:
//   * candfd[p][q]  -- the firstDescendants row of candidate q, written by
//                      workgroup q of the previous iteration (it knew its new
//                      boundary B[r][q] and had that row in LDS);
//   * LA rows B[r][c] .. +32 of chain c -- read straight from la: the
//     previous iteration's window covered them, so they come from L2 / MALL.
// 1024 threads: LPC lanes per candidate, 4 x 16-B pieces of its FD row per
// lane in registers.  The search is over ROWS, for all candidates at once:
// count(k) = #{q : window row k strongly sees q} is monotone in k, and
// B[r+1][c] = the first k with count(k) >= SM.  A probe reads one window row
// (every lane group reads the same 128 B per instruction: an LDS broadcast),
// compares 16 columns per lane, sums over the group with DPP, and counts the
// groups that reach SM with a ballot.  While the search runs, the FD rows of
// the window are loaded; afterwards the workgroup hands over candfd for the
// new boundary.  Windows that do not reach SM fall back to direct loads.
constexpr int HW = 32;  // rows handed over per chain

template <int LPC>
__device__ __forceinline__ int group_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
  if (LPC >= 8) v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, true);  // row_half_mirror
  return v;
}

// The first row j of chain i at or after row `lo` (of [lo, hi)) whose LA
// in column c is >= k, or hi if none: firstDescendants read from the
// column-major LA (FD[(c, k)][i] = min{j : LA[(i, j)][c]
// >= k}, and LA[(i, j)][c] is non-decreasing in j).  `col` = LA[.][c] from
// chain i's first row.  Found by the 16 lanes of every aligned lane group
// with `on` set (col, lo, hi, k uniform over the group); every lane of the
// wave calls it.  One dependent load per pass: a first pass over the 1024
// rows after lo (16 probes 64 apart, when `near`), then 16-ary narrowing,
// spans of <= 64 rows finished with 4 rows a lane.
// GL-lane groups (GL = 16 or 8): GL-ary narrowing, spans of <= 4 GL rows
// finished with 4 rows a lane; `near`: the first pass covers the 64 GL rows
// after lo only (an entry just past a hand-off's loaded rows)
template <int GL>
__device__ __forceinline__ int32_t first_ge_group(const int32_t *col, int32_t lo, int32_t hi, int32_t k, bool on,
                                                  bool near) {
  constexpr uint32_t GM = (1u << GL) - 1u;
  const int lane = threadIdx.x & 63, g = lane & (GL - 1), gb = lane & (64 - GL);
  while (__any(on)) {
    if (on) {
      if (hi - lo <= 4 * GL) {
        const int32_t x = lo + 4 * g;
        int cnt = 0;
#pragma unroll
        for (int v = 0; v < 4; ++v)
          cnt += __popc((uint32_t)(__ballot(x + v < hi && col[x + v] < k) >> gb) & GM);
        lo += cnt;
        on = false;
      } else {
        const int32_t lim = near ? min(hi, lo + 64 * GL) : hi;
        const int32_t s = (lim - lo + GL - 1) / GL;
        const int32_t pr = min(lo + (g + 1) * s, lim) - 1;
        const uint32_t m = (uint32_t)(__ballot(col[pr] >= k) >> gb) & GM;
        if (m) {
          const int f = __builtin_ctz(m);
          hi = min(lo + (f + 1) * s, lim);
          lo += f * s;
        } else {
          lo = lim;
          on = lim < hi;
        }
        near = false;
      }
    }
  }
  return lo;
}

__device__ __forceinline__ int32_t first_ge16(const int32_t *col, int32_t lo, int32_t hi, int32_t k, bool on,
                                              bool near) {
  return first_ge_group<16>(col, lo, hi, k, on, near);
}

// candidates' FD rows for the first iteration of a loop (parity 0): round 0
// (B = 0) or the resume round ST_RESUME (B[r0]), searched in la_col -- one
// workgroup per candidate chain c, a 16-lane group per chain i
__device__ __forceinline__ void cand_row(const Dev &d, int c, int32_t r, int32_t b) {
  const int t = threadIdx.x;
  if (t == 0 && d.c8tag) d.c8tag[c] = d.c8tag[d.n + c] = -1;
  if (d.fd_cols) {
    // the parity-1 hand-off slots, which the loop's iteration 1 must not take
    // for its own: top byte 0 (k_round2p's tag 1 differs) and bit 0 set
    // (k_round_lean's tag bit for iteration 1 is 0)
    for (int i = t; i < d.npad; i += blockDim.x) d.candfd[((int64_t)d.n + c) * d.npad + i] = 1;
    if (t == 0) d.Bp[d.n + c] = 0;
  }
  if (b >= d.chain_len[c]) return;  // no candidate on chain c
  if (d.cla && t < d.npad)  // the candidate's LA row (fame)
    d.cla[cla_row(d, c, r) * d.npad + t] =
        t < d.n ? d.la_col[(int64_t)t * la_col_stride(d) + d.chain_start[c] + b] : -1;
  const int32_t *colc = d.la_col + (int64_t)c * la_col_stride(d);
  int32_t *cf = d.candfd + (int64_t)c * d.npad;
  // the wide loop's rows (wide_cols): 16-bit FD + 1 (0xFFFF: none), the
  // entries up to npad rounded to 8 (cand16's row)
  const int w16 = (d.npad + 7) / 8 * 4;
  uint16_t *c16 = d.wide_cols ? reinterpret_cast<uint16_t *>(d.cand16 + (int64_t)c * w16) : nullptr;
  const int nrow = c16 ? 2 * w16 : d.npad;
  // 8-lane groups when that covers every row in one pass (1024 threads,
  // npad <= 128: the segment start's dependent loads once, not twice)
  const bool g8 = !c16 && nrow * 8 <= (int)blockDim.x;
  const int gsh = g8 ? 3 : 4;
  for (int i0 = 0; i0 < nrow; i0 += blockDim.x >> gsh) {  // (uniform trip count)
    const int i = i0 + (t >> gsh);
    const bool on = i < d.n;
    const int32_t cs = on ? d.chain_start[i] : 0, len = on ? d.chain_len[i] : 0;
    // FD[(c, b)][i] >= B[r][i]: (c, b = B[r][c]) is in round >= r, and so
    // is every event that sees it (a round is the maximum of its parents'
    // or one more) -- the search starts there, and usually ends within the
    // first rows after it (two dependent loads instead of ~5 over the chain)
    const int32_t lo0 = r > 0 && on ? min(d.B[(int64_t)r * d.n + i], len) : 0;
    const int32_t j = g8 ? first_ge_group<8>(colc + cs, lo0, len, b, on && len > lo0, r > 0)
                         : first_ge16(colc + cs, lo0, len, b, on && len > lo0, r > 0);
    const int32_t f = on && j < len ? j : FD_NONE;
    if ((t & ((1 << gsh) - 1)) == 0 && i < nrow) {
      if (c16) c16[i] = (uint16_t)min((uint32_t)f + 1u, 0xFFFFu);
      else cf[i] = d.cand_fe ? (int32_t)fe_encode(f, 0) : f;  // (k_round_lean: iteration 0's tag bit is 0)
    }
  }
}

__global__ __launch_bounds__(1024) void k_cand_rows(Dev d, int from_resume) {
  const int c = blockIdx.x;
  const int32_t r = from_resume ? d.state[ST_RESUME] : 0;
  if (c == 0 && threadIdx.x == 0) d.state[ST_GATE] = d.state[ST_FLOWOVF] == 2 ? 1 : 0;  // (k_round2p's entry gate)
  cand_row(d, c, r, from_resume ? d.B[(int64_t)r * d.n + c] : 0);
}

// A segment's start in one launch (the n <= 128 persistent pipeline, segments
// after the first): the previous segment's resume point (k_resume_point's
// search, made by every workgroup -- the view's seg_lo is the previous
// prefix's lengths, its chain_len this one's), then k_round_resume's and
// k_cand_rows' work for chain c.  Three launches and their dispatch gaps
// were ~70 us between two segments' loops at C3 (profiles/r5_gaps_c3_async.txt).
// The search: 8 lanes per chain, a pass over the last 64 rounds, then 8-ary
// over what is left of [0, R] (B[R][q] >= len_q)
__global__ __launch_bounds__(1024) void k_seg_resume(Dev d) {
  __shared__ int32_t m;
  const int c = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const int n = d.n;
  const int32_t R = d.state[ST_ROUNDS];
  if (t == 0) m = R;
  __syncthreads();
  for (int q0 = 0; q0 < n; q0 += (int)(blockDim.x >> 3)) {  // (uniform trip count)
    const int q = q0 + (t >> 3), g = t & 7, gb = lane & 56;
    const bool on = q < n;
    const int32_t len = on ? d.seg_lo[q] : 0;
    int32_t lo = 0, hi = R;  // the first r in [lo, hi] with B[r][q] >= len
    if (R >= 64) {
      // a first pass over the last 64 rounds (where a segment's boundary
      // usually lies: two dependent loads instead of ~5), rows R - 64 + 8 g
      const bool ge = on && d.B[(int64_t)(R - 64 + 8 * g) * n + q] >= len;
      const uint32_t mk = (uint32_t)(__ballot(ge) >> gb) & 0xFFu;
      if (mk & 1u) {
        hi = R - 64;  // at or before row R - 64: the whole range below
      } else if (mk) {
        const int f = __builtin_ctz(mk);
        lo = R - 64 + 8 * (f - 1) + 1;
        hi = R - 64 + 8 * f;
      } else {
        lo = R - 7;
      }
    }
    bool go = on && lo < hi;
    while (__any(go)) {
      const int32_t s = (hi - lo + 7) >> 3;
      const int32_t pr = min(lo + (g + 1) * s, hi) - 1;
      const bool ge = go && d.B[(int64_t)pr * n + q] >= len;
      const uint32_t mk = (uint32_t)(__ballot(ge) >> gb) & 0xFFu;
      if (go) {
        if (mk) {
          const int f = __builtin_ctz(mk);
          hi = min(lo + (f + 1) * s, hi) - 1;
          lo += f * s;
        } else {
          lo = min(lo + 8 * s, hi);
        }
        go = lo < hi;
      }
    }
    if (on && g == 0) {
      if (c == 0 && d.rq) d.rq[q] = lo;
      if (d.chain_len[q] > len) atomicMin(&m, lo);
    }
  }
  __syncthreads();
  const int32_t r0 = max(d.r0, m - 1);
  const int32_t b = d.B[(int64_t)r0 * n + c];
  if (t == 0) {
    d.Bp[c] = b;
    if (c == 0) {
      // (ST_ROUNDS stays: every workgroup reads it above; the loop sets it)
      d.state[ST_RESUME] = r0;
      d.state[ST_PFAIL] = max(d.state[ST_PFAIL], d.state[ST_ERR]);
      d.state[ST_GATE] = d.state[ST_FLOWOVF] == 2 ? 1 : 0;  // (k_round2p's entry gate)
      d.state[ST_CUR0] = r0;
      d.state[ST_CUR0 + 1] = 0;
      d.state[ST_DONE] = 0;
      d.state[ST_ERR] = 0;
      d.state[ST_ITERS] = r0;
    }
  }
  cand_row(d, c, r0, b);
}

void launch_seg_resume(const Dev &d, hipStream_t s) {
  Dev dd = d;
  dd.cand_fe = cand_fe(d);
  k_seg_resume<<<d.n, 1024, 0, s>>>(dd);
}

// TQ (default): every lane group binary-searches its own T_q (the first
// window row strongly seeing candidate q) with no barrier between probes; one
// 33-bin histogram + prefix then gives B[r+1][c] = the first row where
// #{q : T_q <= row} reaches SM.  !TQ (BH_ROUND_ROWS=1, A/B): the row-probe
// search -- the workgroup binary-searches count(row) together, one barrier
// per probe.  Same compares per probe; the groups of a wave read different
// rows, so each group starts its four 128-B chunks at chunk (q & 3).
// 8 lanes per candidate, PPL 16-B pieces of its FD row per lane (LPC * PPL *
// 4 >= npad columns), 8 npad threads (rounded up to whole waves): the
// workgroup is as wide as its candidates need -- at n = 32 four waves of one
// piece per lane instead of sixteen waves of four pieces.
//
// Round 4: the loop reads only the dataflow's column-major LA (la_col); no
// row-major LA and no firstDescendants table are built for it.
//   * The window: HWL = 32 rows of every column from rb = the window's first
//     row rounded down to 4, one aligned 16-B piece (4 rows of one column)
//     per thread (one load instruction per lane), stored transposed into the
//     row-major LDS window; the search runs over its rows off .. 31 (off =
//     the alignment offset, 29 to 32 rows: on the C3 DAG B[r+1][c] - B[r][c]
//     is 12 on average and at most 28; a later row is found by the fallback,
//     window by window).
//   * The hand-off: the new candidate (c, B[r+1][c])'s FD row.  FD[(c, k)][i]
//     is non-decreasing in k, so it starts at the previous candidate's entry
//     j0 = FD[(c, B[r][c])][i] (its row, candfd[p][c]).  At the start of the
//     iteration every 16-lane group loads FDB = 64 rows of LA[.][c] on chain
//     i from j0 (rounded down to 4); once the boundary is known, the entry is
//     j0 + #{rows < the boundary index} -- one count and a group sum, no
//     dependent load.  A group whose 64 rows all stay below (a jump of more
//     than ~60 rows, e.g. a lagging chain's candidate) searches on
//     (first_ge16: usually two more loads).  Entries beyond the view's chain
//     lengths are MaxInt32, as the prefix semantics need (section 4.9).
constexpr int HWL = HW;     // staged window rows (8 aligned 16-B pieces per column)
constexpr int FDB = 64;      // LA rows per chain loaded for the hand-off

// the first iteration's candidate rows (round 0, or the resume round)
void launch_cand_rows(const Dev &d, int from_resume, hipStream_t s) {
  Dev dd = d;
  dd.cand_fe = cand_fe(d);
  k_cand_rows<<<d.n, 1024, 0, s>>>(dd, from_resume);
}

// The hand-off's per-lane inputs (k_round2 / k_round2p): chain i = t / 8
// (8 lanes per chain, n <= 128 = nt / 8), its first row and view length,
// the previous candidate's entry j0 = FD[(c, B[r][c])][i], and the lane's
// 8 rows of LA[.][c] on chain i: 2 aligned 16-B pieces at ab + 8 (t % 8)
// (ab = chain i's row of j0 rounded down to 4; FDB = 64 rows per chain).
template <int NP = 2>
struct HandInT {
  int32_t j0, cs, len;
  int4 fb[NP];
};
using HandIn = HandInT<2>;

template <int NP>
__device__ __forceinline__ void hand_load(const int32_t *colc, HandInT<NP> &h) {
  const int l8 = threadIdx.x & 7;
  const bool live = h.j0 != FD_NONE;
  const int32_t a = live ? (h.cs + h.j0) & ~3 : 0;
#pragma unroll
  for (int u = 0; u < NP; ++u)
    h.fb[u] = live ? *reinterpret_cast<const int4 *>(colc + (a + 4 * NP * l8 + 4 * u)) : make_int4(0, 0, 0, 0);
}

// FD[(c, row)][i] for the lane's chain i: j0 + #{rows from j0 below `row`}
// among the 32 NP loaded (a count and a group sum); an entry beyond them
// (rare) is searched by the wave, chain by chain (first_ge_wave).  Every lane
// of the chain's group returns it; FD_NONE if no row of the view sees (c, row)
template <int NP>
__device__ __forceinline__ int32_t hand_entry(const int32_t *colc, const HandInT<NP> &h, int i, int c, int32_t row) {
  constexpr int FB = 32 * NP;
  const int lane = threadIdx.x & 63, l8 = lane & 7;
  const bool live = h.j0 != FD_NONE;
  const int32_t a = h.cs + h.j0, ab = a & ~3, end = h.cs + h.len;
  const int32_t x0 = ab + 4 * NP * l8, elo = a - x0, ehi = end - x0;  // rows a .. end - 1 of the lane's 4 NP
  int cnt = 0;
  if (live) {
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      cnt += (4 * u + 0 >= elo) & (4 * u + 0 < ehi) & (h.fb[u].x < row);
      cnt += (4 * u + 1 >= elo) & (4 * u + 1 < ehi) & (h.fb[u].y < row);
      cnt += (4 * u + 2 >= elo) & (4 * u + 2 < ehi) & (h.fb[u].z < row);
      cnt += (4 * u + 3 >= elo) & (4 * u + 3 < ehi) & (h.fb[u].w < row);
    }
  }
  cnt = group_total<8>(cnt);
  const int32_t jn = a + cnt, bend = min(ab + FB, end);
  int32_t fd = FD_NONE;
  bool miss = false;
  if (live) {
    if (i == c) fd = row;  // an event is its own first descendant
    else if (jn < bend) fd = jn - h.cs;
    else miss = bend < end;  // (else: no row of chain i in this view sees the candidate)
  }
  // the entry lies beyond the rows loaded (a lagging chain's candidate jumps
  // far): every such chain's 8 lanes search on at once, the first pass over
  // the 512 rows after them
  if (__any(miss)) {
    const int32_t j = first_ge_group<8>(colc, bend, end, row, miss, true);
    if (miss) fd = j < end ? j - h.cs : FD_NONE;
  }
  return fd;
}

template <int PPL, bool TQ>
__global__ __launch_bounds__(1024) void k_round2(Dev d, int p) {
  constexpr int LPC = 8;
  extern __shared__ __attribute__((aligned(16))) int4 sm4[];
  __shared__ int32_t cntk[16];
  __shared__ int32_t hist[HW + 1];  // TQ: T_q histogram; [HW] = the answer row
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nt = blockDim.x;
  const int c = blockIdx.x;
  const int n = d.n, npad = d.npad, sm = d.sm, q4 = npad / 4;
  const int rs4 = q4 + 1, rs = 4 * rs4;  // window row stride (one spare piece: staging stores spread over banks)
  const int64_t stride = la_col_stride(d);
  int4 *win = sm4;  // [HWL][rs4]: LA rows rb .. rb + HWL - 1
  int32_t *win32 = reinterpret_cast<int32_t *>(sm4);
  const int32_t *Bp = d.Bp + (int64_t)p * n;
  const bool dg = d.diag != nullptr && t == 0;
  const unsigned long long ts0 = dg ? stamp() : 0;
  const unsigned long long rt0 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
  // ---- independent loads ----
  const int done = d.state[ST_DONE];
  const int r = d.state[ST_CUR0 + p];
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  const int32_t k0 = Bp[c];
  const int q = t / LPC, part = t % LPC;
  const int rot = TQ ? (q & (PPL - 1)) : 0;  // piece order of this group (bank spread)
  int32_t bq = 0, lq = 0;
  if (q < n) { bq = Bp[q]; lq = d.chain_len[q]; }
  int4 f[PPL];
  {
    const int4 *cf = reinterpret_cast<const int4 *>(d.candfd) + ((int64_t)p * n + min(q, n - 1)) * q4;
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      const int pc = part + LPC * ((u + rot) & (PPL - 1));
      f[u] = pc < q4 ? cf[pc] : make_int4(FD_NONE, FD_NONE, FD_NONE, FD_NONE);
    }
  }
  // the hand-off's inputs (HandIn): chain t / 8 of this lane
  const int32_t *colc = d.la_col + (int64_t)c * stride;  // LA[.][c]
  HandIn hin{FD_NONE, 0, 0, {}};
  {
    const int i = t >> 3;
    if (i < n && k0 < len) {
      hin.j0 = d.candfd[((int64_t)p * n + c) * npad + i];
      hin.cs = d.chain_start[i];
      hin.len = d.chain_len[i];
    }
  }
  // the window's pieces: thread t stages column t / 8, rows rb + 4 (t % 8) .. + 3
  const int32_t rb = (cs + k0) & ~3;
  const int off = cs + k0 - rb;
  const int wi = t >> 3, wr4 = 4 * (t & 7);
  const int4 wv = wi < n ? *reinterpret_cast<const int4 *>(d.la_col + (int64_t)wi * stride + (rb + wr4))
                         : make_int4(-1, -1, -1, -1);
  if (done) return;
  hand_load(colc, hin);  // the hand-off's 64 rows of LA[.][c] per chain (depend on j0 only)
  const bool act = q < n && bq < lq;
  const int rows = min(HWL - off, max(0, len - k0));  // (the window's rows off .. HWL - 1)
  if (wi < n) {
    win32[(wr4 + 0) * rs + wi] = wv.x;
    win32[(wr4 + 1) * rs + wi] = wv.y;
    win32[(wr4 + 2) * rs + wi] = wv.z;
    win32[(wr4 + 3) * rs + wi] = wv.w;
  }
  if (npad > n)  // columns past n: LA -1 (never >= an FD)
    for (int j = t; j < (npad - n) * HWL; j += nt) win32[(j / (npad - n)) * rs + n + j % (npad - n)] = -1;
  if (t < 16) cntk[t] = 0;
  if (TQ && t <= HW) hist[t] = 0;
  __syncthreads();
  const unsigned long long ts1 = dg ? stamp() : 0;
  const unsigned long long rt1 = dg ? __builtin_amdgcn_s_memrealtime() : 0;  // loads landed
  // does window row x4 strongly see this group's candidate?
  auto ss_row = [&](const int4 *x4) {
    int4 x[PPL];  // all reads first: one LDS round trip per probe
#pragma unroll
    for (int u = 0; u < PPL; ++u) x[u] = x4[min(part + LPC * ((u + rot) & (PPL - 1)), q4 - 1)];
    int lt = 0;
#pragma unroll
    for (int u = 0; u < PPL; ++u) lt += lt4(x[u], f[u]);
    return LPC * PPL * 4 - group_sum<LPC>(lt) >= sm;
  };
  auto probe = [&](const int4 *x4, int slot) {
    const bool s = ss_row(x4);
    const unsigned long long m = __ballot(act && part == 0 && s);
    if (lane == 0 && m) atomicAdd(&cntk[slot], __popcll(m));
    return m;  // this wave's candidates the row strongly sees (fame's S_j)
  };
  {
    const unsigned long long m = __ballot(act && part == 0);
    if (lane == 0 && m) atomicAdd(&cntk[0], __popcll(m));
  }
  const int4 *w0 = win + off * rs4;  // window row 0 = row k0 of chain c
  int slot = 1;
  int32_t res = -1;  // window row of B[r+1][c], or -1
  unsigned long long ssb = 0;  // this wave's ballot of the probe that verified the answer row
  if (TQ && rows > 0) {
    // T_q by a per-group binary search over [0, rows] (rows = none in the window)
    int lo = 0, hi = rows;
    while (__any(lo < hi)) {
      const int mid = (lo + hi) >> 1;
      const bool s = ss_row(w0 + min(mid, rows - 1) * rs4);
      if (lo < hi) {
        hi = s ? mid : hi;
        lo = s ? lo : mid + 1;
      }
    }
    if (act && part == 0 && lo < rows) atomicAdd(&hist[lo], 1);
    __syncthreads();
    if (wave == 0) {
      int h = lane < rows ? hist[lane] : 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int x = __shfl_up(h, o);
        h += lane >= o ? x : 0;
      }
      const unsigned long long hit = __ballot(lane < rows && h >= sm);
      if (lane == 0) hist[HW] = hit ? (int)__builtin_ctzll(hit) : -1;
    }
    __syncthreads();
    res = hist[HW];
    // fame's S_j for the new candidate: the candidates whose T_q is at most its row
    ssb = __ballot(act && part == 0 && res >= 0 && lo <= res);
  } else if (rows > 0) {
    // binary search assuming the window's last row reaches SM (count is
    // monotone); that row is probed only if the search ends on it unverified
    int lo = 0, hi = rows - 1;
    bool hi_ok = false;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      const unsigned long long m = probe(w0 + mid * rs4, slot);
      __syncthreads();
      if (cntk[slot] >= sm) {
        hi = mid;
        hi_ok = true;
        ssb = m;
      } else {
        lo = mid + 1;
      }
      ++slot;
    }
    if (!hi_ok) {
      ssb = probe(w0 + hi * rs4, slot);
      __syncthreads();
      hi_ok = cntk[slot] >= sm;
    }
    if (hi_ok) res = lo;
  } else {
    __syncthreads();
  }
  const int nc = cntk[0];
  const unsigned long long ts2 = dg ? stamp() : 0;
  const unsigned long long rt2 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
  int32_t result = len;
  int lrow = 0;  // the LDS window row holding the result's LA row
  if (res >= 0) {
    result = k0 + res;
    lrow = off + res;
  } else if (nc > 0 && rows == HWL - off) {
    // SM not reached in the window (rare): the next windows of chain c,
    // staged the same way (slot counters are reused per row tested)
    if (d.diag && t == 0) atomicAdd(&d.diag[DG_RD_WMISS], 1ull);
    for (int32_t wk = k0 + rows, wr = 0; wk < len && result == len; wk += wr) {
      const int32_t rb2 = (cs + wk) & ~3;
      const int off2 = cs + wk - rb2;
      wr = min(HWL - off2, len - wk);
      __syncthreads();
      if (wi < n) {
        const int4 v = *reinterpret_cast<const int4 *>(d.la_col + (int64_t)wi * stride + (rb2 + wr4));
        win32[(wr4 + 0) * rs + wi] = v.x;
        win32[(wr4 + 1) * rs + wi] = v.y;
        win32[(wr4 + 2) * rs + wi] = v.z;
        win32[(wr4 + 3) * rs + wi] = v.w;
      }
      if (t < 16) cntk[t] = 0;
      __syncthreads();
      const int4 *x4 = win + off2 * rs4;
      const unsigned long long ml = probe(x4 + (wr - 1) * rs4, 1);
      __syncthreads();
      if (cntk[1] < sm) continue;
      int lo = 0, hi = wr - 1, sl = 1;
      ssb = ml;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        ++sl;
        const unsigned long long m = probe(x4 + mid * rs4, sl);
        __syncthreads();
        if (cntk[sl] >= sm) {
          hi = mid;
          ssb = m;
        } else {
          lo = mid + 1;
        }
      }
      result = wk + lo;
      lrow = off2 + lo;
    }
    __syncthreads();
  }
  // ---- hand-off for the next iteration: FD[(c, result)][i] ----
  if (nc > 0 && r + 1 < d.R_cap && result < len) {
    const int32_t fdv = hand_entry(colc, hin, t >> 3, c, result);
    if ((t & 7) == 0 && (t >> 3) < npad) d.candfd[((int64_t)(p ^ 1) * n + c) * npad + (t >> 3)] = fdv;
    // fame's inputs for the new candidate y = (c, result): its LA row (from
    // the window in LDS) and SS(y, q) over the candidates q of round r = the
    // ballots of the probe that verified y's row.  Raw ballots, one aligned
    // 8-B word per wave (candidate q at bit 8 (q % 8) of word q / 8; fame
    // packs the LPC-strided bits and masks the words of chains >= n, which
    // fewer waves leave unwritten), chain-major [c][round]; issued last,
    // since a later vmcnt wait would include them
    if (t < npad) d.cla[cla_row(d, c, r + 1) * npad + t] = win32[lrow * rs + t];
    if (lane == 0) d.ssm[ballot_row(d, c, r + 1) * 16 + wave] = ssb;
  }
  if (dg) {
    const unsigned long long te = stamp();
    if (r >= TL_R0 && r < TL_R0 + TL_NR && c < 128) {
      unsigned long long *tl = d.diag + DG_TL + ((r - TL_R0) * 128 + c) * 4;
      const unsigned long long fl = (unsigned long long)(min(result - k0, 255) & 255) |
                                    (unsigned long long)(res < 0) << 8 | (unsigned long long)(nc > 0) << 9;
      tl[0] = rt0 | fl << 52; tl[1] = rt2; tl[2] = rt1; tl[3] = __builtin_amdgcn_s_memrealtime();
    } else if (r < TL_R0 - 64 || r >= TL_R0 + TL_NR + 64) {
      // phase counters (device-scope atomics from every workgroup: they
      // stretch the round by several us, so none near the timeline window)
      atomicAdd(&d.diag[DG_RD_B], ts1 - ts0);
      atomicAdd(&d.diag[DG_RD_LOAD], 0ull);
      atomicAdd(&d.diag[DG_RD_COMP], ts2 - ts1);
      atomicAdd(&d.diag[DG_RD_TOTAL], te - ts0);
      atomicAdd(&d.diag[DG_RD_CALLS], 1ull);
    }
  }
  if (t == 0) {
    if (nc == 0) {  // no candidates: R = r
      if (c == 0) { d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; signal_done(d); }
      return;
    }
    if (r + 1 >= d.R_cap) {
      if (c == 0) { d.state[ST_ERR] = 1; d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; signal_done(d); }
      return;
    }
    d.Bp[(int64_t)(p ^ 1) * n + c] = result;
    d.B[(int64_t)(r + 1) * n + c] = result;
    if (c == 0) {
      d.state[ST_CUR0 + (p ^ 1)] = r + 1;
      d.state[ST_ITERS] = r + 1;
    }
  }
}

// k_round2p: the n <= 128 round loop as ONE launch of n workgroups, one per
// chain (default; BH_ROUND_PERSIST=0: one k_round2 launch per iteration).
// Each iteration is k_round2's (TQ search, hand-off counted from 64 LA rows
// per chain); no kernel boundary and no grid barrier between iterations
// (round 5): what crosses from one iteration to the next -- each
// candidate's boundary (Bp) and FD row (candfd) -- is stored sc1 as
// self-validating dwords, the iteration's low 8 bits in the top byte, and a
// consumer reloads (sc1, volatile) until every dword it needs carries the
// tag (MI355X_MICROARCH.md, data-tagged granules: one hop, where a barrier
// costs an arrival, a release and the loads behind it).  Values fit 24 bits
// (chain rows < 2^24 - 1; 0xFFFFFF is FD_NONE).  What a workgroup needs of
// its own chain -- the next window (rows from its new boundary) and the LA
// rows its next hand-off counts from -- is loaded before the wait and staged
// while the candidates' rows are in flight.  Every workgroup sees the same
// candidate count, so each decides the loop's end itself.  The wait is
// bounded (d.pbar_spin polls; ST_ERR = 3: a word never arrived -- the host
// then restores the loop's inputs and runs one launch per iteration).
// Co-residency: n <= 128 workgroups of 16 waves fit the 256 compute units
// beside the segment pipeline's coordinate workgroups, and those never wait
// for the loop, so every loop workgroup is placed.

// F32 search (round 5): LA and FD entries are integers below 2^24, exact in
// f32, so #{LA < FD} over two columns is one packed subtract whose clamp
// output modifier turns each difference FD - LA (an integer) into the
// indicator [LA < FD] -- v_pk_add_f32 with the clamp bit, which the compiler
// does not form from fmin/fmax -- and a packed add accumulates the pairs:
// one instruction per column instead of 2.5 (subtract, shift, 3-way add)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 lt_ind2(f32x2 fd, f32x2 la) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1] clamp" : "=v"(r) : "v"(fd), "v"(la));
  return r;
}
__device__ __forceinline__ f32x2 lo2(int4 v) { return f32x2{__int_as_float(v.x), __int_as_float(v.y)}; }
__device__ __forceinline__ f32x2 hi2(int4 v) { return f32x2{__int_as_float(v.z), __int_as_float(v.w)}; }
__device__ __forceinline__ int4 f32_bits4(int4 v) {
  return make_int4(__float_as_int((float)v.x), __float_as_int((float)v.y), __float_as_int((float)v.z),
                   __float_as_int((float)v.w));
}

// the probe's dependent chain, shortened: window rows of a constant width
// (the row offset a shift and an add -- the compiler had turned __mul24 by
// the runtime width into the quarter-rate v_mul_lo_u32 -- and a lane's four
// pieces at immediate offsets from one address), and the lane group's
// indicator sum in f32 straight through DPP (v_add_f32_dpp: no convert
// before the group sum)
template <int RB>
__device__ __forceinline__ int row_bytes(int m) {  // m * RB by the full-rate 24-bit multiply (the compiler picks a 64-bit mad)
  int r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "i"(RB), "v"(m));
  return r;
}
template <int LPC>
__device__ __forceinline__ float group_total_f(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));  // quad_perm [1,0,3,2]
  if (LPC >= 4) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));
  if (LPC >= 8) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, true));
  return v;
}

template <int PPL, bool F32>
__global__ __launch_bounds__(1024) void k_round2p(Dev d) {
  constexpr int LPC = 8;
  extern __shared__ __attribute__((aligned(16))) int4 sm4[];
  __shared__ int32_t cntk[16];
  __shared__ int32_t hist[HW + 1];
  __shared__ int32_t sh_fail;
  __shared__ uint32_t sh_cur;  // (BH_DIAG: the last wave's inputs-current time this round, low 32 bits)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nt = blockDim.x;
  const int c = blockIdx.x;
  // the segment pipeline enqueues every segment's loop without a host round
  // trip: after a failed one (ST_PFAIL: capacity, or a barrier that gave up)
  // or unfinished coordinates (ST_FLOWOVF = 2: a split block without room),
  // the later ones leave at once -- every workgroup reads the same words,
  // written before the launch by the kernels ahead of it on the loop stream
  // (ST_GATE: the copy of ST_FLOWOVF k_cand_rows / k_seg_resume took; the
  // word itself can change mid-dispatch when a later segment's unpack
  // overflows) -- and the host falls back after the last
  if (d.state[ST_PFAIL] || d.state[ST_GATE]) {
    if (c == 0 && t == 0) {
      d.state[ST_DONE] = 1;
      signal_done(d);
    }
    return;
  }
  const int n = d.n, npad = d.npad, sm = d.sm, q4 = npad / 4;
  // window rows of LPC * PPL pieces whatever npad (columns past n hold -1):
  // a lane's four pieces are one LDS base plus immediate offsets
  constexpr int rs4 = LPC * PPL + 1, rs = 4 * rs4;
  const int64_t stride = la_col_stride(d);
  int4 *win = sm4;
  int32_t *win32 = reinterpret_cast<int32_t *>(sm4);
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  // (one piece order for every candidate: the four pieces' LDS addresses are
  // one base plus immediate offsets, three VALU off each probe's chain)
  const int q = t / LPC, part = t % LPC, rot = 0;
  const int32_t lq = q < n ? d.chain_len[q] : 0;
  const int32_t *colc = d.la_col + (int64_t)c * stride;
  const __amdgpu_buffer_rsrc_t cfr = __builtin_amdgcn_make_buffer_rsrc(d.candfd, (short)0, 0x7fffffff, 0x00020000);
  int32_t r = d.state[ST_CUR0];  // the first iteration has parity 0
  int32_t k0 = d.Bp[c];
  HandIn hin{FD_NONE, 0, 0, {}};  // chain t / 8's hand-off inputs
  if ((t >> 3) < n) {
    hin.cs = d.chain_start[t >> 3];
    hin.len = d.chain_len[t >> 3];
    if (k0 < len) hin.j0 = d.candfd[(int64_t)c * npad + (t >> 3)];
  }
  const int wi = t >> 3, wr4 = 4 * (t & 7);
  const bool wst = wi < n;
  int4 wv;
  auto own_loads = [&]() {  // chain c's window from k0 and its hand-off rows from j0
    const int32_t rb = (cs + k0) & ~3;
    wv = wst && k0 < len ? *reinterpret_cast<const int4 *>(d.la_col + (int64_t)wi * stride + (rb + wr4))
                         : make_int4(-1, -1, -1, -1);
    hand_load(colc, hin);
  };
  own_loads();
  if (t == 0) sh_fail = 0;
  if (4 * LPC * PPL > n)  // columns past n: LA -1 (never >= an FD); the staging never writes them
    for (int j = t; j < (4 * LPC * PPL - n) * HWL; j += nt)
      win32[(j / (4 * LPC * PPL - n)) * rs + n + j % (4 * LPC * PPL - n)] = F32 ? __float_as_int(-1.f) : -1;
  int p = 0;
  // a candidate piece's dwords all carry tag `want` in their top byte
  auto tagged = [](int4 v, uint32_t want) {
    const uint32_t an = (uint32_t)(v.x & v.y & v.z & v.w) >> 24, o = (uint32_t)(v.x | v.y | v.z | v.w) >> 24;
    return an == want && o == want;
  };
  constexpr uint32_t VMASK24 = 0xFFFFFFu;  // value bits of a handed-over dword (0xFFFFFF: FD_NONE)
  for (int it = 0;; ++it) {
    // BH_DIAG timeline (tools/timeline.py): iteration start (inputs current),
    // window staged, search done, hand-off stored -- rounds TL_R0 .. + TL_NR
    const bool dgt = d.diag != nullptr && t == 0 && r >= TL_R0 && r < TL_R0 + TL_NR;
    // round r's candidates: boundaries (Bp) and FD rows (candfd), stored by
    // the other workgroups at the end of round r - 1 as self-validating
    // dwords -- tag `it` & 255 (the launch's iteration) in the top byte, the
    // value below it -- with no barrier: a lane reloads until every dword it
    // needs carries the tag (MI355X_MICROARCH.md, data-tagged granules: one
    // hop instead of a flag or a grid barrier and the loads behind it).  An
    // iteration's buffer (parity p) last held iteration it - 2's rows, whose
    // tag differs, and no workgroup writes it again before every workgroup
    // has published iteration it + 1's -- i.e. has finished reading this
    // one's.  Iteration 0's inputs were written before the launch (untagged
    // values, top byte 0 or 0x7F: the same decode), and k_cand_rows zeroed
    // parity 1 (tag 0), which iteration 1 must not take for its own
    const uint32_t want = (uint32_t)it & 0xFFu;
    uint32_t bqr = 0;
    int4 f[PPL];
    const int32_t row0 = (int32_t)(((int64_t)p * n + min(q, n - 1)) * npad * 4);
    auto load_in = [&]() {
      bqr = q < n ? (uint32_t)__hip_atomic_load(d.Bp + (int64_t)p * n + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
      for (int u = 0; u < PPL; ++u) {
        const int pc = part + LPC * ((u + rot) & (PPL - 1));
        // (sc1, and volatile -- bit 31 -- so the poll below reloads)
        f[u] = pc < q4 ? __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(cfr, row0 + 16 * pc, 0,
                                                                                         (int)0x80000010u))
                       : make_int4(FD_NONE, FD_NONE, FD_NONE, FD_NONE);
      }
    };
    const unsigned long long rtp = dgt ? __builtin_amdgcn_s_memrealtime() : 0;  // waiting starts
    int32_t polls = 0;
    load_in();
    // the window first (its rows were loaded at the end of the last
    // iteration): staged while the candidates' rows are in flight, so each
    // wave starts its search as soon as ITS candidates' rows are current
    const int off = (cs + k0) & 3;
    const int rows = min(HWL - off, max(0, len - k0));
    if (wst) {
      const int4 sv = F32 ? f32_bits4(wv) : wv;
      win32[(wr4 + 0) * rs + wi] = sv.x;
      win32[(wr4 + 1) * rs + wi] = sv.y;
      win32[(wr4 + 2) * rs + wi] = sv.z;
      win32[(wr4 + 3) * rs + wi] = sv.w;
    }
    if (t < 16) cntk[t] = 0;
    if (t <= HW) hist[t] = 0;
    if (t == 0) sh_cur = 0;
    __syncthreads();
    const unsigned long long rt1 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    if (it > 0) {
      for (int32_t spin = 0;; ++spin, ++polls) {
        bool ok = q >= n || (bqr >> 24) == want;
        if (ok && q < n && (int32_t)(bqr & VMASK24) < lq) {  // a live candidate: its row as well
#pragma unroll
          for (int u = 0; u < PPL; ++u)
            ok &= part + LPC * ((u + rot) & (PPL - 1)) >= q4 || tagged(f[u], want);
        }
        if (__all(ok)) break;
        if (spin >= d.pbar_spin) {  // a workgroup never published: the host falls back
          sh_fail = 1;  // (read after the search's first workgroup barrier)
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (!ok) load_in();
      }
    }
    const unsigned long long rt0 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    if (d.diag != nullptr && lane == 0) atomicMax(&sh_cur, (uint32_t)__builtin_amdgcn_s_memrealtime());
    unsigned long long rt2 = 0;
    const int32_t bq = (int32_t)(bqr & VMASK24);
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      f[u] = make_int4(f[u].x & VMASK24, f[u].y & VMASK24, f[u].z & VMASK24, f[u].w & VMASK24);
      if (F32) f[u] = f32_bits4(f[u]);
    }
    const bool act = q < n && bq < lq;
    const float ltmax = (float)(LPC * PPL * 4 - sm);  // the most LA < FD columns a strongly seeing row has
    auto ss_row = [&](const int4 *x4) {
      int4 x[PPL];
#pragma unroll
      for (int u = 0; u < PPL; ++u) x[u] = x4[part + LPC * ((u + rot) & (PPL - 1))];
      int lt = 0;
      if constexpr (F32) {
        // every indicator pair first, then a tree of packed adds (no
        // dependent VOP3P back to back)
        f32x2 a[2 * PPL];
#pragma unroll
        for (int u = 0; u < PPL; ++u) {
          a[2 * u] = lt_ind2(lo2(f[u]), lo2(x[u]));
          a[2 * u + 1] = lt_ind2(hi2(f[u]), hi2(x[u]));
        }
#pragma unroll
        for (int w = 1; w < 2 * PPL; w *= 2)
#pragma unroll
          for (int u = 0; u + w < 2 * PPL; u += 2 * w) a[u] += a[u + w];
        return group_total_f<LPC>(a[0].x + a[0].y) <= ltmax;  // (#{LA >= FD} >= sm)
      } else {
#pragma unroll
        for (int u = 0; u < PPL; ++u) lt += lt4(x[u], f[u]);
      }
      return LPC * PPL * 4 - group_sum<LPC>(lt) >= sm;
    };
    auto probe = [&](const int4 *x4, int slot) {
      const bool sv = ss_row(x4);
      const unsigned long long m = __ballot(act && part == 0 && sv);
      if (lane == 0 && m) atomicAdd(&cntk[slot], __popcll(m));
      return m;
    };
    {
      const unsigned long long m = __ballot(act && part == 0);
      if (lane == 0 && m) atomicAdd(&cntk[0], __popcll(m));
    }
    const int4 *w0 = win + off * rs4;
    int32_t res = -1;
    unsigned long long ssb = 0;
    unsigned long long rs1 = 0, rs2 = 0;  // (BH_DIAG: probes done, histogram complete)
    int nprobe = 0;
    if (rows > 0) {  // T_q per lane group, then the histogram (k_round2's TQ search)
      int lo = 0, hi = rows;
      while (__any(lo < hi)) {
        ++nprobe;
        const int mid = (lo + hi) >> 1;
        const bool sv = ss_row(reinterpret_cast<const int4 *>(reinterpret_cast<const char *>(w0) +
                                                               row_bytes<16 * rs4>(min(mid, rows - 1))));
        if (lo < hi) {
          hi = sv ? mid : hi;
          lo = sv ? lo : mid + 1;
        }
      }
      if (dgt) rs1 = __builtin_amdgcn_s_memrealtime();
      if (act && part == 0 && lo < rows) atomicAdd(&hist[lo], 1);
      __syncthreads();
      if (dgt) rs2 = __builtin_amdgcn_s_memrealtime();
      if (sh_fail) {  // a workgroup never published: ST_ERR = 3, the host falls back
        if (t == 0) {
          d.state[ST_ERR] = 3;
          d.state[ST_ROUNDS] = r;
          d.state[ST_DONE] = 1;
          if (c == 0) signal_done(d);
        }
        break;
      }
      // every wave: the first row whose prefix count reaches SM -- an
      // inclusive DPP scan of the bins (row_shr 1, 2, 4, 8 within 16 lanes,
      // then row_bcast 15 / 31 across them), no second barrier
      {
        int h = lane < rows ? hist[lane] : 0;
        h += __builtin_amdgcn_update_dpp(0, h, 0x111, 0xF, 0xF, true);  // row_shr:1
        h += __builtin_amdgcn_update_dpp(0, h, 0x112, 0xF, 0xF, true);  // row_shr:2
        h += __builtin_amdgcn_update_dpp(0, h, 0x114, 0xF, 0xF, true);  // row_shr:4
        h += __builtin_amdgcn_update_dpp(0, h, 0x118, 0xF, 0xF, true);  // row_shr:8
        h += __builtin_amdgcn_update_dpp(0, h, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
        h += __builtin_amdgcn_update_dpp(0, h, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2, 3
        const unsigned long long hit = __ballot(lane < rows && h >= sm);
        res = hit ? (int)__builtin_ctzll(hit) : -1;
      }
      ssb = __ballot(act && part == 0 && res >= 0 && lo <= res);
    } else {
      __syncthreads();
      if (sh_fail) {  // a workgroup never published: ST_ERR = 3, the host falls back
        if (t == 0) {
          d.state[ST_ERR] = 3;
          d.state[ST_ROUNDS] = r;
          d.state[ST_DONE] = 1;
          if (c == 0) signal_done(d);
        }
        break;
      }
    }
    const int nc = cntk[0];
    if (dgt) rt2 = __builtin_amdgcn_s_memrealtime();
    int32_t result = len;
    int lrow = 0;
    if (res >= 0) {
      result = k0 + res;
      lrow = off + res;
    } else if (nc > 0 && rows == HWL - off) {
      // SM not reached in the window (rare): the next windows, staged alike
      for (int32_t wk = k0 + rows, wr = 0; wk < len && result == len; wk += wr) {
        const int32_t rb2 = (cs + wk) & ~3;
        const int off2 = cs + wk - rb2;
        wr = min(HWL - off2, len - wk);
        __syncthreads();
        if (wst) {
          int4 v = *reinterpret_cast<const int4 *>(d.la_col + (int64_t)wi * stride + (rb2 + wr4));
          if (F32) v = f32_bits4(v);
          win32[(wr4 + 0) * rs + wi] = v.x;
          win32[(wr4 + 1) * rs + wi] = v.y;
          win32[(wr4 + 2) * rs + wi] = v.z;
          win32[(wr4 + 3) * rs + wi] = v.w;
        }
        if (t < 16) cntk[t] = 0;
        __syncthreads();
        const int4 *x4 = win + off2 * rs4;
        const unsigned long long ml = probe(x4 + (wr - 1) * rs4, 1);
        __syncthreads();
        if (cntk[1] < sm) continue;
        int lo = 0, hi = wr - 1, sl = 1;
        ssb = ml;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          ++sl;
          const unsigned long long m = probe(x4 + mid * rs4, sl);
          __syncthreads();
          if (cntk[sl] >= sm) {
            hi = mid;
            ssb = m;
          } else {
            lo = mid + 1;
          }
        }
        result = wk + lo;
        lrow = off2 + lo;
      }
      __syncthreads();
    }
    // the loop's end, the same in every workgroup: no candidates (R = r), or
    // the round table's capacity
    if (nc == 0 || r + 1 >= d.R_cap) {
      if (c == 0 && t == 0) {
        if (nc > 0) d.state[ST_ERR] = 1;
        d.state[ST_ROUNDS] = r;
        d.state[ST_ITERS] = r;
        d.state[ST_DONE] = 1;
        signal_done(d);
      }
      break;
    }
    // ---- hand-off: FD[(c, result)][i] and B[r + 1][c], tagged it + 1 ----
    const uint32_t tagw = (uint32_t)((it + 1) & 0xFF) << 24;
    int32_t fdv = FD_NONE;
    if (result < len) {
      fdv = hand_entry(colc, hin, t >> 3, c, result);
      if ((t & 7) == 0 && (t >> 3) < npad)
        __hip_atomic_store(d.candfd + ((int64_t)(p ^ 1) * n + c) * npad + (t >> 3),
                           (int32_t)(tagw | ((uint32_t)fdv & VMASK24)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0)
      __hip_atomic_store(d.Bp + (int64_t)(p ^ 1) * n + c, (int32_t)(tagw | (uint32_t)result), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    if (dgt && c < 128) {
      unsigned long long *tl = d.diag + DG_TL + ((r - TL_R0) * 128 + c) * 4;
      tl[0] = rt0;
      tl[1] = rt2;
      tl[2] = rt1;
      tl[3] = __builtin_amdgcn_s_memrealtime();
      // the hand-over's phases (tools/timeline.py --tagged): waiting starts,
      // inputs current, polls, this round's rows stored
      unsigned long long *tb = d.diag + DG_TLB + ((int64_t)(r - TL_R0) * 512 + c) * 4;
      tb[0] = rtp;
      tb[1] = rt0;
      tb[2] = (unsigned long long)polls;
      tb[3] = tl[3];
      // the search's phases (tools/timeline.py --tagged): wave 0's probes
      // done, the histogram complete (every wave's probes), probes of wave 0
      unsigned long long *ts = d.diag + DG_TLS + ((int64_t)(r - TL_R0) * 512 + c) * 4;
      ts[0] = rs1;
      ts[1] = rs2;
      ts[2] = (unsigned long long)nprobe | (unsigned long long)(sh_cur - (uint32_t)rt0) << 32;
      ts[3] = rt2;
    }
    // what no workgroup reads inside the loop -- fame's inputs (the new
    // candidate's LA row and its ballots) and the round table
    if (result < len) {
      if (t < npad)
        d.cla[cla_row(d, c, r + 1) * npad + t] = F32 ? (int32_t)__int_as_float(win32[lrow * rs + t]) : win32[lrow * rs + t];
      if (lane == 0) d.ssm[ballot_row(d, c, r + 1) * 16 + wave] = ssb;
    }
    if (t == 0) d.B[(int64_t)(r + 1) * n + c] = result;
    ++r;
    p ^= 1;
    k0 = result;
    hin.j0 = result < len ? fdv : FD_NONE;
    own_loads();  // the next window and hand-off rows: they land while the candidates are awaited
    __syncthreads();  // (the window, cntk and hist are rewritten next)
  }
}

// ---------------------------------------------------------------------------
// k_round_lean<PPL, FULL, DIAG>: k_round2p's loop -- the same search, the
// same tagged hand-off, the same results -- cut down for VALU issue (round
// 6).  What bounds k_round2p's work (profiles/pmc_sq.json, n128_N10000000):
// ~396 VALU instructions per wave per round; 16 waves on 4 SIMDs issue one
// wave-instruction per cycle per CU, so ~6,300 cycles = 2.6 us at 2.4 GHz,
// which is the round's measured work (profiles/r6_timeline_c3_base.txt).
// The loop is VALU-issue-bound on its CU, not LDS- or latency-bound.  Here:
//  * float entries: the producers store each FD entry x as fe_encode's f32
//    2^22 + x + b / 2 (b: a 1-bit tag, iteration it's (it >> 1) & 1, which
//    tells it from the parity buffer's last use, it - 2), and the window
//    stages LA as la + 2^22 + b / 2 (a convert and an add), so a received
//    row is used as it arrives and clamp(FD - LA) (v_pk_add_f32 ... clamp)
//    is the 0/1 indicator [LA < FD] (FD - LA = fd - la, an integer);
//  * the per-candidate search is five fixed probes with no loop control: the
//    probed row is an LDS immediate offset from the lane's address, one add
//    and one select move it; rows past the window's valid ones read +inf (a
//    sentinel that strongly sees everything), so the search is over
//    [0, min(rows, 31)] and 31 or the sentinel row means "not in the window";
//  * window rows at a power-of-two stride with their first 128 B repeated
//    after them: candidates 2 and 3 of every four read their pieces 128 B
//    further on (the repeat covers the wrap), so the 16 lanes of each LDS
//    cycle group of a ds_read_b128 touch 16 different bank quads whichever
//    rows their candidates probe;
//  * the hand-off counts the lane's 8 loaded rows without per-row bounds:
//    rows before the previous entry are below the new boundary (LA is
//    monotone on a chain), so the entry is the block's first row + the
//    group's count; a wave that has a chain within 64 rows of its end takes
//    hand_entry's bounded count;
//  * two windows and histograms by parity.
// Needs chains < 2^22 - 2 (else k_round2p's int32 search).
template <int PPL, bool FULL, bool DIAG>
__global__ __launch_bounds__(1024) void k_round_lean(Dev d) {
  constexpr int LPC = 8, RS4 = LPC * PPL, COLS = 4 * RS4, RB = 16 * RS4;
  constexpr int RST = RB + 128 <= 256 ? 256 : RB + 128 <= 512 ? 512 : 1024;  // window row stride, bytes
  constexpr int RSH = RST == 256 ? 8 : RST == 512 ? 9 : 10;
  constexpr int WR = HWL + 2;  // + two sentinel rows (a probe reaches row off + 30 <= 33)
  constexpr uint32_t WBYTES = (uint32_t)WR * RST;
  constexpr uint32_t BIAS = 0x4B800000u, INF = 0x7F800000u;  // (BIAS: the hand-off count's own domain)
  constexpr float FE_LA0 = 4194304.0f;  // 2^22: a window entry la is la + 2^22 + b / 2 (fe_encode's domain)
  constexpr uint32_t VMASK24 = 0xFFFFFFu;
  // the hand-off's rows per chain: 8 lanes x 4 HNP (32 rows: an entry past them in 6 % of
  // workgroup-rounds, 77 % of rounds, C3 32.0 -> 32.9 ms)
  constexpr int HNP = 2, FBL = 32 * HNP;
  extern __shared__ __attribute__((aligned(16))) int4 sm4[];
  char *const wb = reinterpret_cast<char *>(sm4);
  uint32_t *const wb32 = reinterpret_cast<uint32_t *>(sm4);
  __shared__ int32_t cntk[2][16];
  __shared__ int32_t hist[2][HW + 1];
  __shared__ int32_t sh_fail;
  __shared__ uint32_t sh_cur, sh_pend, sh_st, sh_flags, sh_hs;  // (DIAG: the last wave's inputs current, probes done, hand-off start, store)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nt = blockDim.x;
  const int c = blockIdx.x;
  if (d.state[ST_PFAIL] || d.state[ST_GATE]) {  // (k_round2p's entry gate)
    if (c == 0 && t == 0) {
      d.state[ST_DONE] = 1;
      signal_done(d);
    }
    return;
  }
  const int n = d.n, npad = d.npad, sm = d.sm, q4 = npad / 4;
  const int64_t stride = la_col_stride(d);
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  const int q = t / LPC, part = t % LPC, rot = (q >> 1) & 1;
  const int qc = min(q, n - 1);
  const int32_t lq = q < n ? d.chain_len[q] : 0;
  const int32_t *colc = d.la_col + (int64_t)c * stride;
  const __amdgpu_buffer_rsrc_t cfr = __builtin_amdgcn_make_buffer_rsrc(d.candfd, (short)0, 0x7fffffff, 0x00020000);
  int32_t r = d.state[ST_CUR0];  // the first iteration has parity 0
  int32_t k0 = d.Bp[c];
  const int hc = t >> 3;  // the hand-off's chain
  HandInT<HNP> hin{FD_NONE, 0, 0, {}};
  if (hc < n) {
    hin.cs = d.chain_start[hc];
    hin.len = d.chain_len[hc];
    if (k0 < len) hin.j0 = fe_decode((uint32_t)d.candfd[(int64_t)c * npad + hc]);  // (k_cand_rows: float-encoded)
  }
  // the window's staging: thread t holds rows 4 sg .. 4 sg + 3 of column swi
  // (8 lanes per column: a wave's loads touch 8 cache lines, not 64 -- with
  // one column per lane, 1,024 line requests per round per workgroup slowed
  // the hand-off's loads: hop 1.5 -> 3.0 us.  The LDS writes of a column's
  // 8 lanes then share a bank: 8-way, off the critical path)
  const int swi = t >> 3, sg = t & 7;
  const bool sst = sg < 8 && swi < n;
  const int32_t *scol = d.la_col + (int64_t)(sst ? swi : 0) * stride;
  int4 wv;
  f32x2 hfb[2 * HNP];  // hin.fb biased (the fast hand-off count)
  bool hslow = false;  // the lane's 64-row block is not wholly inside chain hc (hand_entry's bounded count)
  auto own_loads = [&]() {  // chain c's window from k0 and the hand-off rows from j0
    const int32_t rb = (cs + k0) & ~3;
    wv = sst && k0 < len ? *reinterpret_cast<const int4 *>(scol + (rb + 4 * sg)) : make_int4(-1, -1, -1, -1);
    hand_load(colc, hin);
    const int32_t ab = (hin.cs + hin.j0) & ~3;
    hslow = hin.j0 != FD_NONE && (ab < hin.cs || ab + FBL > hin.cs + hin.len);
  };
  own_loads();
  // what no staging writes: columns n .. COLS (and their repeats) LA -1, the
  // two rows after the window +inf, in both parity windows
  for (int j = t; j < (int)(2 * WBYTES / 4); j += nt) {
    const int row = (j / (RST / 4)) % WR, col = j % (RST / 4);
    const int lc = col < COLS ? col : col < COLS + 32 ? col - COLS : COLS;
    if (row >= HWL) wb32[j] = INF;
    else if (lc >= n) wb32[j] = __float_as_uint(FE_LA0 - 1.0f);
  }
  if (t == 0) sh_fail = 0, sh_st = sh_flags = sh_hs = 0;
  const uint32_t lane_off = 16u * part + 128u * rot;  // the lane's first piece (rotated by 128 B for odd pairs)
  const int32_t rowq0 = (int32_t)((int64_t)qc * npad * 4), rowq1 = (int32_t)(((int64_t)n + qc) * npad * 4);
  const float ltmax = (float)(COLS - sm);  // the most LA < FD columns a strongly seeing row has
  // a candidate piece's global index for register u (the LDS read of u is at
  // lane_off + 128 u: piece part + 8 (u + rot), the last one in the repeat)
  auto gpiece = [&](int u) { return part + LPC * ((u + rot) & (PPL - 1)); };
  // the per-iteration stores' addresses, kept as running pointers (no 64-bit
  // multiplies or cla's ring modulo per round in the hand-off's scalar path)
  int32_t *const cfs0 = d.candfd + ((int64_t)n + c) * npad, *const cfs1 = d.candfd + (int64_t)c * npad;
  int32_t *const bps0 = d.Bp + n + c, *const bps1 = d.Bp + c;
  int32_t cla_pos = (r + 1 - d.rbase) % d.cla_span;
  const int32_t cla_span = d.cla_span;
  int32_t *const cla_c = d.cla + (int64_t)c * cla_span * npad;
  auto *ssm_p = d.ssm + ballot_row(d, c, r + 1) * 16 + wave;
  int32_t *b_p = d.B + (int64_t)(r + 1) * n + c;
  int p = 0;
  for (int it = 0;; ++it) {
    const bool dgt = DIAG && d.diag != nullptr && t == 0 && r >= TL_R0 && r < TL_R0 + TL_NR;
    const uint32_t want = (uint32_t)it & 0xFFu;  // (Bp's tag)
    const uint32_t tb = ((uint32_t)it >> 1) & 1u;  // (candfd's tag bit: iterations it and it - 2 differ)
    const float la_off = FE_LA0 + 0.5f * (float)tb;  // a window entry la stages as la + la_off
    uint32_t bqr = 0;
    int4 f[PPL];
    const int32_t row0 = p ? rowq1 : rowq0;
    auto load_in = [&]() {
      bqr = q < n ? (uint32_t)__hip_atomic_load(d.Bp + (int64_t)p * n + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      const int32_t none = (int32_t)fe_encode(FD_NONE, tb);  // (a padding column: FD_NONE, tagged)
#pragma unroll
      for (int u = 0; u < PPL; ++u)
        f[u] = FULL || gpiece(u) < q4 ? __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                    cfr, row0 + 16 * gpiece(u), 0, (int)0x80000010u))
                                      : make_int4(none, none, none, none);
    };
    const unsigned long long rtp = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    int32_t polls = 0;
    // the candidates' loads leave only once this wave's own hand-off stores
    // are acknowledged (~1.8 us after them): issued earlier they reach the
    // rows while the other workgroups are still writing them, and every
    // consumer's polls slow those writes down (k_round2p got this wait from
    // its loop latch; MEASUREMENTS.md round 6: polls 0 -> 2, hop 1.2 -> 4 us
    // without it; with the stores-before-loads barrier, C3 32.1 -> 35.5 ms
    // without it)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long rta = dgt ? __builtin_amdgcn_s_memrealtime() : 0;  // (own stores acknowledged)
    load_in();
    // this iteration's window (parity p), staged while the candidates' rows
    // are in flight; rows at or past the chain's end read +inf
    const uint32_t wbase = (uint32_t)p * WBYTES;
    const int32_t rb = (cs + k0) & ~3;
    const int off = cs + k0 - rb;
    const int rows = min(HWL - off, max(0, len - k0));
    const int R = min(rows, HWL - 1);  // searched rows [0, R); R: not in the window
    if (sst) {
      uint32_t v[4] = {__float_as_uint((float)wv.x + la_off), __float_as_uint((float)wv.y + la_off),
                       __float_as_uint((float)wv.z + la_off), __float_as_uint((float)wv.w + la_off)};
      const int32_t lim = cs + len - rb - 4 * sg;  // (uniform test: the window reaches the chain's end)
      if (cs + len < rb + HWL) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = j >= lim ? INF : v[j];
      }
      uint32_t *w = wb32 + (wbase + (uint32_t)(4 * sg) * RST) / 4 + swi;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j * (RST / 4)] = v[j];
      if (swi < 32) {
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j * (RST / 4) + COLS] = v[j];
      }
    }
    // the hand-off rows in the biased f32 domain (the fast count at the end)
#pragma unroll
    for (int u = 0; u < HNP; ++u) {
      hfb[2 * u] = f32x2{__uint_as_float((uint32_t)hin.fb[u].x + BIAS), __uint_as_float((uint32_t)hin.fb[u].y + BIAS)};
      hfb[2 * u + 1] = f32x2{__uint_as_float((uint32_t)hin.fb[u].z + BIAS), __uint_as_float((uint32_t)hin.fb[u].w + BIAS)};
    }
    if (t < 16) cntk[p][t] = 0;
    if (t <= HW) hist[p][t] = 0;
    if (DIAG && t == 0) sh_cur = sh_pend = 0;
    __syncthreads();
    const unsigned long long rt1 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    // round r's candidates, stored by the other workgroups at the end of
    // round r - 1 as dwords tagged with the iteration (k_round2p): reload
    // until every dword this lane needs carries tag `want`
    if (it > 0) {
      for (int32_t spin = 0;; ++spin) {
        bool ok = q >= n || (bqr >> 24) == want;
        if (ok && q < n && (int32_t)(bqr & VMASK24) < lq) {  // a live candidate: its row as well
          uint32_t an = 0xFFFFFFFFu, o = 0;
#pragma unroll
          for (int u = 0; u < PPL; ++u) {
            an &= (uint32_t)(f[u].x & f[u].y & f[u].z & f[u].w);
            o |= (uint32_t)(f[u].x | f[u].y | f[u].z | f[u].w);
          }
          ok = (an & 1u) == tb && (o & 1u) == tb;
        }
        if (__all(ok)) break;
        if (spin >= d.pbar_spin) {  // a workgroup never published: the host falls back
          sh_fail = 1;  // (read after the search's barrier)
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        ++polls;
        load_in();  // (the whole wave: no per-lane merge of old and new rows; the
                    // buffer is not rewritten before this workgroup publishes)
      }
    }
    const unsigned long long rt0 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    if (DIAG && d.diag != nullptr && lane == 0) atomicMax(&sh_cur, (uint32_t)__builtin_amdgcn_s_memrealtime());
    const int32_t bq = (int32_t)(bqr & VMASK24);
    const bool act = q < n && bq < lq;
    // the candidates' entries are used as they arrive: fe_encode's f32 (the
    // tag bit is the window's half; FD - LA is then an integer)
    f32x2 fd[2 * PPL];
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      fd[2 * u] = f32x2{__uint_as_float((uint32_t)f[u].x), __uint_as_float((uint32_t)f[u].y)};
      fd[2 * u + 1] = f32x2{__uint_as_float((uint32_t)f[u].z), __uint_as_float((uint32_t)f[u].w)};
    }
    // one window row (LDS byte address of the lane's first piece) strongly
    // sees candidate q: #{LA < FD} over its COLS columns <= COLS - SM
    auto ss_row = [&](uint32_t a) {
      f32x2 s[2 * PPL];
#pragma unroll
      for (int u = 0; u < PPL; ++u) {
        const int4 x = *reinterpret_cast<const int4 *>(wb + a + 128u * u);
        s[2 * u] = lt_ind2(fd[2 * u], f32x2{__int_as_float(x.x), __int_as_float(x.y)});
        s[2 * u + 1] = lt_ind2(fd[2 * u + 1], f32x2{__int_as_float(x.z), __int_as_float(x.w)});
      }
#pragma unroll
      for (int w = 1; w < 2 * PPL; w *= 2)
#pragma unroll
        for (int u = 0; u + w < 2 * PPL; u += 2 * w) s[u] += s[u + w];
      return group_total_f<LPC>(s[0].x + s[0].y) <= ltmax;
    };
    {
      const unsigned long long m = __ballot(act && part == 0);
      if (lane == 0 && m) atomicAdd(&cntk[p][0], __popcll(m));
    }
    // T_q: the first row in [0, 31] that strongly sees q (31: none in rows
    // 0 .. 30; rows >= R read +inf), five probes
    const uint32_t a0 = wbase + (uint32_t)off * RST + lane_off;
    uint32_t a = a0;
#pragma unroll
    for (int s = 4; s >= 0; --s) {
      const bool sv = ss_row(a + (uint32_t)((1 << s) - 1) * RST);
      a = sv ? a : a + (uint32_t)(1 << s) * RST;
    }
    const int pos = (int)((a - a0) >> RSH);
    const unsigned long long rs1 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    if (DIAG && d.diag != nullptr && lane == 0) atomicMax(&sh_pend, (uint32_t)__builtin_amdgcn_s_memrealtime());
    if (act && part == 0 && pos < R) atomicAdd(&hist[p][pos], 1);
    __syncthreads();
    const unsigned long long rs2 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    if (sh_fail) {  // a workgroup never published: ST_ERR = 3, the host falls back
      if (t == 0) {
        d.state[ST_ERR] = 3;
        d.state[ST_ROUNDS] = r;
        d.state[ST_DONE] = 1;
        if (c == 0) signal_done(d);
      }
      break;
    }
    // B[r+1][c]: the first row whose prefix count of T_q reaches SM (an
    // inclusive DPP scan of the bins -- lanes < 32 -- in every wave, no
    // second barrier)
    int res;
    {
      int h = lane < R ? hist[p][lane] : 0;
      h += __builtin_amdgcn_update_dpp(0, h, 0x111, 0xF, 0xF, true);  // row_shr:1
      h += __builtin_amdgcn_update_dpp(0, h, 0x112, 0xF, 0xF, true);  // row_shr:2
      h += __builtin_amdgcn_update_dpp(0, h, 0x114, 0xF, 0xF, true);  // row_shr:4
      h += __builtin_amdgcn_update_dpp(0, h, 0x118, 0xF, 0xF, true);  // row_shr:8
      h += __builtin_amdgcn_update_dpp(0, h, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
            const unsigned long long hit = __ballot(lane < R && h >= sm);
      res = hit ? (int)__builtin_ctzll(hit) : -1;
    }
    unsigned long long ssb = __ballot(act && part == 0 && res >= 0 && pos <= res);
    const int nc = cntk[p][0];
    const unsigned long long rt2 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    int32_t result = len;
    int lrow = 0;
    if (res >= 0) {
      result = k0 + res;
      lrow = off + res;
    } else if (nc > 0) {
      // SM not reached in the window (rare): the rows after it, window by
      // window, a row probe per step (every candidate on one row, cntk)
      auto probe = [&](uint32_t ra, int slot) {
        const bool sv = ss_row(ra + lane_off);
        const unsigned long long m = __ballot(act && part == 0 && sv);
        if (lane == 0 && m) atomicAdd(&cntk[p][slot], __popcll(m));
        return m;
      };
      for (int32_t wk = k0 + R, wr = 0; wk < len && result == len; wk += wr) {
        const int32_t rb2 = (cs + wk) & ~3;
        const int off2 = cs + wk - rb2;
        wr = min(HWL - off2, len - wk);
        __syncthreads();
        if (sst) {
          const int4 x = *reinterpret_cast<const int4 *>(scol + (rb2 + 4 * sg));
          uint32_t *w = wb32 + (wbase + (uint32_t)(4 * sg) * RST) / 4 + swi;
          const uint32_t v0 = __float_as_uint((float)x.x + la_off), v1 = __float_as_uint((float)x.y + la_off),
                         v2 = __float_as_uint((float)x.z + la_off), v3 = __float_as_uint((float)x.w + la_off);
          w[0] = v0;
          w[RST / 4] = v1;
          w[2 * (RST / 4)] = v2;
          w[3 * (RST / 4)] = v3;
          if (swi < 32) {
            w[COLS] = v0;
            w[RST / 4 + COLS] = v1;
            w[2 * (RST / 4) + COLS] = v2;
            w[3 * (RST / 4) + COLS] = v3;
          }
        }
        if (t < 16) cntk[p][t] = 0;
        __syncthreads();
        const uint32_t x0 = wbase + (uint32_t)off2 * RST;
        const unsigned long long ml = probe(x0 + (uint32_t)(wr - 1) * RST, 1);
        __syncthreads();
        if (cntk[p][1] < sm) continue;
        int lo = 0, hi = wr - 1, sl = 1;
        ssb = ml;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          ++sl;
          const unsigned long long m = probe(x0 + (uint32_t)mid * RST, sl);
          __syncthreads();
          if (cntk[p][sl] >= sm) {
            hi = mid;
            ssb = m;
          } else {
            lo = mid + 1;
          }
        }
        result = wk + lo;
        lrow = off2 + lo;
      }
      __syncthreads();
    }
    // the loop's end, the same in every workgroup: no candidates (R = r), or
    // the round table's capacity
    if (nc == 0 || r + 1 >= d.R_cap) {
      if (c == 0 && t == 0) {
        if (nc > 0) d.state[ST_ERR] = 1;
        d.state[ST_ROUNDS] = r;
        d.state[ST_ITERS] = r;
        d.state[ST_DONE] = 1;
        signal_done(d);
      }
      break;
    }
    // ---- hand-off: FD[(c, result)][i] and B[r + 1][c], tagged it + 1 ----
    if (DIAG && d.diag != nullptr && lane == 0) atomicMax(&sh_hs, (uint32_t)__builtin_amdgcn_s_memrealtime());
    const uint32_t tagw = (uint32_t)((it + 1) & 0xFF) << 24;  // (Bp's)
    const uint32_t fe_base_n = FE_BASE + (((uint32_t)(it + 1) >> 1) & 1u);  // (candfd's: iteration it + 1's tag bit)
    int32_t fdv = FD_NONE;
    if (result < len) {
      if (__any(hslow)) {
        fdv = hand_entry(colc, hin, hc, c, result);
      } else if (hin.j0 != FD_NONE) {  // rows [ab, cs + j0) are below the boundary: counted
        // #{rows < result}: clamp(result - LA) in the biased f32 domain, the
        // rows converted while the candidates were awaited
        const float rf = __uint_as_float((uint32_t)result + BIAS);
        const f32x2 r2{rf, rf};
        f32x2 e0 = lt_ind2(r2, hfb[0]) + lt_ind2(r2, hfb[1]);
#pragma unroll
        for (int u = 1; u < HNP; ++u) e0 += lt_ind2(r2, hfb[2 * u]) + lt_ind2(r2, hfb[2 * u + 1]);
        const int cnt = (int)group_total_f<8>(e0.x + e0.y);
        const int32_t ab = (hin.cs + hin.j0) & ~3, jn = ab + cnt;
        fdv = hc == c ? result : jn < ab + FBL ? jn - hin.cs : FD_NONE;
        // (jn reaching the block's end: the entry lies further on -- searched
        // by hand_entry's wave search, as there)
        const bool miss = hc != c && jn >= ab + FBL;
        if (__any(miss)) {
          if (DIAG && d.diag != nullptr && lane == 0) atomicOr(&sh_flags, 2u);
          const int32_t j = first_ge_group<8>(colc, ab + FBL, hin.cs + hin.len, result, miss, true);
          if (miss) fdv = j < hin.cs + hin.len ? j - hin.cs : FD_NONE;
        }
      }
      if ((t & 7) == 0 && hc < npad)
        __hip_atomic_store((p ? cfs1 : cfs0) + hc, (int32_t)(fe_base_n + 2u * min((uint32_t)fdv, (uint32_t)FE_NONE_X)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0)
      __hip_atomic_store(p ? bps1 : bps0, (int32_t)(tagw | (uint32_t)result), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (DIAG: the row's last store -- every wave's -- and whether a wave took
    // the bounded count; recorded after the iteration's last barrier)
    if (DIAG && d.diag != nullptr && lane == 0) {
      atomicMax(&sh_st, (uint32_t)__builtin_amdgcn_s_memrealtime());
      if (__any(hslow)) atomicOr(&sh_flags, 1u);
    }
    const int32_t rd = r;
    const unsigned long long rt3 = dgt ? __builtin_amdgcn_s_memrealtime() : 0;
    // fame's inputs (the new candidate's LA row and its ballots) and the
    // round table: nothing inside the loop reads them
    if (result < len) {
      if (t < npad) cla_c[(int64_t)cla_pos * npad + t] = (int32_t)(__uint_as_float(wb32[(wbase + (uint32_t)lrow * RST) / 4 + t]) - la_off);
      if (lane == 0) *ssm_p = ssb;
    }
    if (t == 0) *b_p = result;
    cla_pos = cla_pos + 1 == cla_span ? 0 : cla_pos + 1;
    ssm_p += 16;
    b_p += n;
    ++r;
    p ^= 1;
    k0 = result;
    hin.j0 = result < len ? fdv : FD_NONE;
    // every wave's hand-off stores leave before any wave's next loads: the
    // compute unit's vector memory unit takes instructions in order, and a
    // late wave's row store queued behind the other waves' window and
    // hand-off loads (3 per wave) -- the row completed ~0.9 us after the last
    // wave began its hand-off (loading the hand-off rows after the next
    // candidates instead measured slower: C3 34.4 -> 35.8 ms).  (The next
    // iteration stages the other parity's
    // window and histogram; the barrier also keeps a wave's first candidate
    // loads from leaving while the other workgroups' rows are still being
    // written: polls 0 -> 1, hop 1.2 -> 4.2 us without it, MEASUREMENTS.md)
    __syncthreads();
    own_loads();  // the next window and hand-off rows: they land while this wave's stores are acknowledged
    if (dgt && c < 128) {
      // tl / tb [3]: the row complete (every wave's store); the flags in tb[0] bits 60+
      const unsigned long long st = (rt3 & ~0xFFFFFFFFull) | sh_st;
      unsigned long long *tl = d.diag + DG_TL + ((rd - TL_R0) * 128 + c) * 4;
      tl[0] = rt0;
      tl[1] = rt2;
      tl[2] = rt1;
      tl[3] = st;
      unsigned long long *tb = d.diag + DG_TLB + ((int64_t)(rd - TL_R0) * 512 + c) * 4;
      tb[0] = rtp | (unsigned long long)sh_flags << 60;
      tb[1] = rt0;
      tb[2] = (unsigned long long)polls | (unsigned long long)(rta - rtp) << 32;  // (high: the own-store wait)
      tb[3] = st;
      unsigned long long *ts = d.diag + DG_TLS + ((int64_t)(rd - TL_R0) * 512 + c) * 4;
      ts[0] = rs1;
      ts[1] = rs2;
      // (bit 31: the low word is the last wave's probes-done time, not a probe count)
      ts[2] = (unsigned long long)(0x80000000u | (sh_pend - (uint32_t)rt0)) | (unsigned long long)(sh_cur - (uint32_t)rt0) << 32;
      ts[3] = (rt3 & ~0xFFFFFFFFull) | sh_hs;  // (the last wave's hand-off start)
      sh_st = sh_flags = sh_hs = 0;  // (wave 0 only: the other waves' next atomics come after the next barrier)
    }
  }
}

bool round_lean_eligible(const Dev &d) {
  // float-encoded entries: chain rows <= 2^22 - 3 (fe_encode; FD_NONE is 2^22 - 1)
  return d.round_f32 && d.max_chain_len < (1 << 22) - 2;
}

bool cand_fe(const Dev &d) { return round_persist_eligible(d) && round_lean_eligible(d) && !round_solo_eligible(d); }

// parity 0's candidate rows back to plain entries (run_round_loop: a
// persistent k_round_lean that gave up hands its restored inputs to the
// per-iteration k_round2)
__global__ void k_cand_defe(Dev d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int64_t)d.n * d.npad) d.candfd[i] = fe_decode((uint32_t)d.candfd[i]);
}

void launch_cand_defe(const Dev &d, hipStream_t s) {
  k_cand_defe<<<(unsigned)(((int64_t)d.n * d.npad + 255) / 256), 256, 0, s>>>(d);
}

bool round_persist_eligible(const Dev &d) {
  // (the tagged hand-off carries chain rows in 24 bits: 0xFFFFFF is FD_NONE)
  return d.round_persist && round2_eligible(d) && !d.round_src_rows && d.n <= 256 && d.max_chain_len < 0xFFFFFF;
}

static int lanes_per_candidate(int npad);

// the wide persistent loop (k_round_wide<*, true, 0, 256, true>): the 16-bit
// loop over FDT with byte rows searched in pairs, n workgroups that must all
// be resident at once (two per compute unit at n = 512)
static int wide_resident(int lpc) {
  static int slots[2] = {-1, -1};
  int &s = slots[lpc == 8];
  if (s < 0) {
    int nb = 0, cus = 0, dev = 0;
    const size_t wb16 = (size_t)WROWS * lpc * 9 * 16;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (lpc == 8) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_round_wide<8, true, 0, 256, true>, 256, wb16);
    else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_round_wide<4, true, 0, 256, true>, 256, wb16);
    s = std::min(nb, 8) * cus;
  }
  return s;
}

bool round_wide_persist_eligible(const Dev &d) {
  // (wide_cols 1, the window from la_col, stays one launch per round)
  if (!d.round_persist || d.fd_cols || !d.cand16 || d.fd_rows || d.wide_cols == 1 || !d.round_ilp2 || !d.pbar ||
      !round_p16(d))
    return false;
  const int lpc = lanes_per_candidate(d.npad);
  return d.n > 256 / lpc && (lpc == 4 || lpc == 8) && d.n <= wide_resident(lpc);
}

void launch_round_wide_persist(const Dev &d, hipStream_t s) {
  const int lpc = lanes_per_candidate(d.npad);
  const size_t wb16 = (size_t)WROWS * lpc * 9 * 16;
  (void)hipMemsetAsync(d.pbar, 0, (size_t)PBAR_INTS * 4, s);
  // (ILPK = 4, four searches interleaved per lane group: 256 VGPRs, search
  // 20.1 -> 22.3 us per round -- the probes' LDS reads, not their latency, bound it)
  if (d.wide_cols == 2) {  // the hand-off counted in la_col (no FDT)
    if (lpc == 8) k_round_wide<8, true, 2, 256, true><<<d.n, 256, wb16, s>>>(d, 0);
    else k_round_wide<4, true, 2, 256, true><<<d.n, 256, wb16, s>>>(d, 0);
  } else if (lpc == 8) {
    k_round_wide<8, true, 0, 256, true><<<d.n, 256, wb16, s>>>(d, 0);
  } else {
    k_round_wide<4, true, 0, 256, true><<<d.n, 256, wb16, s>>>(d, 0);
  }
}

// e0 / e1: the launch's own start / stop timestamps (hipExtLaunchKernel: no
// marker packets of their own between the segments' kernels, ~5 us each)
void launch_round_persist(const Dev &d, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  const int ppl = d.npad <= 32 ? 1 : d.npad <= 64 ? 2 : 4;  // (k_round2p's rows: 8 * PPL + 1 pieces)
  uint32_t lds = (uint32_t)(HWL * (8 * ppl + 1) * 16);
  const unsigned nt = (unsigned)((8 * d.npad + 63) / 64 * 64);
  void (*k)(Dev);
  if (round_lean_eligible(d)) {
    // two parity windows of HWL + 2 rows at k_round_lean's stride
    const int rst = ppl == 1 ? 256 : ppl == 2 ? 512 : 1024;
    // (at least 148 KiB: no other kernel's workgroup shares the loop's
    // compute unit -- at 88 VGPRs a k_flow32x2 workgroup otherwise fits
    // beside the loop's 16 waves and takes their VALU issue slots)
    lds = (uint32_t)std::max(2 * (HWL + 2) * rst, 148 * 1024);
    const bool full = d.npad == 32 * ppl, diag = d.diag != nullptr && full;
    if (diag) k = ppl == 1 ? k_round_lean<1, true, true> : ppl == 2 ? k_round_lean<2, true, true> : k_round_lean<4, true, true>;
    else if (full) k = ppl == 1 ? k_round_lean<1, true, false> : ppl == 2 ? k_round_lean<2, true, false> : k_round_lean<4, true, false>;
    else k = ppl == 1 ? k_round_lean<1, false, false> : ppl == 2 ? k_round_lean<2, false, false> : k_round_lean<4, false, false>;
  } else {
    k = d.npad <= 32 ? k_round2p<1, false> : d.npad <= 64 ? k_round2p<2, false> : k_round2p<4, false>;
  }
  if (e0 || e1) hipExtLaunchKernelGGL(k, dim3((unsigned)d.n), dim3(nt), lds, s, e0, e1, 0, d);
  else k<<<d.n, nt, lds, s>>>(d);
}

// k_round2r (BH_ROUND_SRC=rows, A/B): the round-3 iteration, reading its
// window from the row-major LA and its hand-off from the FDT tiles that the
// segments' transpose builds (eager rows); k_round2 reads only la_col
template <int PPL, bool TQ>
__global__ __launch_bounds__(1024) void k_round2r(Dev d, int p) {
  constexpr int LPC = 8;
  extern __shared__ __attribute__((aligned(16))) int4 sm4[];
  __shared__ int32_t cntk[16];
  __shared__ int32_t hist[HW + 1];  // TQ: T_q histogram; [HW] = the answer row
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c = blockIdx.x;
  const int n = d.n, npad = d.npad, sm = d.sm, q4 = npad / 4;
  int4 *win = sm4;              // [HW][q4]: LA rows k0 .. k0 + 31
  // [npad][FDS]: FD rows rb .. rb + 31 by column, for the hand-off after the
  // search -- the window's space (every read of it is behind the search's
  // last barrier), so the workgroup's LDS (18 KiB at n = 128) fits beside a
  // k_flow32 workgroup (133 KiB) on one compute unit: the segment pipeline
  // runs both at once
  int32_t *fdw = reinterpret_cast<int32_t *>(sm4);
  constexpr int FDS = HW + 4;
  const int32_t *Bp = d.Bp + (int64_t)p * n;
  const bool dg = d.diag != nullptr && t == 0;
  const unsigned long long ts0 = dg ? stamp() : 0;
  const unsigned long long rt0 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
  // ---- independent loads ----
  const int done = d.state[ST_DONE];
  const int r = d.state[ST_CUR0 + p];
  const int32_t len = d.chain_len[c], cs = d.chain_start[c];
  const int32_t k0 = Bp[c];
  const int q = t / LPC, part = t % LPC;
  const int rot = TQ ? (q & (PPL - 1)) : 0;  // piece order of this group (bank spread)
  int32_t bq = 0, lq = 0;
  if (q < n) { bq = Bp[q]; lq = d.chain_len[q]; }
  int4 f[PPL];
  {
    const int4 *cf = reinterpret_cast<const int4 *>(d.candfd) + ((int64_t)p * n + min(q, n - 1)) * q4;
#pragma unroll
    for (int u = 0; u < PPL; ++u) {
      const int pc = part + LPC * ((u + rot) & (PPL - 1));
      f[u] = pc < q4 ? cf[pc] : make_int4(FD_NONE, FD_NONE, FD_NONE, FD_NONE);
    }
  }
  const int rows = min(HW, max(0, len - k0));
  const int4 wv = reinterpret_cast<const int4 *>(d.la)[(int64_t)(cs + k0) * q4 + min(t, max(rows * q4 - 1, 0))];
  if (done) return;
  const bool act = q < n && bq < lq;
  // ---- loads for the hand-off (consumed after the search) ----
  // FD rows rb .. rb + 31 (rb = the window's first row rounded down to 4)
  // from the FDT tiles: 16 B = 4 rows of one column per thread, 8 threads
  // per column
  const int64_t rb = (int64_t)(cs + k0) & ~(int64_t)3;
  const int fi = min(t >> 3, n - 1), fp = (t & 7) * 4;
  const int4 fv = *reinterpret_cast<const int4 *>(d.fdt + fdt_pos(rb + fp, fi, npad));
  if (t < rows * q4) win[t] = wv;
  if (t < 16) cntk[t] = 0;
  if (TQ && t <= HW) hist[t] = 0;
  __syncthreads();
  const unsigned long long ts1 = dg ? stamp() : 0;
  const unsigned long long rt1 = dg ? __builtin_amdgcn_s_memrealtime() : 0;  // loads landed
  // count(row) into slot: groups whose candidate `row` strongly sees
  // does window row x4 strongly see this group's candidate?
  auto ss_row = [&](const int4 *x4) {
    int4 x[PPL];  // all reads first: one LDS round trip per probe
#pragma unroll
    for (int u = 0; u < PPL; ++u) x[u] = x4[min(part + LPC * ((u + rot) & (PPL - 1)), q4 - 1)];
    int lt = 0;
#pragma unroll
    for (int u = 0; u < PPL; ++u) lt += lt4(x[u], f[u]);
    return LPC * PPL * 4 - group_sum<LPC>(lt) >= sm;
  };
  auto probe = [&](const int4 *x4, int slot) {
    const bool s = ss_row(x4);
    const unsigned long long m = __ballot(act && part == 0 && s);
    if (lane == 0 && m) atomicAdd(&cntk[slot], __popcll(m));
    return m;  // this wave's candidates the row strongly sees (fame's S_j)
  };
  {
    const unsigned long long m = __ballot(act && part == 0);
    if (lane == 0 && m) atomicAdd(&cntk[0], __popcll(m));
  }
  int slot = 1;
  int32_t res = -1;  // window row of B[r+1][c], or -1
  unsigned long long ssb = 0;  // this wave's ballot of the probe that verified the answer row
  if (TQ && rows > 0) {
    // T_q by a per-group binary search over [0, rows] (rows = none in the window)
    int lo = 0, hi = rows;
    while (__any(lo < hi)) {
      const int mid = (lo + hi) >> 1;
      const bool s = ss_row(win + min(mid, rows - 1) * q4);
      if (lo < hi) {
        hi = s ? mid : hi;
        lo = s ? lo : mid + 1;
      }
    }
    if (act && part == 0 && lo < rows) atomicAdd(&hist[lo], 1);
    __syncthreads();
    if (wave == 0) {
      int h = lane < rows ? hist[lane] : 0;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(h, off);
        h += lane >= off ? o : 0;
      }
      const unsigned long long hit = __ballot(lane < rows && h >= sm);
      if (lane == 0) hist[HW] = hit ? (int)__builtin_ctzll(hit) : -1;
    }
    __syncthreads();
    res = hist[HW];
    // fame's S_j for the new candidate: the candidates whose T_q is at most its row
    ssb = __ballot(act && part == 0 && res >= 0 && lo <= res);
  } else if (rows > 0) {
    // binary search assuming the window's last row reaches SM (count is
    // monotone); that row is probed only if the search ends on it unverified
    int lo = 0, hi = rows - 1;
    bool hi_ok = false;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      const unsigned long long m = probe(win + mid * q4, slot);
      __syncthreads();
      if (cntk[slot] >= sm) {
        hi = mid;
        hi_ok = true;
        ssb = m;
      } else {
        lo = mid + 1;
      }
      ++slot;
    }
    if (!hi_ok) {
      ssb = probe(win + hi * q4, slot);
      __syncthreads();
      hi_ok = cntk[slot] >= sm;
    }
    if (hi_ok) res = lo;
  } else {
    __syncthreads();
  }
  const int nc = cntk[0];
  const unsigned long long ts2 = dg ? stamp() : 0;
  const unsigned long long rt2 = dg ? __builtin_amdgcn_s_memrealtime() : 0;
  int32_t result = len;
  if (res >= 0) {
    result = k0 + res;
  } else if (nc > 0 && rows == HW) {
    // SM not reached in the handed-over window (rare): later windows of
    // chain c, loaded directly (slot counters are reused per row tested)
    int4 *x4 = win;  // rows in LDS: row i of the current window at x4[i * q4]
    for (int32_t wk = k0 + HW; wk < len && result == len; wk += HW) {
      const int wr = min(HW, len - wk);
      __syncthreads();
      for (int i = t; i < wr * q4; i += blockDim.x)
        x4[i] = reinterpret_cast<const int4 *>(d.la)[(int64_t)(cs + wk) * q4 + i];
      if (t < 16) cntk[t] = 0;
      __syncthreads();
      const unsigned long long ml = probe(x4 + (wr - 1) * q4, 1);
      __syncthreads();
      if (cntk[1] < sm) continue;
      int lo = 0, hi = wr - 1, sl = 1;
      ssb = ml;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        ++sl;
        const unsigned long long m = probe(x4 + mid * q4, sl);
        __syncthreads();
        if (cntk[sl] >= sm) {
          hi = mid;
          ssb = m;
        } else {
          lo = mid + 1;
        }
      }
      result = wk + lo;
    }
    __syncthreads();
  }
  // ---- hand-off for the next iteration ----
  if (nc > 0 && r + 1 < d.R_cap && result < len) {
    const int32_t off = result - k0;
    int32_t *cf = d.candfd + ((int64_t)(p ^ 1) * n + c) * npad;
    const int frel = (int)(cs + result - rb);  // row of the candidate in fdw
    // the candidate's LA row for fame (cla), before fdw overwrites the window
    if (t < npad) d.cla[cla_row(d, c, r + 1) * npad + t] = d.la[(int64_t)(cs + result) * npad + t];
    if (off < HW && frel < HW) {  // both from the rows staged during the search
      if (t < n * 8) *reinterpret_cast<int4 *>(fdw + fi * FDS + fp) = fv;
      __syncthreads();
      if (t < npad) cf[t] = t < n ? fdw[t * FDS + frel] : FD_NONE;
    } else {
      if (t < npad) cf[t] = t < n ? d.fdt[fdt_pos(cs + result, t, npad)] : FD_NONE;
    }
    // fame's input for the new candidate y = (c, result): SS(y, q) over
    // the candidates q of round r = the ballots of the probe that verified
    // y's row.  Raw ballots, one aligned 8-B word per wave (candidate q at
    // bit 8 (q % 8) of word q / 8; fame packs the LPC-strided bits and masks
    // the words of chains >= n, which fewer waves leave unwritten),
    // chain-major [c][round]; issued last, since a later vmcnt wait would
    // include them
    if (lane == 0) d.ssm[ballot_row(d, c, r + 1) * 16 + wave] = ssb;
  }
  if (dg) {
    const unsigned long long te = stamp();
    if (r >= TL_R0 && r < TL_R0 + TL_NR && c < 128) {
      unsigned long long *tl = d.diag + DG_TL + ((r - TL_R0) * 128 + c) * 4;
      const unsigned long long fl = (unsigned long long)(min(result - k0, 255) & 255) |
                                    (unsigned long long)(res < 0) << 8 | (unsigned long long)(nc > 0) << 9;
      tl[0] = rt0 | fl << 52; tl[1] = rt2; tl[2] = rt1; tl[3] = __builtin_amdgcn_s_memrealtime();
    } else if (r < TL_R0 - 64 || r >= TL_R0 + TL_NR + 64) {
      // phase counters (device-scope atomics from every workgroup: they
      // stretch the round by several us, so none near the timeline window)
      atomicAdd(&d.diag[DG_RD_B], ts1 - ts0);
      atomicAdd(&d.diag[DG_RD_LOAD], 0ull);
      atomicAdd(&d.diag[DG_RD_COMP], ts2 - ts1);
      atomicAdd(&d.diag[DG_RD_TOTAL], te - ts0);
      atomicAdd(&d.diag[DG_RD_CALLS], 1ull);
    }
  }
  if (t == 0) {
    if (nc == 0) {  // no candidates: R = r
      if (c == 0) { d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; signal_done(d); }
      return;
    }
    if (r + 1 >= d.R_cap) {
      if (c == 0) { d.state[ST_ERR] = 1; d.state[ST_ROUNDS] = r; d.state[ST_DONE] = 1; signal_done(d); }
      return;
    }
    d.Bp[(int64_t)(p ^ 1) * n + c] = result;
    d.B[(int64_t)(r + 1) * n + c] = result;
    if (c == 0) {
      d.state[ST_CUR0 + (p ^ 1)] = r + 1;
      d.state[ST_ITERS] = r + 1;
    }
  }
}

// k_round_solo: the whole round loop of a small hashgraph (n <= 32) in ONE
// workgroup that stays resident until the loop ends.  At n <= 32 a round of
// k_round2 is almost all fixed cost -- the launch boundary, and loads that
// every launch fetches again from MALL because each launch starts with
// invalidated L2s -- so here the state that crosses rounds stays on one
// compute unit:
//   * half-wave c (32 lanes) owns chain c, lane q of it candidate q;
//   * B[r] and the candidates' FD rows live in LDS, double-buffered by
//     round parity (one workgroup barrier per round);
//   * chain c's LA window is a 32-row ring in LDS (slot = row & 31): a round
//     loads only the rows its window gained (the boundary moves by about
//     N / (n R) rows, not 32), from an L2 that no launch boundary invalidates;
//   * the search is over rows, as k_round2's row-probe variant: every lane of
//     a half-wave tests the same ring row (an LDS broadcast) against its own
//     candidate, a ballot counts, B[r+1][c] = the first row reaching SM, and
//     the ballot of the probe that verified it is fame's S_j;
//   * the one dependent load of a round -- the new candidate's FD row -- is
//     issued together with the next window's LA rows, and the round's outputs
//     (B history, ssm ballots in k_round2's raw layout: word k holds
//     candidates 8k + b at bit 8b) are stored after them, so no wait for the
//     loads waits for the stores.
// Windows that do not reach SM continue from global memory (rare).
// Termination: each round ends the loop (no candidates, or a full round
// table) or advances r toward R_cap.
constexpr int SOLO_N = 32;
__global__ __launch_bounds__(1024) void k_round_solo(Dev d) {
  extern __shared__ __attribute__((aligned(16))) int4 ring4[];  // [n][32 rows][q4]
  // candidate rows 144 B apart: the 32 lanes of a half-wave reading 32 rows
  // with ds_read_b128 spread over the banks (128 B apart they would collide)
  constexpr int CS = SOLO_N + 4;
  __shared__ __attribute__((aligned(16))) int32_t cand[2][SOLO_N][CS];
  __shared__ int32_t bsh[2][SOLO_N];
  const int t = threadIdx.x, lane = t & 63;
  const int c = t >> 5, q = t & 31;
  const int n = d.n, npad = d.npad, q4 = npad / 4, sm = d.sm;
  const unsigned long long half = (lane < 32) ? 0xFFFFFFFFull : 0xFFFFFFFF00000000ull;
  const int hs = lane & 32;
  const bool cv = c < n;
  const int32_t len = cv ? d.chain_len[c] : 0, cs = cv ? d.chain_start[c] : 0;
  const int32_t lenq = q < n ? d.chain_len[q] : 0;
  const int4 *la4 = reinterpret_cast<const int4 *>(d.la);
  int4 *ring = ring4 + (int64_t)(cv ? c : 0) * 32 * q4;
  // the new LA rows [from, k0 + rows) of chain c's window into its ring:
  // every load issued before any LDS store
  auto load_ring = [&](int32_t from, int32_t to, int4 *lv) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int it = q + 32 * j;
      const int32_t row = from + it / q4;
      lv[j] = (cv && row < to) ? la4[((int64_t)cs + row) * q4 + (it - (it / q4) * q4)] : make_int4(0, 0, 0, 0);
    }
  };
  auto store_ring = [&](int32_t from, int32_t to, const int4 *lv) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int it = q + 32 * j;
      const int32_t row = from + it / q4;
      if (cv && row < to) ring[(row & 31) * q4 + (it - (it / q4) * q4)] = lv[j];
    }
  };
  int r = d.state[ST_CUR0];  // parity-0 buffers: k_cand_rows (after k_round_resume)
  if (t < n) bsh[0][t] = d.Bp[t];
  for (int i = t; i < n * npad; i += blockDim.x) cand[0][i / npad][i % npad] = d.candfd[i];
  int32_t k0 = cv ? d.Bp[c] : 0;
  int32_t ring_lo = k0;  // rows [ring_lo, ring_lo + 32) of chain c are in the ring
  {
    int4 lv[8];
    load_ring(k0, min(len, k0 + 32), lv);
    store_ring(k0, min(len, k0 + 32), lv);
  }
  int err = 0;
  // BH_DIAG: phase cycles of thread 0 (round start -> FD row read -> search
  // done -> round-end loads + barrier), summed over rounds
  const bool dg = d.diag != nullptr && t == 0;
  unsigned long long c_f = 0, c_s = 0, c_e = 0, nr = 0;
  __syncthreads();
  for (int p = 0;; p ^= 1) {
    const unsigned long long ts0 = dg ? stamp() : 0;
    const int32_t bq = q < n ? bsh[p][q] : 0;
    const bool act = q < n && bq < lenq;
    const int nc = __popcll(__ballot(act) & half);  // the same in every half-wave
    if (nc == 0) break;
    if (r + 1 >= d.R_cap) { err = 1; break; }
    const int rows = cv ? min(32, max(0, len - k0)) : 0;
    int4 f[8];  // candidate q's FD row
#pragma unroll
    for (int u = 0; u < 8; ++u)
      f[u] = (act && u < q4) ? *reinterpret_cast<const int4 *>(&cand[p][q][4 * u])
                             : make_int4(FD_NONE, FD_NONE, FD_NONE, FD_NONE);
    if (dg) { __builtin_amdgcn_s_waitcnt(0xc07f); }
    const unsigned long long ts1 = dg ? stamp() : 0;
    auto ss = [&](const int4 *x4, bool global) {
      int ge = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < q4) ge += ge4(x4[u], f[u]);
      (void)global;
      return act && ge >= sm;
    };
    // first window row whose ballot reaches SM
    int lo = 0, hi = rows;
    unsigned long long ssb = 0;
    while (__any(lo < hi)) {
      const int mid = (lo + hi) >> 1;
      const bool sv = ss(ring + ((k0 + min(mid, max(rows - 1, 0))) & 31) * q4, false);
      const unsigned long long m = __ballot(sv) & half;
      if (lo < hi) {
        if (__popcll(m) >= sm) { hi = mid; ssb = m; }
        else lo = mid + 1;
      }
    }
    int32_t result = lo < rows ? k0 + lo : len;
    // ---- SM not reached in the window (rare): later windows from global ----
    bool need = cv && lo >= rows && rows == 32;
    int32_t wk = k0 + 32;
    while (__any(need)) {
      const int wr = need ? min(32, len - wk) : 0;
      if (need && wr <= 0) need = false;
      int l2 = 0, h2 = need ? wr : 0;
      unsigned long long sb2 = 0;
      while (__any(l2 < h2)) {
        const int mid = (l2 + h2) >> 1;
        const int4 *x4 = la4 + ((int64_t)cs + wk + min(mid, max(wr - 1, 0))) * q4;
        const bool sv = need && ss(x4, true);
        const unsigned long long m = __ballot(sv) & half;
        if (l2 < h2) {
          if (__popcll(m) >= sm) { h2 = mid; sb2 = m; }
          else l2 = mid + 1;
        }
      }
      if (need && l2 < wr) { result = wk + l2; ssb = sb2; need = false; }
      wk += 32;
    }
    const unsigned long long ts2 = dg ? stamp() : 0;
    // ---- round end: the hand-off load and the next window's rows together,
    // then this round's outputs ----
    const int32_t k1 = cv ? result : 0;
    const int32_t from = max(k1, ring_lo + 32), to = min(len, k1 + 32);
    int4 lv[8];
    load_ring(from, to, lv);
    const bool hand = cv && result < len;
    const int32_t v = (hand && q < n) ? d.fdt[fdt_pos((int64_t)cs + result, q, npad)] : FD_NONE;
    if (hand && q < 4) {  // fame's S_j of the new candidate (k_round2's ballot layout, 8 lanes per candidate)
      const uint32_t bits = (uint32_t)((ssb >> hs) >> (8 * q)) & 0xFFu;
      unsigned long long w = 0;
      for (int k = 0; k < 8; ++k) w |= (unsigned long long)((bits >> k) & 1u) << (8 * k);
      d.ssm[ballot_row(d, c, r + 1) * 16 + q] = w;
    } else if (hand && q < 16) {
      d.ssm[ballot_row(d, c, r + 1) * 16 + q] = 0ull;
    }
    if (cv && q == 0) d.B[(int64_t)(r + 1) * n + c] = result;
    store_ring(from, to, lv);
    if (hand && q < npad) cand[p ^ 1][c][q] = v;
    if (cv && q == 0) bsh[p ^ 1][c] = result;
    ring_lo = k1;
    k0 = k1;
    ++r;
    __syncthreads();
    if (dg) {
      const unsigned long long ts3 = stamp();
      c_f += ts1 - ts0; c_s += ts2 - ts1; c_e += ts3 - ts2; ++nr;
    }
  }
  if (dg) {
    atomicAdd(&d.diag[DG_RD_B], c_e);
    atomicAdd(&d.diag[DG_RD_LOAD], c_f);
    atomicAdd(&d.diag[DG_RD_COMP], c_s);
    atomicAdd(&d.diag[DG_RD_TOTAL], c_f + c_s + c_e);
    atomicAdd(&d.diag[DG_RD_CALLS], nr);
  }
  if (t == 0) {
    d.state[ST_ROUNDS] = r;
    d.state[ST_ITERS] = r;
    d.state[ST_ERR] = err;
    d.state[ST_DONE] = 1;
    signal_done(d);
  }
}

// opt-in (BH_ROUND_SOLO=1): measured slower than k_round2 at C2 (DESIGN.md
// section 5, "One resident workgroup"), kept as the measured alternative
bool round_solo_eligible(const Dev &d) {
  const char *e = getenv("BH_ROUND_SOLO");  // (read per loop: the tests switch it)
  return d.fd_cols != 0 && d.n <= SOLO_N && e && atoi(e);
}

void launch_round_solo(const Dev &d, hipStream_t s) {
  const size_t lds = (size_t)d.n * 32 * d.npad * 4;
  k_round_solo<<<1, 1024, lds, s>>>(d);
}

// Resuming the loop after a prefix run (segments).  A
// prefix of the DAG in insertion order is closed under ancestry, so its
// rows' lastAncestors are final; a candidate beyond the prefix cannot be
// strongly seen by a prefix row, and an FD entry beyond the prefix compares
// false against a prefix row's LA either way.  So every boundary the prefix
// run finds INSIDE the prefix (B[r][q] < prefix length) holds for the whole
// DAG, and the loop can resume at the last round whose boundaries all lie
// inside: r0 = min over q of (first r with B[r][q] >= len_q) - 1.
// Only chains that gain events can move a boundary: a chain q with no new
// event keeps B[r][q] for every r (its rows' counts do not change, and a
// boundary at len_q finds no row), so the minimum runs over the chains that
// grow in the next prefix (next_len[q] > len_q; every chain when next_len is
// null).  rq[q] keeps each chain's first r for the host, which takes the
// minimum over the chains a later call extends.  A chain that is empty or
// has stopped growing therefore does not pin the resume point.  floor: the
// closed form's first round (a Reset hashgraph's r0, else 0).
__global__ __launch_bounds__(1024) void k_resume_point(Dev d, int32_t R, const int32_t *next_len) {
  __shared__ int32_t m;
  if (R < 0) R = d.state[ST_ROUNDS];  // (a loop the host did not wait for)
  if (threadIdx.x == 0) m = R;
  __syncthreads();
  for (int q = threadIdx.x; q < d.n; q += blockDim.x) {
    const int32_t len = d.chain_len[q];
    int lo = 0, hi = R;  // B[R][q] = len_q (the last iteration's output)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (d.B[(int64_t)mid * d.n + q] >= len) hi = mid;
      else lo = mid + 1;
    }
    if (d.rq) d.rq[q] = lo;
    if (!next_len || next_len[q] > len) atomicMin(&m, lo);
  }
  __syncthreads();
  if (threadIdx.x == 0) d.state[ST_RESUME] = max(d.r0, m - 1);
}

void launch_resume_point(const Dev &d, int32_t R, const int32_t *next_len, hipStream_t s) {
  k_resume_point<<<1, 1024, 0, s>>>(d, R, next_len);
}

// iteration r0's inputs, parity 0: B[r0] and the candidates' FD rows (from
// FDT, which now covers the longer prefix); the loop state
__global__ __launch_bounds__(256) void k_round_resume(Dev d) {
  const int c = blockIdx.x;
  const int32_t r0 = d.state[ST_RESUME];
  const int32_t b = d.B[(int64_t)r0 * d.n + c], len = d.chain_len[c], cs = d.chain_start[c];
  if (threadIdx.x == 0) {
    d.Bp[c] = b;
    if (d.c8tag) d.c8tag[c] = d.c8tag[d.n + c] = -1;  // cand8 rows of an earlier loop are stale
  }
  // (n <= 128: the candidates' rows are searched in la_col, k_cand_rows)
  if (b < len && !d.fd_cols && !d.wide_cols && d.cand16 && !d.fd_rows)
    gather_cand16(d, (int64_t)cs + b, d.cand16 + (int64_t)c * ((d.npad + 7) / 8 * 4));
  if (c == 0 && threadIdx.x == 0) {
    // the previous segment's failure stays visible to the host (ST_PFAIL)
    d.state[ST_PFAIL] = max(d.state[ST_PFAIL], d.state[ST_ERR]);
    d.state[ST_CUR0] = r0;
    d.state[ST_CUR0 + 1] = 0;
    d.state[ST_DONE] = 0;
    d.state[ST_ROUNDS] = 0;
    d.state[ST_ERR] = 0;
    d.state[ST_ITERS] = r0;
  }
}

void launch_round_resume(const Dev &d, hipStream_t s) {
  k_round_resume<<<d.n, 256, 0, s>>>(d);
  if (d.fd_cols || d.wide_cols) launch_cand_rows(d, 1, s);
}

// A chain with no event in the segment has no last-row tile to write
// "never seen" (MaxInt32) into the new rows of the other chains: done here
// from the LA row of its last event (or -1 everywhere if it has none)
__global__ __launch_bounds__(256) void k_fd_idle(Dev d) {
  const int i = blockIdx.x;
  const int32_t hi_i = d.chain_len[i];
  if (d.seg_lo[i] != hi_i) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t lrow = (int64_t)d.chain_start[i] + hi_i - 1;
  for (int c = wave; c < d.n; c += 4) {
    const int32_t seen = hi_i > 0 ? d.la[lrow * d.npad + c] : -1;
    const int32_t cs = d.chain_start[c];
    for (int32_t j = max(seen + 1, d.seg_lo[c]) + lane; j < d.chain_len[c]; j += 64)
      d.fdt[fdt_pos(cs + j, i, d.npad)] = FD_NONE;
  }
}

void launch_fd_idle(const Dev &d, hipStream_t s) { k_fd_idle<<<d.n, 256, 0, s>>>(d); }

bool round2_eligible(const Dev &d) { return d.fd_cols != 0; }

// the 16-bit wide loop: cand16 exists (n <= 512) and
// every LA / FD value + 1 fits below 0xFFFF
bool round_p16(const Dev &d) { return d.cand16 != nullptr && d.max_chain_len <= P16_MAXLEN && !getenv("BH_NO_P16"); }

// candidate (c, 0) of every chain for the 16-bit wide loop
__global__ __launch_bounds__(256) void k_cand16_init(Dev d) {
  const int c = blockIdx.x;
  if (threadIdx.x == 0 && d.c8tag) d.c8tag[c] = d.c8tag[d.n + c] = -1;
  if (d.chain_len[c] > 0) gather_cand16(d, d.chain_start[c], d.cand16 + (int64_t)c * ((d.npad + 7) / 8 * 4));
}

void launch_round_init(const Dev &d, hipStream_t s) {
  if (round2_eligible(d) || d.wide_cols) launch_cand_rows(d, 0, s);
  else if (d.cand16 && !d.fd_rows) k_cand16_init<<<d.n, 256, 0, s>>>(d);
}

static int lanes_per_candidate(int npad) {
  const int q4 = npad / 4;
  int lpc = 1;
  while (lpc * PIECES < q4) lpc <<= 1;
  return lpc;
}

void configure_round_kernels() {
#define CFG(K) (void)hipFuncSetAttribute((const void *)K, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024)
  CFG(k_round<1>); CFG(k_round<2>); CFG(k_round<4>); CFG(k_round<8>); CFG(k_round<16>);
  CFG((k_round_wide<1, false>)); CFG((k_round_wide<2, false>)); CFG((k_round_wide<4, false>));
  CFG((k_round_wide<8, false>)); CFG((k_round_wide<16, false>));
  CFG((k_round_wide<4, true>)); CFG((k_round_wide<8, true>));
  CFG((k_round_wide<4, true, 1>)); CFG((k_round_wide<8, true, 1>));
  CFG((k_round_wide<4, true, 2>)); CFG((k_round_wide<8, true, 2>));
  CFG((k_round_wide<4, true, 0, 256, true>)); CFG((k_round_wide<8, true, 0, 256, true>));
  CFG((k_round_wide<4, true, 2, 256, true>)); CFG((k_round_wide<8, true, 2, 256, true>));
  CFG((k_round2<1, true>)); CFG((k_round2<2, true>)); CFG((k_round2<4, true>));
  CFG((k_round2<1, false>)); CFG((k_round2<2, false>)); CFG((k_round2<4, false>));
  CFG((k_round2r<1, true>)); CFG((k_round2r<2, true>)); CFG((k_round2r<4, true>));
  CFG((k_round_lean<1, true, false>)); CFG((k_round_lean<2, true, false>)); CFG((k_round_lean<4, true, false>));
  CFG((k_round_lean<1, false, false>)); CFG((k_round_lean<2, false, false>)); CFG((k_round_lean<4, false, false>));
  CFG((k_round_lean<1, true, true>)); CFG((k_round_lean<2, true, true>)); CFG((k_round_lean<4, true, true>));
  CFG((k_round2p<1, false>)); CFG((k_round2p<2, false>)); CFG((k_round2p<4, false>));
  CFG(k_round_solo);
#undef CFG
}

// iteration parity p: the loop state alternates by iteration (every graph
// batch -- ITER_FIRST, ITER_BATCH -- is even, so each starts at parity 0)
void launch_round_iteration(const Dev &d, int p, hipStream_t s) {
  if (round2_eligible(d)) {
    const size_t lds = (size_t)HWL * (d.npad / 4 + 1) * 16;  // the staged window
    const bool rows_search = getenv("BH_ROUND_ROWS") && atoi(getenv("BH_ROUND_ROWS"));  // (read per capture: the tests switch it)
    const unsigned nt = (unsigned)((8 * d.npad + 63) / 64 * 64);  // 8 lanes per candidate
    if (d.round_src_rows) {
      const size_t lds2 = std::max((size_t)HW * (d.npad / 4) * 16, (size_t)d.npad * (HW + 4) * 4);
      if (d.npad <= 32) k_round2r<1, true><<<d.n, nt, lds2, s>>>(d, p);
      else if (d.npad <= 64) k_round2r<2, true><<<d.n, nt, lds2, s>>>(d, p);
      else k_round2r<4, true><<<d.n, nt, lds2, s>>>(d, p);
    } else if (rows_search) {
      if (d.npad <= 32) k_round2<1, false><<<d.n, nt, lds, s>>>(d, p);
      else if (d.npad <= 64) k_round2<2, false><<<d.n, nt, lds, s>>>(d, p);
      else k_round2<4, false><<<d.n, nt, lds, s>>>(d, p);
    } else {
      if (d.npad <= 32) k_round2<1, true><<<d.n, nt, lds, s>>>(d, p);
      else if (d.npad <= 64) k_round2<2, true><<<d.n, nt, lds, s>>>(d, p);
      else k_round2<4, true><<<d.n, nt, lds, s>>>(d, p);
    }
    return;
  }
  const int lpc = lanes_per_candidate(d.npad);
  const bool wide = d.n > 256 / lpc;
  if (wide && round_p16(d) && !d.fd_rows && (lpc == 4 || lpc == 8)) {
    const size_t wb16 = (size_t)WROWS * lpc * 9 * 16;
    if (d.wide_cols == 2) {  // (A/B: window rows from la, hand-off from la_col)
      if (lpc == 4) k_round_wide<4, true, 2><<<d.n, 256, wb16, s>>>(d, p);
      else k_round_wide<8, true, 2><<<d.n, 256, wb16, s>>>(d, p);
    } else if (d.wide_cols) {
      if (lpc == 4) k_round_wide<4, true, 1><<<d.n, 256, wb16, s>>>(d, p);
      else k_round_wide<8, true, 1><<<d.n, 256, wb16, s>>>(d, p);
    } else {
      if (lpc == 4) k_round_wide<4, true><<<d.n, 256, wb16, s>>>(d, p);
      else k_round_wide<8, true><<<d.n, 256, wb16, s>>>(d, p);
    }
    return;
  }
  const size_t wbytes = wide ? (size_t)WROWS * lpc * (PIECES + 1) * 16 : (size_t)WROWS * (d.npad + SCAN_PAD) * 4;
#define L(K) K<<<d.n, 256, wbytes, s>>>(d, p)
#define LW(W) (k_round_wide<W, false>)<<<d.n, 256, wbytes, s>>>(d, p)
  switch (lpc) {
    case 1: if (wide) LW(1); else L(k_round<1>); break;
    case 2: if (wide) LW(2); else L(k_round<2>); break;
    case 4: if (wide) LW(4); else L(k_round<4>); break;
    case 8: if (wide) LW(8); else L(k_round<8>); break;
    default: if (wide) LW(16); else L(k_round<16>); break;
  }
#undef L
#undef LW
}

// ---------------------------------------------------------------------------
// witness tables for DecideFame, once after the loop: W(r) = the candidates
// of round r whose round is exactly r (B[r+1][q] > B[r][q]), in chain order;
// wrow = the row of their firstDescendants in fd (chain_start[q] + B[r][q]).
__device__ __forceinline__ void k_wcount_round(const Dev &d, int r) {
  const int lane = threadIdx.x, n = d.n;
  int cnt = 0;
  for (int q = lane; q < n; q += 64) {
    if (r < d.r0) {  // k_fiat's witnesses (Reset)
      cnt += r >= d.rlo && d.fw[(int64_t)(r - d.rlo) * n + q] >= 0;
      continue;
    }
    const int32_t b0 = d.B[(int64_t)r * n + q], b1 = d.B[(int64_t)(r + 1) * n + q];
    cnt += (b0 < d.chain_len[q] && b1 > b0) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if (lane == 0) d.wcnt[r] = cnt;
}

// R < 0: the loop's round count from the device (ST_ROUNDS, at most R_cap),
// read before the host has it (rounds_pipelined launches the tables ahead of
// its synchronisation); the workgroups stride over the rounds
__device__ __forceinline__ int wt_rounds(const Dev &d, int R) { return R >= 0 ? R : min(d.state[ST_ROUNDS], d.R_cap); }

__global__ __launch_bounds__(64) void k_wcount(Dev d, int R) {
  const int RR = wt_rounds(d, R);
  for (int r = blockIdx.x; r < RR; r += gridDim.x) k_wcount_round(d, r);
}

__global__ __launch_bounds__(1024) void k_wscan(Dev d, int R) {
  __shared__ int32_t part[1024];
  const int t = threadIdx.x;
  R = wt_rounds(d, R);
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

__device__ __forceinline__ void k_wfill_round(const Dev &d, int r) {
  const int lane = threadIdx.x, n = d.n;
  int32_t j = d.wofs[r];
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int q = c0 + lane;
    int32_t b0 = 0;
    bool w = false;
    if (q < n && r < d.r0) {  // k_fiat's witnesses (Reset)
      const int32_t x = r >= d.rlo ? d.fw[(int64_t)(r - d.rlo) * n + q] : -1;
      w = x >= 0;
      b0 = w ? d.index[x] : 0;
    } else if (q < n) {
      b0 = d.B[(int64_t)r * n + q];
      w = b0 < d.chain_len[q] && d.B[(int64_t)(r + 1) * n + q] > b0;
    }
    const unsigned long long m = __ballot(w);
    const int32_t k = j + popc64(m & ((1ull << lane) - 1ull));
    if (w && k < d.W_cap) {  // (W_cap: tables of a loop that failed are never read, but stay in bounds)
      d.wids[k] = d.chain_ids[d.chain_start[q] + b0];
      d.wrow[k] = d.chain_start[q] + b0;  // the witness's LA / FD row
    }
    j += popc64(m);
  }
}

__global__ __launch_bounds__(64) void k_wfill(Dev d, int R) {
  const int RR = wt_rounds(d, R);
  for (int r = blockIdx.x; r < RR; r += gridDim.x) k_wfill_round(d, r);
}

void launch_witness_tables(const Dev &d, int R, hipStream_t s) {
  if (R == 0) return;
  // (R < 0: the device's round count, 2048 workgroups striding over it)
  const unsigned g = R > 0 ? (unsigned)R : (unsigned)std::min(d.R_cap + 1, 2048);
  k_wcount<<<g, 64, 0, s>>>(d, R);
  k_wscan<<<1, 1024, 0, s>>>(d, R);
  k_wfill<<<g, 64, 0, s>>>(d, R);
}

// ---------------------------------------------------------------------------
// per-event round / witness from the boundary table (DivideRounds output,
// hashgraph.go:782-827): round(x) = max r with B[r][c] <= k.  Round and
// witness of an event depend only on its ancestors, so events divided by an
// earlier call get the same values again; only events inserted since
// (e >= n_prev) get their initial fame (Undefined for a witness), round
// received (nil) and consensus position.  A new witness of a round that is
// already processed (r < P) is never queued again (hashgraph.go:809-815) and
// so never decided: it is trapped.
__global__ void k_assign(Dev d, int64_t e_begin, int64_t n_prev, int32_t P) {
  const int64_t e = e_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int32_t R = d.state[ST_ROUNDS];
  const int32_t c = d.creator[e], k = d.index[e];
  const int n = d.n;
  int lo = d.r0;
  bool w;
  if (d.r0 > 0 && k < d.B[(int64_t)d.r0 * n + c]) {
    // below the closed form's first round (Reset): k_fiat's round and witness
    lo = d.round[e];
    w = d.witness[e] != 0;
  } else {
    int hi = R - 1;  // B[r0][c] <= k
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (d.B[(int64_t)mid * n + c] <= k) lo = mid;
      else hi = mid - 1;
    }
    d.round[e] = lo;
    w = d.B[(int64_t)lo * n + c] == k;
    d.witness[e] = w ? 1 : 0;
  }
  if (e >= n_prev) {
    d.fame[e] = w ? 0 : -1;
    d.rr[e] = UNSET;
    d.cons_pos[e] = -1;
    const bool trap = w && lo < P;
    d.trapped[e] = trap ? 1 : 0;
    if (trap) atomicAdd(&d.blocked[lo], 1);
  }
}

void launch_assign_rounds(const Dev &d, int64_t e_begin, int64_t n_prev, int32_t P, hipStream_t s) {
  if (d.N <= e_begin) return;
  k_assign<<<(unsigned)((d.N - e_begin + 255) / 256), 256, 0, s>>>(d, e_begin, n_prev, P);
}

// witnesses of the rounds just processed, [P0, P1), that were still
// Undefined: ProcessDecidedRounds went by the pending round's sticky decided
// flag (hashgraph.go:689-695, 1054-1056) and the round leaves PendingRounds
// for good, so DecideFame never visits them again
__global__ __launch_bounds__(64) void k_trap_processed(Dev d, int32_t P0) {
  const int32_t r = P0 + blockIdx.x;
  const int32_t b = d.wofs[r], cnt = d.wcnt[r];
  for (int i = threadIdx.x; i < cnt; i += 64) {
    const int32_t w = d.wids[b + i];
    if (d.fame[w] == 0 && !d.trapped[w]) {
      d.trapped[w] = 1;
      atomicAdd(&d.blocked[r], 1);
    }
  }
}

// ProcessDecidedRounds' read-back in one buffer (one device-to-host copy
// instead of five): the state words, then frames [P0, P0 + k)'s counts,
// offsets and loaded counts, then their transaction counts (8-byte aligned)
__global__ void k_pack_frames(Dev d, int32_t P0, int32_t k, int32_t *out) {
  const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < ST_COUNT) out[i] = d.state[i];
  if (i >= k) return;
  out[ST_COUNT + i] = d.frame_cnt[P0 + i];
  out[ST_COUNT + k + i] = d.frame_ofs[P0 + i];
  out[ST_COUNT + 2 * k + i] = d.frame_loaded[P0 + i];
  reinterpret_cast<int64_t *>(out + pack_ntx_at(k))[i] = d.frame_ntx[P0 + i];
}

void launch_pack_frames(const Dev &d, int32_t P0, int32_t k, int32_t *out, hipStream_t s) {
  const int32_t m = k > ST_COUNT ? k : ST_COUNT;
  k_pack_frames<<<(unsigned)((m + 255) / 256), 256, 0, s>>>(d, P0, k, out);
}

void launch_trap_processed(const Dev &d, int32_t P0, int32_t P1, hipStream_t s) {
  if (P1 <= P0) return;
  k_trap_processed<<<(unsigned)(P1 - P0), 64, 0, s>>>(d, P0);
}

}  // namespace bh
