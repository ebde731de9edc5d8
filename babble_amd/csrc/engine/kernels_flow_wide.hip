// kernels_flow_wide.hip -- the chain dataflow of kernels_flow.hip for wide
// groups (128 < n <= 512): initEventCoordinates (hashgraph.go:439-507) and
// _lamportTimestamp (:325-379) as one workgroup per LA column (plus one for
// LT), one lane per creator chain, 8 compute waves.
//
// What changes against k_flow32 (n <= 128) is the LDS budget: 512 chains'
// rings must fit one compute unit, so
//   * value rings hold 32 events per chain (one dword: generation (k / 32,
//     11 bits) << 21 | value + 1), 66 KiB;
//   * descriptor rings hold 32 other-parent descriptors per chain (one dword:
//     generation << 21 | LDS byte address of the parent's slot), 66 KiB; the
//     lane forms its own slot's address and generation from k (two VALU ops
//     more per step than k_flow32, whose descriptor entries carry it);
//   * there is no store wave: a compute lane stores each value to
//     column-major LA as it computes it, and publishes (for consumers whose
//     parent has left its 32-slot ring) the events whose stores an
//     `s_waitcnt vmcnt(16)` at its header proves complete -- the stores of
//     two headers ago.
// Two prefetch waves keep the descriptor rings filled, 16 entries per
// refill, loading for all their chains at once (one LDS-DMA per chain
// refill, as k_flow32 does, made the prefetch the bottleneck at 512 chains).  Chains shorter than 0x7FE * 32 = 65,472 events;
// Lamport timestamps at 2^21 are clamped and flagged (ST_FLOWOVF), and the
// host then recomputes the coordinates with the chunked sweep.
#include "engine.h"

#include <cstdlib>
#include <cstring>

namespace bh {

constexpr int FW_R = 32, FW_RS = FW_R + 1;    // value-ring slots per chain (+1 pad)
constexpr int FW_DR = 32, FW_DRS = FW_DR + 1;  // descriptor-ring entries per chain
constexpr int FW_REFILL = 16;                  // entries per descriptor refill
constexpr int FW_PW = 2;                       // prefetch waves
constexpr uint32_t FW_VMASK = 0x1FFFFFu, FW_GMASK = 0xFFE00000u;
constexpr uint32_t FW_GNOOP = 0x7FF, FW_GWAIT = 0x7FE, FW_GINIT = 0x7FF;
constexpr int32_t FW_MAXLEN = 0x7FE * FW_R;
constexpr int32_t FW_LTCLAMP = (1 << 21) - 256;

__host__ __device__ constexpr uint32_t fw_desc(int32_t dch, int32_t j) {
  return ((uint32_t)(j >> 5) << 21) | (uint32_t)((dch * FW_RS + (j & (FW_R - 1))) * 4);
}
// sentinel row n: slot R-1 = "no other-parent" (value -1), slot R-2 never matches
__host__ __device__ constexpr uint32_t fw_noop(int n) { return (FW_GNOOP << 21) | (uint32_t)((n * FW_RS + FW_R - 1) * 4); }
__host__ __device__ constexpr uint32_t fw_wait(int n) { return (FW_GWAIT << 21) | (uint32_t)((n * FW_RS + FW_R - 2) * 4); }

// opdesc[row] = descriptor of the row's other-parent
__global__ void k_flow_descw(Dev d) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int32_t o = d.op[e];
  d.opdesc[d.epos[e]] = (int32_t)(o < 0 ? fw_noop(d.n) : fw_desc(d.creator[o], d.index[o]));
}

struct FlowLdsW {
  uint32_t vring[FW_MAXN + 1][FW_RS];  // 66 KiB, LDS offset 0
  int32_t dring[FW_MAXN][FW_DRS];      // 66 KiB
  int32_t filled[FW_MAXN], consumed[FW_MAXN], pub[FW_MAXN], cs[FW_MAXN];
  int32_t abort_;  // set by a compute wave whose watchdog fired: every wave leaves
};
// a compute wave none of whose lanes advanced for this many headers (~0.6 s;
// a run takes tens of ms) leaves, the workgroup with it, and flags
// ST_FLOWOVF = 2: the host recomputes the coordinates with the chunked sweep

typedef __attribute__((address_space(3))) volatile int lds_vint_w;

template <bool LT>
__device__ __forceinline__ void floww_body(const Dev &d, FlowLdsW &L) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = d.n;
  const int nw = (n + 63) >> 6;
  const int col = d.col0 + (int)blockIdx.x;
  const int64_t stride = d.la_rows + 64;
  int32_t *out = LT ? d.lt_row : d.la_col + (int64_t)col * stride;
  for (int c = t; c < n; c += blockDim.x) {
    const int32_t lo = d.seg_lo[c];
    L.filled[c] = lo;
    L.consumed[c] = lo;
    L.pub[c] = lo;
    L.cs[c] = d.chain_start[c];
    for (int s = 0; s < FW_R; ++s) L.vring[c][s] = FW_GINIT << 21;  // matches no real event
  }
  for (int s = t; s < FW_R; s += blockDim.x) L.vring[n][s] = s == FW_R - 1 ? (FW_GNOOP << 21) : 0u;
  if (t == 0) L.abort_ = 0;
  __syncthreads();
  lds_vint_w *filled = (lds_vint_w *)L.filled, *consumed = (lds_vint_w *)L.consumed, *pub = (lds_vint_w *)L.pub;
  lds_vint_w *abort_ = (lds_vint_w *)&L.abort_;

  if (wave >= nw) {
    // ---------------- prefetch waves: descriptor rings ----------------
    // FW_PW waves, each owning chains lane + 64 h for its share of h; a
    // pass loads the next 16 descriptors of every chain that has room, for
    // all its chains at once (one memory latency per pass), then writes them
    // to the rings and publishes `filled`
    constexpr int H = FW_MAXN / 64 / FW_PW;
    const int h0 = (wave - nw) * H;
    if (h0 >= (n + 63) / 64) return;
    int32_t f[H], len[H], cs[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int c = lane + 64 * (h0 + h);
      len[h] = c < n ? d.chain_len[c] : 0;
      const int32_t lo = c < n ? d.seg_lo[c] : 0;
      f[h] = lo & ~(FW_REFILL - 1);  // refills stay aligned to the ring
      cs[h] = c < n ? d.chain_start[c] : 0;
    }
    for (;;) {
      bool left = false;
      bool need[H];
      int32_t v[H][FW_REFILL];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int c = lane + 64 * (h0 + h);
        const int32_t cons = c < n ? consumed[c] : 0;
        need[h] = f[h] < len[h] && f[h] - cons <= FW_DR - FW_REFILL;
        left |= f[h] < len[h];
        const int32_t *src = d.opdesc + cs[h] + f[h];
#pragma unroll
        for (int i = 0; i < FW_REFILL; ++i) v[h][i] = need[h] ? __builtin_nontemporal_load(src + i) : 0;
      }
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int c = lane + 64 * (h0 + h);
        if (need[h]) {
          int32_t *dst = &L.dring[c][f[h] & (FW_DR - 1)];
#pragma unroll
          for (int i = 0; i < FW_REFILL; ++i) dst[i] = v[h][i];
          f[h] += FW_REFILL;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int c = lane + 64 * (h0 + h);
        if (c < n) filled[c] = min(f[h], len[h]);
      }
      if (!__any(left) || *abort_) break;
      __builtin_amdgcn_s_sleep(1);
    }
    return;
  }
  if (wave > nw) return;
  int32_t stall = 0;

  // ---------------- compute waves: one chain per lane ----------------
  const int c = wave * 64 + lane;
  const bool valid = c < n;
  const int32_t len = valid ? d.chain_len[c] : 0;
  const int cc = valid ? c : 0;
  const int32_t inc = LT ? 1 : (c == col ? 1 : 0);  // LT + 1; LA[e][creator] = index
  const uint32_t ring_c = (uint32_t)(cc * FW_RS * 4);
  const uint32_t wscratch = (uint32_t)((n * FW_RS + (lane & 15)) * 4);
  const uint32_t WAIT = fw_wait(n);
  char *const lds = reinterpret_cast<char *>(&L.vring[0][0]);  // vring is at LDS offset 0
  const int32_t *dring_c = &L.dring[cc][0];
  int32_t *const outc = out + (valid ? d.chain_start[c] : 0);
  int32_t k = valid ? d.seg_lo[c] : 0, cur = 0, lim = 0;
  if (k > 0) cur = outc[k - 1] + 1;
  else if (LT && valid && d.lt_seed) cur = d.lt_seed[c] + 1;  // a Reset root's SelfParent LamportTimestamp
  int32_t k1 = k, k2 = k;  // k at the previous two headers: the stores before k2 are complete
  const bool dg = d.diag != nullptr && col == 0 && wave == 0;
  const unsigned long long t_start = dg ? stamp() : 0;
  int32_t step = 0;
  uint32_t dsc = WAIT;
  const int32_t ltclamp = min(d.flow_ltclamp, FW_LTCLAMP);
  // one step: the other-parent's slot, the next descriptor, the value
  // written to the ring and (by the lanes that advance) to HBM; a lane that
  // does not advance writes the sentinel row
#define FW_STEP()                                                                     \
  do {                                                                                \
    const uint32_t slot_ = *reinterpret_cast<const uint32_t *>(lds + (dsc & 0x1FFFFu)); \
    const int32_t kn_ = k + 1;                                                        \
    const uint32_t dn_ = (uint32_t)dring_c[kn_ & (FW_DR - 1)];                        \
    const bool ready_ = (slot_ ^ dsc) < (1u << 21);                                   \
    const int32_t v_ = max(cur, (int32_t)(slot_ & FW_VMASK)) + inc;                   \
    const uint32_t wa_ = ready_ ? ring_c + ((uint32_t)(k & (FW_R - 1)) << 2) : wscratch; \
    *reinterpret_cast<uint32_t *>(lds + wa_) = ((uint32_t)(k >> 5) << 21) | (uint32_t)v_; \
    if (ready_) outc[k] = v_ - 1;                                                     \
    cur = ready_ ? v_ : cur;                                                          \
    dsc = ready_ ? (kn_ < lim ? dn_ : WAIT) : dsc;                                    \
    k = ready_ ? kn_ : k;                                                             \
  } while (0)
  for (;;) {
    // header: publish, limits, stalled descriptors, LT clamp, read-backs, exit
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    if (valid) {
      pub[c] = k2;
      consumed[c] = k;
    }
    k2 = k1;
    k1 = k;
    lim = valid ? filled[cc] : 0;
    if (dsc == WAIT && k < lim) dsc = (uint32_t)dring_c[k & (FW_DR - 1)];
    if (LT && __builtin_expect(__any(cur > ltclamp), 0)) {
      if (cur > ltclamp) {
        cur = ltclamp;
        atomicMax(&d.state[ST_FLOWOVF], 1);
      }
    }
    if (!__any(k < len)) break;
    stall = __any(k != k2) ? 0 : stall + 1;
    if (stall > d.flow_wd || *abort_) {
      if (lane == 0) {
        *abort_ = 1;
        atomicMax(&d.state[ST_FLOWOVF], 2);
      }
      break;
    }
    {
      // a parent its ring has moved past: read it back once published
      const uint32_t sa = dsc & 0x1FFFFu;
      const uint32_t slot = *reinterpret_cast<const uint32_t *>(lds + sa);
      const int32_t si = (int32_t)(sa >> 2), dd = si / FW_RS;
      const int32_t jj = (int32_t)((dsc >> 21) << 5) | (si - dd * FW_RS);
      const bool far = (slot & FW_GMASK) > (dsc & FW_GMASK) && dd < n && pub[dd] > jj;
      if (__builtin_expect(__any(far), 0)) {
        if (far) {
          const int32_t *fp = out + L.cs[dd] + jj;
          int32_t val;
          asm volatile("global_load_dword %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(val) : "v"(fp) : "memory");
          const int32_t v = max(cur, val + 1) + inc;
          *reinterpret_cast<uint32_t *>(lds + ring_c + ((uint32_t)(k & (FW_R - 1)) << 2)) =
              ((uint32_t)(k >> 5) << 21) | (uint32_t)v;
          outc[k] = v - 1;
          cur = v;
          ++k;
          dsc = k < lim ? (uint32_t)dring_c[k & (FW_DR - 1)] : WAIT;
        }
      }
    }
    FW_STEP(); FW_STEP(); FW_STEP(); FW_STEP();
    FW_STEP(); FW_STEP(); FW_STEP(); FW_STEP();
    step += 8;
  }
#undef FW_STEP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (valid) {
    pub[c] = len;
    consumed[c] = len;
  }
  if (dg && lane == 0) {
    d.diag[DG_FL_STEPS] = step;
    d.diag[DG_FL_CYC] = stamp() - t_start;
  }
}

__global__ __launch_bounds__(64 * (FW_MAXN / 64 + FW_PW)) void k_floww(Dev d) {
  __shared__ FlowLdsW L;  // static: the ring's LDS base is the constant 0
  if ((int)blockIdx.x == d.ncol) floww_body<true>(d, L);
  else floww_body<false>(d, L);
}

// ---------------------------------------------------------------------------
// k_floww2: the same dataflow with two values per workgroup, so that n = 512
// columns + LT need 256 workgroups -- one per compute unit, one pass -- where
// k_floww's 513 take three (its LDS admits one workgroup per compute unit).
// Every column follows the same schedule (a lane advances when the
// other-parent's slot holds its event, whatever the column), so a lane
// carries two values per step; the slot grows to 8 bytes and the value ring
// shrinks to 16 events per chain:
//   low dword  = generation (k / 16, 15 bits) << 17 | A + 1   (17 bits)
//   high dword = B + 1 (32 bits), or B + 1 | (C + 1) << 16 for the one
//                workgroup that carries three LA columns (MODE 1; chain
//                positions < 65,535)
// Workgroups: values 0 .. ncol - 1 are LA columns col0 + v, value ncol is LT
// (always a B: the high dword's 32 bits).  ncol + 1 even: workgroup w takes
// values 2w, 2w + 1; odd: workgroup 0 takes three columns and w >= 1 takes
// 2w + 1, 2w + 2.  A step is one 8-byte slot read, one 8-byte ring write and
// two (three) HBM stores.
constexpr int F2_R = 16, F2_RS = F2_R + 1;
// rows per store group (aligned on the row): at a header at most F2_G - 1
// + 9 (8 steps and a read-back) events are unstored, within the 16-event ring
constexpr int F2_G = 8;
constexpr uint32_t F2_VMASK = 0x1FFFFu;
constexpr uint32_t F2_GNOOP = 0x7FFF, F2_GWAIT = 0x7FFE, F2_GINIT = 0x7FFF;

__host__ __device__ constexpr uint32_t f2_desc(int32_t dch, int32_t j) {
  return ((uint32_t)(j >> 4) << 17) | (uint32_t)((dch * F2_RS + (j & (F2_R - 1))) * 8);
}
__host__ __device__ constexpr uint32_t f2_noop(int n) { return (F2_GNOOP << 17) | (uint32_t)((n * F2_RS + F2_R - 1) * 8); }
__host__ __device__ constexpr uint32_t f2_wait(int n) { return (F2_GWAIT << 17) | (uint32_t)((n * F2_RS + F2_R - 2) * 8); }

__global__ void k_flow_descw2(Dev d) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int32_t o = d.op[e];
  d.opdesc[d.epos[e]] = (int32_t)(o < 0 ? f2_noop(d.n) : f2_desc(d.creator[o], d.index[o]));
}

struct FlowLdsW2 {
  uint2 vring[FW_MAXN + 1][F2_RS];  // 68 KiB, LDS offset 0
  int32_t dring[FW_MAXN][FW_DRS];   // 66 KiB
  int32_t filled[FW_MAXN], consumed[FW_MAXN], pub[FW_MAXN], cs[FW_MAXN];
  int32_t abort_;
};

// MODE 0: LA columns A, B; 1: LA columns A, B, C (16-bit B, C); 2: LA column A, LT in B
template <int MODE>
__device__ __forceinline__ void floww2_body(const Dev &d, FlowLdsW2 &L, int colA, int colB, int colC) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = d.n;
  const int nw = (n + 63) >> 6;
  const int64_t stride = d.la_rows + 64;
  int32_t *const outA = d.la_col + (int64_t)colA * stride;
  int32_t *const outB = MODE == 2 ? d.lt_row : d.la_col + (int64_t)colB * stride;
  int32_t *const outC = MODE == 1 ? d.la_col + (int64_t)colC * stride : outA;
  for (int c = t; c < n; c += blockDim.x) {
    const int32_t lo = d.seg_lo[c];
    L.filled[c] = lo;
    L.consumed[c] = lo;
    L.pub[c] = lo;
    L.cs[c] = d.chain_start[c];
    for (int s = 0; s < F2_R; ++s) L.vring[c][s] = make_uint2(F2_GINIT << 17, 0u);  // matches no real event
  }
  for (int s = t; s < F2_R; s += blockDim.x) L.vring[n][s] = make_uint2(s == F2_R - 1 ? (F2_GNOOP << 17) : 0u, 0u);
  if (t == 0) L.abort_ = 0;
  __syncthreads();
  lds_vint_w *filled = (lds_vint_w *)L.filled, *consumed = (lds_vint_w *)L.consumed, *pub = (lds_vint_w *)L.pub;
  lds_vint_w *abort_ = (lds_vint_w *)&L.abort_;

  if (wave >= nw) {
    // ---------------- prefetch waves: descriptor rings (as k_floww) ----------------
    constexpr int H = FW_MAXN / 64 / FW_PW;
    const int h0 = (wave - nw) * H;
    if (h0 >= (n + 63) / 64) return;
    int32_t f[H], len[H], cs[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int c = lane + 64 * (h0 + h);
      len[h] = c < n ? d.chain_len[c] : 0;
      const int32_t lo = c < n ? d.seg_lo[c] : 0;
      f[h] = lo & ~(FW_REFILL - 1);
      cs[h] = c < n ? d.chain_start[c] : 0;
    }
    for (;;) {
      bool left = false;
      bool need[H];
      int32_t v[H][FW_REFILL];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int c = lane + 64 * (h0 + h);
        const int32_t cons = c < n ? consumed[c] : 0;
        need[h] = f[h] < len[h] && f[h] - cons <= FW_DR - FW_REFILL;
        left |= f[h] < len[h];
        const int32_t *src = d.opdesc + cs[h] + f[h];
#pragma unroll
        for (int i = 0; i < FW_REFILL; ++i) v[h][i] = need[h] ? __builtin_nontemporal_load(src + i) : 0;
      }
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int c = lane + 64 * (h0 + h);
        if (need[h]) {
          int32_t *dst = &L.dring[c][f[h] & (FW_DR - 1)];
#pragma unroll
          for (int i = 0; i < FW_REFILL; ++i) dst[i] = v[h][i];
          f[h] += FW_REFILL;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int c = lane + 64 * (h0 + h);
        if (c < n) filled[c] = min(f[h], len[h]);
      }
      if (!__any(left) || *abort_) break;
      __builtin_amdgcn_s_sleep(1);
    }
    return;
  }
  int32_t stall = 0;

  // ---------------- compute waves: one chain per lane ----------------
  const int c = wave * 64 + lane;
  const bool valid = c < n;
  const int32_t len = valid ? d.chain_len[c] : 0;
  const int cc = valid ? c : 0;
  const int32_t incA = c == colA ? 1 : 0;
  const int32_t incB = MODE == 2 ? 1 : (c == colB ? 1 : 0);
  const int32_t incC = MODE == 1 && c == colC ? 1 : 0;
  const uint32_t ring_c = (uint32_t)(cc * F2_RS * 8);
  const uint32_t wscratch = (uint32_t)((n * F2_RS + (lane & 7)) * 8);  // slots 0..7 of the sentinel row
  const uint32_t WAIT = f2_wait(n);
  char *const lds = reinterpret_cast<char *>(&L.vring[0][0]);
  const int32_t *dring_c = &L.dring[cc][0];
  const int64_t cso = valid ? d.chain_start[c] : 0;
  int32_t k = valid ? d.seg_lo[c] : 0, curA = 0, curB = 0, curC = 0, lim = 0;
  if (k > 0) {
    curA = outA[cso + k - 1] + 1;
    curB = outB[cso + k - 1] + 1;
    if (MODE == 1) curC = outC[cso + k - 1] + 1;
  } else if (MODE == 2 && valid && d.lt_seed) {
    curB = d.lt_seed[c] + 1;  // a Reset root's SelfParent LamportTimestamp
  }
  // the stores: buffer stores at one per-lane byte offset (row * 4) into
  // each value's column (wave-uniform descriptors: no 64-bit address math
  // per store)
  auto rsrc = [&](int32_t *p) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0, (int)(stride * 4), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rA = rsrc(outA), rB = rsrc(outB), rC = rsrc(outC);
  // events [kf, k) are computed but not yet stored: the ring holds them (at
  // most F2_G - 1 + 9 <= 16 at a header); a header stores complete F2_G-row
  // groups (rows cso + kf = 0 mod F2_G: 16-B stores, a quarter of the store
  // instructions -- each one touches 64 chains' lines, which is what bounds a
  // step -- and 32 B of a line at once, fewer partial-line evictions) and
  // single rows at a chain's ends
  int32_t kf = k;
  auto slot_vals = [&](int32_t j, int32_t &a, int32_t &b, int32_t &c3) {
    const uint2 v = *reinterpret_cast<const uint2 *>(lds + ring_c + ((uint32_t)(j & (F2_R - 1)) << 3));
    a = (int32_t)(v.x & F2_VMASK) - 1;
    if constexpr (MODE == 1) {
      b = (int32_t)(v.y & 0xFFFFu) - 1;
      c3 = (int32_t)(v.y >> 16) - 1;
    } else {
      b = (int32_t)v.y - 1;
      c3 = 0;
    }
  };
  auto store1 = [&](int32_t j) {
    int32_t a, b, c3;
    slot_vals(j, a, b, c3);
    const int o = (int)((cso + j) * 4);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)a, rA, o, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)b, rB, o, 0, 0);
    if constexpr (MODE == 1) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)c3, rC, o, 0, 0);
  };
  auto flush = [&](bool tail) {
    for (;;) {  // rows before the first aligned group (a chain's start)
      const bool go = kf < k && ((cso + kf) & (F2_G - 1)) != 0;
      if (!__any(go)) break;
      if (go) { store1(kf); ++kf; }
    }
    for (;;) {
      const bool go = kf + F2_G <= k;
      if (!__any(go)) break;
      if (go) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int h = 0; h < F2_G; h += 4) {  // 16-B stores of one 32-B (F2_G rows) piece, back to back
          int32_t a[4], b[4], c3[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) slot_vals(kf + h + u, a[u], b[u], c3[u]);
          const int o = (int)((cso + kf + h) * 4);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)a[0], (unsigned)a[1], (unsigned)a[2], (unsigned)a[3]}, rA, o, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)b[0], (unsigned)b[1], (unsigned)b[2], (unsigned)b[3]}, rB, o, 0, 0);
          if constexpr (MODE == 1)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)c3[0], (unsigned)c3[1], (unsigned)c3[2], (unsigned)c3[3]}, rC, o, 0, 0);
        }
        kf += F2_G;
      }
    }
    if (tail) {
      for (;;) {
        const bool go = kf < k;
        if (!__any(go)) break;
        if (go) { store1(kf); ++kf; }
      }
    }
  };
  int32_t hdr = 0, k1 = k, k2 = k;  // k at the previous two headers (the watchdog)
  const bool dg = d.diag != nullptr && blockIdx.x == 0 && wave == 0;
  const unsigned long long t_start = dg ? stamp() : 0;
  int32_t step = 0;
  uint32_t dsc = WAIT;
  const int32_t ltclamp = min(d.flow_ltclamp, FW_LTCLAMP);
#define F2_STEP()                                                                          \
  do {                                                                                     \
    const uint2 slot_ = *reinterpret_cast<const uint2 *>(lds + (dsc & 0x1FFFFu));          \
    const int32_t kn_ = k + 1;                                                             \
    const uint32_t dn_ = (uint32_t)dring_c[kn_ & (FW_DR - 1)];                             \
    const bool ready_ = (slot_.x ^ dsc) < (1u << 17);                                      \
    const int32_t a_ = max(curA, (int32_t)(slot_.x & F2_VMASK)) + incA;                    \
    int32_t b_, c_ = 0;                                                                    \
    uint32_t hi_;                                                                          \
    if constexpr (MODE == 1) {                                                             \
      b_ = max(curB, (int32_t)(slot_.y & 0xFFFFu)) + incB;                                 \
      c_ = max(curC, (int32_t)(slot_.y >> 16)) + incC;                                     \
      hi_ = (uint32_t)b_ | ((uint32_t)c_ << 16);                                           \
    } else {                                                                               \
      b_ = max(curB, (int32_t)slot_.y) + incB;                                             \
      hi_ = (uint32_t)b_;                                                                  \
    }                                                                                      \
    const uint32_t wa_ = ready_ ? ring_c + ((uint32_t)(k & (F2_R - 1)) << 3) : wscratch;   \
    *reinterpret_cast<uint2 *>(lds + wa_) = make_uint2(((uint32_t)(k >> 4) << 17) | (uint32_t)a_, hi_); \
    curA = ready_ ? a_ : curA;                                                             \
    curB = ready_ ? b_ : curB;                                                             \
    if constexpr (MODE == 1) curC = ready_ ? c_ : curC;                                    \
    dsc = ready_ ? (kn_ < lim ? dn_ : WAIT) : dsc;                                         \
    k = ready_ ? kn_ : k;                                                                  \
  } while (0)
  for (;;) {
    // header: publish, store, limits, stalled descriptors, LT clamp,
    // read-backs, exit.  Every 4th header drains the stores and publishes
    // what was stored before it (far readers read those from HBM)
    if ((hdr++ & 3) == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (valid) pub[c] = kf;
    }
    if (valid) consumed[c] = k;
    flush(false);
    k2 = k1;
    k1 = k;
    lim = valid ? filled[cc] : 0;
    if (dsc == WAIT && k < lim) dsc = (uint32_t)dring_c[k & (FW_DR - 1)];
    if (MODE == 2 && __builtin_expect(__any(curB > ltclamp), 0)) {
      if (curB > ltclamp) {
        curB = ltclamp;
        atomicMax(&d.state[ST_FLOWOVF], 1);
      }
    }
    if (!__any(k < len)) break;
    stall = __any(k != k2) ? 0 : stall + 1;
    if (stall > d.flow_wd || *abort_) {
      if (lane == 0) {
        *abort_ = 1;
        atomicMax(&d.state[ST_FLOWOVF], 2);
      }
      break;
    }
    {
      // a parent its ring has moved past: read it back once published
      const uint32_t sa = dsc & 0x1FFFFu;
      const uint32_t slot = *reinterpret_cast<const uint32_t *>(lds + sa);
      const int32_t si = (int32_t)(sa >> 3), dd = si / F2_RS;
      const int32_t jj = (int32_t)((dsc >> 17) << 4) | (si - dd * F2_RS);
      const bool far = (slot & ~F2_VMASK) > (dsc & ~F2_VMASK) && dd < n && pub[dd] > jj;
      if (__builtin_expect(__any(far), 0)) {
        if (far) {
          const int64_t pr = (int64_t)L.cs[dd] + jj;
          // one asm statement: the compiler must not touch the destinations
          // before the wait
          int32_t va, vb, vc = -1;
          if constexpr (MODE == 1)
            asm volatile("global_load_dword %0, %3, off nt\n\tglobal_load_dword %1, %4, off nt\n\t"
                         "global_load_dword %2, %5, off nt\n\ts_waitcnt vmcnt(0)"
                         : "=&v"(va), "=&v"(vb), "=&v"(vc)
                         : "v"(outA + pr), "v"(outB + pr), "v"(outC + pr)
                         : "memory");
          else
            asm volatile("global_load_dword %0, %2, off nt\n\tglobal_load_dword %1, %3, off nt\n\ts_waitcnt vmcnt(0)"
                         : "=&v"(va), "=&v"(vb)
                         : "v"(outA + pr), "v"(outB + pr)
                         : "memory");
          const int32_t a = max(curA, va + 1) + incA, b = max(curB, vb + 1) + incB;
          const int32_t c3 = MODE == 1 ? max(curC, vc + 1) + incC : 0;
          const uint32_t hi = MODE == 1 ? ((uint32_t)b | ((uint32_t)c3 << 16)) : (uint32_t)b;
          *reinterpret_cast<uint2 *>(lds + ring_c + ((uint32_t)(k & (F2_R - 1)) << 3)) =
              make_uint2(((uint32_t)(k >> 4) << 17) | (uint32_t)a, hi);
          curA = a;
          curB = b;
          if (MODE == 1) curC = c3;
          ++k;
          dsc = k < lim ? (uint32_t)dring_c[k & (FW_DR - 1)] : WAIT;
        }
      }
    }
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    step += 8;
  }
#undef F2_STEP
  flush(true);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (valid) {
    pub[c] = len;
    consumed[c] = len;
  }
  if (dg && lane == 0) {
    d.diag[DG_FL_STEPS] = step;
    d.diag[DG_FL_CYC] = stamp() - t_start;
  }
}

__global__ __launch_bounds__(64 * (FW_MAXN / 64 + FW_PW)) void k_floww2(Dev d) {
  __shared__ FlowLdsW2 L;  // static: the ring's LDS base is the constant 0
  const int w = (int)blockIdx.x, nc = d.ncol, c0 = d.col0;
  if (((nc + 1) & 1) == 0) {  // values 2w, 2w + 1
    const int v = 2 * w;
    if (v + 1 == nc) floww2_body<2>(d, L, c0 + v, 0, 0);
    else floww2_body<0>(d, L, c0 + v, c0 + v + 1, 0);
  } else if (w == 0) {
    floww2_body<1>(d, L, c0, c0 + 1, c0 + 2);
  } else {
    const int v = 2 * w + 1;
    if (v + 1 == nc) floww2_body<2>(d, L, c0 + v, 0, 0);
    else floww2_body<0>(d, L, c0 + v, c0 + v + 1, 0);
  }
}

// the two-value kernel: at least 4 columns (so that a three-column
// workgroup and the LT workgroup are distinct); BH_FLOWW=1 keeps k_floww
static bool floww2_on(const Dev &d) {
  const bool off = getenv("BH_FLOWW") && atoi(getenv("BH_FLOWW")) == 1;
  return !off && d.ncol >= 4;
}

bool floww_eligible(const Dev &d) {
  const char *e = getenv("BH_SWEEP");
  return d.n > FL_MAXN && d.n <= FW_MAXN && d.max_chain_len <= FW_MAXLEN && !(e && !strcmp(e, "chunk"));
}

const char *floww_kernel(const Dev &d) { return floww2_on(d) ? "k_floww2" : "k_floww"; }

void launch_floww(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  const int nw = (d.n + 63) / 64;
  if (floww2_on(d)) {
    if (d.N > d.e0) k_flow_descw2<<<(unsigned)((d.N - d.e0 + 255) / 256), 256, 0, s>>>(d);
    k_floww2<<<(d.ncol + 1) / 2, (nw + FW_PW) * 64, 0, s>>>(d);
    return;
  }
  if (d.N > d.e0) k_flow_descw<<<(unsigned)((d.N - d.e0 + 255) / 256), 256, 0, s>>>(d);
  k_floww<<<d.ncol + 1, (nw + FW_PW) * 64, 0, s>>>(d);
}

}  // namespace bh
