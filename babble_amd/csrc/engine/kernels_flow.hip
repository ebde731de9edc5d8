// kernels_flow.hip -- event coordinates as a dataflow over creator chains.
//
// Reference: initEventCoordinates (hashgraph.go:439-507): LA[e][j] =
// max(LA[sp][j], LA[op][j]), LA[e][creator] = index; _lamportTimestamp
// (hashgraph.go:325-379): LT[e] = max(LT[sp], LT[op]) + 1.
//
// Mapping (n <= 128, chains shorter than 2^21): one workgroup per LA column
// (plus one for LT), one LANE per creator chain.  Along a chain the
// self-parent is the lane's previous event, so that half of the recurrence
// stays in a register; the other-parent (d, j) is read from chain d's ring
// of recent values in LDS, each slot tagged with the index it holds.  A lane
// advances when the tag matches (the parent is done); otherwise it retries
// on the next step.  Event (c, k) is thus computed at step LT(c, k) + 1:
// the number of serial steps is the DAG's critical path (its Lamport depth),
// and each step is one LDS round trip.  The chunked sweep in
// kernels_coords.hip (used above these limits) needs ~2.2x more steps.
//
// Waves: ceil(n/64) compute waves (64 chains each), one prefetch wave that
// keeps every chain's ring of other-parent descriptors (chain-major, packed
// as below) filled by LDS-DMA, 64 entries per refill, and one store wave
// that follows the value rings by tag and streams finished values to
// column-major LA (chain-major rows).  A parent older than the value ring
// (tag past j) is read back from there once the store wave has published
// (after its vmcnt(0)) that the value is in HBM.
#include "engine.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace bh {

// Stores of the transpose's outputs (LA rows, FDT).  BH_XPOSE_NT builds use
// non-temporal stores: streamed once, read rounds later, they need not
// displace the round loop's working set from L2 / the Infinity Cache while
// the segment pipeline runs both at once.
__device__ __forceinline__ void xstore(int32_t *p, int32_t v) {
#ifdef BH_XPOSE_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void xstore(int4 *p, int4 v) {
#ifdef BH_XPOSE_NT
  typedef int v4i __attribute__((ext_vector_type(4)));
  const v4i w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<v4i *>(p));
#else
  *p = v;
#endif
}

constexpr int FL_R = 64;     // value ring slots per chain (int2 {value, index})
constexpr int FL_DR = 128;   // descriptor ring entries per chain


typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) volatile int lds_vint;

// Descriptor of an other-parent (d, j): bits [31:15] = LDS byte address of
// its ring slot (d * FL_R + j % FL_R) * 8, bits [14:0] = j / FL_R (the slot's
// tag when it holds j), so a step extracts both with one shift and one AND.
// A ring slot is two dwords {value + 1 | (tag & 255) << 24, descriptor of
// the event it holds}: a consumer compares the second dword with its own
// descriptor as is, and the tag sits in both dwords, so a read that races
// the slot's write and sees one dword new and the other old fails the
// check (the slot's previous occupant had tag - 1) and is simply retried on
// the next step.  Values are carried biased by +1 (-1 = none) below 2^24
// (LA indexes < 2^21; LT < N < 2^24); a later occupant of the slot has a
// larger descriptor (same address, larger tag).
// Row n of the value ring is a sentinel chain: slot 63 holds the "no
// other-parent" event (value -1, always matches FL_NOOP), slot 62 = {0, 0}
// never matches FL_WAIT (a lane without a loaded descriptor), slots 0..60
// absorb the ring writes of lanes that did not advance.
constexpr int32_t FL_NOOP = 0x7FFF, FL_WAIT = 0x7FFE;
__host__ __device__ constexpr int32_t flow_desc(int32_t d, int32_t j, int32_t tag) {
  return (((d * 64 + (j & 63)) * 8) << 15) | tag;
}
// slot of event k (biased value vb) of the chain whose ring starts at LDS byte ring_c
__device__ __forceinline__ int2 flow_slot(int32_t vb, uint32_t ring_c, int32_t k) {
  const uint32_t addr = ring_c + ((uint32_t)(k & 63) << 3);
  return make_int2((int32_t)(((uint32_t)vb & 0xFFFFFFu) | ((uint32_t)k << 18 & 0xFF000000u)),
                   (int32_t)(addr << 15 | (uint32_t)(k >> 6)));
}
__device__ __forceinline__ bool flow_match(int2 s, int32_t dsc) {
  return s.y == dsc && ((uint32_t)s.x >> 24) == ((uint32_t)dsc & 255u);
}
__device__ __forceinline__ int32_t flow_vb(int2 s) { return (int32_t)((uint32_t)s.x & 0xFFFFFFu); }

// chain-major other-parent descriptors
__global__ void k_flow_desc(Dev d) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int32_t o = d.op[e];
  d.opdesc[d.epos[e]] = o < 0 ? flow_desc(d.n, 63, FL_NOOP) : flow_desc(d.creator[o], d.index[o], d.index[o] >> 6);
}

struct FlowLds {
  int2 vring[FL_MAXN + 1][FL_R];   // 64.5 KiB
  int32_t dring[FL_MAXN][FL_DR];   // 64 KiB
  int32_t filled[FL_MAXN], consumed[FL_MAXN], pub[FL_MAXN], cs[FL_MAXN], stored[FL_MAXN];
};

template <bool LT>
__device__ __forceinline__ void flow_body(const Dev &d, FlowLds &L, int col) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = d.n;
  const int nw = (n + 63) >> 6;  // compute waves
  const int64_t stride = d.la_rows + 64;
  int32_t *out = LT ? d.lt_row : d.la_col + (int64_t)col * stride;
  for (int c = t; c < n; c += blockDim.x) {
    L.filled[c] = 0;
    L.consumed[c] = 0;
    L.pub[c] = 0;
    L.stored[c] = 0;
    L.cs[c] = d.chain_start[c];
    for (int s = 0; s < FL_R; ++s)  // "before event s": descriptor tag 0, value tag byte 255
      L.vring[c][s] = make_int2((int32_t)0xFF000000u, flow_desc(c, s, 0));
  }
  if (t < FL_R) L.vring[n][t] = t == 63 ? make_int2((int32_t)0xFF000000u, flow_desc(n, 63, FL_NOOP)) : make_int2(0, 0);
  __syncthreads();
  lds_vint *filled = (lds_vint *)L.filled, *consumed = (lds_vint *)L.consumed, *pub = (lds_vint *)L.pub,
           *stored = (lds_vint *)L.stored;

  if (wave == nw) {
    // ---------------- prefetch wave: descriptor rings ----------------
    int32_t f[2] = {0, 0};  // entries filled, chains lane and lane + 64
    int32_t len[2], cs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = lane + 64 * h;
      len[h] = c < n ? d.chain_len[c] : 0;
      cs[h] = c < n ? d.chain_start[c] : 0;
    }
    for (;;) {
      bool left = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane + 64 * h;
        const int32_t cons = c < n ? consumed[c] : 0;
        const bool need = f[h] < len[h] && f[h] - cons <= FL_DR - 64;
        left |= f[h] < len[h];
        unsigned long long m = __ballot(need);
        while (m) {
          const int b = __builtin_ctzll(m);
          m &= m - 1;
          const int cc = b + 64 * h;
          const int32_t fc = __builtin_amdgcn_readlane(f[h], b);
          const int32_t csc = __builtin_amdgcn_readlane(cs[h], b);
          __builtin_amdgcn_global_load_lds((const void *)(d.opdesc + csc + fc + lane),
                                           (lds_void_t *)&L.dring[cc][fc & (FL_DR - 1)], 4, 0, 0);
        }
        if (need) f[h] += 64;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane + 64 * h;
        if (c < n) filled[c] = min(f[h], len[h]);
      }
      if (!__any(left)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    return;
  }
  if (wave == nw + 1) {
    // ---------------- store wave: rings -> HBM ----------------
    // Follows every chain's ring by tag and streams the finished values to
    // column-major LA; `stored` (slot reusable) bounds how far the compute
    // lanes may run ahead, `pub` (store complete: after vmcnt(0)) tells far
    // readers the value is in HBM.
    int32_t sp[2], len[2], cs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = lane + 64 * h;
      len[h] = c < n ? d.chain_len[c] : 0;
      cs[h] = c < n ? d.chain_start[c] : 0;
      sp[h] = c < n ? d.seg_lo[c] : 0;
    }
    for (int pass = 1;; ++pass) {
      bool left = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = min(lane + 64 * h, n);  // row n: sentinel, never matches below
        for (int it = 0; it < 8; ++it) {
          const int2 v = L.vring[c][sp[h] & (FL_R - 1)];
          const bool ok = sp[h] < len[h] && flow_match(v, flow_desc(c, sp[h], sp[h] >> 6));
          if (!__any(ok)) break;
          if (ok) {
            out[cs[h] + sp[h]] = flow_vb(v) - 1;
            ++sp[h];
          }
        }
        left |= sp[h] < len[h];
        if (lane + 64 * h < n) stored[lane + 64 * h] = sp[h];
      }
      if ((pass & 7) == 0 || !__any(left)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (lane + 64 * h < n) pub[lane + 64 * h] = sp[h];
      }
      if (!__any(left)) break;
    }
    return;
  }
  if (wave > nw + 1) return;

  // ---------------- compute waves: one chain per lane ----------------
  // Per step: two LDS reads (the other-parent's ring slot, the next
  // descriptor) and one ring write, all unconditional (lanes that do not
  // advance write the sentinel row), so the loop has no divergent branches;
  // refills, read-backs and the exit test sit in a header every 8 steps (a
  // lone wave issues in order, ~10 cycles per instruction: the step's
  // instruction count is its cost).  A lane may run at most 48 events ahead
  // of the store wave (ring slot reuse).
  static_assert(FL_R == 64, "descriptor packing assumes 64 ring slots");
  const int c = wave * 64 + lane;
  const bool valid = c < n;
  const int32_t len = valid ? d.chain_len[c] : 0;
  const int cc = valid ? c : 0;
  const bool own = !LT && c == col;
  const uint32_t ring_c = (uint32_t)(cc * FL_R * 8);           // LDS byte address of my ring
  const uint32_t wscratch = (uint32_t)((n * FL_R + lane % 61) * 8);
  const int32_t WAIT = flow_desc(n, 62, FL_WAIT);
  char *const lds = reinterpret_cast<char *>(&L.vring[0][0]);  // vring is at LDS offset 0
  const int32_t *dring_c = &L.dring[cc][0];
  int32_t k = 0, cur = 0, lim = 0;  // cur: value of event k-1, biased by +1
  int32_t dsc = WAIT;  // descriptor of event k, or WAIT until it may advance
  const bool dg = d.diag != nullptr && col == 0 && wave == 0;
  const unsigned long long t_start = dg ? stamp() : 0;
  int32_t step = 0;
  // one step of the chain: everything unconditional (a chain that does not
  // advance writes the sentinel row); ~20 VALU ops
#define FLOW_STEP()                                                               \
  do {                                                                          \
    const uint32_t sa_ = (uint32_t)dsc >> 15;                                   \
    const int2 slot_ = *reinterpret_cast<const int2 *>(lds + sa_);             \
    const int32_t kn_ = k + 1;                                                  \
    const int32_t dn_ = dring_c[kn_ & (FL_DR - 1)];                              \
    const bool ready_ = flow_match(slot_, dsc);                                 \
    int32_t v_ = max(cur, flow_vb(slot_));                                      \
    if (LT) v_ += 1;                                                            \
    else v_ = own ? k + 1 : v_; /* LA[e][creator] = index */                    \
    const uint32_t wa_ = ready_ ? ring_c + ((k & (FL_R - 1)) << 3) : wscratch;  \
    *reinterpret_cast<int2 *>(lds + wa_) = flow_slot(v_, ring_c, k);           \
    cur = ready_ ? v_ : cur;                                                    \
    dsc = ready_ ? (kn_ < lim ? dn_ : WAIT) : dsc;                              \
    k = ready_ ? kn_ : k;                                                       \
  } while (0)
  for (;; step += 8) {
    // header, every 8 steps: limits, stalled descriptors, read-backs, exit
    lim = valid ? min(filled[cc], stored[cc] + 48) : 0;
    if (dsc == WAIT && k < lim) dsc = dring_c[k & (FL_DR - 1)];
    if ((step & 63) == 0 && valid) consumed[c] = k;
    if (!__any(k < len)) break;
    {
      // a parent the ring has moved past (tag beyond j): read it back once
      // chain dd has published it, and take the step here (rare; one
      // inline-asm load with its own wait, so the compiler never sees a load
      // in flight across the loop)
      const uint32_t sa = (uint32_t)dsc >> 15;
      const int32_t tag = dsc & 0x7FFF;
      const int2 slot = *reinterpret_cast<const int2 *>(lds + sa);
      const int32_t dd = (int32_t)(sa >> 9), jj = (tag << 6) | ((sa >> 3) & 63);
      const bool far = (uint32_t)slot.y > (uint32_t)dsc && pub[dd] > jj;
      if (__builtin_expect(__any(far), 0)) {
        if (far) {
          const int32_t *fp = out + L.cs[dd] + jj;
          int32_t val;
          asm volatile("global_load_dword %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(val) : "v"(fp) : "memory");
          int32_t v = max(cur, val + 1);
          if (LT) v += 1;
          else v = own ? k + 1 : v;
          *reinterpret_cast<int2 *>(lds + ring_c + ((k & (FL_R - 1)) << 3)) = flow_slot(v, ring_c, k);
          cur = v;
          ++k;
          dsc = k < lim ? dring_c[k & (FL_DR - 1)] : WAIT;
        }
      }
    }
    FLOW_STEP(); FLOW_STEP(); FLOW_STEP(); FLOW_STEP();
    FLOW_STEP(); FLOW_STEP(); FLOW_STEP(); FLOW_STEP();
  }
#undef FLOW_STEP
  if (valid) consumed[c] = len;
  if (dg && lane == 0) {
    d.diag[DG_FL_STEPS] = step;
    d.diag[DG_FL_CYC] = stamp() - t_start;
  }
}

// workgroups 0 .. ncol-1: this shard's columns col0 + b; workgroup ncol (or
// every workgroup when lt_only): the Lamport timestamps
__global__ __launch_bounds__(256) void k_flow(Dev d, int lt_only) {
  __shared__ FlowLds L;  // static: the ring's LDS base is the constant 0
  if (lt_only || (int)blockIdx.x == d.ncol) flow_body<true>(d, L, d.n);
  else flow_body<false>(d, L, d.col0 + (int)blockIdx.x);
}

// ---------------------------------------------------------------------------
// k_flow32: the same dataflow with ONE-dword ring slots, for chains shorter
// than F2_MAXLEN (2^18 - 256) and Lamport timestamps below 2^21.  Rings hold
// 128 events per chain (66 KiB).
//   slot       = generation (k / 128, 11 bits) << 21 | value + 1 (21 bits)
//   descriptor = generation << 21 | LDS byte address of the slot
// A parent is ready when (slot ^ descriptor) < 2^21: one XOR and one
// compare, and a dword cannot be read torn.  Each descriptor-ring entry
// carries the next event's other-parent descriptor AND the current event's
// own slot descriptor (entry k + 1 = {op(k + 1), own(k)}), both prepared by
// k_flow_desc32, so a step spends no instructions encoding its write: 17
// VALU per step against 21 for k_flow (a lone wave issues one VALU per 8
// cycles on gfx950, tools/micro/lat.hip).  LT values that would reach 2^21
// are clamped (the generation bits stay intact, every lane keeps making
// progress) and flagged in ST_FLOWOVF; the host then recomputes LT with
// k_flow (LT workgroup only).
constexpr int F2_DR = 64;                   // descriptor-ring entries (int2) per chain
constexpr uint32_t F2_VMASK = 0x1FFFFFu;    // value bits
constexpr uint32_t F2_GMASK = 0xFFE00000u;  // generation bits
constexpr uint32_t F2_GNOOP = 0x7FF, F2_GWAIT = 0x7FE, F2_GINIT = 0x7FF;
constexpr int F2_R = 128;                   // value-ring slots per chain
// ring rows padded by one slot / one entry: lanes polling rings of
// different chains at similar indices hit different LDS banks
constexpr int F2_RS = F2_R + 1, F2_DRS = F2_DR + 1;
constexpr int32_t F2_MAXLEN = 0x7FE * F2_R;  // generations of real events stay <= 0x7FD
constexpr int32_t F2_LTCLAMP = (1 << 21) - 256;

__host__ __device__ constexpr uint32_t f2_desc(int32_t dch, int32_t j) {
  return ((uint32_t)(j >> 7) << 21) | (uint32_t)((dch * F2_RS + (j & (F2_R - 1))) * 4);
}
// sentinel row n: slot R-1 = "no other-parent" (value -1), slot R-2 never matches
__host__ __device__ constexpr uint32_t f2_noop(int n) { return (F2_GNOOP << 21) | (uint32_t)((n * F2_RS + F2_R - 1) * 4); }
__host__ __device__ constexpr uint32_t f2_wait(int n) { return (F2_GWAIT << 21) | (uint32_t)((n * F2_RS + F2_R - 2) * 4); }

// opw[row] = {descriptor of the row's other-parent, own slot of the row
// before it}; the .y of a chain's first row holds the previous chain's last
// own slot (the chain reads it as entry len)
__global__ void k_flow_desc32(Dev d) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  int2 *opw = reinterpret_cast<int2 *>(d.opdesc);
  const int32_t o = d.op[e], p = d.epos[e];
  opw[p].x = (int32_t)(o < 0 ? f2_noop(d.n) : f2_desc(d.creator[o], d.index[o]));
  opw[p + 1].y = (int32_t)f2_desc(d.creator[e], d.index[e]);
}

struct FlowLds32 {
  uint32_t vring[FL_MAXN + 1][F2_RS];  // 66 KiB, LDS offset 0
  int2 dring[FL_MAXN][F2_DRS];        // 66 KiB
  int32_t filled[FL_MAXN], consumed[FL_MAXN], pub[FL_MAXN], cs[FL_MAXN], stored[FL_MAXN];
};

template <bool LT>
__device__ __forceinline__ void flow32_body(const Dev &d, FlowLds32 &L) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = d.n;
  const int nw = (n + 63) >> 6;
  const int col = d.col0 + (int)blockIdx.x;  // this shard's columns; the LT workgroup is the last
  const int64_t stride = d.la_rows + 64;
  int32_t *out = LT ? d.lt_row : d.la_col + (int64_t)col * stride;
  // a segment resumes chain c at seg_lo[c]: its earlier events are in HBM
  // (published, read back like any parent older than its ring), and a slot
  // still holding GINIT (newer than every real generation) sends a lookup
  // of one of them there
  for (int c = t; c < n; c += blockDim.x) {
    const int32_t lo = d.seg_lo[c];
    L.filled[c] = lo;
    L.consumed[c] = lo;
    L.pub[c] = lo;
    L.stored[c] = lo;
    L.cs[c] = d.chain_start[c];
    for (int s = 0; s < F2_R; ++s) L.vring[c][s] = F2_GINIT << 21;  // matches no real event
  }
  for (int s = t; s < F2_R; s += blockDim.x) L.vring[n][s] = s == F2_R - 1 ? (F2_GNOOP << 21) : 0u;
  __syncthreads();
  lds_vint *filled = (lds_vint *)L.filled, *consumed = (lds_vint *)L.consumed, *pub = (lds_vint *)L.pub,
           *stored = (lds_vint *)L.stored;
  const int2 *opw = reinterpret_cast<const int2 *>(d.opdesc);

  if (wave == nw) {
    // ---------------- prefetch wave: descriptor rings, 32 entries per DMA ----------------
    int32_t f[2], tot[2], cs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = lane + 64 * h;
      const int32_t len = c < n ? d.chain_len[c] : 0;
      const int32_t lo = c < n ? d.seg_lo[c] : 0;
      // a DMA fills 32 ring entries at f & (F2_DR - 1): f stays a multiple of
      // 32 so it never runs past the ring row (entries below lo go unused)
      f[h] = lo & ~31;
      tot[h] = len > lo ? len + 1 : 0;  // entry len carries the last event's own slot
      cs[h] = c < n ? d.chain_start[c] : 0;
    }
    for (;;) {
      bool left = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane + 64 * h;
        const int32_t cons = c < n ? consumed[c] : 0;
        const bool need = f[h] < tot[h] && f[h] - cons <= F2_DR - 32;
        left |= f[h] < tot[h];
        unsigned long long m = __ballot(need);
        while (m) {
          const int b = __builtin_ctzll(m);
          m &= m - 1;
          const int cc = b + 64 * h;
          const int32_t fc = __builtin_amdgcn_readlane(f[h], b);
          const int32_t csc = __builtin_amdgcn_readlane(cs[h], b);
          __builtin_amdgcn_global_load_lds((const void *)(reinterpret_cast<const int32_t *>(opw + csc + fc) + lane),
                                           (lds_void_t *)&L.dring[cc][fc & (F2_DR - 1)], 4, 0, 0);
        }
        if (need) f[h] += 32;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane + 64 * h;
        if (c < n) filled[c] = min(f[h], tot[h]);
      }
      if (!__any(left)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    return;
  }
  if (wave == nw + 1) {
    // ---------------- store wave: rings -> HBM ----------------
    int32_t sp[2], len[2], cs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = lane + 64 * h;
      len[h] = c < n ? d.chain_len[c] : 0;
      cs[h] = c < n ? d.chain_start[c] : 0;
      sp[h] = c < n ? d.seg_lo[c] : 0;
    }
    // rows cs + sp = 0 mod 4 go out as one 16-B store of four events (a
    // store instruction touches a line per chain whatever its width, so this
    // quarters the wave's store work); a chain's first and last rows singly
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(stride * 4), 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    auto gen_ok = [](uint32_t v, int32_t j) { return (v ^ ((uint32_t)(j >> 7) << 21)) < (1u << 21); };
    for (int pass = 1;; ++pass) {
      bool left = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = min(lane + 64 * h, n);
        for (int it = 0; it < 8; ++it) {
          const int32_t j = sp[h];
          const bool grp = ((cs[h] + j) & 3) == 0 && j + 4 <= len[h];
          const uint32_t v3 = L.vring[c][(j + (grp ? 3 : 0)) & (F2_R - 1)];
          const bool ok = j < len[h] && gen_ok(v3, j + (grp ? 3 : 0));
          if (!__any(ok)) break;
          if (ok) {
            if (grp) {
              const uint32_t v0 = L.vring[c][j & (F2_R - 1)], v1 = L.vring[c][(j + 1) & (F2_R - 1)],
                             v2 = L.vring[c][(j + 2) & (F2_R - 1)];
              __builtin_amdgcn_raw_buffer_store_b128(
                  u32x4{(v0 & F2_VMASK) - 1u, (v1 & F2_VMASK) - 1u, (v2 & F2_VMASK) - 1u, (v3 & F2_VMASK) - 1u}, ro,
                  (int)((cs[h] + j) * 4), 0, 0);
              sp[h] = j + 4;
            } else {
              __builtin_amdgcn_raw_buffer_store_b32((v3 & F2_VMASK) - 1u, ro, (int)((cs[h] + j) * 4), 0, 0);
              sp[h] = j + 1;
            }
          }
        }
        left |= sp[h] < len[h];
        if (lane + 64 * h < n) stored[lane + 64 * h] = sp[h];
      }
      if ((pass & 7) == 0 || !__any(left)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (lane + 64 * h < n) pub[lane + 64 * h] = sp[h];
      }
      if (!__any(left)) break;
    }
    return;
  }
  if (wave > nw + 1) return;

  // ---------------- compute waves: one chain per lane ----------------
  const int c = wave * 64 + lane;
  const bool valid = c < n;
  const int32_t len = valid ? d.chain_len[c] : 0;
  const int cc = valid ? c : 0;
  const int32_t inc = LT ? 1 : (c == col ? 1 : 0);  // LT + 1; LA[e][creator] = index
  const uint32_t wscratch = (uint32_t)((n * F2_RS + lane) * 4);
  const uint32_t WAIT = f2_wait(n);
  char *const lds = reinterpret_cast<char *>(&L.vring[0][0]);  // vring is at LDS offset 0
  const int2 *dring_c = &L.dring[cc][0];
  // cur: value of event k-1 + 1 (0: no self-parent); a resumed segment
  // starts from the value its chain's previous event left in HBM
  int32_t k = valid ? d.seg_lo[c] : 0, cur = 0, lim = 0;
  if (k > 0) cur = out[d.chain_start[c] + k - 1] + 1;
  else if (LT && valid && d.lt_seed) cur = d.lt_seed[c] + 1;  // a Reset root's SelfParent LamportTimestamp
  uint32_t dsc = WAIT;
  const int32_t ltclamp = min(d.flow_ltclamp, F2_LTCLAMP);
  const bool dg = d.diag != nullptr && col == 0 && wave == 0;
  const unsigned long long t_start = dg ? stamp() : 0;
  int32_t step = 0;
#define F2_STEP()                                                                   \
  do {                                                                              \
    const uint32_t slot_ = *reinterpret_cast<const uint32_t *>(lds + (dsc & 0x1FFFFu)); \
    const int32_t kn_ = k + 1;                                                      \
    const int2 e_ = dring_c[kn_ & (F2_DR - 1)];                                     \
    const bool ready_ = (slot_ ^ dsc) < (1u << 21);                                 \
    const int32_t v_ = max(cur, (int32_t)(slot_ & F2_VMASK)) + inc;                 \
    const uint32_t wa_ = ready_ ? ((uint32_t)e_.y & 0x1FFFFu) : wscratch;           \
    *reinterpret_cast<uint32_t *>(lds + wa_) = ((uint32_t)e_.y & F2_GMASK) | (uint32_t)v_; \
    cur = ready_ ? v_ : cur;                                                        \
    dsc = ready_ ? (kn_ < lim ? (uint32_t)e_.x : WAIT) : dsc;                       \
    k = ready_ ? kn_ : k;                                                           \
  } while (0)
  for (;; step += 32) {
    // header: limits (entry k + 1 must be loaded: it holds k's own slot),
    // stalled descriptors, LT clamp, read-backs, exit
    lim = valid ? min(filled[cc] - 1, stored[cc] + F2_R - 16) : 0;
    if (dsc == WAIT && k < lim) dsc = (uint32_t)dring_c[k & (F2_DR - 1)].x;
    if (valid) consumed[c] = k;
    if (LT && __builtin_expect(__any(cur > ltclamp), 0)) {
      if (cur > ltclamp) {
        cur = ltclamp;
        d.state[ST_FLOWOVF] = 1;
      }
    }
    if (!__any(k < len)) break;
    {
      const uint32_t sa = dsc & 0x1FFFFu;
      const uint32_t slot = *reinterpret_cast<const uint32_t *>(lds + sa);
      const int32_t si = (int32_t)(sa >> 2), dd = si / F2_RS;
      const int32_t jj = (int32_t)((dsc >> 21) << 7) | (si - dd * F2_RS);
      const bool far = (slot & F2_GMASK) > (dsc & F2_GMASK) && pub[dd] > jj;
      if (__builtin_expect(__any(far), 0)) {
        if (far) {
          const int32_t *fp = out + L.cs[dd] + jj;
          int32_t val;
          asm volatile("global_load_dword %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(val) : "v"(fp) : "memory");
          const int32_t v = max(cur, val + 1) + inc;
          const uint32_t wd = (uint32_t)dring_c[(k + 1) & (F2_DR - 1)].y;
          *reinterpret_cast<uint32_t *>(lds + (wd & 0x1FFFFu)) = (wd & F2_GMASK) | (uint32_t)v;
          cur = v;
          ++k;
          dsc = k < lim ? (uint32_t)dring_c[k & (F2_DR - 1)].x : WAIT;
        }
      }
    }
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
    F2_STEP(); F2_STEP(); F2_STEP(); F2_STEP();
  }
#undef F2_STEP
  if (valid) consumed[c] = len;
  if (dg && lane == 0) {
    d.diag[DG_FL_STEPS] = step;
    d.diag[DG_FL_CYC] = stamp() - t_start;
  }
}

__global__ __launch_bounds__(256) void k_flow32(Dev d) {
  __shared__ FlowLds32 L;  // static: the ring's LDS base is the constant 0
  if ((int)blockIdx.x == d.ncol) flow32_body<true>(d, L);
  else flow32_body<false>(d, L);
}

// ---------------------------------------------------------------------------
// k_flow32x2: k_flow32's dataflow carrying TWO values per workgroup (round
// 5).  Every LA column and LT follow the same schedule -- a lane advances
// when its other-parent's slot holds the event, whatever the value -- so a
// lane can carry two of them per step at three more VALU ops (a max, an add,
// a select), and n columns + LT need (n + 1) / 2 workgroups: at n = 128, 65
// workgroups run the columns AND the Lamport timestamps in one launch (the
// one-value kernel needs 129, so LT ran as a second phase after the columns:
// 129 + the round loop's 128 workgroups exceed 256 compute units).
//   slot (8 B) = {generation (k / 64, 11 bits) << 21 | A + 1 (21 bits),
//                 B + 1 (32 bits)}
// in 64-slot rings (67 KiB, the LDS k_flow32's 128 one-dword slots took); a
// ds_read_b64 / ds_write_b64 of an aligned slot is one LDS access, so the
// generation in the low dword vouches for both (as in k_floww2).  The
// descriptor entries are k_flow32's ({other-parent's slot, own slot of the
// row before}, prepared by k_flow_desc32x2) with 64-slot addresses.  B is
// LT in workgroup 0 (32 bits: no clamp, no fallback) and an LA column
// elsewhere.  Chains up to 0x7FE * 64 = 131,008 events; longer ones (up to
// F2_MAXLEN) take k_flow32.
constexpr int X2_R = 64, X2_RS = X2_R + 1;     // value-ring slots (8 B) per chain, + 1 pad
constexpr int X2_DR = 64, X2_DRS = X2_DR + 1;  // descriptor-ring entries (int2) per chain
constexpr uint32_t X2_VMASK = 0x1FFFFFu, X2_GMASK = 0xFFE00000u;
constexpr uint32_t X2_GNOOP = 0x7FF, X2_GWAIT = 0x7FE, X2_GINIT = 0x7FF;
constexpr int32_t X2_MAXLEN = 0x7FE * X2_R;

__host__ __device__ constexpr uint32_t x2_desc(int32_t dch, int32_t j) {
  return ((uint32_t)(j >> 6) << 21) | (uint32_t)((dch * X2_RS + (j & (X2_R - 1))) * 8);
}
__host__ __device__ constexpr uint32_t x2_noop(int n) { return (X2_GNOOP << 21) | (uint32_t)((n * X2_RS + X2_R - 1) * 8); }
__host__ __device__ constexpr uint32_t x2_wait(int n) { return (X2_GWAIT << 21) | (uint32_t)((n * X2_RS + X2_R - 2) * 8); }

// Dynamic LDS the segments' small kernels ask for and never touch: more than
// the 12 KiB a persistent round-loop workgroup (>= 148 KiB) leaves on its
// compute unit, so their workgroups run on the others instead of taking the
// loop's issue slots (C3: k_flow_desc32x2 beside the loop cost 10-30 us per
// segment).  Ten such workgroups still fit a free compute unit
constexpr size_t GUARD_LDS = 16 * 1024;

__global__ void k_flow_desc32x2(Dev d) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  int2 *opw = reinterpret_cast<int2 *>(d.opdesc);
  const int32_t o = d.op[e], p = d.epos[e];
  opw[p].x = (int32_t)(o < 0 ? x2_noop(d.n) : x2_desc(d.creator[o], d.index[o]));
  opw[p + 1].y = (int32_t)x2_desc(d.creator[e], d.index[e]);
}

struct FlowLdsX2 {
  uint2 vring[FL_MAXN + 1][X2_RS];  // 67 KiB, LDS offset 0
  int2 dring[FL_MAXN][X2_DRS];      // 66.5 KiB
  int32_t filled[FL_MAXN], consumed[FL_MAXN], pub[FL_MAXN], cs[FL_MAXN], stored[FL_MAXN];
};

// colA / colB: the LA columns this workgroup carries (-1: none); ltB: B is LT
__device__ __forceinline__ void flow32x2_body(const Dev &d, FlowLdsX2 &L, int colA, int colB, bool ltB) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n = d.n;
  const int nw = (n + 63) >> 6;
  const int64_t stride = d.la_rows + 64;
  const bool hasA = colA >= 0, hasB = ltB || colB >= 0;
  int32_t *const pA = hasA ? d.la_col + (int64_t)colA * stride : nullptr;
  int32_t *const pB = ltB ? d.lt_row : colB >= 0 ? d.la_col + (int64_t)colB * stride : nullptr;
  // (an absent value reads the other one's array, and is never stored)
  int32_t *const outA = hasA ? pA : pB;
  int32_t *const outB = hasB ? pB : pA;
  for (int c = t; c < n; c += blockDim.x) {
    const int32_t lo = d.seg_lo[c];
    L.filled[c] = lo;
    L.consumed[c] = lo;
    L.pub[c] = lo;
    L.stored[c] = lo;
    L.cs[c] = d.chain_start[c];
    for (int s = 0; s < X2_R; ++s) L.vring[c][s] = make_uint2(X2_GINIT << 21, 0u);  // matches no real event
  }
  for (int s = t; s < X2_R; s += blockDim.x) L.vring[n][s] = make_uint2(s == X2_R - 1 ? (X2_GNOOP << 21) : 0u, 0u);
  __syncthreads();
  lds_vint *filled = (lds_vint *)L.filled, *consumed = (lds_vint *)L.consumed, *pub = (lds_vint *)L.pub,
           *stored = (lds_vint *)L.stored;
  const int2 *opw = reinterpret_cast<const int2 *>(d.opdesc);

  if (wave == nw) {
    // ---------------- prefetch wave: descriptor rings, 32 entries per DMA (as k_flow32) ----------------
    int32_t f[2], tot[2], cs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = lane + 64 * h;
      const int32_t len = c < n ? d.chain_len[c] : 0;
      const int32_t lo = c < n ? d.seg_lo[c] : 0;
      f[h] = lo & ~31;
      tot[h] = len > lo ? len + 1 : 0;  // entry len carries the last event's own slot
      cs[h] = c < n ? d.chain_start[c] : 0;
    }
    for (;;) {
      bool left = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane + 64 * h;
        const int32_t cons = c < n ? consumed[c] : 0;
        const bool need = f[h] < tot[h] && f[h] - cons <= X2_DR - 32;
        left |= f[h] < tot[h];
        unsigned long long m = __ballot(need);
        while (m) {
          const int b = __builtin_ctzll(m);
          m &= m - 1;
          const int cc = b + 64 * h;
          const int32_t fc = __builtin_amdgcn_readlane(f[h], b);
          const int32_t csc = __builtin_amdgcn_readlane(cs[h], b);
          __builtin_amdgcn_global_load_lds((const void *)(reinterpret_cast<const int32_t *>(opw + csc + fc) + lane),
                                           (lds_void_t *)&L.dring[cc][fc & (X2_DR - 1)], 4, 0, 0);
        }
        if (need) f[h] += 32;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane + 64 * h;
        if (c < n) filled[c] = min(f[h], tot[h]);
      }
      if (!__any(left)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    return;
  }
  if (wave == nw + 1) {
    // ---------------- store wave: rings -> HBM, both values ----------------
    int32_t sp[2], len[2], cs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = lane + 64 * h;
      len[h] = c < n ? d.chain_len[c] : 0;
      cs[h] = c < n ? d.chain_start[c] : 0;
      sp[h] = c < n ? d.seg_lo[c] : 0;
    }
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(outA, (short)0, (int)(stride * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(outB, (short)0, (int)(stride * 4), 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    auto gen_ok = [](uint32_t v, int32_t j) { return (v ^ ((uint32_t)(j >> 6) << 21)) < (1u << 21); };
    for (int pass = 1;; ++pass) {
      bool left = false;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = min(lane + 64 * h, n);  // row n: sentinel, never matches below
        const uint2 *ring = &L.vring[c][0];
        for (int it = 0; it < 8; ++it) {
          const int32_t j = sp[h];
          // rows cs + j = 0 mod 4: one 16-B store of four events per value
          const bool grp = ((cs[h] + j) & 3) == 0 && j + 4 <= len[h];
          const uint2 v3 = ring[(j + (grp ? 3 : 0)) & (X2_R - 1)];
          const bool ok = j < len[h] && gen_ok(v3.x, j + (grp ? 3 : 0));
          if (!__any(ok)) break;
          if (ok) {
            const int o = (int)((cs[h] + j) * 4);
            if (grp) {
              const uint2 v0 = ring[j & (X2_R - 1)], v1 = ring[(j + 1) & (X2_R - 1)], v2 = ring[(j + 2) & (X2_R - 1)];
              if (hasA)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{(v0.x & X2_VMASK) - 1u, (v1.x & X2_VMASK) - 1u,
                                                             (v2.x & X2_VMASK) - 1u, (v3.x & X2_VMASK) - 1u},
                                                       rA, o, 0, 0);
              if (hasB) __builtin_amdgcn_raw_buffer_store_b128(u32x4{v0.y - 1u, v1.y - 1u, v2.y - 1u, v3.y - 1u}, rB, o, 0, 0);
              sp[h] = j + 4;
            } else {
              if (hasA) __builtin_amdgcn_raw_buffer_store_b32((v3.x & X2_VMASK) - 1u, rA, o, 0, 0);
              if (hasB) __builtin_amdgcn_raw_buffer_store_b32(v3.y - 1u, rB, o, 0, 0);
              sp[h] = j + 1;
            }
          }
        }
        left |= sp[h] < len[h];
        if (lane + 64 * h < n) stored[lane + 64 * h] = sp[h];
      }
      if ((pass & 7) == 0 || !__any(left)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (lane + 64 * h < n) pub[lane + 64 * h] = sp[h];
      }
      if (!__any(left)) break;
    }
    return;
  }
  if (wave > nw + 1) return;

  // ---------------- compute waves: one chain per lane, two values ----------------
  const int c = wave * 64 + lane;
  const bool valid = c < n;
  const int32_t len = valid ? d.chain_len[c] : 0;
  const int cc = valid ? c : 0;
  const int32_t incA = c == colA ? 1 : 0;               // LA[e][creator] = index
  const int32_t incB = ltB ? 1 : (c == colB ? 1 : 0);  // LT + 1
  // lanes that do not advance write slots 0..31 of the sentinel row (62 and
  // 63 are the WAIT and no-other-parent slots)
  const uint32_t wscratch = (uint32_t)((n * X2_RS + (lane & 31)) * 8);
  const uint32_t WAIT = x2_wait(n);
  char *const lds = reinterpret_cast<char *>(&L.vring[0][0]);  // vring is at LDS offset 0
  const int2 *dring_c = &L.dring[cc][0];
  // cur*: value of event k-1 + 1 (0: no self-parent); a resumed segment
  // starts from the values its chain's previous event left in HBM
  int32_t k = valid ? d.seg_lo[c] : 0, curA = 0, curB = 0, lim = 0;
  if (k > 0) {
    const int64_t r = (int64_t)d.chain_start[c] + k - 1;
    curA = outA[r] + 1;
    curB = outB[r] + 1;
  } else if (ltB && valid && d.lt_seed) {
    curB = d.lt_seed[c] + 1;  // a Reset root's SelfParent LamportTimestamp
  }
  uint32_t dsc = WAIT;
  const bool dg = d.diag != nullptr && blockIdx.x == 0 && wave == 0;
  const unsigned long long t_start = dg ? stamp() : 0;
  int32_t step = 0;
#define X2_STEP()                                                                        \
  do {                                                                                   \
    const uint2 slot_ = *reinterpret_cast<const uint2 *>(lds + (dsc & 0x1FFFFu));        \
    const int32_t kn_ = k + 1;                                                           \
    const int2 e_ = dring_c[kn_ & (X2_DR - 1)];                                          \
    const bool ready_ = (slot_.x ^ dsc) < (1u << 21);                                    \
    const int32_t a_ = max(curA, (int32_t)(slot_.x & X2_VMASK)) + incA;                  \
    const int32_t b_ = max(curB, (int32_t)slot_.y) + incB;                               \
    const uint32_t wa_ = ready_ ? ((uint32_t)e_.y & 0x1FFFFu) : wscratch;                \
    *reinterpret_cast<uint2 *>(lds + wa_) = make_uint2(((uint32_t)e_.y & X2_GMASK) | (uint32_t)a_, (uint32_t)b_); \
    curA = ready_ ? a_ : curA;                                                           \
    curB = ready_ ? b_ : curB;                                                           \
    dsc = ready_ ? (kn_ < lim ? (uint32_t)e_.x : WAIT) : dsc;                            \
    k = ready_ ? kn_ : k;                                                                \
  } while (0)
  for (;; step += 32) {
    // header: limits (entry k + 1 must be loaded: it holds k's own slot),
    // stalled descriptors, read-backs, exit
    lim = valid ? min(filled[cc] - 1, stored[cc] + X2_R - 16) : 0;
    if (dsc == WAIT && k < lim) dsc = (uint32_t)dring_c[k & (X2_DR - 1)].x;
    if (valid) consumed[c] = k;
    if (!__any(k < len)) break;
    {
      // a parent the ring has moved past: read both values back once its
      // chain has published them
      const uint32_t sa = dsc & 0x1FFFFu;
      const uint32_t slot = *reinterpret_cast<const uint32_t *>(lds + sa);
      const int32_t si = (int32_t)(sa >> 3), dd = si / X2_RS;
      const int32_t jj = (int32_t)((dsc >> 21) << 6) | (si - dd * X2_RS);
      const bool far = (slot & X2_GMASK) > (dsc & X2_GMASK) && pub[dd] > jj;
      if (__builtin_expect(__any(far), 0)) {
        if (far) {
          const int64_t pr = (int64_t)L.cs[dd] + jj;
          int32_t va, vb;
          asm volatile("global_load_dword %0, %2, off nt\n\tglobal_load_dword %1, %3, off nt\n\ts_waitcnt vmcnt(0)"
                       : "=&v"(va), "=&v"(vb)
                       : "v"(outA + pr), "v"(outB + pr)
                       : "memory");
          const int32_t a = max(curA, va + 1) + incA, b = max(curB, vb + 1) + incB;
          const uint32_t wd = (uint32_t)dring_c[(k + 1) & (X2_DR - 1)].y;
          *reinterpret_cast<uint2 *>(lds + (wd & 0x1FFFFu)) = make_uint2((wd & X2_GMASK) | (uint32_t)a, (uint32_t)b);
          curA = a;
          curB = b;
          ++k;
          dsc = k < lim ? (uint32_t)dring_c[k & (X2_DR - 1)].x : WAIT;
        }
      }
    }
    X2_STEP(); X2_STEP(); X2_STEP(); X2_STEP();
    X2_STEP(); X2_STEP(); X2_STEP(); X2_STEP();
    X2_STEP(); X2_STEP(); X2_STEP(); X2_STEP();
    X2_STEP(); X2_STEP(); X2_STEP(); X2_STEP();
    X2_STEP(); X2_STEP(); X2_STEP(); X2_STEP();
    X2_STEP(); X2_STEP(); X2_STEP(); X2_STEP();
    X2_STEP(); X2_STEP(); X2_STEP(); X2_STEP();
    X2_STEP(); X2_STEP(); X2_STEP(); X2_STEP();
  }
#undef X2_STEP
  if (valid) consumed[c] = len;
  if (dg && lane == 0) {
    d.diag[DG_FL_STEPS] = step;
    d.diag[DG_FL_CYC] = stamp() - t_start;
  }
}

// values: the LA columns col0 .. col0 + ncol - 1 and, with flow_lt, LT.
// With LT, workgroup 0 carries {col0, LT} and workgroup w >= 1 {col0 + 2w -
// 1, col0 + 2w}; without, workgroup w carries {col0 + 2w, col0 + 2w + 1}.
// The last workgroup of an odd count carries one column.
__global__ __launch_bounds__(256) void k_flow32x2(Dev d) {
  __shared__ FlowLdsX2 L;  // static: the ring's LDS base is the constant 0
  const int w = (int)blockIdx.x, c0 = d.col0, c1 = d.col0 + d.ncol;
  const bool lt = d.flow_lt && w == 0;
  const int a = d.flow_lt ? c0 + 2 * w - 1 : c0 + 2 * w;  // (one call site: one copy of the unrolled loop)
  flow32x2_body(d, L, lt ? (d.ncol > 0 ? c0 : -1) : a, !lt && a + 1 < c1 ? a + 1 : -1, lt);
}

// column-major LA (chain-major rows) -> row-major LA; LT rows -> event
// ids; and the firstDescendants walk (kernels_fd.hip) on the same tile:
// the TR rows staged column-major are exactly what the walk searches, so
// FDT is produced here without a second pass over LA.  A tile may span
// chain boundaries; each run of rows of one chain is a walk segment whose
// column c owns FD entries j in (LA[row before][c], LA[last row][c]].
template <int TR, int BT>
__device__ __forceinline__ void xpose_tile(const Dev &d, const int64_t tix, int32_t *tile, int32_t *rc, int32_t *rj,
                                           uint64_t &segmask, uint64_t &insmask, int32_t *cstart, int32_t *clen) {
  constexpr int IPP = BT / TR;  // columns per load pass
  constexpr int LU = 16;        // load passes in flight
  const int t = threadIdx.x;
  if (tix * TR >= d.rows) return;
  const int64_t row0 = tix * TR;
  const int64_t N = d.rows;  // rows of the layout; the segment's are those with seg_lo <= index < chain_len
  const int n = d.n, npad = d.npad;
  const int64_t stride = d.la_rows + 64;
  const int ro = t % TR;
  const int rows = (int)min<int64_t>(TR, N - row0);
  const int64_t row = min(row0 + ro, N - 1);
  int32_t *prev = tile + npad * (TR + 1);
  if (t < TR) {
    const int32_t e = d.chain_ids[row];  // -1: a gap row of a chain's region
    const int32_t c = e >= 0 ? d.creator[e] : -1, k = e >= 0 ? d.index[e] : 0;
    const bool ins = t < rows && e >= 0 && k >= d.seg_lo[c] && k < d.chain_len[c];
    if (ins) d.lt[e] = d.lt_row[row0 + t];
    rc[t] = c;
    rj[t] = k;
    const uint64_t m = __ballot(ins);
    if (t == 0) insmask = m;
  }
  __syncthreads();
  const uint64_t insm = insmask;
  if (!insm) return;  // no row of this segment in the tile
  for (int i = t; i < n; i += BT) prev[i] = row0 > 0 ? d.la_col[(int64_t)i * stride + row0 - 1] : -1;
  for (int i = t; i < n; i += BT) {
    cstart[i] = d.chain_start[i];
    clen[i] = d.chain_len[i];
  }
  // column i of a load is uniform per wave when TR = 64: scalar base
  // address, 32-bit lane offset (TR = 32: two columns per wave)
  for (int i = TR >= 64 ? __builtin_amdgcn_readfirstlane(t / TR) : t / TR; i < n; i += LU * IPP) {
    int32_t v[LU];
#pragma unroll
    for (int u = 0; u < LU; ++u)
      v[u] = i + IPP * u < n ? __builtin_nontemporal_load(d.la_col + (int64_t)(i + IPP * u) * stride + row) : 0;
#pragma unroll
    for (int u = 0; u < LU; ++u)
      if (i + IPP * u < n) tile[(i + IPP * u) * (TR + 1) + ro] = v[u];
  }
  __syncthreads();
  if (t < 64) {  // segment starts: row 0 and every chain change
    const bool st = t < rows && t < TR && (t == 0 || rc[t] != rc[t - 1]);
    const uint64_t m = __ballot(st);
    if (t == 0) segmask = m;
  }
  {
    // rows out: thread = (row r0 + k * rpp, 4 columns i4); one division
    const int q4 = npad / 4, rpp = BT / q4;
    if (t < rpp * q4) {
      const int r0 = t / q4, i4 = (t - r0 * q4) * 4;
      int4 *dst = reinterpret_cast<int4 *>(d.la + row0 * npad + i4);
      for (int r = r0; r < rows; r += rpp) {
        if (!((insm >> r) & 1)) continue;  // rows of other segments are not (yet / any longer) ours
        int32_t o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = i4 + u < n ? tile[(i4 + u) * (TR + 1) + r] : -1;
        xstore(dst + (int64_t)r * q4, make_int4(o[0], o[1], o[2], o[3]));
      }
    }
  }
  __syncthreads();
  if (!d.xpose_fd) return;  // (the wide loop that counts its hand-off in la_col reads no FDT)
  const uint64_t segs = segmask;
  const int lane = t & 63, wave = t >> 6;
  for (uint64_t m = segs; m; m &= m - 1) {
    const int ra = __builtin_ctzll(m);
    const uint64_t rest = m & (m - 1);
    const int rb0 = rest ? __builtin_ctzll(rest) : rows;  // rows [ra, rb0) of one chain
    const int32_t i = rc[ra];
    if (i < 0) continue;  // gap rows
    // its rows inside the segment: [ra1, rb)
    const int32_t ka0 = rj[ra], lo_i = d.seg_lo[i];
    const int ra1 = ra + max(0, lo_i - ka0), rb = ra + min(rb0 - ra, clen[i] - ka0);
    if (ra1 >= rb) continue;
    const int32_t ka = ka0 + (ra1 - ra);
    if (ka + (rb - ra1) == clen[i])  // chain i's last event (of the prefix): rows it never sees
      for (int c = wave; c < n; c += BT / 64) {
        const int32_t hi = tile[c * (TR + 1) + rb - 1];
        for (int32_t j = hi + 1 + lane; j < clen[c]; j += 64) xstore(d.fdt + fdt_pos(cstart[c] + j, i, npad), FD_NONE);
      }
    // four columns per pass: their binary searches (log2 TR halvings of a
    // <= TR-row segment) interleave, so LDS latency is paid once per
    // four columns; the first 64 entries of each run here, longer runs'
    // remainders after
    for (int c0 = wave * 4; c0 < n; c0 += BT / 16) {
      int32_t lo[4], hi[4], a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = min(c0 + u, n - 1);
        const int32_t *col = tile + c * (TR + 1);
        lo[u] = ka == 0 ? -1 : (ra1 == 0 ? prev[c] : col[ra1 - 1]);
        hi[u] = c0 + u < n ? col[rb - 1] : lo[u];
        a[u] = ra1;
      }
      // the first row a in [ra1, rb) with LA >= j, as a fixed-length
      // lower bound over TR rows (log2 TR halvings, TR a power of two): rows
      // past rb - 1 read as row rb - 1, whose LA hi >= j
#pragma unroll
      for (int half = TR / 2; half >= 1; half >>= 1) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int idx = min(a[u] + half - 1, rb - 1);
          a[u] += tile[(c0 + u) * (TR + 1) + idx] < lo[u] + 1 + lane ? half : 0;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int32_t j = lo[u] + 1 + lane;
        if (j <= hi[u]) xstore(d.fdt + fdt_pos(cstart[c0 + u] + j, i, npad), ka + a[u] - ra1);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (hi[u] - lo[u] <= 64) continue;
        const int32_t *col = tile + (c0 + u) * (TR + 1);
        for (int32_t j0 = lo[u] + 65; j0 <= hi[u]; j0 += 64) {
          const int32_t j = j0 + lane;
          if (j <= hi[u]) {
            int aa = ra1, zz = rb - 1;
            while (aa < zz) {
              const int mm = (aa + zz) >> 1;
              if (col[mm] >= j) zz = mm;
              else aa = mm + 1;
            }
            xstore(d.fdt + fdt_pos(cstart[c0 + u] + j, i, npad), ka + aa - ra1);
          }
        }
      }
    }
  }
}

template <int TR, int BT>
__global__ __launch_bounds__(BT) void k_flow_transpose(Dev d) {
  extern __shared__ int32_t tile[];  // [npad][TR + 1], then prev[npad]
  __shared__ int32_t rc[TR], rj[TR];
  __shared__ uint64_t segmask, insmask;
  __shared__ int32_t cstart[512 + 16], clen[512 + 16];  // up to the wide dataflow's 512 chains
  if (d.tile_list) {
    // a segment's tiles, a contiguous share per
    // workgroup: few workgroups, so the round loop running beside them
    // keeps its compute units; consecutive tiles keep the "row before" in
    // the workgroup's XCD L2
    const int64_t per = (d.ntiles + gridDim.x - 1) / gridDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * per, i1 = min<int64_t>(d.ntiles, i0 + per);
    for (int64_t i = i0; i < i1; ++i) {
      __syncthreads();
      xpose_tile<TR, BT>(d, d.tile_list[i], tile, rc, rj, segmask, insmask, cstart, clen);
    }
    return;
  }
  // XCD-aware tile order: workgroup b runs on XCD b % 8, so give each XCD a
  // contiguous range of tiles -- a tile's "row before" (the previous tile's
  // last row) is then usually already in that XCD's L2
  // (the grid is rounded up to a multiple of 8 workgroups)
  const uint32_t per = gridDim.x / 8;
  const int64_t tix = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  xpose_tile<TR, BT>(d, tix, tile, rc, rj, segmask, insmask, cstart, clen);
}

// 128 chains (one LDS ring row each + the sentinel row within a 17-bit
// address), chains shorter than 2^21 (15-bit tags), values below 2^24
bool flow_eligible(const Dev &d) {
  return d.n <= FL_MAXN && d.max_chain_len < (1 << 21) && d.N < (1 << 24) - 1;
}

// one-dword slots: chains short enough for 11-bit generations
// (BH_SWEEP=flow64 forces the two-dword kernel)
bool flow32_eligible(const Dev &d) {
  const char *e = getenv("BH_SWEEP");
  return flow_eligible(d) && d.max_chain_len <= F2_MAXLEN && !(e && !strcmp(e, "flow64"));
}

// two values per workgroup (k_flow32x2) for chains up to X2_MAXLEN;
// BH_FLOW1=1 keeps the one-value k_flow32 (the fallback for chains up to
// F2_MAXLEN, parity-tested through this switch)
bool flow32x2_eligible(const Dev &d) {
  return flow32_eligible(d) && d.max_chain_len <= X2_MAXLEN && !(getenv("BH_FLOW1") && atoi(getenv("BH_FLOW1")));
}

const char *flow_kernel(const Dev &d) {
  return flow32x2_eligible(d) ? "k_flow32x2" : flow32_eligible(d) ? "k_flow32" : "k_flow";
}

void launch_flow_desc(const Dev &d, hipStream_t s) {
  if (d.N <= d.e0) return;
  // (GUARD_LDS: its workgroups stay off the compute units the round loop holds)
  if (flow32x2_eligible(d)) k_flow_desc32x2<<<(unsigned)((d.N - d.e0 + 255) / 256), 256, GUARD_LDS, s>>>(d);
  else if (flow32_eligible(d)) k_flow_desc32<<<(unsigned)((d.N - d.e0 + 255) / 256), 256, 0, s>>>(d);
  else k_flow_desc<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d);
}

void launch_flow(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  const int nw = (d.n + 63) / 64;
  if (flow32x2_eligible(d)) {
    const int nv = d.ncol + (d.flow_lt ? 1 : 0);
    if (nv > 0) k_flow32x2<<<(nv + 1) / 2, (nw + 2) * 64, 0, s>>>(d);
  } else if (flow32_eligible(d)) {
    k_flow32<<<d.ncol + (d.flow_lt ? 1 : 0), (nw + 2) * 64, 0, s>>>(d);
  } else {
    k_flow<<<d.ncol + 1, (nw + 2) * 64, 0, s>>>(d, 0);
  }
}

// LT overflowed k_flow32's 21-bit values (ST_FLOWOVF): recompute LT with
// the two-dword kernel's LT workgroup alone, then the rows' timestamps
void launch_flow_lt_fallback(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  const int nw = (d.n + 63) / 64;
  k_flow_desc<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d);
  k_flow<<<1, (nw + 2) * 64, 0, s>>>(d, 1);
  launch_flow_transpose(d, s);
}

void launch_flow_transpose(const Dev &d, hipStream_t s) {
  if (d.rows == 0) return;
  if (d.tile_list) {
    if (d.ntiles == 0) return;
    const int64_t wg = std::min<int64_t>(d.ntiles, 512);
    k_flow_transpose<64, 512><<<(unsigned)wg, 512, (size_t)d.npad * 66 * 4, s>>>(d);
    return;
  }
  if (d.npad > 128) {
    // wide rows: 32-row tiles so several workgroups share a compute unit --
    // the walk's LDS round trips are latency, not bandwidth (16- and 64-row
    // tiles measured slower, round 3)
    const unsigned tiles = (unsigned)((d.rows + 31) / 32);
    k_flow_transpose<32, 512><<<(tiles + 7) / 8 * 8, 512, (size_t)d.npad * 34 * 4, s>>>(d);
    return;
  }
  const unsigned tiles = (unsigned)((d.rows + 63) / 64);
  k_flow_transpose<64, 512><<<(tiles + 7) / 8 * 8, 512, (size_t)d.npad * 66 * 4, s>>>(d);
}

// Lamport timestamps of the events [e0, N) from the chain-major LT rows:
// the transpose's side job, for segments that do without it (n <= 128)
__global__ __launch_bounds__(256) void k_lt_rows(Dev d) {
  const int64_t e = d.e0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  d.lt[e] = d.lt_row[(int64_t)d.chain_start[d.creator[e]] + d.index[e]];
}

void launch_lt_rows(const Dev &d, hipStream_t s) {
  if (d.N <= d.e0) return;
  k_lt_rows<<<(unsigned)((d.N - d.e0 + 255) / 256), 256, GUARD_LDS, s>>>(d);
}

void launch_flow_coordinates(const Dev &d, hipStream_t s) {
  launch_flow_desc(d, s);
  launch_flow(d, s);
  launch_flow_transpose(d, s);
}

void configure_flow_kernels() {
  (void)hipFuncSetAttribute((const void *)k_flow_transpose<64, 512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
  (void)hipFuncSetAttribute((const void *)k_flow_transpose<32, 512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
}

}  // namespace bh
