// kernels_coords.hip -- event coordinates (lastAncestors) and Lamport timestamps.
//
// Reference: initEventCoordinates (hashgraph.go:439-507) computes, per event,
// LA[e][j] = max(LA[sp][j], LA[op][j]) with LA[e][creator] = index, and
// _lamportTimestamp (hashgraph.go:325-379) LT[e] = max(LT[sp], LT[op]) + 1.
// firstDescendants (updateAncestorFirstDescendant, :510-544) follow from LA
// in closed form (kernels_fd.hip).
//
// MI355X mapping: each column j depends only on column j of the parents, so
// the columns are split over workgroups that never communicate: one
// workgroup per column walks ALL events in topological order, 64 events
// (one per lane) per chunk, resolving intra-chunk dependencies in `depth`
// sub-steps.  Parents within the last `ring` events are read from an LDS
// ring (the common case: the self-parent is the creator's previous event,
// the other-parent a recent head); older ones from HBM.  One extra
// workgroup computes LT the same way.  The kernel is bound by the DAG's
// critical path (sub-steps x LDS round trip), not by HBM bandwidth -- see
// DESIGN.md.
#include "engine.h"

namespace bh {

// ---------------------------------------------------------------------------
// prep: chain-major id table (ParticipantEventsCache, caches.go:34-129) and
// round-loop state.
__global__ void k_chain_scatter(Dev d, int64_t e_begin) {
  int64_t e = e_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int32_t p = d.chain_start[d.creator[e]] + d.index[e];
  d.chain_ids[p] = (int32_t)e;
  d.epos[e] = p;
}

__global__ void k_state_init(Dev d) {
  int t = threadIdx.x;
  if (t < ST_COUNT) d.state[t] = 0;
  for (int c = t; c < d.n; c += blockDim.x) {
    d.B[c] = 0;  // B[0][c]: every event has round >= 0
    d.Bp[c] = 0;
  }
  if (t == 0) d.wofs[0] = 0;
}

void launch_prep(const Dev &d, hipStream_t s) {
  if (d.rows > 0) (void)hipMemsetAsync(d.chain_ids, 0xFF, (size_t)d.rows * 4, s);  // gap rows: -1
  launch_chain_scatter(d, 0, s);
  k_state_init<<<1, 256, 0, s>>>(d);
}

void launch_chain_scatter(const Dev &d, int64_t e_begin, hipStream_t s) {
  if (d.N > e_begin) k_chain_scatter<<<(unsigned)((d.N - e_begin + 255) / 256), 256, 0, s>>>(d, e_begin);
}

// ---------------------------------------------------------------------------
// intra-chunk dependency depth: one wave per 64-event chunk; parents inside
// the chunk have smaller lanes, so the Jacobi update converges in depth+1.
__global__ __launch_bounds__(256) void k_chunk_depth(Dev d) {
  const int lane = threadIdx.x & 63;
  const int64_t chunk = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t base = chunk * 64;
  if (base >= d.N) return;
  const int64_t e = base + lane;
  const bool valid = e < d.N;
  int psp = -1, pop = -1;
  if (valid) {
    const int32_t s = d.sp[e], o = d.op[e];
    if (s >= base) psp = (int)(s - base);
    if (o >= base) pop = (int)(o - base);
  }
  int dep = 0;
  for (int it = 0; it < 64; ++it) {
    const int ds = __shfl(dep, psp < 0 ? lane : psp);
    const int dop = __shfl(dep, pop < 0 ? lane : pop);
    int nd = 0;
    if (psp >= 0) nd = ds + 1;
    if (pop >= 0) nd = max(nd, dop + 1);
    const bool ch = nd != dep;
    dep = nd;
    if (!__any(ch)) break;
  }
  if (valid) d.depth[e] = (uint8_t)dep;
  int m = valid ? dep : 0;
  for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
  if (lane == 0) d.chunk_maxd[chunk] = (uint8_t)m;
}

// per-event sweep descriptor, 16 B -- everything the compute wave needs,
// precomputed so that its per-chunk work is one LDS read:
//   .x = ring slot of sp | ring slot of op << 16
//   .y = creator | flags << 16
//   .z = index, .w = unused
// Ring slots are (event & (ring-1)); an absent parent, or one that is too
// old to still be in the ring ("far"), maps to the sentinel slot `ring`
// (always -1).  flags = maxd (max intra-chunk depth, chunk-uniform) |
// chunk-has-far << 8 | sp-far << 9 | op-far << 10.
constexpr int SW_FAR = 0x100, SW_SPFAR = 0x200, SW_OPFAR = 0x400;

__global__ __launch_bounds__(256) void k_pack_desc(Dev d) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t base = e & ~(int64_t)63;  // a wave is a chunk
  const bool valid = e < d.N;
  const int ring = 1 << d.ring_log2;
  const int64_t ring_lo = base + 64 - ring;
  int32_t sp = -1, op = -1;
  if (valid) { sp = d.sp[e]; op = d.op[e]; }
  const bool spfar = sp >= 0 && sp < ring_lo, opfar = op >= 0 && op < ring_lo;
  const bool far = __any(spfar || opfar);
  if (!valid) return;
  const int sa = (sp < 0 || spfar) ? ring : (int)(sp & (ring - 1));
  const int sb = (op < 0 || opfar) ? ring : (int)(op & (ring - 1));
  const int fl = (int)d.chunk_maxd[e >> 6] | (far ? SW_FAR : 0) | (spfar ? SW_SPFAR : 0) |
                 (opfar ? SW_OPFAR : 0);
  d.desc[e] = make_int4(sa | (sb << 16), d.creator[e] | (fl << 16), d.index[e], 0);
}

// ---------------------------------------------------------------------------
// The coordinate sweep.  blockIdx.x < n: LA column c = blockIdx.x;
// blockIdx.x == n: Lamport timestamps.  One 32-bit value per lane and
// event, so a sub-step is two ds_read_b32 gathers, one v_max3 and one
// ds_write_b32 -- the shortest LDS round trip the dependency chain allows.
//
// Two specialised waves per workgroup, handing off through LDS counters:
//   wave 0 (compute)  walks the chunks touching only LDS: one descriptor
//                     read per chunk, maxd+1 sub-steps, then ONE coalesced
//                     store of the lane's final value (256 B per chunk) --
//                     its own ring slots need no hand-off, and its vmcnt
//                     holds only those stores (waited on only before the
//                     rare load of a parent older than the ring);
//   wave 1 (prefetch) streams descriptors into the LDS descriptor ring with
//                     LDS-DMA (global_load_lds_dwordx4, 1 KiB = one chunk per
//                     instruction), GROUP chunks per group, two groups in
//                     flight, retired with counted vmcnt waits.
// A wave's LDS operations execute in order, and the CU's LDS serves waves
// through one pipeline, so data written before a counter is visible to a
// reader that has seen the counter.
constexpr int GROUP = 8;    // chunks per prefetch group (= vmcnt step)
static_assert(GROUP == 8, "the prefetch wave's counted wait is vmcnt(8)");
typedef __attribute__((address_space(3))) void lds_void;

// progress counters live in LDS; an explicit address space keeps them ds_*
// ops (through a generic pointer they become flat ops that wait on vmcnt)
typedef __attribute__((address_space(3))) volatile int lds_flag;
__device__ __forceinline__ int lds_poll(lds_flag *p) { return *p; }
#define COMPILER_FENCE() __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront")

enum { F_LANDED = 0, F_CONSUMED = 1 };

template <bool LT, int DRING>
__device__ __forceinline__ void sweep_body(const Dev &d, int32_t *vring, int4 (*dring)[64], int *flags) {
  static_assert((DRING & (DRING - 1)) == 0, "descriptor ring: power of two");
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int col = blockIdx.x;
  const int ring = 1 << d.ring_log2;
  const int32_t N = (int32_t)d.N;  // < 2^31 events (int32 ids)
  const int32_t nchunks = (N + 63) / 64;
  lds_flag *vf = (lds_flag *)flags;
  int32_t *out = LT ? d.lt : d.la_ev + (int64_t)col * (d.la_rows + 64);
  if (threadIdx.x < 2) flags[threadIdx.x] = 0;
  if (threadIdx.x == 0) vring[ring] = -1;  // sentinel slot for absent / far parents
  __syncthreads();
  const bool dgw = d.diag != nullptr && col == 0 && lane == 0;

  if (wave == 1) {
    // ---------------- prefetch wave ----------------
    unsigned long long t_busy = 0, n_idle = 0;
    int32_t issued = 0, freed = DRING;  // chunks issued; slots usable below `freed`
    int inflight = 0;                   // groups in flight
    for (;;) {
      bool can = issued < nchunks;
      if (can && issued + GROUP > freed) {
        freed = lds_poll(&vf[F_CONSUMED]) + DRING;
        can = issued + GROUP <= freed;
      }
      if (can) {
        const unsigned long long ta = dgw ? stamp() : 0;
#pragma unroll
        for (int q = 0; q < GROUP; ++q) {
          const int32_t mq = issued + q;
          const int32_t e = min(mq * 64 + lane, N - 1);
          int4 *dst = mq < nchunks ? &dring[mq & (DRING - 1)][0] : &dring[DRING][0];
          __builtin_amdgcn_global_load_lds((const void *)(d.desc + e), (lds_void *)dst, 16, 0, 0);
        }
        issued += GROUP;
        ++inflight;
        if (dgw) t_busy += stamp() - ta;
      }
      if (inflight == 2 || (!can && inflight > 0)) {
        if (inflight == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        --inflight;
        if (lane == 0) vf[F_LANDED] = min(issued - inflight * GROUP, nchunks);
      } else if (!can) {
        if (issued >= nchunks) break;
        if (dgw) ++n_idle;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (dgw) { d.diag[DG_SW_MEM_PREF] = t_busy; d.diag[DG_SW_MEM_IDLE] = n_idle; }
    return;
  }

  // ---------------- compute wave ----------------
  // Per chunk: the NEXT chunk's descriptor is read before this chunk's
  // sub-steps (LDS returns in order, so it costs no extra wait).  Sub-step s
  // rewrites every lane's slot with max(ring[sa], ring[sb], own) --
  // unconditionally: a lane's value is final from sub-step depth(lane) on
  // (its in-chunk parents are final one sub-step earlier), and nobody needs
  // it before then.  The slots written alias only events older than the
  // ring, which no lane reads (far parents map to the sentinel and are
  // folded into `own` from HBM instead).
  const bool dg = d.diag != nullptr && col == 0;
  unsigned long long t_start = dg ? stamp() : 0, w_desc = 0, nsub = 0, nfar = 0;
  int32_t have = 0;
  while ((have = lds_poll(&vf[F_LANDED])) <= 0) __builtin_amdgcn_s_sleep(1);
  int4 dc = dring[0][lane];
  for (int32_t m = 0; m < nchunks; ++m) {
    const bool nxt = m + 1 < nchunks && (have > m + 1 || (have = lds_poll(&vf[F_LANDED])) > m + 1);
    int4 dn = dc;
    if (nxt) dn = dring[(m + 1) & (DRING - 1)][lane];
    const int sa = dc.x & 0xffff, sb = dc.x >> 16;
    const int fl = __builtin_amdgcn_readfirstlane(dc.y >> 16);
    const int maxd = fl & 0xff;
    const int32_t e = m * 64 + lane;
    const int sw = e & (ring - 1);
    int32_t own = -1;
    if (!LT) own = (dc.y & 0xffff) == col ? dc.z : -1;
    if (__builtin_expect(fl & SW_FAR, 0)) {
      // parents older than the ring: this wave stored them; drain its stores
      // and read them back past L1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int32_t ec = min(e, N - 1);
      if ((dc.y >> 16) & SW_SPFAR) own = max(own, __builtin_nontemporal_load(out + d.sp[ec]));
      if ((dc.y >> 16) & SW_OPFAR) own = max(own, __builtin_nontemporal_load(out + d.op[ec]));
    }
    int32_t v = 0;
    for (int s = 0; s <= maxd; ++s) {
      v = max(max(vring[sa], vring[sb]), own);
      if (LT) v += 1;
      vring[sw] = v;
      COMPILER_FENCE();  // one wave: LDS ops execute in issue order
    }
    if (LT) out[e] = v;
    else out[e] = v;  // lanes past N land in the 64 scratch rows
    if (dg) { nsub += maxd + 1; nfar += (fl & SW_FAR) ? 1 : 0; }
    if (lane == 0) vf[F_CONSUMED] = m + 1;
    if (!nxt && m + 1 < nchunks) {
      const unsigned long long t1 = dg ? stamp() : 0;
      while ((have = lds_poll(&vf[F_LANDED])) <= m + 1) __builtin_amdgcn_s_sleep(1);
      if (dg) w_desc += stamp() - t1;
      dn = dring[(m + 1) & (DRING - 1)][lane];
    }
    dc = dn;
  }
  if (dg && lane == 0) {
    d.diag[DG_SW_TOTAL] = stamp() - t_start;
    d.diag[DG_SW_WAIT_DESC] = w_desc;
    d.diag[DG_SW_WAIT_RING] = 0;
    d.diag[DG_SW_SUBSTEPS] = nsub;
    d.diag[DG_SW_FAR] = nfar;
    d.diag[DG_SW_CHUNKS] = nchunks;
  }
}

void launch_chunk_depth(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  const int64_t nchunks = (d.N + 63) / 64;
  k_chunk_depth<<<(unsigned)((nchunks + 3) / 4), 256, 0, s>>>(d);
  k_pack_desc<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d);
}

// one launch: the column workgroups and the Lamport workgroup run
// concurrently; the branch is uniform per workgroup.  DRING descriptor
// chunks (the LDS budget: 32 with a 16K-event value ring, one workgroup per
// CU; 16 with a 4K ring, four per CU for wide configurations)
template <int DRING>
__global__ __launch_bounds__(128) void k_la_sweep(Dev d) {
  extern __shared__ __attribute__((aligned(16))) int4 swm[];
  __shared__ int flags[2];
  int4(*dring)[64] = reinterpret_cast<int4(*)[64]>(swm);  // [DRING + 1][64]; [DRING] = sink
  int32_t *vring = reinterpret_cast<int32_t *>(swm + (size_t)(DRING + 1) * 64);  // [ring + 1]
  if ((int)blockIdx.x == d.n) sweep_body<true, DRING>(d, vring, dring, flags);
  else sweep_body<false, DRING>(d, vring, dring, flags);
}

// the sweep's column slabs -> chain-major LA rows (the layout the round
// loop's per-chain windows read).  One thread per event: every load
// instruction reads 256 B contiguous from one column; each lane writes its
// own row 16 B at a time in column order.  HBM-bound: 2 x 4*npad B/event.
__global__ __launch_bounds__(256) void k_permute(Dev d) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int n = d.n, npad = d.npad;
  const int64_t stride = d.la_rows + 64;
  const int32_t *src = d.la_ev + e;
  const int64_t row = d.epos[e];
  int4 *dst = reinterpret_cast<int4 *>(d.la + row * npad);
  // n <= 128: the column-major copy too (k_round2 and fame read it; its
  // own allocation there -- wider groups' la_col may be the slabs themselves)
  int32_t *col = d.fd_cols ? d.la_col + row : nullptr;
  int c = 0;
  for (; c + 32 <= n; c += 32) {
    int32_t v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) v[u] = __builtin_nontemporal_load(src + (int64_t)(c + u) * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) dst[c / 4 + u] = make_int4(v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]);
    if (col)
#pragma unroll
      for (int u = 0; u < 32; ++u) col[(int64_t)(c + u) * stride] = v[u];
  }
  for (; c < npad; c += 4) {
    int32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = c + u < n ? src[(int64_t)(c + u) * stride] : -1;
    dst[c / 4] = make_int4(v[0], v[1], v[2], v[3]);
    if (col)
      for (int u = 0; u < 4; ++u)
        if (c + u < n) col[(int64_t)(c + u) * stride] = v[u];
  }
}

void launch_la_sweep(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  const bool big = d.ring_log2 >= 14;
  const int dn = big ? 32 : 16;
  const size_t lds = (size_t)(dn + 1) * 64 * 16 + ((size_t)(1 << d.ring_log2) + 4) * 4;
  if (big) k_la_sweep<32><<<d.n + 1, 128, lds, s>>>(d);
  else k_la_sweep<16><<<d.n + 1, 128, lds, s>>>(d);
}

void configure_coord_kernels() {
  (void)hipFuncSetAttribute((const void *)k_la_sweep<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
  (void)hipFuncSetAttribute((const void *)k_la_sweep<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
}

void launch_permute(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  k_permute<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d);
}

void launch_coordinates(const Dev &d, hipStream_t s) {
  launch_chunk_depth(d, s);
  launch_la_sweep(d, s);
  launch_permute(d, s);
}

}  // namespace bh
