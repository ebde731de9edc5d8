// kernels_coords.hip -- event coordinates (lastAncestors) and Lamport timestamps.
//
// Reference: initEventCoordinates (hashgraph.go:439-507) computes, per event,
// LA[e][j] = max(LA[sp][j], LA[op][j]) with LA[e][creator] = index, and
// _lamportTimestamp (hashgraph.go:325-379) LT[e] = max(LT[sp], LT[op]) + 1.
// firstDescendants (updateAncestorFirstDescendant, :510-544) is only ever
// read for witnesses (stronglySee's y argument); those rows are produced by
// the round loop (kernels_rounds.hip) from LA, so no per-event FD walk runs.
//
// MI355X mapping: each column j depends only on column j of the parents, so
// the columns are split over workgroups that never communicate: one
// workgroup per group of four columns (int4 lanes) walks ALL events in
// topological order, 64 events (one per lane) per chunk, resolving
// intra-chunk dependencies in `depth` sub-steps.  Parents within the last
// VRING events are read from an LDS ring (the common case: the self-parent is
// the creator's previous event, the other-parent a recent head); older ones
// from HBM.  One extra workgroup computes LT the same way.  The kernel is
// bound by the DAG's critical path (levels x LDS latency), not by HBM
// bandwidth -- see DESIGN.md.
#include "engine.h"

namespace bh {

// ---------------------------------------------------------------------------
// prep: chain-major id table (ParticipantEventsCache, caches.go:34-129) and
// round-loop state.
__global__ void k_chain_scatter(Dev d) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int32_t p = d.chain_start[d.creator[e]] + d.index[e];
  d.chain_ids[p] = (int32_t)e;
  d.epos[e] = p;
}

// row of each event's other-parent (so the sweep's prefetch has no dependent load)
__global__ void k_opos(Dev d) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int32_t o = d.op[e];
  d.opos[e] = o >= 0 ? d.epos[o] : 0;
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
  if (d.N > 0) {
    k_chain_scatter<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d);
    k_opos<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d);
  }
  k_state_init<<<1, 256, 0, s>>>(d);
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
//   .z = index, .w = LA row (chain-major position, for the write-back)
// Ring slots are (event & (VRING-1)); an absent parent, or one that is too
// old to still be in the ring ("far"), maps to the sentinel slot VRING (-1s).
// flags = maxd (max intra-chunk depth, chunk-uniform) | chunk-has-far << 8 |
//         sp-far << 9 | op-far << 10.
constexpr int VRING = 4096;  // value ring (events); parents this recent stay on chip
constexpr int SW_FAR = 0x100, SW_SPFAR = 0x200, SW_OPFAR = 0x400;

__global__ __launch_bounds__(256) void k_pack_desc(Dev d) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t base = e & ~(int64_t)63;  // a wave is a chunk
  const bool valid = e < d.N;
  const int64_t ring_lo = base + 64 - VRING;
  int32_t sp = -1, op = -1;
  if (valid) { sp = d.sp[e]; op = d.op[e]; }
  const bool spfar = sp >= 0 && sp < ring_lo, opfar = op >= 0 && op < ring_lo;
  const bool far = __any(spfar || opfar);
  if (!valid) return;
  const int sa = (sp < 0 || spfar) ? VRING : (int)(sp & (VRING - 1));
  const int sb = (op < 0 || opfar) ? VRING : (int)(op & (VRING - 1));
  const int fl = (int)d.chunk_maxd[e >> 6] | (far ? SW_FAR : 0) | (spfar ? SW_SPFAR : 0) |
                 (opfar ? SW_OPFAR : 0);
  d.desc[e] = make_int4(sa | (sb << 16), d.creator[e] | (fl << 16), d.index[e], d.epos[e]);
}

// ---------------------------------------------------------------------------
// The coordinate sweep.  blockIdx.x < ngroups: columns [4g, 4g+4);
// blockIdx.x == ngroups: Lamport timestamps.
//
// Three specialised waves per workgroup, handing off through LDS counters:
//   wave 0 (compute)  walks the chunks touching only LDS: one descriptor
//                     read per chunk, then maxd+1 sub-steps of
//                     2 x ds_read_b128, 4 x v_max3, ds_write_b128;
//   wave 1 (prefetch) streams descriptors into the LDS descriptor ring with
//                     LDS-DMA (global_load_lds_dwordx4, 1 KiB = one chunk per
//                     instruction), GROUP chunks per group, two groups in
//                     flight, retired with counted vmcnt waits;
//   wave 2 (store)    reads finished chunks out of the value ring and writes
//                     them to HBM; it frees ring slots as soon as it has READ
//                     them and publishes HBM visibility separately (needed
//                     only by the rare chunk whose parent left the ring).
// vmcnt is one in-order counter per wave covering loads AND stores, so
// keeping prefetch and stores in different waves means neither ever waits
// for the other's traffic.  A wave's LDS operations execute in order, and
// the CU's LDS serves waves through one pipeline, so data written before a
// counter is visible to a reader that has seen the counter.
constexpr int DRING = 64;   // descriptor ring (chunks); slot DRING is a sink
constexpr int GROUP = 8;    // chunks per prefetch group (= vmcnt step)
static_assert(GROUP == 8, "the prefetch wave's counted wait is vmcnt(8)");
typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int4 nt_load4(const int32_t *p) {  // L1-bypassing 16-B load
  const v4i v = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(p));
  return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ int4 max4(int4 a, int4 b) {
  return make_int4(max(a.x, b.x), max(a.y, b.y), max(a.z, b.z), max(a.w, b.w));
}

// progress counters live in LDS; an explicit address space keeps them ds_*
// ops (through a generic pointer they become flat ops that wait on vmcnt)
typedef __attribute__((address_space(3))) volatile int lds_flag;
__device__ __forceinline__ int lds_poll(lds_flag *p) { return *p; }
#define COMPILER_FENCE() __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront")

enum { F_LANDED = 0, F_COMPUTED = 1, F_READ = 2, F_STORED = 3 };

template <bool LT>
__device__ __forceinline__ void sweep_body(const Dev &d, int4 *vring, int4 (*dring)[64], int *flags) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int ngroups = d.npad / 4;
  const int g = LT ? ngroups : blockIdx.x;
  const int col0 = 4 * g;
  const int64_t N = d.N;
  const int64_t nchunks = (N + 63) / 64;
  lds_flag *vf = (lds_flag *)flags;
  int4 *const slab = reinterpret_cast<int4 *>(d.la_ev) + (int64_t)g * (d.la_rows + 64);
  const int4 none = make_int4(-1, -1, -1, -1);
  if (threadIdx.x < 4) flags[threadIdx.x] = 0;
  if (threadIdx.x == 0) vring[VRING] = none;  // sentinel slot for absent / far parents
  __syncthreads();
  const bool dgw = d.diag != nullptr && g == 0 && lane == 0;

  if (wave == 1) {
    // ---------------- prefetch wave ----------------
    unsigned long long t_busy = 0, n_idle = 0;
    int64_t issued = 0, freed = DRING;  // chunks issued; slots usable below `freed`
    int inflight = 0;                   // groups in flight
    for (;;) {
      bool can = issued < nchunks;
      if (can && issued + GROUP > freed) {
        freed = (int64_t)lds_poll(&vf[F_READ]) + DRING;
        can = issued + GROUP <= freed;
      }
      if (can) {
        const unsigned long long ta = dgw ? stamp() : 0;
#pragma unroll
        for (int q = 0; q < GROUP; ++q) {
          const int64_t mq = issued + q;
          const int64_t e = min(mq * 64 + lane, N - 1);
          int4 *dst = mq < nchunks ? &dring[mq % DRING][0] : &dring[DRING][0];
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
        if (lane == 0) vf[F_LANDED] = (int)min(issued - (int64_t)inflight * GROUP, nchunks);
      } else if (!can) {
        if (issued >= nchunks) break;
        if (dgw) ++n_idle;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (dgw) { d.diag[DG_SW_MEM_PREF] = t_busy; d.diag[DG_SW_MEM_IDLE] = n_idle; }
    return;
  }

  if (wave == 2) {
    // ---------------- store wave ----------------
    unsigned long long t_busy = 0;
    int64_t mstore = 0, computed = 0, published = 0;
    while (mstore < nchunks) {
      if (computed <= mstore) {
        computed = lds_poll(&vf[F_COMPUTED]);
        if (computed <= mstore) {
          if (published < mstore) {  // idle: make the stores visible
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) vf[F_STORED] = (int)mstore;
            published = mstore;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
      }
      const unsigned long long ta = dgw ? stamp() : 0;
      const int64_t hi = min(computed, mstore + 8);
      // all 8 reads first, then 8 unconditional stores: chunks past `hi`
      // re-store chunk hi-1 to its own place (idempotent), and lanes past N
      // land in the 64 scratch rows behind the slab, so no store needs a
      // branch (a branch per store would serialise each LDS read with it)
      int4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t m = min(mstore + q, hi - 1);
        v[q] = vring[(m * 64 + lane) & (VRING - 1)];
      }
      // one contiguous 1 KiB store per chunk (event-major slab of this
      // column group); k_permute builds the chain-major rows afterwards
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t e = min(mstore + q, hi - 1) * 64 + lane;
        if (LT) d.lt[e] = v[q].x;
        else slab[e] = v[q];
      }
      mstore = hi;
      COMPILER_FENCE();
      if (lane == 0) vf[F_READ] = (int)mstore;  // slots read: reusable
      if (mstore - published >= 64) {           // bound what a far reader may wait for
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) vf[F_STORED] = (int)mstore;
        published = mstore;
      }
      if (dgw) t_busy += stamp() - ta;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) vf[F_STORED] = (int)nchunks;
    if (dgw) d.diag[DG_SW_MEM_STORE] = t_busy;
    return;
  }

  // ---------------- compute wave ----------------
  // Per chunk: the NEXT chunk's descriptor is read before this chunk's
  // sub-steps (LDS returns in order, so it costs no extra wait); the other
  // waves' counters are re-polled only when the cached values run out.
  // Sub-step s rewrites every lane's slot with max(ring[sa], ring[sb], own)
  // -- unconditionally: a lane's value is final from sub-step depth(lane) on
  // (its in-chunk parents are final one sub-step earlier), and nobody needs
  // it before then.  The slots written alias only events older than the
  // ring, which no lane reads (far parents map to the sentinel and are
  // folded into `own` from HBM instead).
  int *vring_i = reinterpret_cast<int *>(vring);
  const bool dg = d.diag != nullptr && g == 0;
  unsigned long long t_start = dg ? stamp() : 0, w_desc = 0, w_ring = 0, nsub = 0, nfar = 0;
  int64_t have = 0, readc = 0;
  while ((have = lds_poll(&vf[F_LANDED])) <= 0) __builtin_amdgcn_s_sleep(1);
  int4 dc = dring[0][lane];
  for (int64_t m = 0; m < nchunks; ++m) {
    const unsigned long long t0 = dg ? stamp() : 0;
    const bool nxt = m + 1 < nchunks && (have > m + 1 || (have = lds_poll(&vf[F_LANDED])) > m + 1);
    int4 dn = dc;
    if (nxt) dn = dring[(m + 1) % DRING][lane];
    // chunk m overwrites value-ring slots of chunk m - VRING/64
    const int64_t need = m - VRING / 64 + 1;
    if (readc < need)
      while ((readc = lds_poll(&vf[F_READ])) < need) __builtin_amdgcn_s_sleep(1);
    if (dg) w_ring += stamp() - t0;
    const int sa = dc.x & 0xffff, sb = dc.x >> 16;
    const int own = (dc.y & 0xffff) - col0;
    const int fl = __builtin_amdgcn_readfirstlane(dc.y >> 16);
    const int maxd = fl & 0xff;
    const int sw = (int)((m * 64 + lane) & (VRING - 1));
    if (__builtin_expect(fl & SW_FAR, 0)) {
      // parents older than the ring: wait until their chunks are in HBM
      while (lds_poll(&vf[F_STORED]) < need) __builtin_amdgcn_s_sleep(1);
    }
    if (LT) {
      int farv = -1;
      if (__builtin_expect(fl & SW_FAR, 0)) {  // L1-bypassing loads of rows written by this CU
        const int64_t e = min(m * 64 + lane, N - 1);
        if ((dc.y >> 16) & SW_SPFAR) farv = max(farv, __builtin_nontemporal_load(d.lt + d.sp[e]));
        if ((dc.y >> 16) & SW_OPFAR) farv = max(farv, __builtin_nontemporal_load(d.lt + d.op[e]));
      }
      for (int s = 0; s <= maxd; ++s) {
        vring_i[4 * sw] = max(max(vring_i[4 * sa], vring_i[4 * sb]), farv) + 1;
        COMPILER_FENCE();  // one wave: LDS ops execute in issue order
      }
    } else {
      const int idx = dc.z;
      int4 ownv = make_int4(own == 0 ? idx : -1, own == 1 ? idx : -1, own == 2 ? idx : -1,
                            own == 3 ? idx : -1);
      if (__builtin_expect(fl & SW_FAR, 0)) {
        const int64_t e = min(m * 64 + lane, N - 1);
        if ((dc.y >> 16) & SW_SPFAR) ownv = max4(ownv, nt_load4(reinterpret_cast<const int32_t *>(slab + d.sp[e])));
        if ((dc.y >> 16) & SW_OPFAR) ownv = max4(ownv, nt_load4(reinterpret_cast<const int32_t *>(slab + d.op[e])));
      }
      for (int s = 0; s <= maxd; ++s) {
        vring[sw] = max4(max4(vring[sa], vring[sb]), ownv);
        COMPILER_FENCE();
      }
    }
    if (dg) { nsub += maxd + 1; nfar += (fl & SW_FAR) ? 1 : 0; }
    if (lane == 0) vf[F_COMPUTED] = (int)(m + 1);
    if (!nxt && m + 1 < nchunks) {
      const unsigned long long t1 = dg ? stamp() : 0;
      while ((have = lds_poll(&vf[F_LANDED])) <= m + 1) __builtin_amdgcn_s_sleep(1);
      if (dg) w_desc += stamp() - t1;
      dn = dring[(m + 1) % DRING][lane];
    }
    dc = dn;
  }
  if (dg && lane == 0) {
    d.diag[DG_SW_TOTAL] = stamp() - t_start;
    d.diag[DG_SW_WAIT_DESC] = w_desc;
    d.diag[DG_SW_WAIT_RING] = w_ring;
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

// one launch: column-group workgroups and the Lamport workgroup run
// concurrently; the branch is uniform per workgroup
__global__ __launch_bounds__(192) void k_la_sweep(Dev d) {
  __shared__ int4 vring[VRING + 1];       // 64 KiB results (LT mode: .x); [VRING] = -1s
  __shared__ int4 dring[DRING + 1][64];   // 65 KiB descriptors; [DRING] = prefetch sink
  __shared__ int flags[4];
  if ((int)blockIdx.x == d.npad / 4) sweep_body<true>(d, vring, dring, flags);
  else sweep_body<false>(d, vring, dring, flags);
}

// the sweep's column-group slabs -> chain-major LA rows (the layout the
// round loop's per-chain windows read).  One wave per 64 events: every
// load instruction reads 1 KiB contiguous from a slab; each lane writes its
// own row's 16-B pieces in column order, so a row's lines are complete by
// the time they leave L2.  HBM-bound: 2 x 4*npad bytes per event.
__global__ __launch_bounds__(256) void k_permute(Dev d) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  const int ng = d.npad / 4;
  const int64_t stride = d.la_rows + 64;
  const int4 *src = reinterpret_cast<const int4 *>(d.la_ev) + e;
  int4 *dst = reinterpret_cast<int4 *>(d.la + (int64_t)d.epos[e] * d.npad);
  int g = 0;
  for (; g + 8 <= ng; g += 8) {
    int4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = nt_load4(reinterpret_cast<const int32_t *>(src + (int64_t)(g + u) * stride));
#pragma unroll
    for (int u = 0; u < 8; ++u) dst[g + u] = v[u];
  }
  for (; g < ng; ++g) dst[g] = src[(int64_t)g * stride];
}

void launch_la_sweep(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  k_la_sweep<<<d.npad / 4 + 1, 192, 0, s>>>(d);
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
