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

// per-event sweep descriptor, 32 B: {sp, op, creator, index}, {depth, row,
// other-parent row, max depth of the event's chunk}
__global__ void k_pack_desc(Dev d) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.N) return;
  d.desc[2 * e] = make_int4(d.sp[e], d.op[e], d.creator[e], d.index[e]);
  d.desc[2 * e + 1] = make_int4(d.depth[e], d.epos[e], d.opos[e], d.chunk_maxd[e >> 6]);
}

// ---------------------------------------------------------------------------
// The coordinate sweep.  blockIdx.x < ngroups: columns [4g, 4g+4);
// blockIdx.x == ngroups: Lamport timestamps.
//
// Wave specialisation inside each two-wave workgroup:
//   wave 0 (compute) walks the chunks doing LDS-only work: descriptors from
//          the LDS descriptor ring, parents from the LDS value ring;
//   wave 1 (memory)  prefetches descriptors of upcoming chunks into the
//          descriptor ring and writes finished chunks from the value ring to
//          HBM.
// vmcnt is one in-order counter per wave covering loads AND stores, so a
// single wave that both stores rows and prefetches descriptors drains its
// stores at every descriptor wait (two HBM round trips per chunk, measured
// 1.9 us/chunk).  Split this way, the compute wave issues no stores and
// waits only on LDS.  The waves hand off through LDS counters; a wave's LDS
// operations execute in order, so data written before a counter is visible
// to a reader that has seen the counter.
constexpr int VRING = 4096;  // value ring (events)
constexpr int DRING = 32;    // descriptor ring (chunks)
constexpr int PBATCH = 16;   // chunks prefetched per memory-wave iteration
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int4 nt_load4(const int32_t *p) {  // L1-bypassing 16-B load
  const v4i v = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(p));
  return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ int4 max4(int4 a, int4 b) {
  return make_int4(max(a.x, b.x), max(a.y, b.y), max(a.z, b.z), max(a.w, b.w));
}

__device__ __forceinline__ int4 set_own(int4 v, int own, int idx) {
  if (own == 0) v.x = idx;
  else if (own == 1) v.y = idx;
  else if (own == 2) v.z = idx;
  else if (own == 3) v.w = idx;
  return v;
}

__device__ __forceinline__ int lds_poll(volatile int *p) { return *p; }

template <bool LT>
__device__ __forceinline__ void sweep_body(const Dev &d, int4 *vring, int4 (*dring)[2][64], int *flags) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int ngroups = d.npad / 4;
  const int g = LT ? ngroups : blockIdx.x;
  const bool lt_mode = LT;
  const int col0 = 4 * g;
  const int64_t N = d.N;
  const int64_t nchunks = (N + 63) / 64;
  volatile int *vf = flags;
  const int4 none = make_int4(-1, -1, -1, -1);
  if (threadIdx.x < 4) flags[threadIdx.x] = 0;
  if (threadIdx.x == 0) vring[VRING] = none;  // sentinel slot for absent parents
  __syncthreads();

  if (wave == 1) {
    // ---------------- memory wave ----------------
    int64_t mload = 0, mstore = 0;
    const bool dgm = d.diag != nullptr && g == 0 && lane == 0;
    unsigned long long m_pref = 0, m_store = 0, m_idle = 0;
    while (mstore < nchunks) {
      bool idle = true;
      const unsigned long long ta = dgm ? stamp() : 0;
      // prefetch descriptors into free slots (a slot is free once its chunk
      // has been written back: the store takes the row index from it).  All
      // PBATCH chunks' loads are issued unconditionally (clamped) before the
      // first use, so the wave pays one HBM latency per batch.
      const int64_t room = min((int64_t)PBATCH, min(nchunks - mload, mstore + DRING - mload));
      if (room > 0) {
        int4 pa[PBATCH], pb[PBATCH];
#pragma unroll
        for (int q = 0; q < PBATCH; ++q) {
          const int64_t mq = min(mload + q, nchunks - 1);
          int64_t e = mq * 64 + lane;
          e = e < N ? e : N - 1;
          pa[q] = d.desc[2 * e];
          pb[q] = d.desc[2 * e + 1];
        }
#pragma unroll
        for (int q = 0; q < PBATCH; ++q) {
          if (q < room) {
            int4 b = pb[q];
            if ((mload + q) * 64 + lane >= N) b.x = 255;  // tail lanes never match a sub-step
            dring[(mload + q) % DRING][0][lane] = pa[q];
            dring[(mload + q) % DRING][1][lane] = b;
          }
        }
        mload += room;
        if (lane == 0) vf[0] = (int)mload;
        idle = false;
      }
      const unsigned long long tb = dgm ? stamp() : 0;
      if (dgm) m_pref += tb - ta;
      // write back computed chunks; publish once the stores have drained
      const int64_t computed = lds_poll(&vf[1]);
      if (mstore < computed) {
        for (; mstore < computed; ++mstore) {
          const int64_t e = mstore * 64 + lane;
          if (e < N) {
            const int4 v = vring[e & (VRING - 1)];
            if (lt_mode) d.lt[e] = v.x;
            else {
              const int pos = dring[mstore % DRING][1][lane].y;
              *reinterpret_cast<int4 *>(d.la + (int64_t)pos * d.npad + col0) = v;
            }
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) vf[2] = (int)mstore;
        idle = false;
      }
      if (dgm) m_store += stamp() - tb;
      if (idle) {
        if (dgm) ++m_idle;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (dgm) {
      d.diag[DG_SW_MEM_PREF] = m_pref;
      d.diag[DG_SW_MEM_STORE] = m_store;
      d.diag[DG_SW_MEM_IDLE] = m_idle;
    }
    return;
  }

  // ---------------- compute wave ----------------
  int *vring_i = reinterpret_cast<int *>(vring);
  const bool dg = d.diag != nullptr && g == 0;
  unsigned long long t_start = dg ? stamp() : 0, w_desc = 0, w_ring = 0, nsub = 0, nfar = 0;
  int4 res4 = none;
  for (int64_t m = 0; m < nchunks; ++m) {
    unsigned long long t0 = dg ? stamp() : 0;
    while (lds_poll(&vf[0]) <= m) __builtin_amdgcn_s_sleep(1);
    unsigned long long t1 = dg ? stamp() : 0;
    // chunk m writes value-ring slots last used by chunk m - VRING/64
    while ((int64_t)lds_poll(&vf[2]) < m - VRING / 64 + 1) __builtin_amdgcn_s_sleep(1);
    if (dg) { const unsigned long long t2 = stamp(); w_desc += t1 - t0; w_ring += t2 - t1; }
    const int4 da = dring[m % DRING][0][lane];
    const int4 db = dring[m % DRING][1][lane];
    const int32_t sp = da.x, op = da.y, cr = da.z, idx = da.w;
    const int32_t dep = db.x, pos = db.y, opos = db.z, maxd = db.w;
    const int64_t base = m * 64;
    const int64_t e = base + lane;
    // parents at or after ring_lo are in the value ring; older ones were
    // written back (stored >= m - VRING/64 + 1 covers their chunks)
    const int64_t ring_lo = base + 64 - VRING;
    const bool far = (sp >= 0 && sp < ring_lo) || (op >= 0 && op < ring_lo);
    const int own = cr - col0;
    if (__builtin_expect(!__any(far), 1)) {
      // Common case, branch-free sub-steps: every lane reads its parents'
      // slots (absent parents -> the sentinel slot of -1s) and rewrites its
      // own slot each sub-step, the new value once its depth comes up.  Safe:
      // a lane of depth s only reads parents of depth < s (already final),
      // and the slots this chunk writes alias only events older than
      // ring_lo, which no lane of this chunk reads (no far parent).
      const int sa = sp >= 0 ? (int)(sp & (VRING - 1)) : VRING;
      const int sb = op >= 0 ? (int)(op & (VRING - 1)) : VRING;
      const int sw = (int)(e & (VRING - 1));
      const bool ox = own == 0, oy = own == 1, oz = own == 2, ow = own == 3;
      if (LT) {
        int res1 = -1;
        for (int s = 0; s <= maxd; ++s) {
          const int v = max(vring_i[4 * sa], vring_i[4 * sb]) + 1;
          res1 = dep == s ? v : res1;
          vring_i[4 * sw] = res1;
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
        res4.x = res1;
      } else {
        for (int s = 0; s <= maxd; ++s) {
          int4 v = max4(vring[sa], vring[sb]);
          v.x = ox ? idx : v.x;
          v.y = oy ? idx : v.y;
          v.z = oz ? idx : v.z;
          v.w = ow ? idx : v.w;
          const bool mine = dep == s;
          res4.x = mine ? v.x : res4.x;
          res4.y = mine ? v.y : res4.y;
          res4.z = mine ? v.z : res4.z;
          res4.w = mine ? v.w : res4.w;
          vring[sw] = res4;
          // one wave: LDS ops execute in issue order; compiler ordering only
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
      }
      if (dg) nsub += maxd + 1;
    } else {
      // rare: some parent left the value ring; read it from HBM with
      // L1-bypassing loads (the line may hold bytes written after this CU
      // cached it), predicated per lane
      if (dg) { nsub += maxd + 1; ++nfar; }
      for (int s = 0; s <= maxd; ++s) {
        if (dep == s) {
          if (LT) {
            int a = -1, b = -1;
            if (sp >= 0) a = sp >= ring_lo ? vring_i[4 * (sp & (VRING - 1))] : __builtin_nontemporal_load(d.lt + sp);
            if (op >= 0) b = op >= ring_lo ? vring_i[4 * (op & (VRING - 1))] : __builtin_nontemporal_load(d.lt + op);
            vring_i[4 * (e & (VRING - 1))] = max(a, b) + 1;
          } else {
            int4 a = none, b = none;
            if (sp >= 0)
              a = sp >= ring_lo ? vring[sp & (VRING - 1)] : nt_load4(d.la + (int64_t)(pos - 1) * d.npad + col0);
            if (op >= 0)
              b = op >= ring_lo ? vring[op & (VRING - 1)] : nt_load4(d.la + (int64_t)opos * d.npad + col0);
            vring[e & (VRING - 1)] = set_own(max4(a, b), own, idx);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      }
    }
    if (lane == 0) vf[1] = (int)(m + 1);
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
__global__ __launch_bounds__(128) void k_la_sweep(Dev d) {
  __shared__ int4 vring[VRING + 1];         // 64 KiB results (LT mode: .x); [VRING] = -1s
  __shared__ int4 dring[DRING][2][64];      // 64 KiB {sp,op,cr,idx},{dep,pos,opos,maxd}
  __shared__ int flags[4];                  // [0] desc ready, [1] computed, [2] stored
  if ((int)blockIdx.x == d.npad / 4) sweep_body<true>(d, vring, dring, flags);
  else sweep_body<false>(d, vring, dring, flags);
}

void launch_la_sweep(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  k_la_sweep<<<d.npad / 4 + 1, 128, 0, s>>>(d);
}

void launch_coordinates(const Dev &d, hipStream_t s) {
  launch_chunk_depth(d, s);
  launch_la_sweep(d, s);
}

}  // namespace bh
