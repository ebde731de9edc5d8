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
// the columns are split over workgroups that never communicate: one wave per
// group of four columns (int4 lanes) walks ALL events in topological order,
// 64 events (one per lane) per chunk, resolving intra-chunk dependencies in
// `depth` sub-steps.  Parents within the last RING events are read from an
// LDS ring (the common case: the self-parent is the creator's previous
// event and the other-parent a recent head); older parents from HBM.  One
// extra wave computes LT the same way.  The kernel is bound by the DAG's
// critical path (levels), not by HBM bandwidth -- see DESIGN.md.
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

__global__ void k_state_init(Dev d) {
  int t = threadIdx.x;
  if (t < ST_COUNT) d.state[t] = 0;
  for (int c = t; c < d.n; c += blockDim.x) d.B[c] = 0;  // B[0][c]: every event has round >= 0
  if (t == 0) d.wofs[0] = 0;
}

void launch_prep(const Dev &d, hipStream_t s) {
  if (d.N > 0) k_chain_scatter<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d);
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

// ---------------------------------------------------------------------------
// The coordinate sweep.  blockIdx.x < ngroups: columns [4g, 4g+4);
// blockIdx.x == ngroups: Lamport timestamps.
__device__ __forceinline__ int4 max4(int4 a, int4 b) {
  return make_int4(max(a.x, b.x), max(a.y, b.y), max(a.z, b.z), max(a.w, b.w));
}

__global__ __launch_bounds__(64) void k_la_sweep(Dev d) {
  __shared__ int4 ring[RING];  // 128 KiB
  const int lane = threadIdx.x;
  const int ngroups = d.npad / 4;
  const int g = blockIdx.x;
  const bool lt_mode = g == ngroups;
  const int col0 = 4 * g;
  const int64_t N = d.N;
  const int64_t nchunks = (N + 63) / 64;
  int *ring_i = reinterpret_cast<int *>(ring);
  const int4 none = make_int4(-1, -1, -1, -1);

  // prefetched descriptors of the next chunk
  int64_t e = lane;
  int32_t nsp = -1, nop = -1, ncr = 0, nidx = 0, ndep = 0, nmaxd = 0, npos = 0, nopos = 0;
  if (e < N) {
    nsp = d.sp[e]; nop = d.op[e]; ncr = d.creator[e]; nidx = d.index[e]; ndep = d.depth[e];
    npos = d.epos[e]; nopos = nop >= 0 ? d.epos[nop] : 0;
  }
  if (nchunks > 0) nmaxd = d.chunk_maxd[0];

  for (int64_t m = 0; m < nchunks; ++m) {
    const int64_t base = m * 64;
    e = base + lane;
    const bool valid = e < N;
    const int32_t sp = nsp, op = nop, cr = ncr, idx = nidx, dep = ndep, maxd = nmaxd;
    const int32_t pos = npos, opos = nopos;  // HBM rows (chain-major); sp row = pos - 1
    // prefetch chunk m+1
    const int64_t en = e + 64;
    if (en < N) {
      nsp = d.sp[en]; nop = d.op[en]; ncr = d.creator[en]; nidx = d.index[en]; ndep = d.depth[en];
      npos = d.epos[en]; nopos = nop >= 0 ? d.epos[nop] : 0;
    }
    if (m + 1 < nchunks) nmaxd = d.chunk_maxd[m + 1];
    // parents at or after this bound are still in the ring (the ring slot of
    // a later event of this chunk can alias only older parents)
    const int64_t ring_lo = base + 64 - RING;

    for (int s = 0; s <= maxd; ++s) {
      const bool mine = valid && dep == s;
      const bool far = mine && ((sp >= 0 && sp < ring_lo) || (op >= 0 && op < ring_lo));
      if (__builtin_expect(__any(far), 0)) {
        // rare: a parent left the LDS ring; read its row from HBM (this wave
        // wrote it >= RING events ago).  Kept on its own wave-uniform path so
        // the common path below carries no vmcnt wait (which would also
        // drain this wave's pending LA stores).
        if (mine) {
          if (lt_mode) {
            int a = -1, b = -1;
            if (sp >= 0) a = sp >= ring_lo ? ring_i[sp & (RING - 1)] : d.lt[sp];
            if (op >= 0) b = op >= ring_lo ? ring_i[op & (RING - 1)] : d.lt[op];
            const int v = max(a, b) + 1;
            ring_i[e & (RING - 1)] = v;
            d.lt[e] = v;
          } else {
            int4 a = none, b = none;
            if (sp >= 0)
              a = sp >= ring_lo ? ring[sp & (RING - 1)]
                                : *reinterpret_cast<const int4 *>(d.la + (int64_t)(pos - 1) * d.npad + col0);
            if (op >= 0)
              b = op >= ring_lo ? ring[op & (RING - 1)]
                                : *reinterpret_cast<const int4 *>(d.la + (int64_t)opos * d.npad + col0);
            int4 v = max4(a, b);
            const int own = cr - col0;
            if (own == 0) v.x = idx;
            else if (own == 1) v.y = idx;
            else if (own == 2) v.z = idx;
            else if (own == 3) v.w = idx;
            ring[e & (RING - 1)] = v;
            *reinterpret_cast<int4 *>(d.la + (int64_t)pos * d.npad + col0) = v;
          }
        }
      } else if (mine) {
        if (lt_mode) {
          const int a = sp >= 0 ? ring_i[sp & (RING - 1)] : -1;
          const int b = op >= 0 ? ring_i[op & (RING - 1)] : -1;
          const int v = max(a, b) + 1;
          ring_i[e & (RING - 1)] = v;
          d.lt[e] = v;
        } else {
          const int4 a = sp >= 0 ? ring[sp & (RING - 1)] : none;
          const int4 b = op >= 0 ? ring[op & (RING - 1)] : none;
          int4 v = max4(a, b);
          const int own = cr - col0;
          if (own == 0) v.x = idx;
          else if (own == 1) v.y = idx;
          else if (own == 2) v.z = idx;
          else if (own == 3) v.w = idx;
          ring[e & (RING - 1)] = v;
          *reinterpret_cast<int4 *>(d.la + (int64_t)pos * d.npad + col0) = v;
        }
      }
      // The block is ONE wave: its LDS accesses execute in issue order, so
      // the next sub-step's ds_reads see this sub-step's ds_writes without a
      // hardware barrier.  Only compiler ordering is needed -- a
      // __syncthreads() here would also drain the global LA stores
      // (s_waitcnt vmcnt(0)) on every sub-step.
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
  }
}

void launch_chunk_depth(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  const int64_t nchunks = (d.N + 63) / 64;
  k_chunk_depth<<<(unsigned)((nchunks + 3) / 4), 256, 0, s>>>(d);
}

void launch_la_sweep(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  k_la_sweep<<<d.npad / 4 + 1, 64, 0, s>>>(d);
}

void launch_coordinates(const Dev &d, hipStream_t s) {
  launch_chunk_depth(d, s);
  launch_la_sweep(d, s);
}

}  // namespace bh
