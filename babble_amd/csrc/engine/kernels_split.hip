// kernels_split.hip -- the coordinate split across shards.
//
// Shards 1 .. G-1 ("coordinate shards") run the chain dataflow (k_flow32 at
// n <= 128, k_floww2 up to 512) for a range of LA columns each; shard 0 runs the round loop, fame and order,
// and computes no coordinates.  Per pipeline segment a coordinate shard packs
// the segment's rows of its columns of la_col and ships them to shard 0,
// which unpacks them into its own la_col before the segment's round loop.
//
// What a segment holds: chain c's rows lo_c .. hi_c - 1 (chain positions;
// the prefix of insertion order the segment adds).  Packed index x in
// [0, S) (S = the segment's events) runs over the chains in order: chain c
// owns [P[c], P[c+1]), P[c] = sum of earlier chains' row counts.  A column's
// values along one chain are non-decreasing (LA along a creator's chain), so
// every 64 rows of a chain's run (chunk q, Q[c] <= q < Q[c+1]) are stored as
// 16-bit offsets from the chunk's first value (the chunk header, + 1 so that
// -1 -- "no ancestor on that chain" -- stays >= 0).  A chunk whose values
// span more than 65535 (a chain that ignored another one for 65k of its
// events: never on gossip DAGs, possible on adversarial ones) is sent raw in
// one of OV_CAP overflow slots (header -1 - slot); more overflows than slots
// set the block's error word and the call falls back to the unsplit path.
//
// Block layout (one per coordinate shard and segment; byte offsets from
// split_layout): hdr int32[ncol][NQ] | pay uint16[ncol][S] | ovf count,
// error | ovf int32[OV_CAP][64] | lt int32[S] (the LT owner only).
//
// HBM cost per event: 4 B per column read + 2 B written on the coordinate
// shard; 2 B read + 4 B written on shard 0.  Link bytes per event: 2 B per
// column (+ 4 B of LT, + ~1/16 of headers).
#include "engine.h"

#include <algorithm>

namespace bh {

// the chain of packed index x: the last c with P[c] <= x (P in LDS, n + 1 entries)
__device__ __forceinline__ int split_chain(const int32_t *P, int n, int32_t x) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (P[mid] <= x) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// the segment's P and Q into LDS
__device__ __forceinline__ void split_tables(const int32_t *pq, int n, int32_t *P, int32_t *Q) {
  for (int i = threadIdx.x; i <= n; i += blockDim.x) {
    P[i] = pq[i];
    Q[i] = pq[n + 1 + i];
  }
  __syncthreads();
}

// chunk headers: one thread per (column, chunk); grid (chunks / 256, ncol)
__global__ __launch_bounds__(256) void k_split_hdr(Dev v, const int32_t *pq, SplitBlock b) {
  __shared__ int32_t P[FW_MAXN + 1], Q[FW_MAXN + 1];
  const int n = v.n;
  split_tables(pq, n, P, Q);
  const int32_t q = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  const int col = (int)blockIdx.y;
  if (q >= b.NQ) return;
  const int c = split_chain(Q, n, q);  // Q[c] <= q < Q[c + 1]
  const int32_t r0 = v.seg_lo[c] + 64 * (q - Q[c]), r1 = min(r0 + 64, v.chain_len[c]);
  const int32_t *src = v.la_col + (int64_t)(b.c0 + col) * la_col_stride(v) + v.chain_start[c];
  const int32_t a = src[r0], z = src[r1 - 1];
  int32_t h;
  if ((int64_t)z - a <= b.range) {
    h = a + 1;
  } else {
    const int32_t slot = atomicAdd(b.ovf_count, 1);
    if (slot < SPLIT_OV_CAP) {
      h = -1 - slot;
    } else {
      h = -1 - SPLIT_OV_CAP;  // (unpacked as garbage: the error word fails the call)
      atomicExch(b.err, 1);
    }
  }
  b.hdr[(int64_t)col * b.NQ + q] = h;
}

// payload: one thread per (column, packed index); grid (S / 256, ncol); the
// LT owner's block also carries the segment's LT rows (blockIdx.y == ncol)
__global__ __launch_bounds__(256) void k_split_pack(Dev v, const int32_t *pq, SplitBlock b) {
  __shared__ int32_t P[FW_MAXN + 1], Q[FW_MAXN + 1];
  const int n = v.n;
  split_tables(pq, n, P, Q);
  const int32_t x = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  const int col = (int)blockIdx.y;
  if (x >= b.S) return;
  const int c = split_chain(P, n, x);
  const int32_t j = v.seg_lo[c] + (x - P[c]);
  const int64_t row = (int64_t)v.chain_start[c] + j;
  if (col >= b.ncol) {  // LT rows
    if (b.lt_on) b.lt[x] = v.lt_row[row];
    return;
  }
  const int32_t val = v.la_col[(int64_t)(b.c0 + col) * la_col_stride(v) + row];
  const int32_t q = Q[c] + (j - v.seg_lo[c]) / 64;
  const int32_t h = b.hdr[(int64_t)col * b.NQ + q];
  if (h >= 0) {
    b.pay[(int64_t)col * b.S + x] = (uint16_t)(val - (h - 1));
  } else if (-1 - h < SPLIT_OV_CAP) {
    b.ovf[(int64_t)(-1 - h) * 64 + (j - v.seg_lo[c]) % 64] = val;
  }
}

// shard 0: a block into la_col columns [c0, c0 + ncol) (and lt_row);
// grid (S / 256, ncol [+ 1])
__global__ __launch_bounds__(256) void k_split_unpack(Dev v, const int32_t *pq, SplitBlock b) {
  __shared__ int32_t P[FW_MAXN + 1], Q[FW_MAXN + 1];
  const int n = v.n;
  split_tables(pq, n, P, Q);
  const int32_t x = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  const int col = (int)blockIdx.y;
  if (x == 0 && col == 0) {
    // the sender's flags: overflow slots exhausted (the call is recomputed
    // unsplit, ST_FLOWOVF = 2 as a dataflow watchdog), and the sender's own
    // ST_FLOWOVF -- 1: LT beyond the dataflow's range (the LT fallback), 2:
    // its dataflow's watchdog (unfinished columns: recomputed unsplit)
    if (b.err[0]) atomicMax(&v.state[ST_FLOWOVF], 2);
    if (b.err[1]) atomicMax(&v.state[ST_FLOWOVF], min(b.err[1], 2));
  }
  if (x >= b.S) return;
  const int c = split_chain(P, n, x);
  const int32_t j = v.seg_lo[c] + (x - P[c]);
  const int64_t row = (int64_t)v.chain_start[c] + j;
  if (col >= b.ncol) {
    if (b.lt_on) v.lt_row[row] = b.lt[x];
    return;
  }
  const int32_t q = Q[c] + (j - v.seg_lo[c]) / 64;
  const int32_t h = b.hdr[(int64_t)col * b.NQ + q];
  int32_t val;
  if (h >= 0) val = (h - 1) + (int32_t)b.pay[(int64_t)col * b.S + x];
  else val = b.ovf[(int64_t)min(-1 - h, SPLIT_OV_CAP - 1) * 64 + (j - v.seg_lo[c]) % 64];
  v.la_col[(int64_t)(b.c0 + col) * la_col_stride(v) + row] = val;
}

size_t split_layout(int ncol, int64_t S, int64_t NQ, bool lt, SplitBlock *b, uint8_t *base) {
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = 0;
  const size_t o_hdr = o; o += up((size_t)ncol * NQ * 4);
  const size_t o_pay = o; o += up((size_t)ncol * S * 2);
  const size_t o_cnt = o; o += 256;
  const size_t o_ovf = o; o += up((size_t)SPLIT_OV_CAP * 64 * 4);
  const size_t o_lt = o; o += lt ? up((size_t)S * 4) : 0;
  if (b) {
    b->S = S;
    b->NQ = NQ;
    b->ncol = ncol;
    b->lt_on = lt;
    b->hdr = reinterpret_cast<int32_t *>(base + o_hdr);
    b->pay = reinterpret_cast<uint16_t *>(base + o_pay);
    b->ovf_count = reinterpret_cast<int32_t *>(base + o_cnt);
    b->err = reinterpret_cast<int32_t *>(base + o_cnt + 4);
    b->ovf = reinterpret_cast<int32_t *>(base + o_ovf);
    b->lt = lt ? reinterpret_cast<int32_t *>(base + o_lt) : nullptr;
  }
  return o;
}

void launch_split_pack(const Dev &v, const int32_t *pq, const SplitBlock &b, hipStream_t s) {
  (void)hipMemsetAsync(b.ovf_count, 0, 12, s);  // count, err[0], err[1] (the flags travel even in an empty block)
  if (b.S > 0 && b.ncol > 0) k_split_hdr<<<dim3((unsigned)((b.NQ + 255) / 256), (unsigned)b.ncol), 256, 0, s>>>(v, pq, b);
  const unsigned ny = (unsigned)(b.ncol + (b.lt_on ? 1 : 0));
  if (b.S > 0 && ny) k_split_pack<<<dim3((unsigned)((b.S + 255) / 256), ny), 256, 0, s>>>(v, pq, b);
  // every sender's dataflow flags travel (a watchdog on any shard leaves its
  // columns unfinished)
  (void)hipMemcpyAsync(b.err + 1, v.state + ST_FLOWOVF, 4, hipMemcpyDeviceToDevice, s);
}

void launch_split_unpack(const Dev &v, const int32_t *pq, const SplitBlock &b, hipStream_t s) {
  const unsigned ny = (unsigned)std::max(1, b.ncol + (b.lt_on ? 1 : 0));  // (one workgroup reads the flags)
  k_split_unpack<<<dim3((unsigned)std::max<int64_t>(1, (b.S + 255) / 256), ny), 256, 0, s>>>(v, pq, b);
}

}  // namespace bh
