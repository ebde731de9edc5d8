// kernels_fd.hip -- firstDescendants of every event.
//
// Reference: updateAncestorFirstDescendant (hashgraph.go:510-544) walks, for
// every new event, the self-parent chains of its last ancestors and sets
// FD[y][creator] the first time a descendant on that chain appears.  The same
// vector in closed form: FD[y][i] = min{k : LA[(i,k)][creator(y)] >= index(y)}
// (event (i,k) sees y), MaxInt32 when no event of chain i sees y.
//
// LA[(i,k)][c] is non-decreasing in k, so for a fixed (chain i, column c)
// one pass over chain i yields FD[(c,j)][i] for every j: the rows k at which
// the column steps from v' to v own the j in (v', v].  That pass is HBM
// streaming work with no serial dependency between segments of a chain:
//   k_fd_walk       workgroup = (chain i, 64-row segment) staged in LDS; the
//                   entries of column c form one contiguous run of
//                   FDT[i][row(c,j)], written 256 B per wave instruction;
//   k_fd_transpose  64-row tiles of FDT through LDS into chain-major FD rows
//                   (the layout the round loop gathers candidates from),
//                   substituting MaxInt32 where j exceeds what the chain's
//                   last event sees (lastLA), which the walk never writes.
// Algorithmic bytes: walk 4n (read LA row) + 4n (write FDT) per event,
// transpose 4n + 4n per event: 16n B/event, HBM-bound.
#include "engine.h"

#include <algorithm>
#include <cstdlib>

namespace bh {


// lastLA[i][c] = LA[(i, len_i - 1)][c] (-1 for an empty chain); the row
// [n] below the table holds min_i lastLA[i][c]: rows with j at most that
// need no substitution at all
__global__ void k_last_la(Dev d) {
  const int i = blockIdx.x;
  const int32_t len = d.chain_len[i], cs = d.chain_start[i];
  for (int c = threadIdx.x; c < d.npad; c += blockDim.x) {
    const int32_t v = len > 0 ? d.la[(int64_t)(cs + len - 1) * d.npad + c] : -1;
    d.last_la[(int64_t)i * d.npad + c] = v;
    atomicMin(&d.last_la[(int64_t)d.n * d.npad + c], v);
  }
}

__global__ void k_last_la_init(Dev d) {
  for (int c = threadIdx.x; c < d.npad; c += blockDim.x) d.last_la[(int64_t)d.n * d.npad + c] = INT32_MAX;
}

// One workgroup per (chain i, 64-row segment).  The segment's LA rows (and
// the row before it) are staged in LDS transposed, one column per LDS row
// (stride WSEG + 1: the 64 lanes of a wave searching one column hit
// distinct banks); column c then owns the FD entries j in
// (LA[k0-1][c], LA[k0+63][c]], a contiguous run of FDT[i][row(c, j)].  A
// wave writes that run 64 entries per instruction (256 B coalesced), each
// lane finding its k by binary search down column c.
constexpr int WSEG = 64;
constexpr int WST = WSEG + 1;  // LDS stride of a staged column (odd)

__global__ __launch_bounds__(256) void k_fd_walk(Dev d) {
  extern __shared__ int32_t seg[];  // [npad][WST]: seg[c][0] = LA[k0 - 1][c], seg[c][1 + k] = LA[k0 + k][c]
  const int i = blockIdx.y;
  const int32_t len = d.chain_len[i];
  const int32_t k0 = blockIdx.x * WSEG;
  if (k0 >= len) return;
  const int rows = min(WSEG, len - k0);
  const int32_t cs = d.chain_start[i];
  const int npad = d.npad, q4 = npad / 4, t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  {
    const int4 *src = reinterpret_cast<const int4 *>(d.la + (int64_t)(cs + k0) * npad);
    const int tot = rows * q4;
    for (int b = 0; b < tot; b += 4 * 256) {
      int4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        typedef int v4i __attribute__((ext_vector_type(4)));
        const v4i x = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(src + min(b + u * 256 + t, tot - 1)));
        v[u] = make_int4(x.x, x.y, x.z, x.w);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = b + u * 256 + t;
        if (e < tot) {
          const int r = e / q4, c = (e - r * q4) * 4;
          seg[(c + 0) * WST + 1 + r] = v[u].x;
          seg[(c + 1) * WST + 1 + r] = v[u].y;
          seg[(c + 2) * WST + 1 + r] = v[u].z;
          seg[(c + 3) * WST + 1 + r] = v[u].w;
        }
      }
    }
    for (int c = t; c < npad; c += 256) seg[c * WST] = k0 > 0 ? d.la[(int64_t)(cs + k0 - 1) * npad + c] : -1;
  }
  __syncthreads();
  const bool last = k0 + rows == len;
  for (int c = wave; c < d.n; c += 4) {
    const int32_t *col = seg + c * WST;
    const int32_t lo = col[0], hi = col[rows];  // run (lo, hi]
    const int64_t rc0 = d.chain_start[c];
    if (last && d.fd_cols)  // rows (c, j) no event of chain i sees
      for (int32_t j = hi + 1 + lane; j < d.chain_len[c]; j += 64) d.fdt[fdt_pos(rc0 + j, i, npad)] = FD_NONE;
    for (int32_t j0 = lo + 1; j0 <= hi; j0 += 64) {
      const int32_t j = j0 + lane;
      if (j <= hi) {
        // first segment row k (1-based) with LA[k][c] >= j
        int a = 1, z = rows;
        while (a < z) {
          const int m = (a + z) >> 1;
          if (col[m] >= j) z = m;
          else a = m + 1;
        }
        d.fdt[fdt_pos(rc0 + j, i, npad)] = k0 + a - 1;
      }
    }
  }
}

// FD[row][i] for a TR_ROWS-row tile; rows are chain-major (row of (c, j) =
// chain_start[c] + j) over the whole layout (d.rows; gap rows of a chain's
// region have chain_ids -1 and are skipped); creator/index of a row come
// from chain_ids.
template <int TR_ROWS>
__global__ __launch_bounds__(256) void k_fd_transpose(Dev d) {
  extern __shared__ int32_t tile[];  // [npad][TR_ROWS + 1]
  constexpr int IPP = 256 / TR_ROWS;  // columns i per pass
  __shared__ int32_t rc[TR_ROWS], rj[TR_ROWS], rfast[TR_ROWS];
  const int t = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * TR_ROWS;
  const int64_t N = d.rows > 0 ? d.rows : d.N;
  const int n = d.n, npad = d.npad;
  const int ro = t % TR_ROWS;
  const int64_t row = min(row0 + ro, N - 1);
  if (t < TR_ROWS) {
    const int32_t e = d.chain_ids[row];
    const bool gap = e < 0 || row0 + t >= N;
    const int32_t c = gap ? -1 : d.creator[e], j = gap ? 0 : d.index[e];
    rc[t] = c;
    rj[t] = j;
    rfast[t] = !gap && j <= d.last_la[(int64_t)n * npad + c];  // every chain sees (c, j)
  }
  // phase 1: FDT[i][row0 .. row0+TR_ROWS) -> tile[i][*]; IPP columns per
  // pass, 4 passes of loads in flight
  for (int i = t / TR_ROWS; i < n; i += 4 * IPP) {
    int32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ii = min(i + IPP * u, n - 1);
      v[u] = __builtin_nontemporal_load(d.fdt + fdt_pos(row, ii, npad));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + IPP * u < n) tile[(i + IPP * u) * (TR_ROWS + 1) + ro] = v[u];
  }
  __syncthreads();
  // phase 2: rows out, 16 B per thread, columns i..i+3
  const int q4 = npad / 4;
  for (int p = t; p < TR_ROWS * q4; p += blockDim.x) {
    const int r = p / q4, i4 = (p - r * q4) * 4;
    if (row0 + r >= N || rc[r] < 0) continue;
    const int32_t c = rc[r], j = rj[r];
    const bool fast = rfast[r];
    int32_t o[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ii = i4 + u;
      int32_t x = FD_NONE;
      if (ii < n && (fast || j <= d.last_la[(int64_t)ii * npad + c])) x = tile[ii * (TR_ROWS + 1) + r];
      o[u] = x;
    }
    if (d.fd_rows) *reinterpret_cast<int4 *>(d.fd + (row0 + r) * npad + i4) = make_int4(o[0], o[1], o[2], o[3]);
  }
}

void launch_first_descendants(const Dev &d, hipStream_t s, bool walked) {
  if (d.N == 0) return;
  if (!walked) {
    dim3 g((unsigned)((d.max_chain_len + WSEG - 1) / WSEG), (unsigned)d.n);
    k_fd_walk<<<g, 256, (size_t)WST * d.npad * 4, s>>>(d);
  }
  if (d.fd_cols) return;  // FDT complete; no chain-major rows
  k_last_la_init<<<1, 256, 0, s>>>(d);
  k_last_la<<<d.n, 256, 0, s>>>(d);
  // the 16-bit wide loop gathers its candidates' rows from the complete FDT
  // (cand16); chain-major rows are written only for the 32-bit loop
  if (!d.fd_rows) return;
  // tile rows: LDS is npad x (TR + 1) words, so wide groups take short
  // tiles and several workgroups per compute unit (the kernel is bound by
  // its loads' latency: n = 512 with 64-row tiles left one 4-wave workgroup
  // per CU, 1.2 TB/s)
  const int64_t rows = d.rows > 0 ? d.rows : d.N;  // the layout's rows, gaps included
  if (d.npad <= 128)
    k_fd_transpose<64><<<(unsigned)((rows + 63) / 64), 256, (size_t)d.npad * 65 * 4, s>>>(d);
  else
    k_fd_transpose<16><<<(unsigned)((rows + 15) / 16), 256, (size_t)d.npad * 17 * 4, s>>>(d);
}

void configure_fd_kernels() {
  (void)hipFuncSetAttribute((const void *)k_fd_walk, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
  (void)hipFuncSetAttribute((const void *)k_fd_transpose<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
}

}  // namespace bh
