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
//   k_fd_walk       workgroup = (chain i, segment of rows), thread = column c;
//                   writes FDT[i][row(c,j)] = k -- each thread appends to its
//                   own run of chain c, so lines are completed in L2;
//   k_fd_transpose  64-row tiles of FDT through LDS into chain-major FD rows
//                   (the layout the round loop gathers candidates from),
//                   substituting MaxInt32 where j exceeds what the chain's
//                   last event sees (lastLA), which the walk never writes.
// Algorithmic bytes: walk 4n (read LA row) + 4n (write FDT) per event,
// transpose 4n + 4n per event: 16n B/event, HBM-bound.
#include "engine.h"

#include <algorithm>

namespace bh {

constexpr int FD_SEG = 256;  // chain rows per walk workgroup

// lastLA[i][c] = LA[(i, len_i - 1)][c] (-1 for an empty chain)
__global__ void k_last_la(Dev d) {
  const int i = blockIdx.x;
  const int32_t len = d.chain_len[i], cs = d.chain_start[i];
  for (int c = threadIdx.x; c < d.npad; c += blockDim.x)
    d.last_la[(int64_t)i * d.npad + c] = len > 0 ? d.la[(int64_t)(cs + len - 1) * d.npad + c] : -1;
}

__global__ __launch_bounds__(256) void k_fd_walk(Dev d) {
  const int i = blockIdx.y;
  const int32_t len = d.chain_len[i];
  const int32_t k0 = blockIdx.x * FD_SEG;
  if (k0 >= len) return;
  const int32_t k1 = min(len, k0 + FD_SEG);
  const int32_t cs = d.chain_start[i];
  const int64_t stride = d.la_rows + 64;  // FDT row stride
  int32_t *fdt = d.fdt + (int64_t)i * stride;
  for (int c = threadIdx.x; c < d.n; c += blockDim.x) {
    const int32_t *col = d.la + (int64_t)cs * d.npad + c;
    int32_t prev = k0 > 0 ? col[(int64_t)(k0 - 1) * d.npad] : -1;
    int32_t *out = fdt + d.chain_start[c];
    int32_t k = k0;
    // 8 rows of loads in flight per thread
    for (; k + 8 <= k1; k += 8) {
      int32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(col + (int64_t)(k + u) * d.npad);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        for (; prev < v[u]; ) out[++prev] = k + u;
    }
    for (; k < k1; ++k) {
      const int32_t v = col[(int64_t)k * d.npad];
      for (; prev < v; ) out[++prev] = k;
    }
  }
}

// FD[row][i] for a TR_ROWS-row tile; rows are chain-major (row of (c, j) =
// chain_start[c] + j); creator/index of a row come from chain_ids.
template <int TR_ROWS>
__global__ __launch_bounds__(256) void k_fd_transpose(Dev d) {
  extern __shared__ int32_t tile[];  // [npad][TR_ROWS + 1]
  constexpr int IPP = 256 / TR_ROWS;  // columns i per pass
  __shared__ int32_t rc[TR_ROWS], rj[TR_ROWS];
  const int t = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * TR_ROWS;
  const int64_t N = d.N;
  const int n = d.n, npad = d.npad;
  const int64_t stride = d.la_rows + 64;
  const int ro = t % TR_ROWS;
  const int64_t row = min(row0 + ro, N - 1);
  if (t < TR_ROWS) {
    const int32_t e = d.chain_ids[row];
    rc[t] = d.creator[e];
    rj[t] = d.index[e];
  }
  // phase 1: FDT[i][row0 .. row0+TR_ROWS) -> tile[i][*]; IPP columns per
  // pass, 4 passes of loads in flight
  for (int i = t / TR_ROWS; i < n; i += 4 * IPP) {
    int32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ii = min(i + IPP * u, n - 1);
      v[u] = __builtin_nontemporal_load(d.fdt + (int64_t)ii * stride + row);
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
    if (row0 + r >= N) continue;
    const int32_t c = rc[r], j = rj[r];
    int32_t o[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ii = i4 + u;
      int32_t x = FD_NONE;
      if (ii < n && j <= d.last_la[(int64_t)ii * npad + c]) x = tile[ii * (TR_ROWS + 1) + r];
      o[u] = x;
    }
    *reinterpret_cast<int4 *>(d.fd + (row0 + r) * npad + i4) = make_int4(o[0], o[1], o[2], o[3]);
  }
}

void launch_first_descendants(const Dev &d, hipStream_t s) {
  if (d.N == 0) return;
  k_last_la<<<d.n, 256, 0, s>>>(d);
  const int wt = std::min(256, (d.n + 63) / 64 * 64);
  dim3 g((unsigned)((d.max_chain_len + FD_SEG - 1) / FD_SEG), (unsigned)d.n);
  k_fd_walk<<<g, wt, 0, s>>>(d);
  if (d.npad <= 512)
    k_fd_transpose<64><<<(unsigned)((d.N + 63) / 64), 256, (size_t)d.npad * 65 * 4, s>>>(d);
  else
    k_fd_transpose<32><<<(unsigned)((d.N + 31) / 32), 256, (size_t)d.npad * 33 * 4, s>>>(d);
}

void configure_fd_kernels() {
  (void)hipFuncSetAttribute((const void *)k_fd_transpose<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
  (void)hipFuncSetAttribute((const void *)k_fd_transpose<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
}

}  // namespace bh
