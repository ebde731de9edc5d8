// kernels_query.hip -- the Hashgraph's private predicates over event pairs
// (hashgraph.go:80-191, 382-395), evaluated from the device coordinates:
//   ancestor(x, y)      LA[x][creator(y)] >= index(y), or x == y   (_ancestor :93-118)
//   selfAncestor(x, y)  same creator and index(x) >= index(y)       (_selfAncestor :134-149)
//   see(x, y)           = ancestor (no forks get inserted)          (see :152-157)
//   stronglySee(x, y)   #{i : LA[x][i] >= FD[y][i]} >= SM           (_stronglySee :172-191)
//   roundDiff(x, y)     round(x) - round(y)                         (roundDiff :382-395)
// One thread per pair; the reference's LRU caches have nothing to add.
#include "engine.h"

namespace bh {

// lastAncestors / firstDescendants entry of event e, column i, in whichever
// layout the coordinate path left them: LA rows are chain-major (`la`), FD
// rows are the FDT tiles (n <= 128) or chain-major `fd`
__device__ __forceinline__ int32_t la_at(const Dev &d, int32_t e, int i) {
  return d.la[(int64_t)d.epos[e] * d.npad + i];
}
__device__ __forceinline__ int32_t fd_at(const Dev &d, int32_t e, int i) {
  const int64_t row = d.epos[e];
  return d.fd_cols || !d.fd_rows ? d.fdt[fdt_pos(row, i, d.npad)] : d.fd[row * d.npad + i];
}

__global__ __launch_bounds__(256) void k_query(Dev d, int32_t kind, int64_t count, const int64_t *xs,
                                               const int64_t *ys, int32_t *out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= count) return;
  const int32_t x = (int32_t)xs[k], y = (int32_t)ys[k];
  int32_t r = 0;
  switch (kind) {
    case 0:  // ancestor
    case 2:  // see
      r = x == y || la_at(d, x, d.creator[y]) >= d.index[y];
      break;
    case 1:  // selfAncestor
      r = x == y || (d.creator[x] == d.creator[y] && d.index[x] >= d.index[y]);
      break;
    case 3: {  // stronglySee
      int c = 0;
      for (int i = 0; i < d.n; ++i) c += la_at(d, x, i) >= fd_at(d, y, i);
      r = c >= d.sm;
      break;
    }
    default: {  // roundDiff
      const int32_t rx = d.round[x], ry = d.round[y];
      r = rx == UNSET || ry == UNSET ? UNSET : rx - ry;
    }
  }
  out[k] = r;
}

void launch_query(const Dev &d, int32_t kind, int64_t count, const int64_t *x, const int64_t *y, int32_t *out,
                  hipStream_t s) {
  if (count > 0) k_query<<<(unsigned)((count + 255) / 256), 256, 0, s>>>(d, kind, count, x, y, out);
}

}  // namespace bh
