// kernels_reset.hip -- a hashgraph Reset from a Frame (FastSync; SURVEY
// 8(f) row 4): Hashgraph.Reset (hashgraph.go:1324-1369) installs the frame's
// Roots, whose SelfParent / NextRound / Others stand for the events the
// hashgraph no longer holds (root.go; the six cases of docs/fastsync.rst:
// 140-175).
//
// k_reset_coords: the events whose other-parent only Root.Others knows (the
// frame's, inserted first) have no chain dataflow parent to wait for, and
// their Lamport timestamps take the Others entry's (_lamportTimestamp,
// :358-375).  They are a prefix of the insertion order; one workgroup
// computes their lastAncestors column by column (a thread per column
// follows the events in order: LA[e][j] depends on column j of its parents
// only, initEventCoordinates :439-507, parents the Store lacks contribute
// nothing) and their Lamport timestamps (one thread); the dataflow kernels
// then resume every chain after them, as a segment does.
//
// k_fiat: rounds below r0.  A root-attached event takes Root.NextRound by
// fiat (:229-236), and an other-parent in Root.Others counts as NextRound
// (:246-256), so the closed form's premise -- a candidate of round > r
// strongly sees SM witnesses of round r -- holds only above F, the highest
// NextRound / SelfParent.Round of any root.  Below
// r0 = F + 1 every event's round is computed as _round does, in insertion
// order (a topological order), against the witnesses found so far; a chain
// is done at its first event of round >= r0 (rounds are monotone along a
// chain), which is B[r0][c] for the loop.  Events of done chains are skipped
// 1024 at a time.
#include "engine.h"

namespace bh {

__global__ __launch_bounds__(1024) void k_reset_coords(Dev d) {
  const int t = threadIdx.x, n = d.n;
  const int64_t stride = d.la_rows + 64;
  if (t < n) {  // column t of lastAncestors
    int32_t *col = d.la_col + (int64_t)t * stride;
    for (int64_t e = 0; e < d.N; ++e) {
      const int32_t sp = d.sp[e], op = d.op[e];
      int32_t v = -1;
      if (sp >= 0) v = col[d.epos[sp]];
      if (op >= 0) v = max(v, col[d.epos[op]]);
      if (d.creator[e] == t) v = d.index[e];
      col[d.epos[e]] = v;
    }
  } else if (t == 1023) {  // Lamport timestamps by chain-major row
    for (int64_t e = 0; e < d.N; ++e) {
      const int32_t sp = d.sp[e], op = d.op[e], c = d.creator[e];
      int32_t lt = sp >= 0 ? d.lt_row[d.epos[sp]] : d.lt_seed[c];
      if (op >= 0) lt = max(lt, d.lt_row[d.epos[op]]);
      else if (d.ext_lt[e] != UNSET) lt = max(lt, d.ext_lt[e]);
      d.lt_row[d.epos[e]] = lt + 1;
    }
  }
}

void launch_reset_coords(const Dev &d, hipStream_t s) {
  if (d.N > 0) k_reset_coords<<<1, 1024, 0, s>>>(d);
}

constexpr int FI_MAXN = 512;

__global__ __launch_bounds__(1024) void k_fiat(Dev d) {
  __shared__ int32_t done[FI_MAXN], bfirst[FI_MAXN];
  __shared__ int32_t list[1024], wcnt[16];
  __shared__ int32_t sh_cnt, sh_ndone, sh_pr, sh_ss, sh_stop;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, n = d.n, npad = d.npad;
  const int32_t r0 = d.r0, rlo = d.rlo;
  for (int c = t; c < n; c += 1024) {
    done[c] = 0;
    bfirst[c] = d.chain_len[c];
  }
  if (t == 0) { sh_ndone = 0; sh_stop = 0; }
  __syncthreads();
  // round of an event processed before x: its stored round, or "at least
  // r0" if its chain was done at or before it
  auto round_of = [&](int32_t y) -> int32_t {
    const int32_t cy = d.creator[y];
    return (done[cy] && d.index[y] >= bfirst[cy]) ? r0 : d.round[y];
  };
  for (int64_t base = 0; base < d.N; base += 1024) {
    // the chunk's events on chains not done yet, in order
    const int64_t e = base + t;
    const bool need = e < d.N && !done[d.creator[e]];
    const unsigned long long m = __ballot(need);
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int32_t pos = __popcll(m & ((1ull << lane) - 1ull));
    for (int w = 0; w < wave; ++w) pos += wcnt[w];
    if (need) list[pos] = (int32_t)e;
    if (t == 0) {
      int32_t tot = 0;
      for (int w = 0; w < 16; ++w) tot += wcnt[w];
      sh_cnt = tot;
    }
    __syncthreads();
    const int32_t cnt = sh_cnt;
    __syncthreads();
    for (int32_t j = 0; j < cnt; ++j) {
      const int32_t x = list[j], c = d.creator[x];
      if (done[c]) continue;  // uniform: done[] only changes behind barriers
      if (t == 0) {
        const int32_t sp = d.sp[x], op = d.op[x];
        const bool oth = d.rflag[x] & 1;               // Root.Others[x] names x's other-parent
        const bool op_empty = op < 0 && !(d.rflag[x] & 2);  // no other-parent at all
        int32_t pr;
        if (sp < 0 && (oth || op_empty)) {
          pr = -1 - d.root_next[c];  // attached to the Root: NextRound by fiat (encoded < 0)
        } else {
          pr = sp < 0 ? d.root_sp_round[c] : round_of(sp);
          if (oth) pr = max(pr, d.root_next[c]);
          else if (op >= 0) pr = max(pr, round_of(op));
        }
        sh_pr = pr;
        sh_ss = 0;
      }
      __syncthreads();
      const int32_t pr = sh_pr;
      if (pr >= 0 && pr < r0) {
        // #witnesses of round pr that x strongly sees (_stronglySee :172-191)
        const int64_t rx = d.epos[x];
        for (int q = wave; q < n; q += 16) {
          const int32_t w = pr >= rlo ? d.fw[(int64_t)(pr - rlo) * n + q] : -1;
          if (w < 0) continue;
          const int64_t rw = d.epos[w];
          int cntc = 0;
          for (int i = lane; i < n; i += 64) cntc += d.la[rx * npad + i] >= d.fdt[fdt_pos(rw, i, npad)];
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) cntc += __shfl_xor(cntc, off);
          if (lane == 0 && cntc >= d.sm) atomicAdd(&sh_ss, 1);
        }
      }
      __syncthreads();
      if (t == 0) {
        int32_t r;
        if (pr < 0) r = -1 - pr;
        else r = pr < r0 && sh_ss >= d.sm ? pr + 1 : pr;
        const int32_t k = d.index[x];
        if (r >= r0) {  // x opens round >= r0 on its chain: the closed form's candidate
          done[c] = 1;
          bfirst[c] = k;
          if (++sh_ndone == n) sh_stop = 1;
        } else {
          const int32_t spr = d.sp[x] < 0 ? d.root_sp_round[c] : d.round[d.sp[x]];
          const bool w = r > spr;  // witness (hashgraph.go:281-296)
          d.round[x] = r;
          d.witness[x] = w ? 1 : 0;
          d.rexists[r] = 1;
          if (w) d.fw[(int64_t)(r - rlo) * n + c] = x;
          if (r > d.state[ST_FIATMAX]) d.state[ST_FIATMAX] = r;
        }
      }
      __syncthreads();
    }
    if (sh_stop) break;
  }
  __syncthreads();
  for (int c = t; c < n; c += 1024) d.B[(int64_t)r0 * n + c] = bfirst[c];
  if (t == 0) d.state[ST_RESUME] = r0;
}

void launch_fiat(const Dev &d, hipStream_t s) {
  k_fiat<<<1, 1024, 0, s>>>(d);
}

}  // namespace bh
