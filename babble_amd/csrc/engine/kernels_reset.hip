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
constexpr int FI_CACHE_N = 128;  // witness FD rows of one round cached in LDS up to this many chains

struct FiatLds {
  int32_t done[FI_MAXN], bfirst[FI_MAXN];
  // the chunk's events (1024 ids from `base`) and the previous chunk's
  // (slot (id - base + 1024) of 2048): creator, index (chain position) and
  // the rounds this pass gave them; parents and flags of the current chunk
  int32_t list[1024], wcnt[16];
  int32_t cc[2048], ck[2048], crd[2048];
  int32_t csp[1024], cop[1024];
  int8_t cfl[1024];
  // FD rows of round cache_r's witnesses (n <= FI_CACHE_N): fdc[j][i] for
  // the j-th witness in chain order
  int32_t fdc[FI_CACHE_N][FI_CACHE_N];
  int32_t wl[FI_CACHE_N];  // those witnesses' ids
  int32_t cache_r, cache_nw;
  int32_t cnt, ndone, pr, ss, stop, fmax;
};

__global__ __launch_bounds__(1024) void k_fiat(Dev d) {
  __shared__ FiatLds L;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, n = d.n, npad = d.npad;
  const int32_t r0 = d.r0, rlo = d.rlo;
  const bool cached = n <= FI_CACHE_N;
  for (int c = t; c < n; c += 1024) {
    L.done[c] = 0;
    L.bfirst[c] = d.chain_len[c];
  }
  if (t == 0) { L.ndone = 0; L.stop = 0; L.cache_r = -1; L.cache_nw = 0; L.fmax = -1; }
  for (int i = t; i < 1024; i += 1024) L.cc[i] = -1;
  __syncthreads();
  for (int64_t base = 0; base < d.N; base += 1024) {
    // the chunk's events, staged (the previous chunk's move down); those on
    // chains not done yet listed in order
    const int64_t e = base + t;
    bool need = false;
    if (base > 0) {
      L.cc[t] = L.cc[1024 + t];
      L.ck[t] = L.ck[1024 + t];
      L.crd[t] = L.crd[1024 + t];
    }
    __syncthreads();
    if (e < d.N) {
      const int32_t c = d.creator[e];
      L.cc[1024 + t] = c;
      L.ck[1024 + t] = d.index[e];
      L.csp[t] = d.sp[e];
      L.cop[t] = d.op[e];
      L.cfl[t] = d.rflag[e];
      L.crd[1024 + t] = UNSET;
      need = !L.done[c];
    }
    const unsigned long long m = __ballot(need);
    if (lane == 0) L.wcnt[wave] = __popcll(m);
    __syncthreads();
    int32_t pos = __popcll(m & ((1ull << lane) - 1ull));
    for (int w = 0; w < wave; ++w) pos += L.wcnt[w];
    if (need) L.list[pos] = t;
    if (t == 0) {
      int32_t tot = 0;
      for (int w = 0; w < 16; ++w) tot += L.wcnt[w];
      L.cnt = tot;
    }
    __syncthreads();
    const int32_t cnt = L.cnt;
    for (int32_t j = 0; j < cnt; ++j) {
      const int32_t xi = L.list[j];
      const int32_t x = (int32_t)(base + xi), c = L.cc[1024 + xi];
      if (L.done[c]) continue;  // uniform: done[] only changes behind barriers
      // x's lastAncestors, loaded while lane 0 works out its parent round
      const int64_t rx = d.epos[x];
      const int32_t la0 = lane < n ? d.la[rx * npad + lane] : -1;
      const int32_t la1 = lane + 64 < n ? d.la[rx * npad + lane + 64] : -1;
      if (t == 0) {
        // round of an event before x: "at least r0" if its chain was done at
        // or before it, else the round this pass gave it
        auto round_of = [&](int32_t y) -> int32_t {
          int32_t cy, ky, ry;
          if (y >= base - (base > 0 ? 1024 : 0)) {
            const int32_t sl = (int32_t)(y - base + 1024);
            cy = L.cc[sl]; ky = L.ck[sl]; ry = L.crd[sl];
          } else {
            cy = d.creator[y]; ky = d.index[y]; ry = d.round[y];
          }
          return (L.done[cy] && ky >= L.bfirst[cy]) ? r0 : ry;
        };
        const int32_t sp = L.csp[xi], op = L.cop[xi];
        const bool oth = L.cfl[xi] & 1;                 // Root.Others[x] names x's other-parent
        const bool op_empty = op < 0 && !(L.cfl[xi] & 2);  // no other-parent at all
        int32_t pr;
        if (sp < 0 && (oth || op_empty)) {
          pr = -1 - d.root_next[c];  // attached to the Root: NextRound by fiat (encoded < 0)
        } else {
          pr = sp < 0 ? d.root_sp_round[c] : round_of(sp);
          if (oth) pr = max(pr, d.root_next[c]);
          else if (op >= 0) pr = max(pr, round_of(op));
        }
        L.pr = pr;
        L.ss = 0;
      }
      __syncthreads();
      const int32_t pr = L.pr;
      if (pr >= 0 && pr < r0 && pr >= rlo) {
        // #witnesses of round pr that x strongly sees (_stronglySee :172-191)
        const int32_t *wrow = d.fw + (int64_t)(pr - rlo) * n;
        if (cached) {
          if (L.cache_r != pr) {  // stage round pr's witness FD rows
            __syncthreads();
            if (t == 0) {
              int32_t k = 0;
              for (int q = 0; q < n; ++q)
                if (wrow[q] >= 0) L.wl[k++] = wrow[q];
              L.cache_nw = k;
            }
            __syncthreads();
            const int32_t nw = L.cache_nw;
            for (int p = t; p < nw * n; p += 1024) {
              const int32_t jw = p / n, i = p - jw * n;
              L.fdc[jw][i] = d.fdt[fdt_pos(d.epos[L.wl[jw]], i, npad)];
            }
            __syncthreads();
            if (t == 0) L.cache_r = pr;
            __syncthreads();
          }
          const int32_t nw = L.cache_nw;
          for (int jw = wave; jw < nw; jw += 16) {
            int cntc = (lane < n && la0 >= L.fdc[jw][lane]) + (lane + 64 < n && la1 >= L.fdc[jw][lane + 64]);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) cntc += __shfl_xor(cntc, off);
            if (lane == 0 && cntc >= d.sm) atomicAdd(&L.ss, 1);
          }
        } else {
          for (int q = wave; q < n; q += 16) {
            const int32_t w = wrow[q];
            if (w < 0) continue;
            const int64_t rw = d.epos[w];
            int cntc = 0;
            for (int i = lane; i < n; i += 64) cntc += d.la[rx * npad + i] >= d.fdt[fdt_pos(rw, i, npad)];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) cntc += __shfl_xor(cntc, off);
            if (lane == 0 && cntc >= d.sm) atomicAdd(&L.ss, 1);
          }
        }
      }
      __syncthreads();
      if (t == 0) {
        int32_t r;
        if (pr < 0) r = -1 - pr;
        else r = pr < r0 && L.ss >= d.sm ? pr + 1 : pr;
        const int32_t k = L.ck[1024 + xi];
        if (r >= r0) {  // x opens round >= r0 on its chain: the closed form's candidate
          L.done[c] = 1;
          L.bfirst[c] = k;
          if (++L.ndone == n) L.stop = 1;
        } else {
          const int32_t sp = L.csp[xi];
          const int32_t spr = sp < 0 ? d.root_sp_round[c]
                            : sp >= base - (base > 0 ? 1024 : 0) ? L.crd[sp - base + 1024] : d.round[sp];
          const bool w = r > spr;  // witness (hashgraph.go:281-296)
          d.round[x] = r;
          d.witness[x] = w ? 1 : 0;
          L.crd[1024 + xi] = r;
          d.rexists[r] = 1;
          if (w) {
            d.fw[(int64_t)(r - rlo) * n + c] = x;
            if (r == L.cache_r) L.cache_r = -1;  // the cached round gained a witness
          }
          L.fmax = max(L.fmax, r);
        }
      }
      __syncthreads();
    }
    if (L.stop) break;
  }
  __syncthreads();
  for (int c = t; c < n; c += 1024) d.B[(int64_t)r0 * n + c] = L.bfirst[c];
  if (t == 0) {
    d.state[ST_RESUME] = r0;
    d.state[ST_FIATMAX] = L.fmax;
  }
}

void launch_fiat(const Dev &d, hipStream_t s) {
  k_fiat<<<1, 1024, 0, s>>>(d);
}

}  // namespace bh
