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

#include <cstdlib>
#include <cstring>

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
constexpr int FI_CN = 128;               // one round's witness FD rows held in LDS up to this many chains
constexpr int32_t PR_SKIP = INT32_MIN;  // L.pr of an event on a done chain (or none)

// a workgroup barrier that waits for LDS traffic only: the per-event
// hand-offs of k_fiat go through LDS, so loads in flight (the next event's
// lastAncestors) and stores (its results) keep going across it.  Where global
// data one wave stored is read by another (fw) a full __syncthreads
// stays.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct FiatLds {
  int32_t done[FI_MAXN], bfirst[FI_MAXN];
  // the chunk's events (1024 ids from `base`) and the previous chunk's
  // (slot (id - base + 1024) of 2048): creator, index (chain position) and
  // the rounds this pass gave them; parents and flags of the current chunk
  int32_t list[1024], wcnt[16];
  int32_t cc[2048], ck[2048], crd[2048];
  int32_t csp[1024], cop[1024], cep[1024];
  int8_t cfl[1024];
  int32_t rnext[FI_MAXN], rspr[FI_MAXN];  // Root.NextRound / SelfParent.Round
  int32_t cnt, ndone, pr, ss, stop, fmax, nvis, nch, neww, newslot, cache_r;
  // n <= FI_CN: round cache_r's witnesses (cw[q], -1 none) and their FD rows
  // (fdc[q][i], FD_NONE past n), the counts' operand read from LDS: the whole
  // round is read per event, which from global memory is a compute unit's
  // load bandwidth (≈ 2k cycles per event at n = 128)
  int32_t cw[FI_CN], fdc[FI_CN * FI_CN];
};

__global__ __launch_bounds__(1024) void k_fiat(Dev d) {
  __shared__ FiatLds L;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, n = d.n, npad = d.npad;
  const int32_t r0 = d.r0, rlo = d.rlo;
  for (int c = t; c < n; c += 1024) {
    L.done[c] = 0;
    L.bfirst[c] = d.chain_len[c];
    L.rnext[c] = d.root_next[c];
    L.rspr[c] = d.root_sp_round[c];
  }
  if (t == 0) { L.ndone = 0; L.stop = 0; L.fmax = -1; L.nvis = 0; L.nch = 0; L.neww = -1; L.cache_r = -1; }
  const bool cached = n <= FI_CN;
  // thread 0: the event counted last, finalized at the next event
  bool pend = false;
  int32_t p_pr = 0, p_spr = 0, p_c = 0, p_k = 0, p_xi = 0;
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
      L.cep[t] = d.epos[e];
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
      L.nch++;
    }
    __syncthreads();
    const int32_t cnt = L.cnt;
    // lastAncestors of the next listed event, loaded one event ahead
    int32_t nla0 = -1, nla1 = -1;
    if (cnt > 0) {
      const int64_t rx = L.cep[L.list[0]];
      if (lane < n) nla0 = d.la[rx * npad + lane];
      if (lane + 64 < n) nla1 = d.la[rx * npad + lane + 64];
    }
    // Event j: thread 0 first finalizes event j-1 (its round from the count
    // j-1's waves left in L.ss: witness flag, fw, done) and then computes
    // j's parent round pr; a new witness's FD row is copied; the waves count
    // j's strongly-seen witnesses.  Two LDS barriers per event; j == cnt
    // finalizes the chunk's last event only.
    for (int32_t j = 0; j <= cnt; ++j) {
      const bool have = j < cnt;
      const int32_t xi = have ? L.list[j] : 0;
      const int32_t la0 = nla0, la1 = nla1;
      if (j + 1 < cnt) {
        const int64_t rn = L.cep[L.list[j + 1]];
        if (lane < n) nla0 = d.la[rn * npad + lane];
        if (lane + 64 < n) nla1 = d.la[rn * npad + lane + 64];
      }
      const int64_t rx = L.cep[xi];
      const bool dg = d.diag != nullptr && t == 0;
      const unsigned long long q0t = dg ? __builtin_amdgcn_s_memtime() : 0;
      if (t == 0) {
        if (pend) {  // finalize the previous event
          pend = false;
          int32_t r;
          if (p_pr < 0) r = -1 - p_pr;
          else r = p_pr < r0 && L.ss >= d.sm ? p_pr + 1 : p_pr;
          if (r >= r0) {  // it opens round >= r0 on its chain: the closed form's candidate
            L.done[p_c] = 1;
            L.bfirst[p_c] = p_k;
            if (++L.ndone == n) L.stop = 1;
          } else {
            const bool w = r > p_spr;  // witness (hashgraph.go:281-296)
            d.round[base + p_xi] = r;
            d.witness[base + p_xi] = w ? 1 : 0;
            L.crd[1024 + p_xi] = r;
            d.rexists[r] = 1;
            if (w) {
              d.fw[(int64_t)(r - rlo) * n + p_c] = (int32_t)(base + p_xi);
              L.neww = (int32_t)(base + p_xi);
              L.newslot = (r - rlo) * n + p_c;
            }
            L.fmax = max(L.fmax, r);
          }
        }
        int32_t pr = PR_SKIP;
        const int32_t c = have ? L.cc[1024 + xi] : 0;
        if (have && !L.done[c]) {
          // round of an event before x: "at least r0" if its chain was done at
          // or before it, else the round this pass gave it
          auto round_of = [&](int32_t y) -> int32_t {
            int32_t cy, ky, ry;
            if (y >= base - (base > 0 ? 1024 : 0)) {
              const int32_t sl = (int32_t)(y - base + 1024);
              cy = L.cc[sl]; ky = L.ck[sl]; ry = L.crd[sl];
            } else {
              cy = d.creator[y]; ky = d.index[y]; ry = __builtin_nontemporal_load(d.round + y);
            }
            return (L.done[cy] && ky >= L.bfirst[cy]) ? r0 : ry;
          };
          const int32_t sp = L.csp[xi], op = L.cop[xi];
          const bool oth = L.cfl[xi] & 1;                 // Root.Others[x] names x's other-parent
          const bool op_empty = op < 0 && !(L.cfl[xi] & 2);  // no other-parent at all
          // the self-parent's round (x's chain is not done: the round this pass gave it)
          const int32_t spr = sp < 0 ? L.rspr[c] : round_of(sp);
          if (sp < 0 && (oth || op_empty)) {
            pr = -1 - L.rnext[c];  // attached to the Root: NextRound by fiat (encoded < 0)
          } else {
            pr = spr;
            if (oth) pr = max(pr, L.rnext[c]);
            else if (op >= 0) pr = max(pr, round_of(op));
          }
          pend = true;
          p_pr = pr; p_spr = spr; p_c = c; p_k = L.ck[1024 + xi]; p_xi = xi;
          L.ss = 0;
          L.nvis++;
        }
        L.pr = pr;
      }
      lds_barrier();
      const unsigned long long q1t = dg ? __builtin_amdgcn_s_memtime() : 0;
      if (L.neww >= 0) {  // a new witness of the staged round: its FD row into the LDS copy
        const int64_t rw = L.cep[L.neww - base];
        const bool inc = cached && L.newslot / n + rlo == L.cache_r;
        const int q = L.newslot % n;
        if (inc)
          for (int i = t; i < FI_CN; i += 1024) L.fdc[q * FI_CN + i] = i < n ? d.fdt[fdt_pos(rw, i, npad)] : FD_NONE;
        if (inc && t == 0) L.cw[q] = L.neww;
        __syncthreads();  // (fw stored, then loaded within the workgroup: one compute unit's cache)
        if (t == 0) L.neww = -1;
        __syncthreads();
      }
      const unsigned long long q2t = dg ? __builtin_amdgcn_s_memtime() : 0;
      const int32_t pr = L.pr;
      if (pr == PR_SKIP) continue;  // uniform
      if (pr >= 0 && pr < r0 && pr >= rlo && cached) {
        if (L.cache_r != pr) {  // stage round pr (chain-major rows, coalesced)
          // the round's witnesses' FD rows, gathered from FDT (complete: the
          // walks write MaxInt32 where no event of a chain sees a row)
          const int32_t *wrow = d.fw + (int64_t)(pr - rlo) * n;
          for (int k = t; k < n * FI_CN; k += 1024) {
            const int q = k / FI_CN, i = k % FI_CN;
            const int32_t w = __builtin_nontemporal_load(wrow + q);  // (vector load: see fiat_count)
            L.fdc[k] = i < n && w >= 0 ? d.fdt[fdt_pos(d.epos[w], i, npad)] : FD_NONE;
          }
          if (t < FI_CN) L.cw[t] = t < n ? wrow[t] : -1;
          lds_barrier();
          if (t == 0) L.cache_r = pr;
          if (dg) d.diag[31] += 1;
        }
        // #witnesses of round pr that x strongly sees: a wave takes every 16th
        // witness row (q = wave + 16u; rows past n are absent), a lane two
        // columns; every LDS read of the wave issued before the first use
        int32_t w[FI_CN / 16], f0[FI_CN / 16], f1[FI_CN / 16];
#pragma unroll
        for (int u = 0; u < FI_CN / 16; ++u) {
          const int q = wave + 16 * u;
          w[u] = L.cw[q];
          f0[u] = L.fdc[q * FI_CN + lane];
          f1[u] = L.fdc[q * FI_CN + lane + 64];
        }
        int ssw = 0;
#pragma unroll
        for (int u = 0; u < FI_CN / 16; ++u) {
          const int cntc = __popcll(__ballot(la0 >= f0[u])) + __popcll(__ballot(la1 >= f1[u]));
          ssw += w[u] >= 0 && wave + 16 * u < n && cntc >= d.sm;
        }
        if (lane == 0 && ssw) atomicAdd(&L.ss, ssw);
      } else if (pr >= 0 && pr < r0 && pr >= rlo) {
        // #witnesses of round pr that x strongly sees (_stronglySee :172-191)
        // the round's witnesses' FD rows from FDT (fw names each witness): a
        // wave takes every 16th chain, loads all its rows' columns first,
        // then counts columns by ballot
        const int32_t *wrow = d.fw + (int64_t)(pr - rlo) * n;
        int ssw = 0;
        for (int q0 = wave; q0 < n; q0 += 16 * 8) {
          int32_t f0[8], f1[8];
          int64_t wr[8];
          bool has[8];
          // every load of the batch issued at once (one cache round trip): rows
          // of absent witnesses are read too and masked after
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int q = min(q0 + 16 * u, n - 1);
            const int32_t w = __builtin_nontemporal_load(wrow + q);  // (vector load: see fiat_count)
            has[u] = w >= 0 && q0 + 16 * u < n;
            wr[u] = d.epos[max(w, 0)];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            f0[u] = d.fdt[fdt_pos(wr[u], min(lane, npad - 1), npad)];
            f1[u] = d.fdt[fdt_pos(wr[u], min(lane + 64, npad - 1), npad)];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (!has[u] || lane >= n) f0[u] = FD_NONE;
            if (!has[u] || lane + 64 >= n) f1[u] = FD_NONE;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            int cntc = __popcll(__ballot(la0 >= f0[u])) + __popcll(__ballot(la1 >= f1[u]));
            for (int i0 = 128; i0 < n; i0 += 64) {  // chains beyond 128 (n <= 512)
              const int i = i0 + lane;
              cntc += __popcll(__ballot(has[u] && i < n && d.la[rx * npad + i] >= d.fdt[fdt_pos(wr[u], min(i, npad - 1), npad)]));
            }
            ssw += has[u] && cntc >= d.sm;
          }
        }
        if (lane == 0 && ssw) atomicAdd(&L.ss, ssw);
      }
      lds_barrier();
      if (dg) {  // phase cycles (BH_DIAG): finalize + pr, witness rows, counts
        const unsigned long long q3t = __builtin_amdgcn_s_memtime();
        d.diag[24] += q1t - q0t;
        d.diag[25] += q2t - q1t;
        d.diag[26] += q3t - q2t;
        d.diag[28] += 1;
      }
    }
    if (L.stop) break;
  }
  __syncthreads();
  for (int c = t; c < n; c += 1024) d.B[(int64_t)r0 * n + c] = L.bfirst[c];
  if (t == 0) {
    d.state[ST_RESUME] = r0;
    d.state[ST_FIATMAX] = L.fmax;
    d.state[ST_FIATDONE] = L.ndone;
    d.state[ST_FIATEV] = L.nvis;
    d.state[ST_FIATCH] = L.nch;
  }
}

// ---------------------------------------------------------------------------
// k_fiat_ls: the same rounds, level-synchronously.  An event's round depends
// only on its ancestors (the witnesses it can strongly see are ancestors:
// LA[x][i] >= FD[w][i] means x has an ancestor descending from w), so any
// topological order gives Go's rounds, and every event whose parents are
// done can be computed at once.  A step: (A) each chain's next event, if its
// other-parent is done, takes pr from its parents; (B) the counts, as items
// (ready event, block of witnesses) spread over the waves, each item's
// witness FD rows loaded at once from FDT; (C) one wave per ready event sets
// its round and, for a new witness, fw (and its FD row in the LDS copy) --
// after every count of the step (a same-step witness is no ancestor of a
// same-step event, so it would count zero, but a half-written row must not
// be read).  Steps ~ the fiat region's depth instead of its events.
constexpr int FL_MAXREADY = FI_MAXN;
constexpr int FL_WC = 56 * 1024;   // 16-bit witness FD entries cached in LDS (112 KiB)
constexpr int FL_WFL = 4096;       // witness presence flags ((r0 - rlo) n)

struct FiatLsLds {
  int32_t cur[FI_MAXN], done[FI_MAXN], bfirst[FI_MAXN], lastr[FI_MAXN];
  int32_t rnext[FI_MAXN], rspr[FI_MAXN], len[FI_MAXN], cs[FI_MAXN];
  int32_t rx[FL_MAXREADY], rc[FL_MAXREADY], rpr[FL_MAXREADY], rsp[FL_MAXREADY], ss[FL_MAXREADY];
  int32_t rcnt[2], ndone, fmax, nvis, steps;
  // the fiat rounds' witness FD rows as 16-bit FD + 1 (0xFFFF: none), when
  // they fit ((r0 - rlo) n npad <= FL_WC and chains <= P16_MAXLEN), and
  // their presence flags: the counts then read LDS instead of L2
  uint16_t wc[FL_WC];
  int8_t wfl[FL_WFL];
};

// #witnesses q0 .. q0 + IW - 1 of round pr that the event at chain-major row
// xrow strongly sees (_stronglySee :172-191): LA row in registers (NV
// 64-column groups), the IW witness FD rows loaded at once
template <int NV, int IW>
__device__ __forceinline__ int fiat_count(const Dev &d, int64_t xrow, int32_t pr, int q0, int lane) {
  const int n = d.n, npad = d.npad, rlo = d.rlo;
  int32_t la[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int i = lane + 64 * v;
    la[v] = i < n ? d.la[xrow * npad + i] : -1;
  }
  const int32_t *wrow = d.fw + (int64_t)(pr - rlo) * n;
  // which of the block's witnesses exist: one lane-indexed (vector) load --
  // fw is stored by this kernel, and a wave-uniform load could be served by
  // the scalar cache, which vector stores do not update
  const int32_t wl = lane < IW && q0 + lane < n ? wrow[q0 + lane] : -1;
  const unsigned long long hm = __ballot(wl >= 0);
  // each witness's FD row straight from FDT (its chain-major row from epos)
  const int64_t wrl = d.epos[max(wl, 0)];
  int32_t f[IW][NV];
#pragma unroll
  for (int u = 0; u < IW; ++u) {
    const int64_t wr = __shfl(wrl, u);
#pragma unroll
    for (int v = 0; v < NV; ++v) f[u][v] = d.fdt[fdt_pos(wr, min(lane + 64 * v, npad - 1), npad)];
  }
  int ssw = 0;
#pragma unroll
  for (int u = 0; u < IW; ++u) {
    int cnt = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v) cnt += __popcll(__ballot(lane + 64 * v < n && la[v] >= f[u][v]));
    ssw += ((hm >> u) & 1) && cnt >= d.sm;
  }
  return ssw;
}

// NV: 64-column groups of a row (n <= 64 NV), one instantiation per width
// (all four in one kernel spill registers)
// fiat_count over the LDS copy: LA + 1 against FD + 1, 16-bit
template <int NV, int IW>
__device__ __forceinline__ int fiat_count_lds(const Dev &d, const uint16_t *wc, const int8_t *wfl, int64_t xrow,
                                              int32_t pr, int q0, int lane) {
  const int n = d.n, npad = d.npad, rlo = d.rlo;
  int32_t la[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int i = lane + 64 * v;
    la[v] = i < n ? d.la[xrow * npad + i] + 1 : 0;
  }
  const uint16_t *frow = wc + (int64_t)(pr - rlo) * n * npad;
  const int8_t *wrow = wfl + (pr - rlo) * n;
  // every LDS read of the item first (one round trip), then the compares
  int32_t f[IW][NV];
  const int32_t wl = lane < IW && q0 + lane < n ? wrow[q0 + lane] : 0;
  const unsigned long long hm = __ballot(wl != 0);
#pragma unroll
  for (int u = 0; u < IW; ++u) {
    const int q = min(q0 + u, n - 1);
#pragma unroll
    for (int v = 0; v < NV; ++v) f[u][v] = frow[q * npad + min(lane + 64 * v, npad - 1)];
  }
  int ssw = 0;
#pragma unroll
  for (int u = 0; u < IW; ++u) {
    int cnt = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v) cnt += __popcll(__ballot(lane + 64 * v < n && la[v] >= f[u][v]));
    ssw += ((hm >> u) & 1) && cnt >= d.sm;
  }
  return ssw;
}

template <int NV>
__global__ __launch_bounds__(1024) void k_fiat_ls(Dev d) {
  __shared__ FiatLsLds L;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, n = d.n, npad = d.npad;
  const int32_t r0 = d.r0, rlo = d.rlo;
  for (int c = t; c < n; c += 1024) {
    L.cur[c] = 0;
    L.done[c] = 0;
    L.bfirst[c] = d.chain_len[c];
    L.lastr[c] = 0;
    L.rnext[c] = d.root_next[c];
    L.rspr[c] = d.root_sp_round[c];
    L.len[c] = d.chain_len[c];
    L.cs[c] = d.chain_start[c];
  }
  if (t == 0) { L.rcnt[0] = L.rcnt[1] = 0; L.ndone = 0; L.fmax = -1; L.nvis = 0; L.steps = 0; }
  const bool cached = (int64_t)(r0 - rlo) * n * npad <= FL_WC && (r0 - rlo) * n <= FL_WFL && d.max_chain_len <= P16_MAXLEN;
  if (cached)
    for (int i = t; i < (r0 - rlo) * n; i += 1024) L.wfl[i] = 0;
  __syncthreads();
  const bool dg = d.diag != nullptr && t == 0;
  for (int s = 0;; ++s) {
    const int par = s & 1;
    const unsigned long long q0t = dg ? __builtin_amdgcn_s_memtime() : 0;
    // (A) each chain's next event, if its other-parent is done: the parents' round
    if (t < n && !L.done[t] && L.cur[t] < L.len[t]) {
      const int c = t, k = L.cur[c];
      const int32_t x = d.chain_ids[L.cs[c] + k];
      const int32_t op = d.op[x], sp = d.sp[x];
      const int8_t fl = d.rflag[x];
      bool ready = true;
      int32_t opr = 0;
      if (op >= 0) {
        const int32_t cy = d.creator[op], ky = d.index[op];
        ready = ky < L.cur[cy] || L.done[cy];
        // a parent at or past its chain's first event of round >= r0 counts as r0
        if (ready) opr = (L.done[cy] && ky >= L.bfirst[cy]) ? r0 : __builtin_nontemporal_load(d.round + op);
      }
      if (ready) {
        const int32_t spr = sp < 0 ? L.rspr[c] : L.lastr[c];  // the self-parent: chain c's previous event
        const bool oth = fl & 1, op_empty = op < 0 && !(fl & 2);
        int32_t pr;
        if (sp < 0 && (oth || op_empty)) {
          pr = -1 - L.rnext[c];  // attached to the Root: NextRound by fiat (encoded < 0)
        } else {
          pr = spr;
          if (oth) pr = max(pr, L.rnext[c]);  // Root.Others names the other-parent
          else if (op >= 0) pr = max(pr, opr);
        }
        const int j = atomicAdd(&L.rcnt[par], 1);
        L.rx[j] = x;
        L.rc[j] = c;
        L.rpr[j] = pr;
        L.rsp[j] = spr;
        L.ss[j] = 0;
      }
    }
    __syncthreads();
    const int cnt = L.rcnt[par];
    if (cnt == 0) break;  // every chain done or exhausted
    const unsigned long long q1t = dg ? __builtin_amdgcn_s_memtime() : 0;
    // (B) counts: items (ready event j, a block of IW witnesses) over the waves
    {
      constexpr int IW = 64 / NV;  // witnesses per item (64 FD values per lane in flight)
      const int per = (n + IW - 1) / IW;
      for (int it = wave; it < cnt * per; it += 16) {
        const int j = it / per, q0 = (it - j * per) * IW;
        const int32_t pr = L.rpr[j];
        if (!(pr >= 0 && pr < r0 && pr >= rlo)) continue;
        const int32_t c = L.rc[j];
        const int64_t xrow = (int64_t)L.cs[c] + L.cur[c];
        const int ssw = cached ? fiat_count_lds<NV, IW>(d, L.wc, L.wfl, xrow, pr, q0, lane)
                               : fiat_count<NV, IW>(d, xrow, pr, q0, lane);
        if (lane == 0 && ssw) atomicAdd(&L.ss[j], ssw);
      }
    }
    __syncthreads();
    const unsigned long long q2t = dg ? __builtin_amdgcn_s_memtime() : 0;
    // (C) one wave per ready event: its round; a new witness's FD row, then fw
    for (int j = wave; j < cnt; j += 16) {
      const int32_t x = L.rx[j], c = L.rc[j], pr = L.rpr[j];
      const int32_t k = L.cur[c];
      const int64_t xrow = (int64_t)L.cs[c] + k;
      const int32_t r = pr < 0 ? -1 - pr : (pr < r0 && L.ss[j] >= d.sm ? pr + 1 : pr);
      const bool w = r < r0 && r > L.rsp[j];  // witness (hashgraph.go:281-296)
      if (w) {
        const int64_t slot = (int64_t)(r - rlo) * n + c;
        if (cached)
          for (int i = lane; i < npad; i += 64) {
            const int32_t v = i < n ? d.fdt[fdt_pos(xrow, i, npad)] : FD_NONE;
            L.wc[slot * npad + i] = (uint16_t)min((uint32_t)v + 1u, 0xFFFFu);  // FD_NONE + 1 wraps to 2^31
          }
        if (lane == 0) {
          d.fw[slot] = x;
          if (cached) L.wfl[slot] = 1;
        }
      }
      if (lane == 0) {
        atomicAdd(&L.nvis, 1);
        if (r >= r0) {  // x opens round >= r0 on its chain: the closed form's candidate
          L.done[c] = 1;
          L.bfirst[c] = k;
          atomicAdd(&L.ndone, 1);
        } else {
          d.round[x] = r;
          d.witness[x] = w ? 1 : 0;
          d.rexists[r] = 1;
          L.lastr[c] = r;
          L.cur[c] = k + 1;
          atomicMax(&L.fmax, r);
        }
      }
    }
    if (t == 0) {
      L.rcnt[par ^ 1] = 0;
      L.steps = s + 1;
    }
    __syncthreads();  // (rounds / fw stored before the next step loads them)
    if (dg) {  // phase cycles per step (BH_DIAG): A, B, C
      const unsigned long long q3t = __builtin_amdgcn_s_memtime();
      d.diag[24] += q1t - q0t;
      d.diag[25] += q2t - q1t;
      d.diag[26] += q3t - q2t;
      d.diag[28] += 1;
    }
  }
  for (int c = t; c < n; c += 1024) d.B[(int64_t)r0 * n + c] = L.bfirst[c];
  if (t == 0) {
    d.state[ST_RESUME] = r0;
    d.state[ST_FIATMAX] = L.fmax;
    d.state[ST_FIATDONE] = L.ndone;
    d.state[ST_FIATEV] = L.nvis;
    d.state[ST_FIATCH] = L.steps;
  }
}

// BH_FIAT=serial: the event-by-event pass (A/B; the tests run both)
void launch_fiat(const Dev &d, hipStream_t s) {
  const char *e = getenv("BH_FIAT");
  if (e && !strcmp(e, "serial")) k_fiat<<<1, 1024, 0, s>>>(d);
  else if (d.n <= 64) k_fiat_ls<1><<<1, 1024, 0, s>>>(d);
  else if (d.n <= 128) k_fiat_ls<2><<<1, 1024, 0, s>>>(d);
  else if (d.n <= 256) k_fiat_ls<4><<<1, 1024, 0, s>>>(d);
  else k_fiat_ls<8><<<1, 1024, 0, s>>>(d);
}

}  // namespace bh
