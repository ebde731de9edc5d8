// kernels_order.hip -- DecideRoundReceived + ProcessDecidedRounds / GetFrame.
//
// Round received (hashgraph.go:951-1036): x is received in the first round
// i > round(x) such that rounds round(x)+1..i all have their witnesses
// decided, round i has >= 1 famous witness, and every famous witness of i
// sees x.  see(w, x) = LA[w][creator(x)] >= index(x), so the last condition
// is index(x) <= minLA[i][creator(x)] (min over the famous witnesses of i,
// published by k_fame).  One thread per event; the loop over i stops at the
// first undecided round, usually after one or two rounds.
//
// ProcessDecidedRounds (hashgraph.go:1041-1122) walks PendingRounds (all
// rounds, ascending, in the batch schedule) while they are decided: rounds
// [0, P) are processed.  Frame r = events received in r (GetFrame,
// :1125-1231), ordered ByLamportTimestamp (event.go:332-347): Lamport
// timestamp, then the signature's r as a big integer (8 big-endian words
// here).  A block is emitted per non-empty frame (:1083-1107).  Implementation:
// histogram of rr -> exclusive scan -> scatter into frame buckets -> one
// workgroup per frame sorts its bucket (bitonic, keys staged in LDS; frames
// larger than FRAME_LDS_MAX sort in place in HBM with the same network).
#include "engine.h"

namespace bh {

__global__ void k_round_received(Dev d, int32_t R) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= d.N) return;
  const int32_t r = d.round[x], c = d.creator[x], k = d.index[x];
  int32_t res = UNSET;
  for (int32_t i = r + 1; i < R; ++i) {
    if (!d.decided[i]) break;
    if (d.nfam[i] > 0 && k <= d.minla[(int64_t)i * d.npad + c]) { res = i; break; }
  }
  d.rr[x] = res;
}

void launch_round_received(const Dev &d, int32_t R, hipStream_t s) {
  if (d.N == 0) return;
  k_round_received<<<(unsigned)((d.N + 255) / 256), 256, 0, s>>>(d, R);
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_prefix(Dev d, int32_t R) {
  __shared__ int32_t p;
  if (threadIdx.x == 0) p = R;
  __syncthreads();
  for (int32_t r = threadIdx.x; r < R; r += blockDim.x)
    if (!d.decided[r]) atomicMin(&p, r);
  __syncthreads();
  for (int32_t r = threadIdx.x; r < R; r += blockDim.x) { d.frame_cnt[r] = 0; d.frame_cur[r] = 0; }
  if (threadIdx.x == 0) {
    d.state[ST_P] = p;
    d.counters[0] = 0;
    d.counters[1] = 0;
    d.counters[2] = 0;
  }
}

__global__ void k_frame_count(Dev d) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t rr = x < d.N ? d.rr[x] : UNSET;
  // events received (in any round): they leave UndeterminedEvents
  const unsigned long long m = __ballot(rr != UNSET);
  if ((threadIdx.x & 63) == 0 && m)
    atomicAdd(reinterpret_cast<unsigned long long *>(&d.counters[2]), (unsigned long long)__popcll(m));
  if (rr != UNSET && rr < d.state[ST_P]) atomicAdd(&d.frame_cnt[rr], 1);
}

// exclusive scans of frame sizes and of non-empty flags (block indices)
__global__ __launch_bounds__(1024) void k_frame_scan(Dev d) {
  __shared__ int32_t part[1024], partb[1024];
  const int t = threadIdx.x;
  const int32_t P = d.state[ST_P];
  const int32_t per = (P + 1023) / 1024;
  const int32_t lo = min(P, t * per), hi = min(P, lo + per);
  int32_t s = 0, sb = 0;
  for (int32_t r = lo; r < hi; ++r) { s += d.frame_cnt[r]; sb += d.frame_cnt[r] > 0; }
  part[t] = s;
  partb[t] = sb;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int32_t a = t >= off ? part[t - off] : 0, b = t >= off ? partb[t - off] : 0;
    __syncthreads();
    part[t] += a;
    partb[t] += b;
    __syncthreads();
  }
  int32_t run = part[t] - s, runb = partb[t] - sb;
  for (int32_t r = lo; r < hi; ++r) {
    d.frame_ofs[r] = run;
    d.blk_of_frame[r] = d.frame_cnt[r] > 0 ? runb : -1;
    run += d.frame_cnt[r];
    runb += d.frame_cnt[r] > 0;
  }
  if (t == 1023) { d.state[ST_NCONS] = part[1023]; d.state[ST_NBLOCKS] = partb[1023]; }
}

__global__ void k_frame_scatter(Dev d) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= d.N) return;
  const int32_t rr = d.rr[x];
  if (rr == UNSET || rr >= d.state[ST_P]) return;
  const int32_t slot = atomicAdd(&d.frame_cur[rr], 1);
  d.order[d.frame_ofs[rr] + slot] = (int32_t)x;
}

// ByLamportTimestamp.Less; equal keys (same r, impossible for distinct
// signatures) fall back to the id to stay deterministic
struct Key {
  int32_t lt;
  uint32_t w[8];
  int32_t id;
};
__device__ __forceinline__ bool key_less(const Key &a, const Key &b) {
  if (a.lt != b.lt) return a.lt < b.lt;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (a.w[q] != b.w[q]) return a.w[q] < b.w[q];
  return a.id < b.id;
}
__device__ __forceinline__ Key load_key(const Dev &d, int32_t e) {
  Key k;
  k.lt = d.lt[e];
  const uint4 *s = reinterpret_cast<const uint4 *>(d.sigw + (int64_t)e * 8);
  const uint4 a = s[0], b = s[1];
  k.w[0] = a.x; k.w[1] = a.y; k.w[2] = a.z; k.w[3] = a.w;
  k.w[4] = b.x; k.w[5] = b.y; k.w[6] = b.z; k.w[7] = b.w;
  k.id = e;
  return k;
}

// bitonic network in its "flip" form: every comparator puts the smaller key
// at the lower index, so padding past `cnt` is never touched
template <bool LDS>
__device__ void bitonic(Key *keys, int32_t *ids, int32_t cnt, const Dev &d) {
  int32_t p2 = 1;
  while (p2 < cnt) p2 <<= 1;
  for (int32_t k = 2; k <= p2; k <<= 1) {
    for (int32_t j = k >> 1; j > 0; j >>= 1) {
      for (int32_t i = threadIdx.x; i < p2; i += blockDim.x) {
        int32_t partner;
        if (j == (k >> 1)) partner = i ^ (k - 1);
        else partner = i ^ j;
        if (partner <= i || partner >= cnt) continue;
        if (LDS) {
          if (key_less(keys[partner], keys[i])) {
            const Key tmp = keys[i];
            keys[i] = keys[partner];
            keys[partner] = tmp;
          }
        } else {
          const int32_t a = ids[i], b = ids[partner];
          if (key_less(load_key(d, b), load_key(d, a))) { ids[i] = b; ids[partner] = a; }
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(256) void k_frame_sort(Dev d) {
  extern __shared__ __attribute__((aligned(16))) unsigned char osm[];
  __shared__ unsigned long long sh_ntx, sh_loaded;
  const int32_t f = blockIdx.x;
  const int32_t cnt = d.frame_cnt[f];
  if (cnt == 0) return;
  const int32_t off = d.frame_ofs[f];
  int32_t *ids = d.order + off;
  if (threadIdx.x == 0) { sh_ntx = 0; sh_loaded = 0; }
  if (cnt <= FRAME_LDS_MAX) {
    Key *keys = reinterpret_cast<Key *>(osm);
    for (int32_t i = threadIdx.x; i < cnt; i += blockDim.x) keys[i] = load_key(d, ids[i]);
    __syncthreads();
    bitonic<true>(keys, nullptr, cnt, d);
    for (int32_t i = threadIdx.x; i < cnt; i += blockDim.x) ids[i] = keys[i].id;
    __syncthreads();
  } else {
    __syncthreads();
    bitonic<false>(nullptr, ids, cnt, d);
  }
  unsigned long long ntx = 0, loaded = 0;
  for (int32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
    const int32_t e = ids[i];
    d.cons_pos[e] = (int64_t)off + i;
    const int32_t t = d.ntx[e];
    ntx += t;
    loaded += (d.index[e] == 0 || t > 0);  // IsLoaded, event.go:169-178
  }
  if (ntx) atomicAdd(&sh_ntx, ntx);
  if (loaded) atomicAdd(&sh_loaded, loaded);
  __syncthreads();
  if (threadIdx.x == 0) {
    d.frame_ntx[f] = (int64_t)sh_ntx;
    atomicAdd(reinterpret_cast<unsigned long long *>(&d.counters[0]), (unsigned long long)sh_ntx);
    atomicAdd(reinterpret_cast<unsigned long long *>(&d.counters[1]), (unsigned long long)sh_loaded);
  }
}

void configure_order_kernels() {
  (void)hipFuncSetAttribute((const void *)k_frame_sort, hipFuncAttributeMaxDynamicSharedMemorySize,
                            FRAME_LDS_MAX * sizeof(Key));
}

void launch_order(const Dev &d, int32_t R, hipStream_t s) {
  if (R <= 0) return;
  k_prefix<<<1, 1024, 0, s>>>(d, R);
  const unsigned g = (unsigned)((d.N + 255) / 256);
  k_frame_count<<<g, 256, 0, s>>>(d);
  k_frame_scan<<<1, 1024, 0, s>>>(d);
  k_frame_scatter<<<g, 256, 0, s>>>(d);
  // frames [0, P); P <= R.  Launch R blocks: frames >= P have cnt 0.
  k_frame_sort<<<R, 256, FRAME_LDS_MAX * sizeof(Key), s>>>(d);
}

}  // namespace bh
