// kernels_sha.hip -- batched SHA-256 of event bodies (insert-side hashing).
//
// Reference: Event.Hash() = SHA-256 of the Go-JSON encoding of the event
// body (event.go:50-56), computed for every event InsertEvent receives
// (hashgraph.go:716-721: the hash keys the event, feeds the signature check
// and its byte 16 is the fame coin, middleBit hashgraph.go:1526-1535).
// SURVEY §8(f) row 2.  FIPS 180-4 SHA-256, one thread per message: the
// messages are a few hundred bytes, so a lane walks its message in 64-byte
// blocks; each block is read as 17 dword loads from the 4-byte-aligned
// address below it and realigned with v_alignbyte, then byte-swapped to the
// big-endian schedule words.  Integer-only, bit-exact by construction
// (checked against hashlib and the generator's digests).
#include "engine.h"

namespace bh {

__constant__ uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_amdgcn_perm(0, x, 0x00010203); }

// data: message bytes (at least 68 readable bytes past every message end),
// off[i] / len[i]: message i; out: 32 bytes per message
__global__ __launch_bounds__(256) void k_sha256(const uint8_t *data, const int64_t *off, const int32_t *len,
                                                int64_t count, uint8_t *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t m0 = off[i];
  const int32_t L = len[i];
  const int nb = (L + 8) / 64 + 1;
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  for (int b = 0; b < nb; ++b) {
    const int64_t m = m0 + 64 * b;
    const uint32_t *a = reinterpret_cast<const uint32_t *>(data + (m & ~(int64_t)3));
    const int s = (int)(m & 3);
    uint32_t dw[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) dw[k] = a[k];
    uint32_t w[64];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      // bytes 64b + 4k .. +3 of the message, little-endian in dw, realigned
      const uint32_t le = (uint32_t)(((uint64_t)dw[k + 1] << 32 | dw[k]) >> (8 * s));
      uint32_t x = bswap(le);
      const int pos = 64 * b + 4 * k;
      const int nv = min(max(L - pos, 0), 4);  // message bytes in this word
      if (nv < 4) {
        x = nv == 0 ? 0u : (x & ~(0xFFFFFFFFu >> (8 * nv)));
        if (L - pos >= 0 && L - pos < 4) x |= 0x80u << (24 - 8 * nv);  // the 1 bit after the message
      }
      w[k] = x;
    }
    if (b == nb - 1) {  // bit length, big-endian 64-bit
      const uint64_t bits = (uint64_t)L * 8;
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
#pragma unroll
    for (int k = 16; k < 64; ++k) {
      const uint32_t s0 = rotr(w[k - 15], 7) ^ rotr(w[k - 15], 18) ^ (w[k - 15] >> 3);
      const uint32_t s1 = rotr(w[k - 2], 17) ^ rotr(w[k - 2], 19) ^ (w[k - 2] >> 10);
      w[k] = w[k - 16] + s0 + w[k - 7] + s1;
    }
    uint32_t A = h[0], B = h[1], C = h[2], D = h[3], E = h[4], F = h[5], G = h[6], H = h[7];
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      const uint32_t S1 = rotr(E, 6) ^ rotr(E, 11) ^ rotr(E, 25);
      const uint32_t ch = (E & F) ^ (~E & G);
      const uint32_t t1 = H + S1 + ch + SHA_K[k] + w[k];
      const uint32_t S0 = rotr(A, 2) ^ rotr(A, 13) ^ rotr(A, 22);
      const uint32_t mj = (A & B) ^ (A & C) ^ (B & C);
      const uint32_t t2 = S0 + mj;
      H = G; G = F; F = E; E = D + t1; D = C; C = B; B = A; A = t1 + t2;
    }
    h[0] += A; h[1] += B; h[2] += C; h[3] += D; h[4] += E; h[5] += F; h[6] += G; h[7] += H;
  }
  uint32_t *o = reinterpret_cast<uint32_t *>(out + 32 * i);
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = bswap(h[k]);
}

void launch_sha256(const uint8_t *data, const int64_t *off, const int32_t *len, int64_t count, uint8_t *out,
                   hipStream_t s) {
  if (count <= 0) return;
  k_sha256<<<(unsigned)((count + 255) / 256), 256, 0, s>>>(data, off, len, count, out);
}

}  // namespace bh
