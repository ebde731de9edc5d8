// kernels_ecdsa.hip -- batched ECDSA P-256 signature verification.
//
// Reference: Event.Verify() (event.go:194-209) decodes the creator's public
// key and the signature (r, s) and calls crypto.Verify -> Go's
// ecdsa.Verify(pub, hash, r, s) (crypto/utils.go:43-51), for every event
// InsertEvent receives (hashgraph.go:716-721).  SURVEY 8(f) row 2.
// ecdsa.Verify: r, s in [1, n-1]; e = the 32-byte hash as an integer (the
// P-256 order has 256 bits, so no truncation); w = s^-1 mod n;
// (x1, y1) = (e w) G + (r w) Q; valid iff the point is finite and
// x1 mod n == r.
//
// One thread per signature.  Field and scalar elements are 8 x 32-bit limbs
// in Montgomery form (CIOS multiplication, R = 2^256); points in Jacobian
// coordinates with a = -3 (dbl-2001-b) and mixed additions of the affine
// G and Q (madd-2007-bl, with its doubling / infinity cases); u1 G + u2 Q by
// Shamir's interleaving (256 doublings); inverses by Fermat exponentiation.
// Integer-only: the result is exact, checked against the generator's
// signatures and a pure-Python verify.
#include "engine.h"

namespace bh {

struct F {
  uint32_t v[8];  // little-endian limbs
};

__constant__ uint32_t EC_P[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0x00000000u,
                                 0x00000000u, 0x00000000u, 0x00000001u, 0xffffffffu};
__constant__ uint32_t EC_N[8] = {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                                 0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu};
__constant__ uint32_t EC_R2P[8] = {0x00000003u, 0x00000000u, 0xffffffffu, 0xfffffffbu,
                                   0xfffffffeu, 0xffffffffu, 0xfffffffdu, 0x00000004u};
__constant__ uint32_t EC_R2N[8] = {0xbe79eea2u, 0x83244c95u, 0x49bd6fa6u, 0x4699799cu,
                                   0x2b6bec59u, 0x2845b239u, 0xf3d95620u, 0x66e12d94u};
__constant__ uint32_t EC_GX[8] = {0x18a9143cu, 0x79e730d4u, 0x5fedb601u, 0x75ba95fcu,  // Montgomery
                                  0x77622510u, 0x79fb732bu, 0xa53755c6u, 0x18905f76u};
__constant__ uint32_t EC_GY[8] = {0xce95560au, 0xddf25357u, 0xba19e45cu, 0x8b4ab8e4u,
                                  0xdd21f325u, 0xd2e88688u, 0x25885d85u, 0x8571ff18u};
__constant__ uint32_t EC_ONEP[8] = {0x00000001u, 0x00000000u, 0x00000000u, 0xffffffffu,  // R mod p
                                    0xffffffffu, 0xffffffffu, 0xfffffffeu, 0x00000000u};
__constant__ uint32_t EC_PM2[8] = {0xfffffffdu, 0xffffffffu, 0xffffffffu, 0x00000000u,
                                   0x00000000u, 0x00000000u, 0x00000001u, 0xffffffffu};
__constant__ uint32_t EC_NM2[8] = {0xfc63254fu, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                                   0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu};
constexpr uint32_t EC_MINV_P = 0x1u, EC_MINV_N = 0xee00bc4fu;

__device__ __forceinline__ F fconst(const uint32_t *c) {
  F r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = c[i];
  return r;
}
__device__ __forceinline__ F fsmall(uint32_t x) {
  F r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = i == 0 ? x : 0u;
  return r;
}
__device__ __forceinline__ bool fzero(const F &a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i];
  return o == 0;
}
__device__ __forceinline__ bool feq(const F &a, const F &b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i] ^ b.v[i];
  return o == 0;
}
__device__ __forceinline__ bool fless(const F &a, const uint32_t *m) {  // a < m
  for (int i = 7; i >= 0; --i)
    if (a.v[i] != m[i]) return a.v[i] < m[i];
  return false;
}

// Montgomery product a b R^-1 mod m (a < R, b < m)
__device__ __noinline__ F mmul(F a, F b, const uint32_t *m, uint32_t minv) {
  uint32_t t[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) t[k] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t C = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t x = (uint64_t)a.v[j] * b.v[i] + t[j] + C;
      t[j] = (uint32_t)x;
      C = x >> 32;
    }
    uint64_t x = (uint64_t)t[8] + C;
    t[8] = (uint32_t)x;
    t[9] = (uint32_t)(x >> 32);
    const uint32_t mq = t[0] * minv;
    x = (uint64_t)mq * m[0] + t[0];
    C = x >> 32;
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      x = (uint64_t)mq * m[j] + t[j] + C;
      t[j - 1] = (uint32_t)x;
      C = x >> 32;
    }
    x = (uint64_t)t[8] + C;
    t[7] = (uint32_t)x;
    t[8] = t[9] + (uint32_t)(x >> 32);
  }
  F s, r;
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t x = (uint64_t)t[j] - m[j] - br;
    s.v[j] = (uint32_t)x;
    br = (x >> 63) & 1;
  }
  const bool ge = t[8] != 0 || br == 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = ge ? s.v[j] : t[j];
  return r;
}

__device__ __forceinline__ F pmul(const F &a, const F &b) { return mmul(a, b, EC_P, EC_MINV_P); }
__device__ __forceinline__ F psqr(const F &a) { return mmul(a, a, EC_P, EC_MINV_P); }

__device__ __noinline__ F padd(F a, F b) {  // (a + b) mod p
  F s, r;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t x = (uint64_t)a.v[j] + b.v[j] + c;
    s.v[j] = (uint32_t)x;
    c = x >> 32;
  }
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t x = (uint64_t)s.v[j] - EC_P[j] - br;
    r.v[j] = (uint32_t)x;
    br = (x >> 63) & 1;
  }
  const bool ge = c != 0 || br == 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = ge ? r.v[j] : s.v[j];
  return r;
}

__device__ __noinline__ F psub(F a, F b) {  // (a - b) mod p
  F s, r;
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t x = (uint64_t)a.v[j] - b.v[j] - br;
    s.v[j] = (uint32_t)x;
    br = (x >> 63) & 1;
  }
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t x = (uint64_t)s.v[j] + EC_P[j] + c;
    r.v[j] = (uint32_t)x;
    c = x >> 32;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) r.v[j] = br ? r.v[j] : s.v[j];
  return r;
}

// a^e in Montgomery form (e: constant exponent limbs), MSB first
__device__ F mpow(F a, const uint32_t *e, const uint32_t *m, uint32_t minv, F one) {
  F r = one;
  for (int i = 255; i >= 0; --i) {
    r = mmul(r, r, m, minv);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = mmul(r, a, m, minv);
  }
  return r;
}

struct J {
  F x, y, z;  // Jacobian, Montgomery; z == 0: infinity
};

__device__ J pdbl(const J &p) {
  const F delta = psqr(p.z), gamma = psqr(p.y), beta = pmul(p.x, gamma);
  const F t2 = pmul(psub(p.x, delta), padd(p.x, delta));
  const F alpha = padd(padd(t2, t2), t2);
  const F b2 = padd(beta, beta), b4 = padd(b2, b2), b8 = padd(b4, b4);
  J r;
  r.x = psub(psqr(alpha), b8);
  r.z = psub(psub(psqr(padd(p.y, p.z)), gamma), delta);
  const F gg = psqr(gamma), g2 = padd(gg, gg), g4 = padd(g2, g2), g8 = padd(g4, g4);  // 8 gamma^2
  r.y = psub(pmul(alpha, psub(b4, r.x)), g8);
  return r;
}

__device__ J pmadd(const J &p, const F &x2, const F &y2) {
  if (fzero(p.z)) return J{x2, y2, fconst(EC_ONEP)};
  const F z1z1 = psqr(p.z);
  const F u2 = pmul(x2, z1z1);
  const F s2 = pmul(y2, pmul(p.z, z1z1));
  const F h = psub(u2, p.x), rr = psub(s2, p.y);
  if (fzero(h)) {
    if (fzero(rr)) return pdbl(p);
    return J{fconst(EC_ONEP), fconst(EC_ONEP), fsmall(0)};
  }
  const F hh = psqr(h), hh2 = padd(hh, hh), i4 = padd(hh2, hh2);
  const F jj = pmul(h, i4), r2 = padd(rr, rr), v = pmul(p.x, i4);
  J r;
  r.x = psub(psub(psqr(r2), jj), padd(v, v));
  const F y1j = pmul(p.y, jj);
  r.y = psub(pmul(r2, psub(v, r.x)), padd(y1j, y1j));
  r.z = psub(psub(psqr(padd(p.z, h)), z1z1), hh);
  return r;
}

__device__ __forceinline__ F load_be(const uint8_t *b) {  // 32 big-endian bytes
  F r;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint8_t *q = b + 28 - 4 * i;
    r.v[i] = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  }
  return r;
}

// hash / r / s: 32 B big-endian per signature; key[i] selects the public
// key pub[key][0..64) = x || y big-endian; ok[i] = 1 if it verifies
__global__ __launch_bounds__(128) void k_ecdsa_verify(const uint8_t *hash, const uint8_t *sr, const uint8_t *ss,
                                                      const int32_t *key, const uint8_t *pub, int64_t count,
                                                      uint8_t *ok) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const F e = load_be(hash + 32 * i), r = load_be(sr + 32 * i), s = load_be(ss + 32 * i);
  const uint8_t *pk = pub + 64 * (int64_t)key[i];
  const F qx = load_be(pk), qy = load_be(pk + 32);
  bool valid = !fzero(r) && !fzero(s) && fless(r, EC_N) && fless(s, EC_N);
  if (valid) {
    const F one_n = mmul(fconst(EC_R2N), fsmall(1), EC_N, EC_MINV_N);  // R mod n
    const F sm = mmul(s, fconst(EC_R2N), EC_N, EC_MINV_N);             // s R
    const F wm = mpow(sm, EC_NM2, EC_N, EC_MINV_N, one_n);             // s^-1 R
    const F u1 = mmul(e, wm, EC_N, EC_MINV_N), u2 = mmul(r, wm, EC_N, EC_MINV_N);  // plain form
    const F qxm = pmul(qx, fconst(EC_R2P)), qym = pmul(qy, fconst(EC_R2P));
    const F gx = fconst(EC_GX), gy = fconst(EC_GY);
    J acc{fconst(EC_ONEP), fconst(EC_ONEP), fsmall(0)};
    for (int b = 255; b >= 0; --b) {
      acc = pdbl(acc);
      if ((u1.v[b >> 5] >> (b & 31)) & 1u) acc = pmadd(acc, gx, gy);
      if ((u2.v[b >> 5] >> (b & 31)) & 1u) acc = pmadd(acc, qxm, qym);
    }
    if (fzero(acc.z)) {
      valid = false;
    } else {
      const F zi = mpow(acc.z, EC_PM2, EC_P, EC_MINV_P, fconst(EC_ONEP));
      F x = pmul(pmul(acc.x, psqr(zi)), fsmall(1));  // affine x, plain form
      if (!fless(x, EC_N)) {                         // x mod n (x < p < 2n)
        uint64_t br = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint64_t t = (uint64_t)x.v[j] - EC_N[j] - br;
          x.v[j] = (uint32_t)t;
          br = (t >> 63) & 1;
        }
      }
      valid = feq(x, r);
    }
  }
  ok[i] = valid ? 1 : 0;
}

void launch_ecdsa_verify(const uint8_t *hash, const uint8_t *r, const uint8_t *s, const int32_t *key,
                         const uint8_t *pub, int64_t count, uint8_t *ok, hipStream_t st) {
  if (count <= 0) return;
  k_ecdsa_verify<<<(unsigned)((count + 127) / 128), 128, 0, st>>>(hash, r, s, key, pub, count, ok);
}

}  // namespace bh
