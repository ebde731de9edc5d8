// Micro-benchmark: issue/latency of a lone wave on gfx950 (VALU dependent
// chains, independent VALU, LDS pointer chasing).  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long *out, int iters, int seed) {
  __shared__ int lds[4096];
  const int t = threadIdx.x;
  for (int i = t; i < 4096; i += blockDim.x) lds[i] = (i * 7 + 1) & 4095;
  __syncthreads();
  if (t >= 64) return;
  int v = seed + t, w = seed * 3 + t, x = t, y = t + 5, z = t + 9;
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {  // 8 dependent VALU
    v += 0x9E37; v ^= v >> 3; v += t; v ^= v >> 2;
    v += 0x9E37; v ^= v >> 3; v += t; v ^= v >> 2;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {  // 4 independent chains x 2 ops
    w ^= w >> 1; x ^= x >> 2; y ^= y >> 3; z ^= z >> 1;
  }
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  int p = t;
  for (int i = 0; i < iters; ++i) {  // LDS pointer chase
    p = lds[p]; p = lds[p]; p = lds[p]; p = lds[p];
  }
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  int q = t;
  for (int i = 0; i < iters; ++i) {  // LDS chase + 1 VALU between
    q = lds[q] + 1; q = lds[q & 4095] + 1; q = lds[q & 4095] + 1; q = lds[q & 4095] + 1; q &= 4095;
  }
  unsigned long long t4 = __builtin_amdgcn_s_memtime();
  unsigned long long r4 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    out[5] = t4 - t0; out[6] = r4 - r0;
    out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3;
  }
  if (v == 12345 && w == 1 && x == 2 && y == 3 && z == 4 && p == 77 && q == 5) out[4] = 1;
}
int main() {
  unsigned long long *o, h[8] = {0};
  (void)hipMalloc(&o, 64);
  (void)hipMemset(o, 0, 64);
  const int iters = 10000;
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, o, iters, 3);
  (void)hipMemcpy(h, o, 64, hipMemcpyDeviceToHost);
  printf("memtime MHz: %.0f\n", h[5] * 100.0 / h[6]);
  printf("dep VALU (8/iter): %.2f cyc/instr\n", h[0] / (8.0 * iters));
  printf("indep VALU (8/iter, 4 chains): %.2f cyc/instr\n", h[1] / (8.0 * iters));
  printf("LDS chase: %.1f cyc/read\n", h[2] / (4.0 * iters));
  printf("LDS chase +VALU: %.1f cyc/read\n", h[3] / (4.0 * iters));
  return 0;
}
