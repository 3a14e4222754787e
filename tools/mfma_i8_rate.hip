// Measured int8 MFMA rate on gfx950 (the exact GRM's roofline reference):
// v_mfma_i32_16x16x64_i8 back to back on register operands (random bytes), 2 waves per SIMD, with the
// exact GEMM's accumulator count (36 = 9 slices x 4), without and with its one v_perm per MFMA.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_i8_rate.hip -o tools/mfma_i8_rate ; run: tools/mfma_i8_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <bool PERM>
__global__ void __launch_bounds__(256, 2) rate(int* out, int iters, unsigned seed, long long* clk) {
  unsigned x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return (int)(x & 0x3F3F3F3F); };
  i32x4 af[4], bf, w1, w2;
  for (int m = 0; m < 4; m++) af[m] = (i32x4){rnd(), rnd(), rnd(), rnd()};
  bf = (i32x4){rnd() & 0x0C0C0C0C, rnd() & 0x07070707, rnd() & 0x03030303, rnd() & 0x04040404};
  w1 = (i32x4){rnd(), rnd(), rnd(), rnd()};
  w2 = (i32x4){rnd(), rnd(), rnd(), rnd()};
  i32x4 acc[9][4];
  for (int s = 0; s < 9; s++)
    for (int m = 0; m < 4; m++) acc[s][m] = (i32x4){0, 0, 0, 0};
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int s = 0; s < 9; s++) {
      i32x4 bs = bf;
      if (PERM) {
#pragma unroll
        for (int e = 0; e < 4; e++) bs[e] = (int)__builtin_amdgcn_perm((unsigned)w1[e], (unsigned)w2[e], (unsigned)bf[e]);
        w1 = w1 + 1;  // keeps the perms in the loop
      }
#pragma unroll
      for (int m = 0; m < 4; m++) acc[s][m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[m], bs, acc[s][m], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int s = 0;
  for (int k = 0; k < 9; k++)
    for (int m = 0; m < 4; m++) s += acc[k][m][0] + acc[k][m][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && clk) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = cus * 2, threads = 256, iters = 20000;
  int* out;
  long long* clk;
  CK(hipMalloc(&out, (size_t)blocks * threads * 4));
  CK(hipMalloc(&clk, (size_t)blocks * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int perm = 0; perm < 2; perm++) {
    for (int rep = 0; rep < 3; rep++) {
      CK(hipEventRecord(a));
      if (perm) rate<true><<<blocks, threads>>>(out, iters, 12345 + rep, clk);
      else rate<false><<<blocks, threads>>>(out, iters, 12345 + rep, clk);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double ops = (double)blocks * 4 /*waves*/ * iters * 36.0 * 16 * 16 * 64 * 2;
      long long h[2];
      CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
      const double ghz = (double)h[0] / (double)h[1] * 0.1;  // memrealtime ticks at 100 MHz
      printf("{\"perm\": %d, \"rep\": %d, \"ms\": %.3f, \"tops\": %.1f, \"clock_ghz_block0\": %.3f}\n", perm, rep, ms,
             ops / (ms * 1e-3) / 1e12, ghz);
    }
  }
  return 0;
}
