// int8 MFMA issue rate with fewer v_perms per MFMA (probe for the exact GEMM's digit-half layout):
// v_mfma_i32_16x16x64_i8 back to back, 2 waves per SIMD, each wave R row blocks x SD digits of accumulators
// (R x SD x 4 registers), one B fragment (4 v_perms) per digit shared by the R row blocks:
//   R = 4, SD = 9: the shipped kernel's ratio (1 v_perm per MFMA); R = 8, SD = 5: the digit-half kernel (1/2).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_i8_rate_dh.hip -o tools/mfma_i8_rate_dh
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int R, int SD, bool PERM>
__global__ void __launch_bounds__(256, 2) rate(int* out, int iters, unsigned seed, long long* clk) {
  unsigned x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return (int)(x & 0x3F3F3F3F); };
  i32x4 af[R], bf, w1, w2;
  for (int m = 0; m < R; m++) af[m] = (i32x4){rnd(), rnd(), rnd(), rnd()};
  bf = (i32x4){rnd() & 0x0C0C0C0C, rnd() & 0x07070707, rnd() & 0x03030303, rnd() & 0x04040404};
  w1 = (i32x4){rnd(), rnd(), rnd(), rnd()};
  w2 = (i32x4){rnd(), rnd(), rnd(), rnd()};
  i32x4 acc[SD][R];
  for (int s = 0; s < SD; s++)
    for (int m = 0; m < R; m++) acc[s][m] = (i32x4){0, 0, 0, 0};
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int s = 0; s < SD; s++) {
      i32x4 bs = bf;
      if (PERM) {
#pragma unroll
        for (int e = 0; e < 4; e++) bs[e] = (int)__builtin_amdgcn_perm((unsigned)w1[e], (unsigned)w2[e], (unsigned)bf[e]);
        w1 = w1 + 1;
      }
#pragma unroll
      for (int m = 0; m < R; m++) acc[s][m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[m], bs, acc[s][m], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int s = 0;
  for (int k = 0; k < SD; k++)
    for (int m = 0; m < R; m++) s += acc[k][m][0] + acc[k][m][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && clk) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int R, int SD, bool PERM>
void run(int blocks, int* out, long long* clk) {
  const int threads = 256, iters = 20000 * 36 / (R * SD);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(a));
    rate<R, SD, PERM><<<blocks, threads>>>(out, iters, 12345 + rep, clk);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double ops = (double)blocks * 4 * iters * (double)(R * SD) * 16 * 16 * 64 * 2;
    long long h[2];
    CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    printf("{\"R\": %d, \"SD\": %d, \"perm\": %d, \"rep\": %d, \"ms\": %.3f, \"tops\": %.1f, \"clock_ghz_block0\": %.3f}\n",
           R, SD, (int)PERM, rep, ms, ops / (ms * 1e-3) / 1e12, (double)h[0] / (double)h[1] * 0.1);
  }
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = cus * 2;
  int* out;
  long long* clk;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CK(hipMalloc(&clk, (size_t)blocks * 16));
  run<4, 9, false>(blocks, out, clk);
  run<4, 9, true>(blocks, out, clk);
  run<8, 5, false>(blocks, out, clk);
  run<8, 5, true>(blocks, out, clk);
  run<8, 4, true>(blocks, out, clk);
  return 0;
}
