// Microbenchmark + layout check for v_mfma_f64_16x16x4_f64 on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_probe.hip -o tools/mfma_f64_probe
// Prints the measured back-to-back f64 MFMA and f64 VALU FMA rates (TFLOP/s), which
// DESIGN.md quotes next to the 78.6 TFLOP/s datasheet peak.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__global__ void layout_kernel(const double* A, const double* B, double* C) {
  int l = threadIdx.x;
  // A is 16x4 row-major, B is 4x16 row-major
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; r++) {
    int row = (l >> 4) + 4 * r, col = l & 15;
    C[row * 16 + col] = acc[r];
  }
}

template <int NACC>
__global__ void __launch_bounds__(256) mfma_rate(double* out, int iters, double seed) {
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  d4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; i++) acc[i] = (d4){0, 0, 0, 0};
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// GEMM-shaped: 4x4 accumulators fed by 4 A and 4 B fragments per k-step (the GRM inner loop)
__global__ void __launch_bounds__(256, 2) mfma_rate_gemm(double* out, int iters, double seed) {
  double af[4], bf[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    af[i] = seed + threadIdx.x * 1e-3 + i;
    bf[i] = seed - threadIdx.x * 1e-3 - i;
  }
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = 0; b < 4; b++) acc[a][b] = (d4){0, 0, 0, 0};
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 4; b++) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      af[i] = af[i] * 0.999 + 1e-3;
      bf[i] = bf[i] * 0.999 - 1e-3;
    }
  }
  double s = 0;
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = 0; b < 4; b++) s += acc[a][b][0] + acc[a][b][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Mixed: even waves run the GEMM-shaped MFMA loop, odd waves a VALU f64 FMA loop, to see whether
// the f64 matrix and vector pipes add up on gfx950.
__global__ void __launch_bounds__(256, 2) mixed_rate(double* out, int iters_m, int iters_v, double seed, int mode) {
  const int wave = threadIdx.x >> 6;
  double s = 0;
  const bool do_mfma = (mode == 0) ? true : (mode == 1 ? false : ((wave & 1) == 0));
  if (do_mfma) {
    double af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; i++) { af[i] = seed + threadIdx.x * 1e-3 + i; bf[i] = seed - threadIdx.x * 1e-3 - i; }
    d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 4; b++) acc[a][b] = (d4){0, 0, 0, 0};
    for (int it = 0; it < iters_m; it++) {
#pragma unroll
      for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 4; b++) s += acc[a][b][0] + acc[a][b][3];
  } else {
    double x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = seed + i + threadIdx.x;
    const double m = 0.999999, c = 1e-7;
    for (int it = 0; it < iters_v; it++) {
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = fma(x[i], m, c);
    }
#pragma unroll
    for (int i = 0; i < 16; i++) s += x[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) valu_rate(double* out, int iters, double seed) {
  double x[8];
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = seed + i + threadIdx.x;
  double m = 0.999999, c = 1e-7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = fma(x[i], m, c);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  // ---- layout check with asymmetric integer data ----
  double hA[64], hB[64], hC[256], ref[256];
  for (int i = 0; i < 16; i++) for (int k = 0; k < 4; k++) hA[i * 4 + k] = i * 4 + k + 1;
  for (int k = 0; k < 4; k++) for (int j = 0; j < 16; j++) hB[k * 16 + j] = (k + 1) * 100 + j * 3 + 1;
  for (int i = 0; i < 16; i++) for (int j = 0; j < 16; j++) {
    double s = 0; for (int k = 0; k < 4; k++) s += hA[i * 4 + k] * hB[k * 16 + j];
    ref[i * 16 + j] = s;
  }
  double *dA, *dB, *dC, *dO;
  CK(hipMalloc(&dA, sizeof hA)); CK(hipMalloc(&dB, sizeof hB)); CK(hipMalloc(&dC, sizeof hC));
  CK(hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice));
  layout_kernel<<<1, 64>>>(dA, dB, dC);
  CK(hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 256; i++) bad += hC[i] != ref[i];
  printf("{\"probe\":\"layout\",\"mismatches\":%d}\n", bad);

  // ---- throughput ----
  int dev; hipDeviceProp_t prop; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&prop, dev));
  int cus = prop.multiProcessorCount;
  const int maxblocks = cus * 8;
  CK(hipMalloc(&dO, (size_t)maxblocks * 256 * sizeof(double)));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int iters = 20000;
  float ms;
  for (int rep = 0; rep < 2; rep++) {
    for (int bpc = 1; bpc <= 4; bpc *= 2) {
      int blocks = cus * bpc;  // bpc blocks of 4 waves per CU -> bpc waves / SIMD
#define RUN(NA) \
      mfma_rate<NA><<<blocks, 256>>>(dO, iters, 1.0); \
      CK(hipEventRecord(e0)); \
      mfma_rate<NA><<<blocks, 256>>>(dO, iters, 1.0); \
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); \
      CK(hipEventElapsedTime(&ms, e0, e1)); \
      printf("{\"probe\":\"mfma_f64_16x16x4\",\"waves_per_simd\":%d,\"nacc\":%d,\"tflops\":%.2f,\"ms\":%.3f}\n", \
             bpc, NA, (double)blocks * 4 * iters * NA * 2.0 * 16 * 16 * 4 / ms / 1e9, ms);
      RUN(1) RUN(4) RUN(8)
    }
    for (int bpc = 1; bpc <= 2; bpc++) {
      int blocks = cus * bpc;
      int it2 = 5000;
      mfma_rate_gemm<<<blocks, 256>>>(dO, it2, 1.0);
      CK(hipEventRecord(e0));
      mfma_rate_gemm<<<blocks, 256>>>(dO, it2, 1.0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"probe\":\"mfma_f64_gemm_4x4acc\",\"waves_per_simd\":%d,\"tflops\":%.2f,\"ms\":%.3f}\n", bpc,
             (double)blocks * 4 * it2 * 16 * 2.0 * 16 * 16 * 4 / ms / 1e9, ms);
    }
    for (int bpc = 1; bpc <= 8; bpc *= 2) {
      int blocks = cus * bpc;
      valu_rate<<<blocks, 256>>>(dO, iters, 1.0);
      CK(hipEventRecord(e0));
      valu_rate<<<blocks, 256>>>(dO, iters, 1.0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      double flops = (double)blocks * 256 * iters * 8 * 2.0;
      printf("{\"probe\":\"valu_fma_f64\",\"waves_per_simd\":%d,\"tflops\":%.2f,\"ms\":%.3f}\n", bpc, flops / ms / 1e9, ms);
    }
  }
  {
    // mixed MFMA + VALU: per wave, MFMA work = it_m*16*2048 flops, VALU work = it_v*16*2*64 flops
    const int it_m = 5000, it_v = 40000;
    const int blocks = cus * 2;
    for (int mode = 0; mode < 3; mode++) {
      mixed_rate<<<blocks, 256>>>(dO, it_m, it_v, 1.0, mode);
      CK(hipEventRecord(e0));
      mixed_rate<<<blocks, 256>>>(dO, it_m, it_v, 1.0, mode);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double wm = (double)it_m * 16 * 2048, wv = (double)it_v * 16 * 2 * 64;
      const double waves = (double)blocks * 4;
      double fl = mode == 0 ? waves * wm : (mode == 1 ? waves * wv : waves / 2 * (wm + wv));
      printf("{\"probe\":\"mixed\",\"mode\":\"%s\",\"tflops\":%.2f,\"ms\":%.3f}\n",
             mode == 0 ? "mfma_only" : (mode == 1 ? "valu_only" : "half_half"), fl / ms / 1e9, ms);
    }
  }
  return bad ? 1 : 0;
}
