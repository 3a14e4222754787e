// Probe (timing only, not part of libgbm): the GRM tile loop's MFMA rate with operands streamed from HBM, for
// the shipped shape — 128 x 128 tiles, two workgroups per CU, BK = 16 loci per LDS stage, two stages — against
// a 128 x 256 tile on one workgroup per CU (each wave 64 x 128, 32 accumulators in AGPRs) with a three-stage
// LDS ring (48 KB per stage), i.e. half the barriers per MFMA and 25 % fewer operand bytes per MFMA.
// Build: hipcc --offload-arch=gfx950 -O3 tools/syrk_tile_probe.hip -o tools/syrk_tile_probe
// Run:   tools/syrk_tile_probe [p=50000] [reps=5]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);       \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

constexpr int NCOL = 5120;  // Zt row length (individuals)
constexpr int BK = 16;
constexpr int LROW = 130;

// ---- the shipped shape (tile_pass, grm.hip): 128 x 128, 2 stages, 2 workgroups per CU
__global__ void __launch_bounds__(256, 2) tile128(const double* __restrict__ U, int64_t K, double* out) {
  __shared__ __attribute__((aligned(16))) double lds[2 * 2 * BK * LROW];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1, fr = lane >> 4, fc = lane & 15;
  const int64_t i0 = (blockIdx.x % 40) * 128, j0 = ((blockIdx.x / 40) % 40) * 128;
  constexpr int STAGE = 2 * BK * LROW;
  auto stage_rows = [&](int64_t st, int buf) {
#pragma unroll
    for (int rr = 0; rr < BK / 4; rr++) {
      const int r = wave * (BK / 4) + rr;
      const double* src = U + (st * BK + r) * NCOL;
      __builtin_amdgcn_global_load_lds((const void*)(src + i0 + lane * 2), (void*)(lds + buf * STAGE + r * LROW), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(src + j0 + lane * 2), (void*)(lds + buf * STAGE + (BK + r) * LROW), 16, 0, 0);
    }
  };
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = 0; b < 4; b++) acc[a][b] = (d4){0, 0, 0, 0};
  const int64_t nst = K / BK;
  stage_rows(0, 0);
  __syncthreads();
  for (int64_t st = 0; st < nst; st++) {
    const int buf = (int)(st & 1);
    if (st + 1 < nst) stage_rows(st + 1, buf ^ 1);
    const double* A = lds + buf * STAGE;
    const double* B = A + BK * LROW;
#pragma unroll
    for (int ks = 0; ks < BK / 4; ks++) {
      const int kr = ks * 4 + fr;
      const double2 a01 = *reinterpret_cast<const double2*>(&A[kr * LROW + wm * 64 + 4 * fc]);
      const double2 a23 = *reinterpret_cast<const double2*>(&A[kr * LROW + wm * 64 + 4 * fc + 2]);
      const double2 b01 = *reinterpret_cast<const double2*>(&B[kr * LROW + wn * 64 + 4 * fc]);
      const double2 b23 = *reinterpret_cast<const double2*>(&B[kr * LROW + wn * 64 + 4 * fc + 2]);
      const double af[4] = {a01.x, a01.y, a23.x, a23.y}, bf[4] = {b01.x, b01.y, b23.x, b23.y};
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int m = 0; m < 4; m++)
#pragma unroll
        for (int q = 0; q < 4; q++) acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[q], acc[m][q], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
  }
  if (K < 0) {
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 4; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) out[((a * 4 + b) * 4 + r) * 256 + threadIdx.x] = acc[a][b][r];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0][0][0];
}

// ---- 128 x 256 on one workgroup per CU: wave (wm, wn) owns rows 64 wm.., columns 128 wn.. (two 64-column halves,
// each read like the shipped B fragments); a 3-stage ring, stage s + 2 issued after the barrier that ends s − 1
constexpr int BROW = 258;
__global__ void __launch_bounds__(256, 1) tile256(const double* __restrict__ U, int64_t K, double* out) {
  constexpr int SA = BK * LROW, SB = BK * BROW, STAGE = SA + SB;
  __shared__ __attribute__((aligned(16))) double lds[3 * STAGE];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1, fr = lane >> 4, fc = lane & 15;
  const int64_t i0 = (blockIdx.x % 40) * 128, j0 = ((blockIdx.x / 40) % 20) * 256;
  // 16 k-rows x (1 KB of A + 2 KB of B) per stage = 48 pieces of 1 KB, 12 per wave
  auto stage_rows = [&](int64_t st, int buf) {
    double* base = lds + buf * STAGE;
#pragma unroll
    for (int rr = 0; rr < BK / 4; rr++) {
      const int r = wave * (BK / 4) + rr;
      const double* src = U + (st * BK + r) * NCOL;
      __builtin_amdgcn_global_load_lds((const void*)(src + i0 + lane * 2), (void*)(base + r * LROW), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(src + j0 + lane * 2), (void*)(base + SA + r * BROW), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(src + j0 + 128 + lane * 2), (void*)(base + SA + r * BROW + 128), 16,
                                       0, 0);
    }
  };
  d4 acc[4][8];
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = 0; b < 8; b++) acc[a][b] = (d4){0, 0, 0, 0};
  const int64_t nst = K / BK;
  stage_rows(0, 0);
  if (nst > 1) stage_rows(1, 1);
  for (int64_t st = 0; st < nst; st++) {
    // stage st landed for this wave (stage st + 1's 12 pieces may stay in flight), then for every wave
    if (st + 1 < nst) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (st + 2 < nst) stage_rows(st + 2, (int)((st + 2) % 3));
    const double* A = lds + (st % 3) * STAGE;
    const double* B = A + SA;
    // fragments of k-step ks + 1 read before k-step ks's MFMAs (one wave per SIMD: nothing else hides the
    // LDS latency)
    double af[2][4], bf[2][8];
    auto frag = [&](int ks, double (&a)[4], double (&b)[8]) {
      const int kr = ks * 4 + fr;
      const double2 a01 = *reinterpret_cast<const double2*>(&A[kr * LROW + wm * 64 + 4 * fc]);
      const double2 a23 = *reinterpret_cast<const double2*>(&A[kr * LROW + wm * 64 + 4 * fc + 2]);
      const double2 b01 = *reinterpret_cast<const double2*>(&B[kr * BROW + wn * 128 + 4 * fc]);
      const double2 b23 = *reinterpret_cast<const double2*>(&B[kr * BROW + wn * 128 + 4 * fc + 2]);
      const double2 b45 = *reinterpret_cast<const double2*>(&B[kr * BROW + wn * 128 + 64 + 4 * fc]);
      const double2 b67 = *reinterpret_cast<const double2*>(&B[kr * BROW + wn * 128 + 64 + 4 * fc + 2]);
      a[0] = a01.x, a[1] = a01.y, a[2] = a23.x, a[3] = a23.y;
      b[0] = b01.x, b[1] = b01.y, b[2] = b23.x, b[3] = b23.y, b[4] = b45.x, b[5] = b45.y, b[6] = b67.x, b[7] = b67.y;
    };
    frag(0, af[0], bf[0]);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ks++) {
      if (ks + 1 < BK / 4) frag(ks + 1, af[(ks + 1) & 1], bf[(ks + 1) & 1]);
#pragma unroll
      for (int m = 0; m < 4; m++)
#pragma unroll
        for (int q = 0; q < 8; q++)
          acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[ks & 1][m], bf[ks & 1][q], acc[m][q], 0, 0, 0);
    }
  }
  // every accumulator stored (only when K < 0, never: the MFMAs must stay live without a reduction tree
  // holding extra registers)
  if (K < 0) {
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 8; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) out[((a * 8 + b) * 4 + r) * 256 + threadIdx.x] = acc[a][b][r];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0][0][0];
}

int main(int argc, char** argv) {
  const int64_t p = argc > 1 ? atoll(argv[1]) : 50000;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  double *U = nullptr, *out = nullptr;
  CK(hipMalloc((void**)&U, (size_t)p * NCOL * 8));
  CK(hipMalloc((void**)&out, (size_t)2 * cus * 256 * 8));
  CK(hipMemset(U, 0x3F, (size_t)p * NCOL * 8));  // every double ≈ 0.496
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double flops = 2.0 * cus * 128.0 * 256.0 * (double)p;  // both launches: cus x 128 x 256 outputs over p
  for (int variant = 0; variant < 2; variant++) {
    std::vector<float> ts;
    for (int r = 0; r <= reps; r++) {
      CK(hipEventRecord(a, 0));
      if (variant == 0) tile128<<<2 * cus, 256>>>(U, p, out);
      else tile256<<<cus, 256>>>(U, p, out);
      CK(hipGetLastError());
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r) ts.push_back(ms);
    }
    float best = ts[0];
    for (float t : ts) best = t < best ? t : best;
    printf("{\"probe\": \"%s\", \"p\": %lld, \"ms\": %.3f, \"tflops\": %.2f}\n", variant ? "tile256_1wg_3stage" : "tile128_2wg_2stage",
           (long long)p, best, flops / best / 1e9);
  }
  return 0;
}
