// Marker back-solve and linear predictor (HBM-bound GEMV streams over the locus rows).
//   B[t, j] = (z_j · a_t) / (q s_j)  — Fit.b_hat (pattern of reference src/linear.jl:218-221)
//   msum[t] = Σ_j m_j B[t, j]        — b0 = μ̂ − msum makes `predict` exact
//   out[t, i] = b0_t + Σ_j X[i, j] b_t[j]   — reference src/prediction.jl:228
#include <type_traits>

#include "gbm_internal.h"

namespace gbm {

// The streamed fit's rows: int8 dosages, z = (d·xs − m)·r rebuilt exactly as the standardisation
// computed it (x rounded on its own, r = 1/s), so B is bit-identical to the fp64-Z kernel's.
__device__ __forceinline__ double dosage_z(int8_t d, double xs, double m, double r) {
#pragma clang fp contract(off)
  const double x = (double)d * xs;
  return (x - m) * r;
}

// R locus rows per wave (round 6); each lane takes four consecutive individuals per pass, i = 4·lane + 256·k
// (T = double: the standardised row, two 16-byte loads; T = int8_t: the dosage row, one 4-byte load, z rebuilt in
// registers), and the trait vectors' values for them are loaded once for the wave's R rows. Every row is summed in
// the same order whatever R and T — per lane fma(z_i, a_i, ·) over its individuals in order, then an xor-shuffle
// tree — so B is bit-identical between the fp64 rows and the dosage bytes. Up to 4 traits per pass over the rows.
// (Round 5 ran one row per wave with 2 individuals per lane: the int8 variant issued two byte loads per lane per
// 128 individuals and re-read the trait vector from L2 for every locus, 0.29 ms at C2 for 250 MB of bytes.)
// rows per wave of the dosage-byte and fp64 variants (timing variants: tools/build_effects_variants.sh; C2 exact
// path, single trait: 0.31 ms in round 5, R = 4 0.26, R = 2 0.19, R = 1 0.19 ms; the fp64 rows are HBM-bound at
// ≈ 5.5 TB/s, 0.365 ms, whatever R)
#ifndef GBM_EFF_R_I8
#define GBM_EFF_R_I8 2
#endif
#ifndef GBM_EFF_R_F64
#define GBM_EFF_R_F64 1
#endif
#ifndef GBM_EFF_UNROLL
#define GBM_EFF_UNROLL 1  // passes of the individuals loop unrolled (loads of the next pass in flight)
#endif
template <typename T, int R, int TU>  // TU: traits per pass over the rows (1: the single-trait fit, fewer registers)
__global__ void __launch_bounds__(256) marker_effects_kernel(const T* __restrict__ Zt, int64_t ldz, int64_t p,
                                                             int64_t n, const double* __restrict__ A, int64_t lda,
                                                             int64_t nrhs, double inv_q,
                                                             const int64_t* __restrict__ q_dev,
                                                             const double* __restrict__ mean,
                                                             const double* __restrict__ sd,
                                                             const int32_t* __restrict__ keep,
                                                             double* __restrict__ B, int64_t ldb, double xs) {
  constexpr bool kI8 = std::is_same<T, int8_t>::value;
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  if (q_dev) inv_q = 1.0 / (double)(*q_dev);
  for (int64_t j0 = wave_g * R; j0 < p; j0 += nwaves * R) {
    const T* z[R];
    bool kp[R], any = false;
    double m[R], r[R];
#pragma unroll
    for (int q = 0; q < R; q++) {
      const int64_t j = j0 + q < p ? j0 + q : p - 1;  // (a row past p repeats the last one; never stored)
      z[q] = Zt + j * ldz;
      kp[q] = j0 + q < p && keep[j] != 0;
      any |= kp[q];
      m[q] = kI8 ? mean[j] : 0.0;
      r[q] = kI8 && kp[q] ? 1.0 / sd[j] : 0.0;
    }
    for (int64_t t0 = 0; t0 < nrhs; t0 += TU) {
      double acc[R][TU];
#pragma unroll
      for (int q = 0; q < R; q++)
#pragma unroll
        for (int u = 0; u < TU; u++) acc[q][u] = 0.0;
      if (any) {
#pragma unroll GBM_EFF_UNROLL
        for (int64_t i = (int64_t)lane * 4; i < n; i += 256) {
          const bool whole = i + 4 <= n;
          double zv[R][4];
#pragma unroll
          for (int q = 0; q < R; q++) {
            if constexpr (kI8) {
              const int8_t* zr = z[q] + i;
              int8_t d[4];
              if (whole && ((uintptr_t)zr & 3) == 0) {
                const uint32_t w = *reinterpret_cast<const uint32_t*>(zr);
#pragma unroll
                for (int e = 0; e < 4; e++) d[e] = (int8_t)(w >> (8 * e));
              } else {
#pragma unroll
                for (int e = 0; e < 4; e++) d[e] = i + e < n ? zr[e] : 0;
              }
#pragma unroll
              for (int e = 0; e < 4; e++) zv[q][e] = i + e < n ? dosage_z(d[e], xs, m[q], r[q]) : 0.0;
            } else {
              const double* zr = z[q] + i;
              if (whole) {
                const double2 v0 = *reinterpret_cast<const double2*>(zr);
                const double2 v1 = *reinterpret_cast<const double2*>(zr + 2);
                zv[q][0] = v0.x;
                zv[q][1] = v0.y;
                zv[q][2] = v1.x;
                zv[q][3] = v1.y;
              } else {
#pragma unroll
                for (int e = 0; e < 4; e++) zv[q][e] = i + e < n ? zr[e] : 0.0;
              }
            }
          }
#pragma unroll
          for (int u = 0; u < TU; u++)
            if (t0 + u < nrhs) {
              const double* ar = A + (t0 + u) * lda + i;
              double av[4];
              if (whole) {
                const double2 a0 = *reinterpret_cast<const double2*>(ar);
                const double2 a1 = *reinterpret_cast<const double2*>(ar + 2);
                av[0] = a0.x;
                av[1] = a0.y;
                av[2] = a1.x;
                av[3] = a1.y;
              } else {
#pragma unroll
                for (int e = 0; e < 4; e++) av[e] = i + e < n ? ar[e] : 0.0;
              }
#pragma unroll
              for (int q = 0; q < R; q++)
#pragma unroll
                for (int e = 0; e < 4; e++) acc[q][u] = __builtin_fma(zv[q][e], av[e], acc[q][u]);
            }
        }
      }
#pragma unroll
      for (int q = 0; q < R; q++)
#pragma unroll
        for (int u = 0; u < TU; u++) {
          double v = acc[q][u];
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
          if (lane == 0 && t0 + u < nrhs && j0 + q < p) B[(t0 + u) * ldb + j0 + q] = kp[q] ? v * inv_q / sd[j0 + q] : 0.0;
        }
    }
  }
}

// msum[t] = Σ_j mean_j B[t, j]: one workgroup per trait, fixed reduction order. Each thread's terms j = tid,
// tid + 1024, ... are added in that order; their loads are issued WS at a time instead of one per term: same bits,
// C2 effects stage 0.366 → 0.360 ms fp64, 0.189 → 0.185 ms exact (profiles/r06_wsum_batch_ab.txt)
#ifndef GBM_WSUM_BATCH
#define GBM_WSUM_BATCH 8
#endif
__global__ void __launch_bounds__(1024) weighted_sum_kernel(const double* __restrict__ mean,
                                                            const double* __restrict__ B, int64_t ldb, int64_t p,
                                                            double* __restrict__ msum) {
  constexpr int WS = GBM_WSUM_BATCH;
  __shared__ double red[16];
  const int64_t t = blockIdx.x;
  double s = 0.0;
  for (int64_t j0 = threadIdx.x; j0 < p; j0 += 1024 * WS) {
    double mv[WS], bv[WS];
#pragma unroll
    for (int u = 0; u < WS; u++) {
      const int64_t j = j0 + (int64_t)u * 1024;
      mv[u] = j < p ? mean[j] : 0.0;
      bv[u] = j < p ? B[t * ldb + j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < WS; u++)
      if (j0 + (int64_t)u * 1024 < p) s += mv[u] * bv[u];
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int w = 0; w < 16; w++) tot += red[w];
    msum[t] = tot;
  }
}

// partial[c, t, i] = Σ_{j in chunk c} Xt[j, i] b_t[j]
__global__ void __launch_bounds__(256) predict_partial_kernel(const double* __restrict__ Xt, int64_t ldx, int64_t p,
                                                              int64_t n, const double* __restrict__ b,
                                                              int64_t ldb, int64_t nrhs, int64_t chunk,
                                                              double* __restrict__ partial) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t c = blockIdx.y;
  const int64_t j0 = c * chunk;
  const int64_t j1 = j0 + chunk < p ? j0 + chunk : p;
  for (int64_t t0 = 0; t0 < nrhs; t0 += 4) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (i < n) {
      for (int64_t j = j0; j < j1; j++) {
        const double x = Xt[j * ldx + i];
#pragma unroll
        for (int u = 0; u < 4; u++)
          if (t0 + u < nrhs) acc[u] += x * b[(t0 + u) * ldb + 1 + j];
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (t0 + u < nrhs) partial[(c * nrhs + t0 + u) * n + i] = acc[u];
    }
  }
}

__global__ void __launch_bounds__(256) predict_reduce_kernel(const double* __restrict__ partial, int64_t nchunks,
                                                             int64_t n, const double* __restrict__ b, int64_t ldb,
                                                             int64_t nrhs, double* __restrict__ out, int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t t = blockIdx.y;
  if (i >= n) return;
  double s = 0.0;
  for (int64_t c = 0; c < nchunks; c++) s += partial[(c * nrhs + t) * n + i];
  out[t * ldo + i] = b[t * ldb] + s;
}

int launch_predict(const double* Xt, int64_t ldx, int64_t p, int64_t n, const double* b, int64_t ldb, int64_t nrhs,
                   double* partial, int64_t nchunks, double* out, int64_t ldo, hipStream_t s) {
  const int64_t chunk = (p + nchunks - 1) / nchunks;
  const unsigned gx = (unsigned)((n + 255) / 256);
  predict_partial_kernel<<<dim3(gx, (unsigned)nchunks), 256, 0, s>>>(Xt, ldx, p, n, b, ldb, nrhs, chunk, partial);
  GBM_LAUNCH_CHECK();
  predict_reduce_kernel<<<dim3(gx, (unsigned)nrhs), 256, 0, s>>>(partial, nchunks, n, b, ldb, nrhs, out, ldo);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// B rows of p loci (rows of Zt: standardised fp64, ldz even) / msum = Σ_j mean_j B[t, j] (in a
// separate launch, so a streamed fit computes B chunk by chunk and msum once over all its loci).
int launch_marker_rows(const double* Zt, int64_t ldz, int64_t p, int64_t n, const double* A, int64_t lda, int64_t nrhs,
                       double inv_q, const int64_t* q_dev, const double* sd, const int32_t* keep, double* B,
                       int64_t ldb, hipStream_t s) {
  if (p < 1) return GBM_OK;
  constexpr int R = GBM_EFF_R_F64;  // rows per wave (the trait vector's loads shared by them)
  const int64_t groups = (p + R - 1) / R, blocks = (groups + 3) / 4 < 8192 ? (groups + 3) / 4 : 8192;
  if (nrhs == 1)
    marker_effects_kernel<double, R, 1><<<(unsigned)blocks, 256, 0, s>>>(Zt, ldz, p, n, A, lda, nrhs, inv_q, q_dev,
                                                                         nullptr, sd, keep, B, ldb, 1.0);
  else
    marker_effects_kernel<double, R, 4><<<(unsigned)blocks, 256, 0, s>>>(Zt, ldz, p, n, A, lda, nrhs, inv_q, q_dev,
                                                                         nullptr, sd, keep, B, ldb, 1.0);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

int launch_marker_rows_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, const double* A, int64_t lda,
                          int64_t nrhs, double inv_q, const int64_t* q_dev, const double* mean, const double* sd,
                          const int32_t* keep, double* B, int64_t ldb, hipStream_t s) {
  if (p < 1) return GBM_OK;
  constexpr int R = GBM_EFF_R_I8;
  const int64_t groups = (p + R - 1) / R, blocks = (groups + 3) / 4 < 8192 ? (groups + 3) / 4 : 8192;
  if (nrhs == 1)
    marker_effects_kernel<int8_t, R, 1><<<(unsigned)blocks, 256, 0, s>>>(D, ldd, p, n, A, lda, nrhs, inv_q, q_dev, mean,
                                                                         sd, keep, B, ldb, 1.0 / ploidy);
  else
    marker_effects_kernel<int8_t, R, 4><<<(unsigned)blocks, 256, 0, s>>>(D, ldd, p, n, A, lda, nrhs, inv_q, q_dev, mean,
                                                                         sd, keep, B, ldb, 1.0 / ploidy);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

int launch_weighted_sum(const double* mean, const double* B, int64_t ldb, int64_t p, int64_t nrhs, double* msum,
                        hipStream_t s) {
  weighted_sum_kernel<<<(unsigned)nrhs, 1024, 0, s>>>(mean, B, ldb, p, msum);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

int64_t predict_chunks(int64_t n, int64_t p) {
  const int64_t col_blocks = (n + 255) / 256;
  int64_t c = (2048 + col_blocks - 1) / col_blocks;
  if (c > p) c = p;
  return c < 1 ? 1 : c;
}

}  // namespace gbm

using namespace gbm;

extern "C" int gbm_dev_marker_effects(const double* Zt, int64_t ldz, int64_t p, int64_t n, const double* A,
                                      int64_t lda, int64_t nrhs, double inv_q, const int64_t* q_dev,
                                      const double* mean, const double* sd,
                                      const int32_t* keep, double* B, int64_t ldb, double* msum, void* stream) {
  if (!Zt || !A || !mean || !sd || !keep || !B || !msum || p < 1 || n < 1 || ldz < n || (ldz & 1) ||
      lda < ldz || (lda & 1) || nrhs < 1 || ldb < p || !(q_dev || inv_q > 0.0))
    return fail(GBM_E_ARG, "gbm_dev_marker_effects: bad arguments (need ldz >= n even, lda >= ldz even, ldb >= p)");
  hipStream_t s = (hipStream_t)stream;
  GBM_TRY(launch_marker_rows(Zt, ldz, p, n, A, lda, nrhs, inv_q, q_dev, sd, keep, B, ldb, s));
  return launch_weighted_sum(mean, B, ldb, p, nrhs, msum, s);
}

extern "C" int gbm_dev_marker_effects_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy,
                                         const double* A, int64_t lda, int64_t nrhs, double inv_q,
                                         const int64_t* q_dev, const double* mean, const double* sd,
                                         const int32_t* keep, double* B, int64_t ldb, double* msum, void* stream) {
  if (!D || !A || !mean || !sd || !keep || !B || !msum || p < 1 || n < 1 || ldd < n || ploidy < 1 ||
      lda < gbm::npad_of(n) || (lda & 1) || nrhs < 1 || ldb < p || !(q_dev || inv_q > 0.0))
    return fail(GBM_E_ARG, "gbm_dev_marker_effects_i8: bad arguments (need ldd >= n, lda >= npad(n) even, ldb >= p)");
  hipStream_t s = (hipStream_t)stream;
  GBM_TRY(launch_marker_rows_i8(D, ldd, p, n, ploidy, A, lda, nrhs, inv_q, q_dev, mean, sd, keep, B, ldb, s));
  return launch_weighted_sum(mean, B, ldb, p, nrhs, msum, s);
}
