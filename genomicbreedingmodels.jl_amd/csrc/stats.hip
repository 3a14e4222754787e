// Locus-row streaming kernels: synthetic genotypes, int8 dosage expansion and the column
// standardisation of reference src/gwas.jl:112-115,127-130 (HBM-bound; one pass over X).
#include <type_traits>

#include "gbm_internal.h"

namespace gbm {

// ---- counter-based genotype generator (bit-identical to oracle/gbm_oracle.c) -------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// One workgroup strip of 1024 columns of one locus row per blockIdx.x; rows grid-strided on y.
__global__ void __launch_bounds__(256) synth_kernel(double* __restrict__ Xt, int64_t ldx, int64_t p,
                                                    int64_t n, uint64_t seed, int64_t j0) {
  for (int64_t j = blockIdx.y; j < p; j += gridDim.y) {
    const uint64_t base = mix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)(j0 + j));
    const uint64_t thr = 214748364ull + (((base >> 32) * 1932735283ull) >> 32);
    double* row = Xt + j * ldx;
    for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < (int64_t)(blockIdx.x + 1) * 1024 && i < ldx;
         i += 256) {
      double v = 0.0;
      if (i < n) {
        const uint64_t h = mix64(base ^ ((uint64_t)i * 0x8CB92BA72F3D8DD7ull));
        const int d = ((h & 0xFFFFFFFFull) < thr) + ((h >> 32) < thr);
        v = 0.5 * (double)d;
      }
      row[i] = v;
    }
  }
}

// The same generator's dosages d (0, 1, 2) as bytes, column-major n x p (ldd): locus j0 + j's n
// dosages at D + j*ldd. X = d/2 of synth_kernel exactly, at 1 B per cell: the device-resident input
// of the loci-streamed fit (C3 on one GPU: 30 GB instead of 240 GB of fp64).
__global__ void __launch_bounds__(256) synth_i8_kernel(int8_t* __restrict__ D, int64_t ldd, int64_t p, int64_t n,
                                                       uint64_t seed, int64_t j0) {
  for (int64_t j = blockIdx.y; j < p; j += gridDim.y) {
    const uint64_t base = mix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)(j0 + j));
    const uint64_t thr = 214748364ull + (((base >> 32) * 1932735283ull) >> 32);
    int8_t* col = D + j * ldd;
    for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < (int64_t)(blockIdx.x + 1) * 1024 && i < n;
         i += 256) {
      const uint64_t h = mix64(base ^ ((uint64_t)i * 0x8CB92BA72F3D8DD7ull));
      col[i] = (int8_t)(((h & 0xFFFFFFFFull) < thr) + ((h >> 32) < thr));
    }
  }
}

// D column-major n x p int8 (ldd) -> Xt row-major p x ldx, X = d / ploidy.
__global__ void __launch_bounds__(256) expand_i8_kernel(const int8_t* __restrict__ D, int64_t ldd,
                                                        int64_t n, int64_t p, double inv_ploidy,
                                                        double* __restrict__ Xt, int64_t ldx) {
  for (int64_t j = blockIdx.y; j < p; j += gridDim.y) {
    const int8_t* col = D + j * ldd;
    double* row = Xt + j * ldx;
    for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < (int64_t)(blockIdx.x + 1) * 1024 && i < ldx;
         i += 256)
      row[i] = i < n ? (double)col[i] * inv_ploidy : 0.0;
  }
}

// ---- standardisation ---------------------------------------------------------------------
template <int BS>
__device__ __forceinline__ double block_sum(double v, double* red) {
  // wave reduction (64 lanes) then across the BS/64 waves through LDS
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < BS / 64; k++) s += red[k];  // fixed order: deterministic
  return s;
}

// One workgroup per locus row (grid-strided). NPT = values cached in registers per thread
// (0 = generic path re-reading the row from L2/MALL). T = int8_t reads dosage rows directly,
// x = d·xs (the value expand_i8_kernel would have stored: bit-identical, without the fp64 copy).
// The dosage product d·xs is rounded on its own (never fused into the caller's x − m): the value
// expand_i8_kernel stores, so every kernel that rebuilds z from the bytes (standardise, the
// streamed marker effects) gets the same bits as one that reads the expanded fp64 row.
__device__ __forceinline__ double dosage_x(int8_t d, double xs) {
#pragma clang fp contract(off)
  return (double)d * xs;
}

// The fp64 row read and the Z row written with the nontemporal hint (GBM_STD_NT: 1 both, the default; 2 reads
// only, 3 writes only, 0 neither): X is read once and Z is next read by the GRM after 4 GB of other traffic, so
// neither is worth a cache line. C2, same bits: 0.740 → 0.699 ms (reads only 0.728, writes only 0.718), step
// 21.06 → 21.02 ms (profiles/r06_standardize_nt_ab.txt)
#ifndef GBM_STD_NT
#define GBM_STD_NT 1
#endif
template <typename T>
__device__ __forceinline__ double load_x(const T* row, int64_t i, double xs) {
  if constexpr (std::is_same<T, int8_t>::value)
    return dosage_x(row[i], xs);
  else if constexpr (GBM_STD_NT == 1 || GBM_STD_NT == 2)
    return __builtin_nontemporal_load(row + i);
  else
    return row[i];
}
__device__ __forceinline__ void store_z(double* z, double v) {
  if constexpr (GBM_STD_NT == 1 || GBM_STD_NT == 3)
    __builtin_nontemporal_store(v, z);
  else
    *z = v;
}

template <int BS, int NPT, bool GATHER, typename T>
__global__ void __launch_bounds__(BS) standardize_kernel(const T* Xt, int64_t ldx, int64_t p,
                                                         const int32_t* __restrict__ idx,
                                                         int64_t n, double* Zt, int64_t ldz,
                                                         double* __restrict__ mean,
                                                         double* __restrict__ sd, int32_t* __restrict__ keep,
                                                         unsigned long long* __restrict__ q_dev, int center_only,
                                                         double xs) {
  __shared__ double red[BS / 64];
  unsigned long long kept_local = 0;
  for (int64_t j = blockIdx.x; j < p; j += gridDim.x) {
    const T* row = Xt + j * ldx;
    double* zrow = Zt + j * ldz;  // may alias row (in place, T = double)
    double m, v;
    if constexpr (NPT > 0) {
      double x[NPT];
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < NPT; k++) {
        const int64_t i = (int64_t)k * BS + threadIdx.x;
        x[k] = i < n ? load_x(row, GATHER ? idx[i] : i, xs) : 0.0;
        s += x[k];
      }
      m = block_sum<BS>(s, red) / (double)n;
      double ss = 0.0;
#pragma unroll
      for (int k = 0; k < NPT; k++) {
        const int64_t i = (int64_t)k * BS + threadIdx.x;
        const double d = x[k] - m;
        ss += i < n ? d * d : 0.0;
      }
      v = n > 1 ? sqrt(block_sum<BS>(ss, red) / (double)(n - 1)) : __builtin_nan("");
      if (center_only) v = 1.0;  // glmnet standardize=false: centre only, keep every column
      const bool kp = (v > 2.220446049250313e-16) && isfinite(v);
      const double r = kp ? 1.0 / v : 0.0;
#pragma unroll
      for (int k = 0; k < NPT; k++) {
        const int64_t i = (int64_t)k * BS + threadIdx.x;
        if (i < ldz) store_z(zrow + i, (kp && i < n) ? (x[k] - m) * r : 0.0);
      }
      for (int64_t i = (int64_t)NPT * BS + threadIdx.x; i < ldz; i += BS) store_z(zrow + i, 0.0);
      if (threadIdx.x == 0) {
        mean[j] = m;
        sd[j] = v;
        keep[j] = kp ? 1 : 0;
        kept_local += kp ? 1 : 0;
      }
    } else {
      double s = 0.0;
      for (int64_t i = threadIdx.x; i < n; i += BS) s += load_x(row, GATHER ? idx[i] : i, xs);
      m = block_sum<BS>(s, red) / (double)n;
      double ss = 0.0;
      for (int64_t i = threadIdx.x; i < n; i += BS) {
        const double d = load_x(row, GATHER ? idx[i] : i, xs) - m;
        ss += d * d;
      }
      v = n > 1 ? sqrt(block_sum<BS>(ss, red) / (double)(n - 1)) : __builtin_nan("");
      if (center_only) v = 1.0;  // glmnet standardize=false: centre only, keep every column
      const bool kp = (v > 2.220446049250313e-16) && isfinite(v);
      const double r = kp ? 1.0 / v : 0.0;
      for (int64_t i = threadIdx.x; i < ldz; i += BS) zrow[i] = (kp && i < n) ? (load_x(row, GATHER ? idx[i] : i, xs) - m) * r : 0.0;
      if (threadIdx.x == 0) {
        mean[j] = m;
        sd[j] = v;
        keep[j] = kp ? 1 : 0;
        kept_local += kp ? 1 : 0;
      }
    }
  }
  if (threadIdx.x == 0 && kept_local) atomicAdd(q_dev, kept_local);
}

// One locus row per wave: NPL values per lane in registers (lane l holds individuals 64k + l), mean
// and variance by xor butterflies over the wave (every lane ends with the same bits: each level adds
// the same two partial sums), no LDS and no workgroup barrier; four rows at a time per workgroup.
// Same per-row semantics as standardize_kernel (two-pass ddof = 1 variance, eps filter).
template <int NPL, bool GATHER, typename T>
__global__ void __launch_bounds__(256) standardize_wave_kernel(const T* Xt, int64_t ldx, int64_t p,
                                                               const int32_t* __restrict__ idx, int64_t n,
                                                               double* Zt, int64_t ldz, double* __restrict__ mean,
                                                               double* __restrict__ sd, int32_t* __restrict__ keep,
                                                               unsigned long long* __restrict__ q_dev,
                                                               int center_only, double xs) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  unsigned long long kept_local = 0;
  for (int64_t j = w0; j < p; j += nw) {
    const T* row = Xt + j * ldx;
    double* zrow = Zt + j * ldz;  // may alias row (in place, T = double)
    double x[NPL];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NPL; k++) {
      const int64_t i = (int64_t)k * 64 + lane;
      x[k] = i < n ? load_x(row, GATHER ? idx[i] : i, xs) : 0.0;
      s += x[k];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    const double m = s / (double)n;
    double ss = 0.0;
#pragma unroll
    for (int k = 0; k < NPL; k++) {
      const int64_t i = (int64_t)k * 64 + lane;
      const double d = x[k] - m;
      ss += i < n ? d * d : 0.0;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ss += __shfl_xor(ss, off, 64);
    double v = n > 1 ? sqrt(ss / (double)(n - 1)) : __builtin_nan("");
    if (center_only) v = 1.0;  // glmnet standardize=false: centre only, keep every column
    const bool kp = (v > 2.220446049250313e-16) && isfinite(v);
    const double r = kp ? 1.0 / v : 0.0;
#pragma unroll
    for (int k = 0; k < NPL; k++) {
      const int64_t i = (int64_t)k * 64 + lane;
      if (i < ldz) zrow[i] = (kp && i < n) ? (x[k] - m) * r : 0.0;
    }
    for (int64_t i = (int64_t)NPL * 64 + lane; i < ldz; i += 64) zrow[i] = 0.0;
    if (lane == 0) {
      mean[j] = m;
      sd[j] = v;
      keep[j] = kp ? 1 : 0;
      kept_local += kp ? 1 : 0;
    }
  }
  if (lane == 0 && kept_local) atomicAdd(q_dev, kept_local);
}

static dim3 row_grid(int64_t ldx, int64_t p) {
  const int64_t gx = (ldx + 1023) / 1024;
  const int64_t gy = p < 65535 ? p : 65535;
  return dim3((unsigned)gx, (unsigned)(gy > 0 ? gy : 1));
}

}  // namespace gbm

using namespace gbm;

extern "C" int gbm_dev_synth_genotypes(double* Xt, int64_t ldx, int64_t p, int64_t n, uint64_t seed,
                                       int64_t j0, void* stream) {
  if (!Xt || p < 0 || n < 0 || ldx < n) return fail(GBM_E_ARG, "gbm_dev_synth_genotypes: bad arguments");
  if (p == 0 || ldx == 0) return GBM_OK;
  synth_kernel<<<row_grid(ldx, p), 256, 0, (hipStream_t)stream>>>(Xt, ldx, p, n, seed, j0);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

extern "C" int gbm_dev_synth_dosage_i8(int8_t* D, int64_t ldd, int64_t p, int64_t n, uint64_t seed, int64_t j0,
                                       void* stream) {
  if (!D || p < 0 || n < 0 || ldd < n) return fail(GBM_E_ARG, "gbm_dev_synth_dosage_i8: bad arguments");
  if (p == 0 || n == 0) return GBM_OK;
  synth_i8_kernel<<<row_grid(n, p), 256, 0, (hipStream_t)stream>>>(D, ldd, p, n, seed, j0);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

extern "C" int gbm_dev_expand_dosage_i8(const int8_t* D, int64_t ldd, int64_t n, int64_t p, int ploidy,
                                        double* Xt, int64_t ldx, void* stream) {
  if (!D || !Xt || p < 0 || n < 0 || ldd < n || ldx < n || ploidy < 1)
    return fail(GBM_E_ARG, "gbm_dev_expand_dosage_i8: bad arguments");
  if (p == 0 || ldx == 0) return GBM_OK;
  expand_i8_kernel<<<row_grid(ldx, p), 256, 0, (hipStream_t)stream>>>(D, ldd, n, p, 1.0 / ploidy, Xt, ldx);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

template <bool GATHER, typename T = double>
static int launch_standardize(const T* Xt, int64_t ldx, int64_t p, const int32_t* idx, int64_t n, double* Zt,
                              int64_t ldz, double* mean, double* sd, int32_t* keep, int64_t* q_dev, int center_only,
                              hipStream_t s, double xs = 1.0) {
  const unsigned grid = (unsigned)(p < 256 * 16 ? p : 256 * 16);
  auto q = reinterpret_cast<unsigned long long*>(q_dev);
#ifndef GBM_STD_WAVE
#define GBM_STD_WAVE 0
#endif
  if (GBM_STD_WAVE && n <= 64 * 128) {
    const int64_t wg = (p + 3) / 4;
    const unsigned g4 = (unsigned)(wg < 4096 ? wg : 4096);
#define GBM_STD_W(NPL)                                                                                              \
  standardize_wave_kernel<NPL, GATHER, T><<<g4, 256, 0, s>>>(Xt, ldx, p, idx, n, Zt, ldz, mean, sd, keep, q, center_only, xs)
    if (n <= 64 * 16) GBM_STD_W(16);
    else if (n <= 64 * 32) GBM_STD_W(32);
    else if (n <= 64 * 48) GBM_STD_W(48);
    else if (n <= 64 * 64) GBM_STD_W(64);
    else if (n <= 64 * 80) GBM_STD_W(80);
    else if (n <= 64 * 96) GBM_STD_W(96);
    else GBM_STD_W(128);
#undef GBM_STD_W
    GBM_LAUNCH_CHECK();
    return GBM_OK;
  }
  if (n <= 256 * 4)
    standardize_kernel<256, 4, GATHER, T><<<grid, 256, 0, s>>>(Xt, ldx, p, idx, n, Zt, ldz, mean, sd, keep, q, center_only, xs);
  else if (n <= 256 * 8)
    standardize_kernel<256, 8, GATHER, T><<<grid, 256, 0, s>>>(Xt, ldx, p, idx, n, Zt, ldz, mean, sd, keep, q, center_only, xs);
  else if (n <= 256 * 16)
    standardize_kernel<256, 16, GATHER, T><<<grid, 256, 0, s>>>(Xt, ldx, p, idx, n, Zt, ldz, mean, sd, keep, q, center_only, xs);
  else if (n <= 256 * 32)
    standardize_kernel<256, 32, GATHER, T><<<grid, 256, 0, s>>>(Xt, ldx, p, idx, n, Zt, ldz, mean, sd, keep, q, center_only, xs);
  else
    standardize_kernel<256, 0, GATHER, T><<<grid, 256, 0, s>>>(Xt, ldx, p, idx, n, Zt, ldz, mean, sd, keep, q, center_only, xs);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

namespace gbm {
int launch_center_columns(const double* Xt, int64_t ldx, int64_t p, int64_t n, double* Zt, int64_t ldz, double* mean,
                          double* sd, int32_t* keep, int64_t* q_dev, hipStream_t s) {
  if (p == 0) return GBM_OK;
  return launch_standardize<false>(Xt, ldx, p, nullptr, n, Zt, ldz, mean, sd, keep, q_dev, 1, s);
}

int launch_standardize_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, double* Zt, int64_t ldz,
                          double* mean, double* sd, int32_t* keep, int64_t* q_dev, hipStream_t s) {
  if (!D || !Zt || !mean || !sd || !keep || !q_dev || p < 0 || n < 1 || ldd < n || ldz < n || ploidy < 1)
    return fail(GBM_E_ARG, "standardize (int8 dosages): bad arguments");
  if (p == 0) return GBM_OK;
  return launch_standardize<false, int8_t>(D, ldd, p, nullptr, n, Zt, ldz, mean, sd, keep, q_dev, 0, s, 1.0 / ploidy);
}
}  // namespace gbm

extern "C" int gbm_dev_standardize(const double* Xt, int64_t ldx, int64_t p, int64_t n, double* Zt, int64_t ldz,
                                   double* mean, double* sd, int32_t* keep, int64_t* q_dev, void* stream) {
  if (!Xt || !Zt || !mean || !sd || !keep || !q_dev || p < 0 || n < 1 || ldx < n || ldz < n ||
      ((const double*)Zt == Xt && ldz != ldx))
    return fail(GBM_E_ARG, "gbm_dev_standardize: bad arguments");
  if (p == 0) return GBM_OK;
  return launch_standardize<false>(Xt, ldx, p, nullptr, n, Zt, ldz, mean, sd, keep, q_dev, 0, (hipStream_t)stream);
}

extern "C" int gbm_dev_standardize_gather(const double* Xt, int64_t ldx, int64_t p, const int32_t* idx, int64_t n,
                                          double* Zt, int64_t ldz, double* mean, double* sd, int32_t* keep,
                                          int64_t* q_dev, int center_only, void* stream) {
  if (!Xt || !idx || !Zt || !mean || !sd || !keep || !q_dev || p < 0 || n < 1 || ldz < n ||
      (const double*)Zt == Xt)
    return fail(GBM_E_ARG, "gbm_dev_standardize_gather: bad arguments (out of place only)");
  if (p == 0) return GBM_OK;
  return launch_standardize<true>(Xt, ldx, p, idx, n, Zt, ldz, mean, sd, keep, q_dev, center_only,
                                  (hipStream_t)stream);
}

extern "C" int gbm_dev_standardize_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, double* Zt,
                                      int64_t ldz, double* mean, double* sd, int32_t* keep, int64_t* q_dev,
                                      void* stream) {
  return launch_standardize_i8(D, ldd, p, n, ploidy, Zt, ldz, mean, sd, keep, q_dev, (hipStream_t)stream);
}
