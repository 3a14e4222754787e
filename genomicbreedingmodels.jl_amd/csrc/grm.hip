// GRM build: G = Σ_j z_j z_jᵀ over the standardised locus rows of Zt — an fp64 SYRK on the
// CDNA4 matrix cores (v_mfma_f64_16x16x4_f64), the dominant cost of the path.
//
// Geometry (DESIGN.md "GRM kernel"):
//   * workgroup tile 128 x 128 of G (upper-triangular tiles only: nt(nt+1)/2 tiles),
//     256 threads = 4 waves in 2 x 2, each wave a 64 x 64 sub-tile = 4 x 4 MFMA 16x16 tiles
//     (16 f64x4 accumulators per lane);
//   * K (= loci) consumed in stages of 16 rows; each stage is 2 x 16 rows x 1 KB of Zt brought
//     straight into LDS by global_load_lds_dwordx4 (one wave-instruction = one 1-KB locus row
//     segment), double-buffered; LDS rows padded to 1152 B so the two 16-lane halves of a
//     ds_read_b64 fragment load land on disjoint bank halves;
//   * split-K over loci ("slices") when the triangular tile count alone cannot fill the
//     256 CUs x 2 resident workgroups; slices write private slabs that a second kernel sums in
//     a fixed order (deterministic, no float atomics).
#include <cstdlib>

#include "chol_device.h"

namespace gbm {

constexpr int BT = 128;            // tile edge
#ifndef GBM_BK
#define GBM_BK 16
#endif
#ifndef GBM_WPS
#define GBM_WPS 2
#endif
constexpr int BK = GBM_BK;         // loci per stage
constexpr int WPS = GBM_WPS;       // target waves per SIMD (= resident 256-thread workgroups per CU)
constexpr int LROW = BT + 16;      // LDS row pitch in doubles (1152 B)
constexpr int STAGE = 2 * BK * LROW;  // doubles per stage (A rows then B rows)

__device__ __forceinline__ void tile_of(int64_t t, int64_t& ti, int64_t& tj) {
  // t -> upper-triangular tile (ti <= tj): enumerate the lower triangle row-major, then swap
  int64_t r = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) r++;
  while (r * (r + 1) / 2 > t) r--;
  tj = r;
  ti = t - r * (r + 1) / 2;
}

enum SyrkMode { kStore = 0, kSlab = 1, kSub = 2 };

// One kernel, three epilogues:
//   kStore  C[i][j]  = Σ_k U[k][i] U[k][j]     (the GRM, single slice)
//   kSlab   slab     = Σ_{k in slice} ...      (the GRM, split over loci)
//   kSub    C[i][j] -= Σ_k U[k][i] U[k][j]     (the upper-Cholesky trailing update, K = 64)
// U is k-major: row k holds columns c contiguous (U[k*ldu + c]); the tiles are the upper
// (ti <= tj) BT x BT tiles of the square [c0, c0 + lim)^2, in absolute column coordinates of U
// and C. Wave quadrants entirely outside `lim` skip their MFMAs and stores (padding / ragged
// last tile); their operand columns may be read past `lim` (the caller guarantees those reads
// stay inside the allocation).
template <int MODE>
__global__ void __launch_bounds__(256, WPS)
syrk_kernel(const double* __restrict__ U, int64_t ldu, int64_t K, int64_t c0, int64_t lim,
            double* __restrict__ C, int64_t ldc, double* __restrict__ slab, int64_t ntiles, int64_t steps_per_slice,
            double* __restrict__ Ld, double* __restrict__ Dinv, int32_t* __restrict__ info, int64_t fk0) {
  // 2 stages (72 KB at BK = 16); kSub's first workgroup reuses it for the 64x64 factor image
  constexpr int LDS_DOUBLES = (2 * STAGE > CNB * PS + CNB) ? 2 * STAGE : CNB * PS + CNB;
  __shared__ __attribute__((aligned(16))) double lds[LDS_DOUBLES];

  const int64_t wg = blockIdx.x;
  const int s = (int)(wg / ntiles);
  const int64_t t = wg - (int64_t)s * ntiles;
  int64_t ti, tj;
  tile_of(t, ti, tj);
  const bool diag = (ti == tj);
  const int64_t i0 = c0 + ti * BT, j0 = c0 + tj * BT;

  const int64_t nsteps_total = (K + BK - 1) / BK;
  const int64_t kstep0 = (int64_t)s * steps_per_slice;
  int64_t kstep1 = kstep0 + steps_per_slice;
  if (kstep1 > nsteps_total) kstep1 = nsteps_total;
  const int64_t nsteps = kstep1 > kstep0 ? kstep1 - kstep0 : 0;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // (the strictly-lower quadrant of a diagonal tile is never needed: upper storage)
  const bool active = (i0 - c0 + wm * 64 < lim) && (j0 - c0 + wn * 64 < lim) && !(diag && wm == 1 && wn == 0);

  // each wave stages BK/4 rows r = wave*BK/4 .. of A (and of B off-diagonal)
  auto stage = [&](int64_t kstep, int buf) {
    double* base = lds + buf * STAGE;
#pragma unroll
    for (int rr = 0; rr < BK / 4; rr++) {
      const int r = wave * (BK / 4) + rr;
      const int64_t k = kstep * BK + r;
      double* la = base + r * LROW;
      double* lb = base + (BK + r) * LROW;
      if (k < K) {
        const double* src = U + k * ldu;
        __builtin_amdgcn_global_load_lds((const void*)(src + i0 + lane * 2), (void*)la, 16, 0, 0);
        if (!diag) __builtin_amdgcn_global_load_lds((const void*)(src + j0 + lane * 2), (void*)lb, 16, 0, 0);
      } else {
        *reinterpret_cast<double2*>(la + lane * 2) = make_double2(0.0, 0.0);
        if (!diag) *reinterpret_cast<double2*>(lb + lane * 2) = make_double2(0.0, 0.0);
      }
    }
  };

  const int frag_row = lane >> 4;  // k within a 4-deep MFMA step
  const int frag_col = lane & 15;
  const int64_t rlim = c0 + lim;

  d4 acc[4][4];
  if constexpr (MODE == kSub) {
    // the C tile goes straight into the accumulators (its loads overlap the operand staging)
    // and the A fragments are negated below: the MFMA chain produces C − Σ_k U[k][i] U[k][j]
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = i0 + wm * 64 + m * 16 + frag_row + 4 * r;
          const int64_t col = j0 + wn * 64 + q * 16 + frag_col;
          acc[m][q][r] = (active && row < rlim && col < rlim) ? C[row * ldc + col] : 0.0;
        }
  } else {
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 4; b++) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
  }

  if (nsteps > 0) stage(kstep0, 0);
  __syncthreads();

  for (int64_t st = 0; st < nsteps; st++) {
    const int buf = (int)(st & 1);
    if (st + 1 < nsteps) stage(kstep0 + st + 1, buf ^ 1);
    if (active) {
      const double* A = lds + buf * STAGE;
      const double* B = diag ? A : A + BK * LROW;
#pragma unroll
      for (int ks = 0; ks < BK / 4; ks++) {
        const int kr = ks * 4 + frag_row;
        double af[4], bf[4];
#pragma unroll
        for (int m = 0; m < 4; m++) {
          af[m] = A[kr * LROW + wm * 64 + m * 16 + frag_col];
          if constexpr (MODE == kSub) af[m] = -af[m];
        }
#pragma unroll
        for (int q = 0; q < 4; q++) bf[q] = B[kr * LROW + wn * 64 + q * 16 + frag_col];
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
          for (int q = 0; q < 4; q++)
            acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[q], acc[m][q], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // kSub, first workgroup (tile (0,0)), fk0 >= 0: factor the next diagonal block afterwards
  const bool factor_next = (MODE == kSub) && fk0 >= 0 && wg == 0;
  if (!active && !factor_next) return;

  // epilogue: f64 MFMA C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
  if constexpr (MODE == kSlab) {
    double* out = slab + ((int64_t)s * ntiles + t) * (int64_t)(BT * BT);
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = wm * 64 + m * 16 + frag_row + 4 * r;
          const int col = wn * 64 + q * 16 + frag_col;
          out[row * BT + col] = acc[m][q][r];
        }
  } else {
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = i0 + wm * 64 + m * 16 + frag_row + 4 * r;
          const int64_t col = j0 + wn * 64 + q * 16 + frag_col;
          if (active && row < rlim && col < rlim) {
            C[row * ldc + col] = acc[m][q][r];
          }
        }
  }
  if constexpr (MODE == kSub) {
    if (factor_next) {
      // the next panel's diagonal block [c0, c0+64)^2 is wave (0,0)'s 64x64 quadrant of this tile
      double* Us = lds;  // the staging buffers are free now (last loop iteration ended in a barrier)
      double* rinv = lds + CNB * PS;
      if (wave == 0) {
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
          for (int q = 0; q < 4; q++)
#pragma unroll
            for (int r = 0; r < 4; r++) Us[(m * 16 + frag_row + 4 * r) * PS + q * 16 + frag_col] = acc[m][q][r];
      }
      __syncthreads();
      const int bad = factor_diag_block(Us, rinv, threadIdx.x);
      if (threadIdx.x == 0 && bad >= 0) atomicCAS(info, 0, (int32_t)(fk0 + bad + 1));
      store_factor(Us, rinv, Ld + fk0 * CNB, Dinv + (fk0 / 16) * 256, threadIdx.x);
    }
  }
}

// G tile = Σ_s slab[s][tile] in slice order (deterministic).
__global__ void __launch_bounds__(256) grm_slab_reduce_kernel(const double* __restrict__ slab, int64_t ntiles,
                                                              int nslices, double* __restrict__ G, int64_t ldg) {
  const int64_t t = blockIdx.x;
  int64_t ti, tj;
  tile_of(t, ti, tj);
  const int64_t per = (int64_t)BT * BT;
  for (int e = threadIdx.x * 2; e < BT * BT; e += 256 * 2) {
    double2 acc = make_double2(0.0, 0.0);
    for (int s = 0; s < nslices; s++) {
      const double2 v = *reinterpret_cast<const double2*>(slab + ((int64_t)s * ntiles + t) * per + e);
      acc.x += v.x;
      acc.y += v.y;
    }
    const int row = e / BT, col = e % BT;
    *reinterpret_cast<double2*>(G + (ti * BT + row) * ldg + tj * BT + col) = acc;
  }
}

static int resident_wgs() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
  }
  return cus * WPS;  // WPS workgroups per CU (LDS 2 x 2 x BK x 1152 B each)
}

static void plan(int64_t n, int64_t p, int64_t& ntiles, int& nslices, int64_t& steps_per_slice) {
  const int64_t nt = npad_of(n) / BT;
  ntiles = nt * (nt + 1) / 2;
  const int64_t nsteps = (p + BK - 1) / BK;
  const int64_t R = resident_wgs();
  int best = 1;
  double best_eff = 0.0;
  for (int S = 1; S <= 8; S++) {
    if (S > 1 && nsteps / S < 16) break;  // keep >= 16 stages per workgroup
    const int64_t w = ntiles * S;
    const double eff = (double)w / (double)(R * ((w + R - 1) / R));
    if (eff > best_eff + 0.05) {
      best_eff = eff;
      best = S;
    }
    if (eff >= 0.92) break;
  }
  nslices = best;
  steps_per_slice = (nsteps + nslices - 1) / nslices;
}

// Small-tile variant of the Cholesky trailing update (64x64 upper tiles, K = 64, 4 waves of
// 32x32): more workgroups for the small trailing matrices of late panels. The C tile is loaded
// into the accumulators first and the A fragments are negated, so the MFMA chain itself
// produces C − Σ_k U[k][i] U[k][j] (no separate read-modify-write).
constexpr int P64 = 80;  // LDS pitch: the two 16-lane halves of a fragment read hit disjoint banks
__global__ void __launch_bounds__(256, 2)
syrk64_sub_kernel(const double* __restrict__ U, int64_t ldu, int64_t c0, int64_t lim, double* __restrict__ C,
                  int64_t ldc, double* __restrict__ Ld, double* __restrict__ Dinv, int32_t* __restrict__ info,
                  int64_t fk0) {
  __shared__ __attribute__((aligned(16))) double As[64 * P64];
  __shared__ __attribute__((aligned(16))) double Bs[64 * P64];
  int64_t ti, tj;
  tile_of(blockIdx.x, ti, tj);
  const bool diag = ti == tj;
  const int64_t i0 = c0 + ti * 64, j0 = c0 + tj * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane >> 4, fc = lane & 15;
  const int64_t rlim = c0 + lim;
  const bool active = (i0 + wm * 32 < rlim) && (j0 + wn * 32 < rlim);
  d4 acc[2][2];
  if (active) {
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
      for (int q = 0; q < 2; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = i0 + wm * 32 + m * 16 + fr + 4 * r;
          const int64_t col = j0 + wn * 32 + q * 16 + fc;
          acc[m][q][r] = (row < rlim && col < rlim) ? C[row * ldc + col] : 0.0;
        }
  }
  {
    const int k = tid >> 2, quarter = tid & 3;
    const double* sa = U + k * ldu + i0 + quarter * 16;
    const double* sb = U + k * ldu + j0 + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      *reinterpret_cast<double2*>(&As[k * P64 + quarter * 16 + e]) = *reinterpret_cast<const double2*>(sa + e);
      if (!diag)
        *reinterpret_cast<double2*>(&Bs[k * P64 + quarter * 16 + e]) = *reinterpret_cast<const double2*>(sb + e);
    }
  }
  __syncthreads();
  const bool factor_next = fk0 >= 0 && blockIdx.x == 0;
  if (!active && !factor_next) return;
  const double* B = diag ? As : Bs;
#pragma unroll
  for (int ks = 0; ks < (active ? 16 : 0); ks++) {
    double af[2], bf[2];
#pragma unroll
    for (int m = 0; m < 2; m++) af[m] = -As[(ks * 4 + fr) * P64 + wm * 32 + m * 16 + fc];
#pragma unroll
    for (int q = 0; q < 2; q++) bf[q] = B[(ks * 4 + fr) * P64 + wn * 32 + q * 16 + fc];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
      for (int q = 0; q < 2; q++) acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[q], acc[m][q], 0, 0, 0);
  }
#pragma unroll
  for (int m = 0; m < 2; m++)
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int64_t row = i0 + wm * 32 + m * 16 + fr + 4 * r;
        const int64_t col = j0 + wn * 32 + q * 16 + fc;
        if (active && row < rlim && col < rlim) C[row * ldc + col] = acc[m][q][r];
      }
  if (factor_next) {
    // this tile is the next panel's diagonal block: factor it straight from the accumulators
    __syncthreads();  // every wave is done reading As/Bs
    double* Us = As;  // pitch P64 == PS
    double* rinv = Bs;
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
      for (int q = 0; q < 2; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) Us[(wm * 32 + m * 16 + fr + 4 * r) * PS + wn * 32 + q * 16 + fc] = acc[m][q][r];
    __syncthreads();
    const int bad = factor_diag_block(Us, rinv, tid);
    if (tid == 0 && bad >= 0) atomicCAS(info, 0, (int32_t)(fk0 + bad + 1));
    store_factor(Us, rinv, Ld + fk0 * CNB, Dinv + (fk0 / 16) * 256, tid);
  }
}

// Upper-Cholesky trailing update: C[k1:gdim, k1:gdim] (upper tiles) -= U[k0:k1, k1:]ᵀ U[k0:k1, k1:]
int launch_chol_update(double* G, int64_t ldg, int64_t k0, int64_t nb, int64_t gdim, double* Ld, double* Dinv,
                       int32_t* info, int64_t next_k0, hipStream_t s) {
  const int64_t k1 = k0 + nb;
  const int64_t lim = gdim - k1;
  if (lim <= 0) return GBM_OK;
  static const int64_t small_lim = [] {
    const char* e = getenv("GBM_UPD64_LIM");
    return e ? (int64_t)atoll(e) : (int64_t)2048;
  }();
  if (nb == 64 && lim <= small_lim) {
    const int64_t m = (lim + 63) / 64;
    syrk64_sub_kernel<<<(unsigned)(m * (m + 1) / 2), 256, 0, s>>>(G + k0 * ldg, ldg, k1, lim, G, ldg, Ld, Dinv, info,
                                                                  next_k0);
    GBM_LAUNCH_CHECK();
    return GBM_OK;
  }
  const int64_t m = (lim + BT - 1) / BT;
  const int64_t ntiles = m * (m + 1) / 2;
  const int64_t steps = (nb + BK - 1) / BK;
  syrk_kernel<kSub><<<(unsigned)ntiles, 256, 0, s>>>(G + k0 * ldg, ldg, nb, k1, lim, G, ldg, nullptr, ntiles, steps,
                                                     Ld, Dinv, info, next_k0);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

int64_t grm_workspace_bytes(int64_t n, int64_t p) {
  int64_t ntiles, sps;
  int S;
  plan(n, p, ntiles, S, sps);
  return S > 1 ? (int64_t)S * ntiles * BT * BT * (int64_t)sizeof(double) : 0;
}

static int check_grm_args(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg) {
  const int64_t npad = npad_of(n);
  if (!Zt || !G || p < 1 || n < 1 || ldz < npad || ldg < npad || (ldz & 1))
    return fail(GBM_E_ARG, "gbm_dev_grm: bad arguments (need ldz, ldg >= npad(n), even ldz)");
  if (((uintptr_t)Zt & 15) != 0) return fail(GBM_E_ARG, "gbm_dev_grm: Zt must be 16-byte aligned");
  return GBM_OK;
}

// stage 1: the MFMA SYRK (writes G directly, or per-slice slabs into ws when split over loci)
int launch_grm_syrk(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg, void* ws,
                    int64_t ws_bytes, hipStream_t s) {
  int rc = check_grm_args(Zt, ldz, p, n, G, ldg);
  if (rc != GBM_OK) return rc;
  int64_t ntiles, sps;
  int S;
  plan(n, p, ntiles, S, sps);
  const int64_t need = S > 1 ? (int64_t)S * ntiles * BT * BT * (int64_t)sizeof(double) : 0;
  if (need > 0 && (!ws || ws_bytes < need))
    return fail(GBM_E_ARG, "gbm_dev_grm: workspace too small (" + std::to_string(ws_bytes) + " < " +
                               std::to_string(need) + ")");
  if (S == 1)
    syrk_kernel<kStore><<<(unsigned)ntiles, 256, 0, s>>>(Zt, ldz, p, 0, n, G, ldg, nullptr, ntiles, sps, nullptr,
                                                         nullptr, nullptr, -1);
  else
    syrk_kernel<kSlab><<<(unsigned)(ntiles * S), 256, 0, s>>>(Zt, ldz, p, 0, n, G, ldg, (double*)ws, ntiles, sps,
                                                              nullptr, nullptr, nullptr, -1);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// stage 2: sum the slabs (no-op when the plan did not split over loci)
int launch_grm_reduce(int64_t n, int64_t p, double* G, int64_t ldg, const void* ws, hipStream_t s) {
  int64_t ntiles, sps;
  int S;
  plan(n, p, ntiles, S, sps);
  if (S > 1) {
    grm_slab_reduce_kernel<<<(unsigned)ntiles, 256, 0, s>>>((const double*)ws, ntiles, S, G, ldg);
    GBM_LAUNCH_CHECK();
  }
  return GBM_OK;
}

int launch_grm(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg, void* ws,
               int64_t ws_bytes, hipStream_t s) {
  int rc = launch_grm_syrk(Zt, ldz, p, n, G, ldg, ws, ws_bytes, s);
  if (rc != GBM_OK) return rc;
  return launch_grm_reduce(n, p, G, ldg, ws, s);
}

}  // namespace gbm

extern "C" int64_t gbm_dev_grm_workspace(int64_t n, int64_t p) { return gbm::grm_workspace_bytes(n, p); }

extern "C" int gbm_dev_grm(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
                           void* workspace, int64_t ws_bytes, void* stream) {
  return gbm::launch_grm(Zt, ldz, p, n, G, ldg, workspace, ws_bytes, (hipStream_t)stream);
}

extern "C" int gbm_dev_grm_syrk(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
                                void* workspace, int64_t ws_bytes, void* stream) {
  return gbm::launch_grm_syrk(Zt, ldz, p, n, G, ldg, workspace, ws_bytes, (hipStream_t)stream);
}

extern "C" int gbm_dev_grm_reduce(int64_t n, int64_t p, double* G, int64_t ldg, const void* workspace, void* stream) {
  if (!G || n < 1 || p < 1 || ldg < gbm::npad_of(n)) return gbm::fail(GBM_E_ARG, "gbm_dev_grm_reduce: bad arguments");
  return gbm::launch_grm_reduce(n, p, G, ldg, workspace, (hipStream_t)stream);
}

extern "C" int gbm_dev_grm_slices(int64_t n, int64_t p) {
  int64_t ntiles, sps;
  int S;
  gbm::plan(n, p, ntiles, S, sps);
  return S;
}

namespace gbm {
// out[i, j] = inv_q * G[min(i,j), max(i,j)] for i, j < n (full symmetric export of the upper-stored GRM)
__global__ void __launch_bounds__(256) grm_export_kernel(const double* __restrict__ G, int64_t ldg, int64_t n,
                                                         double inv_q, double* __restrict__ out, int64_t ldo) {
  const int64_t i = blockIdx.x;
  for (int64_t j = threadIdx.x; j < n; j += 256)
    out[i * ldo + j] = inv_q * (j >= i ? G[i * ldg + j] : G[j * ldg + i]);
}

int launch_grm_export(const double* G, int64_t ldg, int64_t n, double inv_q, double* out, int64_t ldo, hipStream_t s) {
  grm_export_kernel<<<(unsigned)n, 256, 0, s>>>(G, ldg, n, inv_q, out, ldo);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}
}  // namespace gbm
