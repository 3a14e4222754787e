// GBLUP solve: upper Cholesky V = UᵀU of the bordered matrix (row-major, upper triangle stored)
//
//        [ V    R ]      V = G/q + λI  (npad x npad; padding rows/cols = identity)
//   M =  [ Rᵀ   0 ]      R = [1, y_1, ..., y_t, 0...]  (npad x 64, extra columns)
//
// Right-looking blocked factorisation over the first npad rows, panel height NB = 64:
//   panel k:  U_kk = chol(A_kk)ᵀ (64x64), U_k,J = U_kk⁻ᵀ A_k,J for every column block J > k —
//             including the R columns, which turns them into W = U⁻ᵀR = L⁻¹R (the forward
//             substitution is fused into the factorisation);
//   update k: A_IJ -= U_kIᵀ U_kJ (I <= J) — the same fp64-MFMA SYRK kernel as the GRM
//             (k-major operands: the panel rows), see grm.hip syrk_kernel<kSub>.
// The bottom-right block ends as −WᵀW, so 1ᵀV⁻¹1 and 1ᵀV⁻¹y come out of the factorisation
// (GLS intercept of reference src/gwas.jl:596-597 with X = 1). Then a = U⁻¹(W_y − μ̂ W_1) by
// a blocked back substitution, and GEBV = μ̂ + (y − μ̂) − λa (= μ̂ + G a).
// The reference inverts V with pinv/SVD (src/gwas.jl:472,595); for λ > 0 V is SPD and the
// Cholesky solution is the same up to rounding.
#include "gbm_internal.h"

namespace gbm {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int NB = kCholNB;  // 64
constexpr int MAXRHS = 63;

int launch_chol_update(double* G, int64_t ldg, int64_t k0, int64_t nb, int64_t gdim, hipStream_t s);

__device__ __forceinline__ double rsqrt_nr(double a) {  // v_rsq_f64 + one Newton step
  double y = __builtin_amdgcn_rsq(a);
  const double h = 0.5 * a * y;
  return y * fma(-h, y, 1.5);
}
__device__ __forceinline__ double rcp_nr(double a) {  // v_rcp_f64 + one Newton step
  double y = __builtin_amdgcn_rcp(a);
  const double e = fma(-a, y, 1.0);
  return fma(y, e, y);
}
__device__ __forceinline__ double readlane_d(double x, int lane) {
  union {
    double d;
    int i[2];
  } u;
  u.d = x;
  u.i[0] = __builtin_amdgcn_readlane(u.i[0], lane);
  u.i[1] = __builtin_amdgcn_readlane(u.i[1], lane);
  return u.d;
}

// ---- V = G/q + λI (upper part), padding = identity, bordered R columns -----------------------
__global__ void __launch_bounds__(256) prepare_v_kernel(double* __restrict__ G, int64_t ld, int64_t n,
                                                        int64_t npad, int64_t gdim, double inv_q,
                                                        const int64_t* __restrict__ q_dev, double lambda,
                                                        const double* __restrict__ Y, int64_t ldy, int64_t nrhs,
                                                        int32_t* __restrict__ info) {
  const int64_t i = blockIdx.x;  // row
  if (i == 0 && threadIdx.x == 0) *info = 0;
  if (q_dev) inv_q = 1.0 / (double)(*q_dev);
  double* row = G + i * ld;
  const int64_t jbeg = (i / NB) * NB;  // from the start of the diagonal block
  for (int64_t j = jbeg + threadIdx.x; j < gdim; j += 256) {
    double v = 0.0;
    if (i < npad) {
      if (j < i) v = 0.0;
      else if (j < npad) v = (i < n && j < n) ? row[j] * inv_q + (i == j ? lambda : 0.0) : (i == j ? 1.0 : 0.0);
      else if (i < n) {
        const int64_t t = j - npad;
        v = t == 0 ? 1.0 : (t <= nrhs ? Y[(t - 1) * ldy + i] : 0.0);
      }
    }
    row[j] = v;
  }
}

// ---- panel k ---------------------------------------------------------------------------------
// Workgroup 0: factor the 64x64 diagonal block and store U_kk into the scratch Ld (not in place:
// the other workgroups of this launch read the unfactored block from G). Workgroup g >= 1:
// factor the same block redundantly (4 x 16-row sub-panels, MFMA for the inner updates), then
// solve its 64-column chunk X = A[k0:k0+64, k0+64g : k0+64g+64] in place: X <- U_kk⁻ᵀ X.
// LDS images are U-layout (row i, column j, upper part valid); pitch 80 doubles puts the two
// 16-lane halves of every MFMA fragment read on disjoint bank halves.
constexpr int PS = NB + 16;

// D(16x16 at (r0, c0) of dst) -= Σ_k S[kb + k][ra + row] T[kb + k][cb + col], k < 4*ksteps
__device__ __forceinline__ void mfma_tile_sub_t(double* dst, int r0, int c0, const double* S, int ra,
                                                const double* T, int cb, int kb, int ksteps, int lane) {
  d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
  const int fr = lane >> 4, fc = lane & 15;
  for (int ks = 0; ks < ksteps; ks++) {
    const double a = S[(kb + ks * 4 + fr) * PS + ra + fc];
    const double b = T[(kb + ks * 4 + fr) * PS + cb + fc];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) dst[(r0 + fr + 4 * r) * PS + c0 + fc] -= acc[r];
}

__global__ void __launch_bounds__(256) chol_panel_kernel(double* __restrict__ G, int64_t ld, int64_t k0,
                                                         double* __restrict__ Ld, int32_t* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) double Us[NB * PS];
  __shared__ __attribute__((aligned(16))) double X[NB * PS];
  __shared__ double rinv[NB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool diag_wg = blockIdx.x == 0;
  {
    const int row = tid >> 2, quarter = tid & 3;
    const double* sa = G + (k0 + row) * ld + k0 + quarter * 16;
    const double* sx = G + (k0 + row) * ld + k0 + (int64_t)blockIdx.x * NB + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      *reinterpret_cast<double2*>(&Us[row * PS + quarter * 16 + e]) = *reinterpret_cast<const double2*>(sa + e);
      if (!diag_wg)
        *reinterpret_cast<double2*>(&X[row * PS + quarter * 16 + e]) = *reinterpret_cast<const double2*>(sx + e);
    }
  }
  __syncthreads();
  bool bad = false;
  int badcol = 0;
  for (int kb = 0; kb < 4; kb++) {
    const int o = kb * 16;
    if (wave == 0) {
      // right-looking factorisation of the 16-row sub-panel U[o:o+16, o:64]: lane r owns
      // column o + r (= row o + r of L = Uᵀ); columns o..o+15 form the diagonal sub-block, the
      // others are solved in the same 16-step loop (u_cs broadcast from lane s by v_readlane)
      const int ncols = NB - o;
      const int cc = o + (lane < ncols ? lane : 0);
      double x[16];
#pragma unroll
      for (int t = 0; t < 16; t++) x[t] = Us[(o + t) * PS + cc];
#pragma unroll
      for (int c = 0; c < 16; c++) {
        const double piv = readlane_d(x[c], c);
        if (!(piv > 0.0) || !isfinite(piv)) {
          if (!bad) badcol = o + c;
          bad = true;
        }
        const double lc = x[c] * rsqrt_nr(piv);  // lane c: piv/sqrt(piv) = U[c][c]
#pragma unroll
        for (int sidx = c + 1; sidx < 16; sidx++) x[sidx] -= lc * readlane_d(lc, sidx);
        x[c] = lc;
      }
      if (lane < ncols) {
#pragma unroll
        for (int t = 0; t < 16; t++) Us[(o + t) * PS + cc] = (lane < 16 && t > lane) ? 0.0 : x[t];
      }
      if (lane < 16) rinv[o + lane] = rcp_nr(x[lane & 15]);
    }
    __syncthreads();
    // trailing update of the block's remaining upper 16x16 tiles on the matrix cores:
    // U[i][j] -= Σ_{t in [o, o+16)} U[t][i] U[t][j]
    const int m = 3 - kb;
    const int ntile = m * (m + 1) / 2;
    for (int t = wave; t < ntile; t += 4) {
      int a = 0;
      while ((a + 1) * (a + 2) / 2 <= t) a++;
      const int b = t - a * (a + 1) / 2;  // b <= a  -> tile (row b, col a)
      const int r0 = o + 16 + b * 16, c0 = o + 16 + a * 16;
      mfma_tile_sub_t(Us, r0, c0, Us, r0, Us, c0, o, 4, lane);
    }
    __syncthreads();
  }
  if (diag_wg) {
    if (bad && tid == 0) atomicCAS(info, 0, (int32_t)(k0 + badcol + 1));
    const int row = tid >> 2, quarter = tid & 3;
    double* dst = Ld + (k0 + row) * NB + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      const int c = quarter * 16 + e;
      *reinterpret_cast<double2*>(dst + e) =
          make_double2(c >= row ? Us[row * PS + c] : 0.0, c + 1 >= row ? Us[row * PS + c + 1] : 0.0);
    }
    return;
  }
  // X <- U_kk⁻ᵀ X, 16-row block by 16-row block
  for (int rb = 0; rb < 4; rb++) {
    const int o = rb * 16;
    // X[o:o+16, :] -= U[0:o, o:o+16]ᵀ X[0:o, :]   (wave w: columns 16w..16w+15)
    if (rb > 0) mfma_tile_sub_t(X, o, wave * 16, Us, o, X, wave * 16, 0, rb * 4, lane);
    __syncthreads();
    if (wave == 0) {
      // forward substitution on the 16x16 diagonal sub-block, lane = column of X
      double x[16];
#pragma unroll
      for (int t = 0; t < 16; t++) x[t] = X[(o + t) * PS + lane];
#pragma unroll
      for (int c = 0; c < 16; c++) {
        x[c] *= rinv[o + c];
#pragma unroll
        for (int sidx = c + 1; sidx < 16; sidx++) x[sidx] -= Us[(o + c) * PS + o + sidx] * x[c];
      }
#pragma unroll
      for (int t = 0; t < 16; t++) X[(o + t) * PS + lane] = x[t];
    }
    __syncthreads();
  }
  {
    const int row = tid >> 2, quarter = tid & 3;
    double* dx = G + (k0 + row) * ld + k0 + (int64_t)blockIdx.x * NB + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2)
      *reinterpret_cast<double2*>(dx + e) = *reinterpret_cast<const double2*>(&X[row * PS + quarter * 16 + e]);
    // the same chunk transposed into the (otherwise unused) lower triangle: L = Uᵀ row-major,
    // so the back substitution and the μ̂ kernel read coalesced rows. Never overwritten later:
    // every later trailing update covers only rows/cols >= its own k1 > these columns.
    double* dl = G + (k0 + (int64_t)blockIdx.x * NB + row) * ld + k0 + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2)
      *reinterpret_cast<double2*>(dl + e) =
          make_double2(X[(quarter * 16 + e) * PS + row], X[(quarter * 16 + e + 1) * PS + row]);
  }
}

// ---- inverses of all diagonal blocks U_bb (one workgroup per block, all in parallel) --------
// lane = column j: X[i][j] = (δ_ij − Σ_{k>i} U[i][k] X[k][j]) / U[i][i], the dot product split
// over 4 partial sums so the dependent chain is a quarter of its length.
__global__ void __launch_bounds__(64) diag_inverse_kernel(const double* __restrict__ Ld, double* __restrict__ Linv) {
  __shared__ double Ub[NB][NB + 1];
  const int lane = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * NB;
  for (int r = 0; r < NB; r++) Ub[r][lane] = Ld[(b0 + r) * NB + lane];
  __syncthreads();
  double x[NB];
#pragma unroll
  for (int i = NB - 1; i >= 0; i--) {
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
    for (int k = i + 1; k < NB; k += 4) {
      p0 = fma(Ub[i][k], x[k], p0);
      if (k + 1 < NB) p1 = fma(Ub[i][k + 1], x[k + 1], p1);
      if (k + 2 < NB) p2 = fma(Ub[i][k + 2], x[k + 2], p2);
      if (k + 3 < NB) p3 = fma(Ub[i][k + 3], x[k + 3], p3);
    }
    x[i] = (i <= lane) ? (((lane == i) ? 1.0 : 0.0) - ((p0 + p1) + (p2 + p3))) * rcp_nr(Ub[i][i]) : 0.0;
  }
#pragma unroll
  for (int i = 0; i < NB; i++) Linv[(b0 + i) * NB + lane] = x[i];
}

// ---- μ̂ and the back-substitution right-hand sides w_t = W_{1+t} − μ̂_t W_0 ---------------------
// W_s is column npad + s of the factored rows (row npad + s of the lower copy); the Schur
// block holds −W_sᵀW_t.
__global__ void __launch_bounds__(256) gls_mu_kernel(const double* __restrict__ G, int64_t ld, int64_t npad,
                                                     int64_t nrhs, double* __restrict__ W, int64_t lda,
                                                     double* __restrict__ mu) {
  const int64_t t = blockIdx.y;
  const double c11 = -G[npad * ld + npad];
  const double c1y = -G[npad * ld + npad + 1 + t];
  const double m = c1y / c11;
  if (blockIdx.x == 0 && threadIdx.x == 0) mu[t] = m;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < lda; i += (int64_t)gridDim.x * 256)
    W[t * lda + i] = i < npad ? G[(npad + 1 + t) * ld + i] - m * G[npad * ld + i] : 0.0;
}

// ---- back substitution Lᵀ a = w (L = Uᵀ in the lower triangle) over super-blocks --------------
// Per super-block [s0, s0 + 64*nsub), last to first, two launches:
//   back_diag_kernel (1 workgroup): solve the super-block — diagonal 64-blocks from Ld (stored as
//     U_bb, read transposed), in-super-block couplings w_i -= Σ_r L[s0+64sb+r][i] a_r as
//     column-parallel GEMVs over coalesced rows of L; writes a.
//   back_update_kernel (s0/64 workgroups): w_i -= Σ_r L[s0 + r][i] a_r for i < s0, a 64-column
//     slice per workgroup, rows split over the 4 waves and reduced through LDS.
constexpr int SB = 4;  // 64-blocks per super-block
constexpr int RC = 4;  // right-hand sides per chunk
__global__ void __launch_bounds__(256) back_diag_kernel(const double* __restrict__ G, int64_t ld,
                                                        const double* __restrict__ Linv, int64_t s0, int nsub,
                                                        const double* __restrict__ W, double* __restrict__ A,
                                                        int64_t lda, int64_t nrhs) {
  __shared__ double Ui[SB][NB][NB + 1];  // Ui[sb][i][j] = (U_bb⁻¹)[i][j], b = s0/64 + sb
  __shared__ double wl[RC][SB * NB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int len = nsub * NB;
  for (int e = tid * 2; e < len * NB; e += 512) {
    const int rr = e / NB, cc = e % NB;
    const double2 v = *reinterpret_cast<const double2*>(Linv + (s0 + rr) * NB + cc);
    Ui[rr / NB][rr % NB][cc] = v.x;
    Ui[rr / NB][rr % NB][cc + 1] = v.y;
  }
  for (int64_t t0 = 0; t0 < nrhs; t0 += RC) {
    const int tc = (int)(nrhs - t0 < RC ? nrhs - t0 : RC);
    for (int e = tid; e < tc * len; e += 256) wl[e / len][e % len] = W[(t0 + e / len) * lda + s0 + e % len];
    __syncthreads();
    for (int sb = nsub - 1; sb >= 0; sb--) {
      if (wave == 0) {
        // a_b = U_bb⁻ᵀ... in Lᵀ-form: Lᵀ = U, so a_b = U_bb⁻¹ w_b — a 64x64 GEMV, no serial chain
        for (int t = 0; t < tc; t++) {
          double acc = 0.0;
#pragma unroll 16
          for (int j = 0; j < NB; j++) acc += Ui[sb][lane][j] * wl[t][sb * NB + j];
          wl[t][sb * NB + lane] = acc;
        }
      }
      __syncthreads();
      if (sb > 0 && tid < sb * NB) {  // earlier rows of the super-block (column tid)
        double acc[RC] = {0.0, 0.0, 0.0, 0.0};
        const double* lp = G + (s0 + sb * NB) * ld + s0 + tid;
        double l[NB];
#pragma unroll
        for (int u = 0; u < NB; u++) l[u] = lp[(int64_t)u * ld];
#pragma unroll
        for (int u = 0; u < NB; u++)
#pragma unroll
          for (int t = 0; t < RC; t++)
            if (t < tc) acc[t] += l[u] * wl[t][sb * NB + u];
        for (int t = 0; t < tc; t++) wl[t][tid] -= acc[t];
      }
      __syncthreads();
    }
    for (int e = tid; e < tc * len; e += 256) A[(t0 + e / len) * lda + s0 + e % len] = wl[e / len][e % len];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) back_update_kernel(const double* __restrict__ G, int64_t ld, int64_t s0,
                                                          int len, double* __restrict__ W,
                                                          const double* __restrict__ A, int64_t lda, int64_t nrhs) {
  __shared__ double part[4][RC][64];
  __shared__ double as[RC][SB * NB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  const int rows_per_wave = len / 4;
  for (int64_t t0 = 0; t0 < nrhs; t0 += RC) {
    const int tc = (int)(nrhs - t0 < RC ? nrhs - t0 : RC);
    for (int e = tid; e < tc * len; e += 256) as[e / len][e % len] = A[(t0 + e / len) * lda + s0 + e % len];
    __syncthreads();
    double acc[RC] = {0.0, 0.0, 0.0, 0.0};
    if (i < s0) {
      const double* lp = G + (s0 + wave * rows_per_wave) * ld + i;
      for (int r = 0; r < rows_per_wave; r += 16) {
        double l[16];
#pragma unroll
        for (int u = 0; u < 16; u++) l[u] = lp[(int64_t)(r + u) * ld];
#pragma unroll
        for (int u = 0; u < 16; u++)
#pragma unroll
          for (int t = 0; t < RC; t++)
            if (t < tc) acc[t] += l[u] * as[t][wave * rows_per_wave + r + u];
      }
    }
#pragma unroll
    for (int t = 0; t < RC; t++) part[wave][t][lane] = acc[t];
    __syncthreads();
    if (wave == 0 && i < s0)
      for (int t = 0; t < tc; t++)
        W[(t0 + t) * lda + i] -= ((part[0][t][lane] + part[1][t][lane]) + part[2][t][lane]) + part[3][t][lane];
    __syncthreads();
  }
}

// ---- GEBV = μ̂ + (y − μ̂) − λ a ------------------------------------------------------------
__global__ void __launch_bounds__(256) gebv_kernel(const double* __restrict__ Y, int64_t ldy, int64_t n,
                                                   const double* __restrict__ A, double* __restrict__ gebv,
                                                   int64_t lda, const double* __restrict__ mu, double lambda) {
  const int64_t t = blockIdx.y;
  const double m = mu[t];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < lda; i += (int64_t)gridDim.x * 256)
    gebv[t * lda + i] = i < n ? m + (Y[t * ldy + i] - m) - lambda * A[t * lda + i] : 0.0;
}

}  // namespace gbm

using namespace gbm;

extern "C" int64_t gbm_dev_npad(int64_t n) { return npad_of(n); }
extern "C" int64_t gbm_dev_gdim(int64_t n) { return gdim_of(n); }
// scratch: the factored 64x64 diagonal blocks and their inverses, 2 x npad x 64 doubles
extern "C" int64_t gbm_dev_solve_workspace(int64_t n, int64_t nrhs) {
  (void)nrhs;
  return 2 * npad_of(n) * NB * (int64_t)sizeof(double);
}

extern "C" int gbm_dev_gblup_solve(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev,
                                   double lambda, const double* Y, int64_t ldy, int64_t nrhs, double* A_out,
                                   double* gebv, int64_t lda, double* mu, int32_t* info, void* workspace,
                                   int64_t ws_bytes, void* stream) {
  const int64_t npad = npad_of(n), gdim = gdim_of(n);
  if (!G || !Y || !A_out || !gebv || !mu || !info || n < 1 || ldg < gdim || ldy < n || lda < npad || nrhs < 1 ||
      nrhs > MAXRHS || !(lambda > 0.0) || !(q_dev || inv_q > 0.0))
    return fail(GBM_E_ARG, "gbm_dev_gblup_solve: bad arguments (need ldg >= gdim(n), lda >= npad(n), "
                           "1 <= nrhs <= 63, lambda > 0, inv_q > 0)");
  if ((ldg & 1) || ((uintptr_t)G & 15)) return fail(GBM_E_ARG, "gbm_dev_gblup_solve: G must be 16-byte aligned, even ld");
  if (!workspace || ws_bytes < 2 * npad * NB * (int64_t)sizeof(double) || ((uintptr_t)workspace & 15))
    return fail(GBM_E_ARG, "gbm_dev_gblup_solve: workspace too small (see gbm_dev_solve_workspace)");
  double* Ld = (double*)workspace;
  double* Linv = Ld + npad * NB;
  hipStream_t s = (hipStream_t)stream;
  prepare_v_kernel<<<(unsigned)gdim, 256, 0, s>>>(G, ldg, n, npad, gdim, inv_q, q_dev, lambda, Y, ldy, nrhs, info);
  GBM_LAUNCH_CHECK();
  const int64_t nb = npad / NB;
  for (int64_t kb = 0; kb < nb; kb++) {
    const int64_t k0 = kb * NB;
    const int64_t col_blocks = (gdim - k0) / NB;  // diagonal block + column chunks
    chol_panel_kernel<<<(unsigned)col_blocks, 256, 0, s>>>(G, ldg, k0, Ld, info);
    GBM_LAUNCH_CHECK();
    int rc = launch_chol_update(G, ldg, k0, NB, gdim, s);
    if (rc != GBM_OK) return rc;
  }
  diag_inverse_kernel<<<(unsigned)nb, 64, 0, s>>>(Ld, Linv);
  GBM_LAUNCH_CHECK();
  const unsigned gx = (unsigned)((lda + 255) / 256 < 1024 ? (lda + 255) / 256 : 1024);
  // the gebv buffer doubles as the w scratch: gebv_kernel (last) reads only Y and A
  gls_mu_kernel<<<dim3(gx, (unsigned)nrhs), 256, 0, s>>>(G, ldg, npad, nrhs, gebv, lda, mu);
  GBM_LAUNCH_CHECK();
  for (int64_t end_blk = nb; end_blk > 0;) {
    const int nsub = (int)(end_blk >= SB ? SB : end_blk);
    const int64_t s0 = (end_blk - nsub) * NB;
    back_diag_kernel<<<1, 256, 0, s>>>(G, ldg, Linv, s0, nsub, gebv, A_out, lda, nrhs);
    GBM_LAUNCH_CHECK();
    if (s0 > 0) {
      back_update_kernel<<<(unsigned)(s0 / 64), 256, 0, s>>>(G, ldg, s0, nsub * NB, gebv, A_out, lda, nrhs);
      GBM_LAUNCH_CHECK();
    }
    end_blk -= nsub;
  }
  gebv_kernel<<<dim3(gx, (unsigned)nrhs), 256, 0, s>>>(Y, ldy, n, A_out, gebv, lda, mu, lambda);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}
