// GBLUP solve on the bordered matrix
//
//        [ V    Rᵀ ]      V = G/q + λI  (npad x npad, padding rows/cols = identity)
//   M =  [ R    0  ]      R = [1; y_1; ...; y_t; 0...]  (64 rows)
//
// A right-looking blocked Cholesky over the first npad columns of M (panel width 64) turns
// the R rows into W = (L⁻¹Rᵀ)ᵀ (forward substitution fused into the factorisation) and the
// bottom-right block into −W Wᵀ, from which the GLS intercept follows directly:
//   1ᵀV⁻¹1 = ‖W_0‖², 1ᵀV⁻¹y = W_0·W_y  (reference src/gwas.jl:596-597 with X = 1).
// Then a = L⁻ᵀ(W_y − μ̂ W_0) by a blocked back substitution, one launch per 64-row block,
// and GEBV = μ̂ + (y − μ̂) − λa (= μ̂ + G a since (G + λI) a = y − μ̂).
// The reference inverts V with pinv/SVD (src/gwas.jl:472,595); for λ > 0 V is SPD and the
// Cholesky solution is the same up to rounding.
#include "gbm_internal.h"

namespace gbm {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int NB = kCholNB;  // 64

// ---- V = G/q + λI, padding = identity, bordered RHS rows ------------------------------
__global__ void __launch_bounds__(256) prepare_v_kernel(double* __restrict__ G, int64_t ld, int64_t n,
                                                        int64_t npad, int64_t gdim, double inv_q,
                                                        const int64_t* __restrict__ q_dev, double lambda,
                                                        const double* __restrict__ Y, int64_t ldy, int64_t nrhs,
                                                        int32_t* __restrict__ info) {
  const int64_t i = blockIdx.x;  // row
  if (q_dev) inv_q = 1.0 / (double)(*q_dev);
  if (i == 0 && threadIdx.x == 0) *info = 0;
  double* row = G + i * ld;
  if (i < npad) {
    const int64_t jend = (i / NB + 1) * NB;  // through the end of the diagonal block
    for (int64_t j = threadIdx.x; j < jend; j += 256) {
      double v;
      if (j > i) v = 0.0;
      else if (i < n && j < n) v = row[j] * inv_q + (i == j ? lambda : 0.0);
      else v = (i == j) ? 1.0 : 0.0;
      row[j] = v;
    }
  } else {
    const int64_t t = i - npad;
    for (int64_t j = threadIdx.x; j < gdim; j += 256) {
      double v = 0.0;
      if (j < n) {
        if (t == 0) v = 1.0;
        else if (t <= nrhs) v = Y[(t - 1) * ldy + j];
      }
      row[j] = v;
    }
  }
}

// ---- panel: factor the 64x64 diagonal block (every workgroup, redundantly) and solve the
//      64 panel rows of this workgroup: L21 = A21 L11⁻ᵀ. One wave per workgroup, lane = row.
__global__ void __launch_bounds__(64) chol_panel_kernel(double* __restrict__ G, int64_t ld, int64_t k0,
                                                        double* __restrict__ Ld, int32_t* __restrict__ info) {
  __shared__ double colbuf[2][NB];
  __shared__ double Ls[NB][NB + 1];
  const int r = threadIdx.x;
  double a[NB];
  {
    const double* src = G + (k0 + r) * ld + k0;
#pragma unroll
    for (int t = 0; t < NB; t += 2) {
      const double2 v = *reinterpret_cast<const double2*>(src + t);
      a[t] = v.x;
      a[t + 1] = v.y;
    }
  }
  bool bad = false;
  int badcol = 0;
#pragma unroll
  for (int c = 0; c < NB; c++) {
    colbuf[c & 1][r] = a[c];
    __syncthreads();
    const double piv = colbuf[c & 1][c];
    if (!(piv > 0.0) || !isfinite(piv)) {
      if (!bad) badcol = c;
      bad = true;
    }
    const double d = sqrt(piv);
    const double rd = 1.0 / d;
    const double lr = (r > c) ? a[c] * rd : (r == c ? d : 0.0);
    a[c] = lr;
#pragma unroll
    for (int s = c + 1; s < NB; s++) a[s] -= lr * (colbuf[c & 1][s] * rd);
    __builtin_amdgcn_sched_barrier(0);  // keep each column's LDS reads local (register pressure)
  }
  // L11 into LDS (lower part; zeros above)
#pragma unroll
  for (int t = 0; t < NB; t++) Ls[r][t] = (t <= r) ? a[t] : 0.0;
  if (blockIdx.x == 0) {
    // The factored block goes to the scratch Ld (not in place): the other workgroups of this
    // launch are still reading the unfactored block from G.
    if (bad && r == 0) atomicCAS(info, 0, (int32_t)(k0 + badcol + 1));
    double* dst = Ld + (k0 + r) * NB;
#pragma unroll
    for (int t = 0; t < NB; t += 2)
      *reinterpret_cast<double2*>(dst + t) = make_double2(t <= r ? a[t] : 0.0, t + 1 <= r ? a[t + 1] : 0.0);
    return;
  }
  __syncthreads();
  // panel rows: x Lᵀ = a  ->  x_c = (a_c − Σ_{t<c} x_t L[c][t]) / L[c][c]
  double* rowp = G + (k0 + (int64_t)blockIdx.x * NB + r) * ld + k0;
  double x[NB];
#pragma unroll
  for (int t = 0; t < NB; t += 2) {
    const double2 v = *reinterpret_cast<const double2*>(rowp + t);
    x[t] = v.x;
    x[t + 1] = v.y;
  }
#pragma unroll
  for (int c = 0; c < NB; c++) {
    x[c] = x[c] / Ls[c][c];
#pragma unroll
    for (int s = c + 1; s < NB; s++) x[s] -= x[c] * Ls[s][c];
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int t = 0; t < NB; t += 2) *reinterpret_cast<double2*>(rowp + t) = make_double2(x[t], x[t + 1]);
}

// ---- trailing update: C -= L21 L21ᵀ on lower 64x64 tiles of rows/cols >= k1 (fp64 MFMA) ----
constexpr int UPS = NB + 2;  // LDS row pitch (66 doubles): conflict-free ds_read_b64 fragments

__device__ __forceinline__ void tri_of(int64_t t, int64_t& ti, int64_t& tj) {
  int64_t r = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) r++;
  while (r * (r + 1) / 2 > t) r--;
  ti = r;
  tj = t - r * (r + 1) / 2;
}

__global__ void __launch_bounds__(256) chol_update_kernel(double* __restrict__ G, int64_t ld, int64_t k0) {
  __shared__ __attribute__((aligned(16))) double As[NB * UPS];
  __shared__ __attribute__((aligned(16))) double Bs[NB * UPS];
  int64_t ti, tj;
  tri_of(blockIdx.x, ti, tj);
  const bool diag = ti == tj;
  const int64_t k1 = k0 + NB;
  const int64_t i0 = k1 + ti * NB, j0 = k1 + tj * NB;
  {
    const int row = threadIdx.x >> 2, quarter = threadIdx.x & 3;
    const double* sa = G + (i0 + row) * ld + k0 + quarter * 16;
    const double* sb = G + (j0 + row) * ld + k0 + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      *reinterpret_cast<double2*>(&As[row * UPS + quarter * 16 + e]) = *reinterpret_cast<const double2*>(sa + e);
      if (!diag)
        *reinterpret_cast<double2*>(&Bs[row * UPS + quarter * 16 + e]) = *reinterpret_cast<const double2*>(sb + e);
    }
  }
  __syncthreads();
  const double* B = diag ? As : Bs;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane >> 4, fc = lane & 15;
  d4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; m++)
#pragma unroll
    for (int q = 0; q < 2; q++) acc[m][q] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < NB / 4; ks++) {
    double af[2], bf[2];
#pragma unroll
    for (int m = 0; m < 2; m++) af[m] = As[(wm * 32 + m * 16 + fc) * UPS + ks * 4 + fr];
#pragma unroll
    for (int q = 0; q < 2; q++) bf[q] = B[(wn * 32 + q * 16 + fc) * UPS + ks * 4 + fr];
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
        G[row * ld + col] -= acc[m][q][r];
      }
}

// ---- μ̂ and the back-substitution right-hand sides w_t = W_{1+t} − μ̂_t W_0 ------------
__global__ void __launch_bounds__(256) gls_mu_kernel(const double* __restrict__ G, int64_t ld, int64_t npad,
                                                     int64_t nrhs, double* __restrict__ W, int64_t lda,
                                                     double* __restrict__ mu) {
  const int64_t t = blockIdx.y;
  const double c11 = -G[npad * ld + npad];
  const double c1y = -G[(npad + 1 + t) * ld + npad];
  const double m = c1y / c11;
  if (blockIdx.x == 0 && threadIdx.x == 0) mu[t] = m;
  const double* w0 = G + npad * ld;
  const double* wy = G + (npad + 1 + t) * ld;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < lda; i += (int64_t)gridDim.x * 256)
    W[t * lda + i] = i < npad ? wy[i] - m * w0[i] : 0.0;
}

// ---- back substitution Lᵀ a = w, block b (rows [b*64, b*64+64)), all right-hand sides --
// Every workgroup solves the 64x64 diagonal system (cheap, redundant) from W (read-only for
// rows >= b*64 in this launch), workgroup 0 stores a_b into A, and each workgroup then updates
// its 256-column chunk of w[0, b*64):
//   w_i -= Σ_r L[b*64 + r][i] a_b[r].
constexpr int MAXRHS = 63;
__global__ void __launch_bounds__(256) back_subst_kernel(const double* __restrict__ G, int64_t ld,
                                                         const double* __restrict__ Ld, int64_t b,
                                                         double* __restrict__ W, double* __restrict__ A,
                                                         int64_t lda, int64_t nrhs) {
  __shared__ double Lb[NB][NB + 1];
  __shared__ double ab[MAXRHS][NB];
  const int64_t r0 = b * NB;
  for (int e = threadIdx.x; e < NB * NB; e += 256) {
    const int rr = e / NB, cc = e % NB;
    Lb[rr][cc] = Ld[(r0 + rr) * NB + cc];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int r = threadIdx.x;
    for (int64_t t = 0; t < nrhs; t++) {
      double x = W[t * lda + r0 + r];
      for (int i = NB - 1; i >= 0; i--) {
        const double xi = x / Lb[i][i];
        const double ai = __shfl(xi, i, 64);
        if (r == i) x = ai;
        else if (r < i) x -= Lb[i][r] * ai;
      }
      ab[t][r] = x;
      if (blockIdx.x == 0) A[t * lda + r0 + r] = x;
    }
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < r0) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int64_t t0 = 0; t0 < nrhs; t0 += 4) {
      for (int r = 0; r < NB; r++) {
        const double l = G[(r0 + r) * ld + i];
#pragma unroll
        for (int u = 0; u < 4; u++)
          if (t0 + u < nrhs) acc[u] += l * ab[t0 + u][r];
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (t0 + u < nrhs) {
          W[(t0 + u) * lda + i] -= acc[u];
          acc[u] = 0.0;
        }
    }
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
// scratch: the factored 64x64 diagonal blocks, npad x 64 doubles
extern "C" int64_t gbm_dev_solve_workspace(int64_t n, int64_t nrhs) {
  (void)nrhs;
  return npad_of(n) * NB * (int64_t)sizeof(double);
}

extern "C" int gbm_dev_gblup_solve(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev,
                                   double lambda,
                                   const double* Y, int64_t ldy, int64_t nrhs, double* A_out, double* gebv,
                                   int64_t lda, double* mu, int32_t* info, void* workspace, int64_t ws_bytes,
                                   void* stream) {
  const int64_t npad = npad_of(n), gdim = gdim_of(n);
  if (!G || !Y || !A_out || !gebv || !mu || !info || n < 1 || ldg < gdim || ldy < n || lda < npad || nrhs < 1 ||
      nrhs > MAXRHS || !(lambda > 0.0) || !(q_dev || inv_q > 0.0))
    return fail(GBM_E_ARG, "gbm_dev_gblup_solve: bad arguments (need ldg >= gdim(n), lda >= npad(n), "
                           "1 <= nrhs <= 63, lambda > 0, inv_q > 0)");
  if ((ldg & 1) || ((uintptr_t)G & 15)) return fail(GBM_E_ARG, "gbm_dev_gblup_solve: G must be 16-byte aligned, even ld");
  if (!workspace || ws_bytes < npad * NB * (int64_t)sizeof(double) || ((uintptr_t)workspace & 15))
    return fail(GBM_E_ARG, "gbm_dev_gblup_solve: workspace too small (see gbm_dev_solve_workspace)");
  double* Ld = (double*)workspace;
  hipStream_t s = (hipStream_t)stream;
  prepare_v_kernel<<<(unsigned)gdim, 256, 0, s>>>(G, ldg, n, npad, gdim, inv_q, q_dev, lambda, Y, ldy, nrhs, info);
  GBM_LAUNCH_CHECK();
  const int64_t nb = npad / NB;
  for (int64_t kb = 0; kb < nb; kb++) {
    const int64_t k0 = kb * NB;
    const int64_t rows_blocks = (gdim - k0) / NB;  // diagonal block + panel blocks
    chol_panel_kernel<<<(unsigned)rows_blocks, 64, 0, s>>>(G, ldg, k0, Ld, info);
    GBM_LAUNCH_CHECK();
    const int64_t nt2 = rows_blocks - 1;
    if (nt2 > 0) {
      chol_update_kernel<<<(unsigned)(nt2 * (nt2 + 1) / 2), 256, 0, s>>>(G, ldg, k0);
      GBM_LAUNCH_CHECK();
    }
  }
  const unsigned gx = (unsigned)((lda + 255) / 256 < 1024 ? (lda + 255) / 256 : 1024);
  // the gebv buffer doubles as the w scratch: gebv_kernel (last) reads only Y and A
  gls_mu_kernel<<<dim3(gx, (unsigned)nrhs), 256, 0, s>>>(G, ldg, npad, nrhs, gebv, lda, mu);
  GBM_LAUNCH_CHECK();
  for (int64_t b = nb - 1; b >= 0; b--) {
    const int64_t chunks = (b * NB + 255) / 256;
    back_subst_kernel<<<(unsigned)(chunks > 0 ? chunks : 1), 256, 0, s>>>(G, ldg, Ld, b, gebv, A_out, lda, nrhs);
    GBM_LAUNCH_CHECK();
  }
  gebv_kernel<<<dim3(gx, (unsigned)nrhs), 256, 0, s>>>(Y, ldy, n, A_out, gebv, lda, mu, lambda);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}
