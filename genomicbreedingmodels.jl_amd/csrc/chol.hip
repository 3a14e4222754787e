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

// ---- panel: 256 threads, 64x64 diagonal block factored as four
//      16-wide sub-panels whose trailing updates run on the matrix cores; the 64 panel rows of
//      this workgroup are then solved against L11 block-column by block-column (MFMA for the
//      off-diagonal part, a 16-column lane-per-row substitution for the diagonal part).
//      The serial chain is 4 x (16 short columns) instead of 64 long ones.
constexpr int PS = NB + 2;  // LDS pitch (66 doubles): MFMA fragment reads conflict-free

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

// C(16x16 at (r0, c0) of dst) -= A(rows ra.., k) * B(rows rb.., k)ᵀ for k in [k0, k0 + 4*ksteps)
__device__ __forceinline__ void mfma_tile_sub(double* dst, int r0, int c0, const double* A, int ra,
                                              const double* B, int rb, int kbase, int ksteps, int lane) {
  d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
  const int fr = lane >> 4, fc = lane & 15;
  for (int ks = 0; ks < ksteps; ks++) {
    const double a = A[(ra + fc) * PS + kbase + ks * 4 + fr];
    const double b = B[(rb + fc) * PS + kbase + ks * 4 + fr];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) dst[(r0 + fr + 4 * r) * PS + c0 + fc] -= acc[r];
}

__global__ void __launch_bounds__(256) chol_panel_blocked_kernel(double* __restrict__ G, int64_t ld, int64_t k0,
                                                                 double* __restrict__ Ld,
                                                                 int32_t* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) double L[NB * PS];
  __shared__ __attribute__((aligned(16))) double X[NB * PS];
  __shared__ double rinv[NB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool diag_wg = blockIdx.x == 0;
  {
    const int row = tid >> 2, quarter = tid & 3;
    const double* sa = G + (k0 + row) * ld + k0 + quarter * 16;
    const double* sx = G + (k0 + (int64_t)blockIdx.x * NB + row) * ld + k0 + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      *reinterpret_cast<double2*>(&L[row * PS + quarter * 16 + e]) = *reinterpret_cast<const double2*>(sa + e);
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
      // (a+b) right-looking factorisation of the tall 16-column sub-panel L11[o:64, o:o+16]:
      // lane r owns row o + r; rows o..o+15 form the diagonal sub-block, the rest are solved
      // in the same 16-step loop (l_sc broadcast from lane s by v_readlane).
      const int nrows = NB - o;
      const int rr = o + (lane < nrows ? lane : 0);
      double x[16];
#pragma unroll
      for (int t = 0; t < 16; t++) x[t] = L[rr * PS + o + t];
#pragma unroll
      for (int c = 0; c < 16; c++) {
        const double piv = readlane_d(x[c], c);
        if (!(piv > 0.0) || !isfinite(piv)) {
          if (!bad) badcol = o + c;
          bad = true;
        }
        const double lc = x[c] * rsqrt_nr(piv);  // lane c: piv/sqrt(piv) = L[c][c]
#pragma unroll
        for (int sidx = c + 1; sidx < 16; sidx++) x[sidx] -= lc * readlane_d(lc, sidx);
        x[c] = lc;
      }
      if (lane < nrows) {
#pragma unroll
        for (int t = 0; t < 16; t++) L[rr * PS + o + t] = (lane < 16 && t > lane) ? 0.0 : x[t];
      }
      if (lane < 16) rinv[o + lane] = rcp_nr(x[lane & 15]);
    }
    __syncthreads();
    // (c) trailing update of L11 (16x16 lower tiles of block rows/cols > kb) on the matrix cores
    const int m = 3 - kb;
    const int ntile = m * (m + 1) / 2;
    for (int t = wave; t < ntile; t += 4) {
      int ti = 0;
      while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
      const int tj = t - ti * (ti + 1) / 2;
      const int r0 = o + 16 + ti * 16, c0 = o + 16 + tj * 16;
      mfma_tile_sub(L, r0, c0, L, r0, L, c0, o, 4, lane);
    }
    __syncthreads();
  }
  if (diag_wg) {
    if (bad && lane == 0 && wave == 0) atomicCAS(info, 0, (int32_t)(k0 + badcol + 1));
    // factored block -> scratch Ld (other workgroups of this launch still read G's copy)
    const int row = tid >> 2, quarter = tid & 3;
    double* dst = Ld + (k0 + row) * NB + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2)
      *reinterpret_cast<double2*>(dst + e) = *reinterpret_cast<const double2*>(&L[row * PS + quarter * 16 + e]);
    return;
  }
  // panel rows: X L11ᵀ = A21, block column by block column
  for (int cb = 0; cb < 4; cb++) {
    const int o = cb * 16;
    if (cb > 0) mfma_tile_sub(X, wave * 16, o, X, wave * 16, L, o, 0, cb * 4, lane);
    __syncthreads();
    if (wave == 0) {
      double x[16];
#pragma unroll
      for (int t = 0; t < 16; t++) x[t] = X[lane * PS + o + t];
#pragma unroll
      for (int c = 0; c < 16; c++) {
        x[c] *= rinv[o + c];
#pragma unroll
        for (int sidx = c + 1; sidx < 16; sidx++) x[sidx] -= x[c] * L[(o + sidx) * PS + o + c];
      }
#pragma unroll
      for (int t = 0; t < 16; t++) X[lane * PS + o + t] = x[t];
    }
    __syncthreads();
  }
  {
    const int row = tid >> 2, quarter = tid & 3;
    double* dx = G + (k0 + (int64_t)blockIdx.x * NB + row) * ld + k0 + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2)
      *reinterpret_cast<double2*>(dx + e) = *reinterpret_cast<const double2*>(&X[row * PS + quarter * 16 + e]);
  }
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
// ---- back substitution Lᵀ a = w over super-blocks of up to 4 x 64 rows --------------------
// Launch per super-block [s0, s0 + 64*nsub), last to first. Every workgroup redundantly solves
// the super-block's triangular system in LDS (4 diagonal 64-blocks from Ld + the in-block GEMV
// updates read from G), workgroup 0 stores a, and each workgroup then applies the super-block's
// contribution to its 256 columns of w[0, s0):  w_i -= Σ_r L[s0 + r][i] a_r.
// Right-hand sides are processed in chunks of 8 (LDS: 4 x 32 KB L blocks + 16 KB of w).
constexpr int SB = 4;   // 64-blocks per super-block
constexpr int RC = 8;   // rhs per chunk
__global__ void __launch_bounds__(256) back_subst_kernel(const double* __restrict__ G, int64_t ld,
                                                         const double* __restrict__ Ld, int64_t s0, int nsub,
                                                         double* __restrict__ W, double* __restrict__ A,
                                                         int64_t lda, int64_t nrhs) {
  __shared__ __attribute__((aligned(16))) double Lb[SB][NB][NB];
  __shared__ double wl[RC][SB * NB];
  __shared__ double rdiag[SB * NB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int len = nsub * NB;
  for (int e = tid * 2; e < len * NB; e += 512) {
    const int rr = e / NB, cc = e % NB;  // row within the super-block, column within its block
    *reinterpret_cast<double2*>(&Lb[rr / NB][rr % NB][cc]) =
        *reinterpret_cast<const double2*>(Ld + (s0 + rr) * NB + cc);
  }
  __syncthreads();
  if (tid < len) rdiag[tid] = rcp_nr(Lb[tid / NB][tid % NB][tid % NB]);
  for (int64_t t0 = 0; t0 < nrhs; t0 += RC) {
    const int tc = (int)(nrhs - t0 < RC ? nrhs - t0 : RC);
    for (int e = tid; e < tc * len; e += 256) wl[e / len][e % len] = W[(t0 + e / len) * lda + s0 + e % len];
    __syncthreads();
    for (int sb = nsub - 1; sb >= 0; sb--) {
      if (wave == 0) {
        for (int t = 0; t < tc; t++) {
          double x = wl[t][sb * NB + lane];
#pragma unroll
          for (int i = NB - 1; i >= 0; i--) {
            const double ai = readlane_d(x, i) * rdiag[sb * NB + i];
            x = (lane < i) ? x - Lb[sb][i][lane] * ai : (lane == i ? ai : x);
          }
          wl[t][sb * NB + lane] = x;
        }
      }
      __syncthreads();
      if (sb > 0 && tid < sb * NB) {  // in-super-block update of earlier rows (column tid)
        double acc[RC];
#pragma unroll
        for (int t = 0; t < RC; t++) acc[t] = 0.0;
        const double* lp = G + (s0 + sb * NB) * ld + s0 + tid;
        for (int r = 0; r < NB; r += 16) {
          double l[16];
#pragma unroll
          for (int u = 0; u < 16; u++) l[u] = lp[(int64_t)(r + u) * ld];
#pragma unroll
          for (int u = 0; u < 16; u++)
#pragma unroll
            for (int t = 0; t < RC; t++) acc[t] += l[u] * wl[t][sb * NB + r + u];
        }
        for (int t = 0; t < tc; t++) wl[t][tid] -= acc[t];
      }
      __syncthreads();
    }
    if (blockIdx.x == 0)
      for (int e = tid; e < tc * len; e += 256) A[(t0 + e / len) * lda + s0 + e % len] = wl[e / len][e % len];
    const int64_t i = (int64_t)blockIdx.x * 256 + tid;
    if (i < s0) {
      double acc[RC];
#pragma unroll
      for (int t = 0; t < RC; t++) acc[t] = 0.0;
      const double* lp = G + s0 * ld + i;
      for (int r = 0; r < len; r += 16) {
        double l[16];
#pragma unroll
        for (int u = 0; u < 16; u++) l[u] = lp[(int64_t)(r + u) * ld];
#pragma unroll
        for (int u = 0; u < 16; u++)
#pragma unroll
          for (int t = 0; t < RC; t++) acc[t] += l[u] * wl[t][r + u];
      }
      for (int t = 0; t < tc; t++) W[(t0 + t) * lda + i] -= acc[t];
    }
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
    chol_panel_blocked_kernel<<<(unsigned)rows_blocks, 256, 0, s>>>(G, ldg, k0, Ld, info);
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
  for (int64_t end_blk = nb; end_blk > 0;) {
    const int nsub = (int)(end_blk >= SB ? SB : end_blk);
    const int64_t s0 = (end_blk - nsub) * NB;
    const int64_t chunks = (s0 + 255) / 256;
    back_subst_kernel<<<(unsigned)(chunks > 0 ? chunks : 1), 256, 0, s>>>(G, ldg, Ld, s0, nsub, gebv, A_out, lda, nrhs);
    GBM_LAUNCH_CHECK();
    end_blk -= nsub;
  }
  gebv_kernel<<<dim3(gx, (unsigned)nrhs), 256, 0, s>>>(Y, ldy, n, A_out, gebv, lda, mu, lambda);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}
