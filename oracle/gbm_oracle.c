/*
 * gbm_oracle.c — independent plain-C (OpenMP) restatement of the GRM + GBLUP hot path.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ and __graft_entry__.smoke() as a checker; the
 * product (libgbm.so) never links or calls it. Parity against the Julia reference itself is
 * UNPINNED (julia absent, GRM in the un-vendored GenomicBreedingCore):
 * this is the second of two restatements (the other is oracle/oracle.py, numpy/LAPACK) that
 * check each other and the GPU path.
 *
 * Restates:
 *   colstats        reference src/gwas.jl:112-113 (std with ddof = 1, keep = std > eps && finite)
 *   standardise     src/gwas.jl:114,129
 *   GRM             north_star G = Z Zᵀ / q (Core grmsimple is called at src/gwas.jl:124)
 *   V, GLS, BLUP    src/gwas.jl:462-472,591-597 (V = G + λI, μ̂ = 1ᵀV⁻¹y/1ᵀV⁻¹1)
 *   b_hat layout    src/linear.jl:218-221 ([intercept; b]), predictor src/prediction.jl:228
 *
 * Build: make -C oracle   (gcc -O2 -fopenmp -shared -fPIC -> oracle/build/libgbm_oracle.so)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

/* ---- synthetic genotype generator: bit-identical to oracle.py and the HIP kernel ---- */
static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
#define KJ 0xD1B54A32D192ED03ull
#define KI 0x8CB92BA72F3D8DD7ull
#define F_LO 214748364ull
#define F_SPAN 1932735283ull

double gbm_ref_synth_genotype(uint64_t seed, int64_t i, int64_t j) {
  uint64_t base = mix64(seed * KJ + (uint64_t)j);
  uint64_t thr = F_LO + (((base >> 32) * F_SPAN) >> 32);
  uint64_t h = mix64(base ^ ((uint64_t)i * KI));
  int d = ((h & 0xFFFFFFFFull) < thr) + ((h >> 32) < thr);
  return 0.5 * (double)d;
}

/* X n x p column-major (ldx >= n), loci j0 .. j0+p-1 */
void gbm_ref_synth_matrix(uint64_t seed, int64_t n, int64_t p, int64_t j0, double* X, int64_t ldx) {
#pragma omp parallel for schedule(static)
  for (int64_t j = 0; j < p; j++)
    for (int64_t i = 0; i < n; i++) X[i + j * ldx] = gbm_ref_synth_genotype(seed, i, j0 + j);
}

/* ---- column statistics (two-pass, ddof = 1) ---- */
int64_t gbm_ref_colstats(const double* X, int64_t n, int64_t p, int64_t ldx, double* mean,
                         double* sd, uint8_t* keep) {
  int64_t q = 0;
#pragma omp parallel for schedule(static) reduction(+ : q)
  for (int64_t j = 0; j < p; j++) {
    const double* x = X + j * ldx;
    double s = 0.0;
    for (int64_t i = 0; i < n; i++) s += x[i];
    double m = s / (double)n;
    double ss = 0.0;
    for (int64_t i = 0; i < n; i++) {
      double d = x[i] - m;
      ss += d * d;
    }
    double v = n > 1 ? sqrt(ss / (double)(n - 1)) : NAN;
    int k = (v > DBL_EPSILON) && isfinite(v);
    mean[j] = m;
    sd[j] = v;
    keep[j] = (uint8_t)k;
    q += k;
  }
  return q;
}

/* Z (n x q column-major, compacted kept columns) */
static double* standardise(const double* X, int64_t n, int64_t p, int64_t ldx, const double* m,
                           const double* s, const uint8_t* keep, int64_t q, int64_t* colmap) {
  double* Z = (double*)malloc(sizeof(double) * (size_t)n * (size_t)(q > 0 ? q : 1));
  int64_t c = 0;
  for (int64_t j = 0; j < p; j++)
    if (keep[j]) colmap[c++] = j;
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < q; k++) {
    int64_t j = colmap[k];
    double inv = 1.0 / s[j];
    for (int64_t i = 0; i < n; i++) Z[i + k * n] = (X[i + j * ldx] - m[j]) * inv;
  }
  return Z;
}

/* G (n x n, full symmetric, column-major) = Z Zᵀ / q, blocked over (i, j) tiles */
static void syrk_scaled(const double* Z, int64_t n, int64_t q, double* G) {
  const int64_t BT = 64, BK = 256;
  int64_t nt = (n + BT - 1) / BT;
  double invq = 1.0 / (double)q;
#pragma omp parallel for schedule(dynamic)
  for (int64_t t = 0; t < nt * nt; t++) {
    int64_t ti = t / nt, tj = t % nt;
    if (tj > ti) continue;
    int64_t i0 = ti * BT, j0 = tj * BT;
    int64_t ib = (i0 + BT < n ? BT : n - i0), jb = (j0 + BT < n ? BT : n - j0);
    double acc[64 * 64];
    memset(acc, 0, sizeof acc);
    for (int64_t k0 = 0; k0 < q; k0 += BK) {
      int64_t kb = k0 + BK < q ? BK : q - k0;
      for (int64_t k = k0; k < k0 + kb; k++) {
        const double* zc = Z + k * n;
        for (int64_t jj = 0; jj < jb; jj++) {
          double b = zc[j0 + jj];
          double* a = acc + jj * 64;
          for (int64_t ii = 0; ii < ib; ii++) a[ii] += zc[i0 + ii] * b;
        }
      }
    }
    for (int64_t jj = 0; jj < jb; jj++)
      for (int64_t ii = 0; ii < ib; ii++) {
        double v = acc[jj * 64 + ii] * invq;
        G[(i0 + ii) + (j0 + jj) * n] = v;
        G[(j0 + jj) + (i0 + ii) * n] = v;
      }
  }
}

/* In-place lower Cholesky of V (n x n column-major), right-looking blocked. Returns 0 or the
 * 1-based failing pivot. */
static int64_t cholesky(double* V, int64_t n) {
  const int64_t NB = 64;
  for (int64_t k0 = 0; k0 < n; k0 += NB) {
    int64_t kb = k0 + NB < n ? NB : n - k0;
    /* factor the diagonal block */
    for (int64_t c = k0; c < k0 + kb; c++) {
      double d = V[c + c * n];
      for (int64_t t = k0; t < c; t++) d -= V[c + t * n] * V[c + t * n];
      if (!(d > 0.0) || !isfinite(d)) return c + 1;
      d = sqrt(d);
      V[c + c * n] = d;
      for (int64_t r = c + 1; r < k0 + kb; r++) {
        double s = V[r + c * n];
        for (int64_t t = k0; t < c; t++) s -= V[r + t * n] * V[c + t * n];
        V[r + c * n] = s / d;
      }
    }
    /* panel: rows below, L21 = A21 L11^-T */
#pragma omp parallel for schedule(static)
    for (int64_t r = k0 + kb; r < n; r++) {
      for (int64_t c = k0; c < k0 + kb; c++) {
        double s = V[r + c * n];
        for (int64_t t = k0; t < c; t++) s -= V[r + t * n] * V[c + t * n];
        V[r + c * n] = s / V[c + c * n];
      }
    }
    /* trailing update A22 -= L21 L21ᵀ (lower triangle) */
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t c = k0 + kb; c < n; c++) {
      for (int64_t t = k0; t < k0 + kb; t++) {
        double b = V[c + t * n];
        const double* l = V + t * n;
        double* col = V + c * n;
        for (int64_t r = c; r < n; r++) col[r] -= l[r] * b;
      }
    }
  }
  return 0;
}

static void chol_solve(const double* L, int64_t n, double* x) {
  for (int64_t i = 0; i < n; i++) {
    double s = x[i];
    for (int64_t t = 0; t < i; t++) s -= L[i + t * n] * x[t];
    x[i] = s / L[i + i * n];
  }
  for (int64_t i = n - 1; i >= 0; i--) {
    double s = x[i];
    for (int64_t t = i + 1; t < n; t++) s -= L[t + i * n] * x[t];
    x[i] = s / L[i + i * n];
  }
}

/* GRM only: G n x n column-major (ldg >= n). Returns q (0 = no polymorphic locus). */
int64_t gbm_ref_grm(const double* X, int64_t n, int64_t p, int64_t ldx, double* G_out, int64_t ldg) {
  double* m = (double*)malloc(sizeof(double) * p);
  double* s = (double*)malloc(sizeof(double) * p);
  uint8_t* keep = (uint8_t*)malloc(p);
  int64_t* colmap = (int64_t*)malloc(sizeof(int64_t) * p);
  int64_t q = gbm_ref_colstats(X, n, p, ldx, m, s, keep);
  if (q > 0) {
    double* Z = standardise(X, n, p, ldx, m, s, keep, q, colmap);
    double* G = (double*)malloc(sizeof(double) * n * n);
    syrk_scaled(Z, n, q, G);
    for (int64_t j = 0; j < n; j++) memcpy(G_out + j * ldg, G + j * n, sizeof(double) * n);
    free(G);
    free(Z);
  }
  free(m); free(s); free(keep); free(colmap);
  return q;
}

/*
 * Full GBLUP fit. Y n x nrhs column-major (ldy >= n); b_hat (p+1) x nrhs column-major;
 * y_pred n x nrhs column-major; mu nrhs. Returns 0, -1 (no polymorphic locus) or
 * -(1 + pivot) for a non-PD V. *q_out receives q.
 */
int64_t gbm_ref_gblup_fit(const double* X, int64_t n, int64_t p, int64_t ldx, const double* Y,
                          int64_t ldy, int64_t nrhs, double lambda, double* b_hat, double* y_pred,
                          double* mu, int64_t* q_out) {
  double* m = (double*)malloc(sizeof(double) * p);
  double* s = (double*)malloc(sizeof(double) * p);
  uint8_t* keep = (uint8_t*)malloc(p);
  int64_t* colmap = (int64_t*)malloc(sizeof(int64_t) * p);
  int64_t q = gbm_ref_colstats(X, n, p, ldx, m, s, keep);
  if (q_out) *q_out = q;
  if (q == 0) {
    free(m); free(s); free(keep); free(colmap);
    return -1;
  }
  double* Z = standardise(X, n, p, ldx, m, s, keep, q, colmap);
  double* V = (double*)malloc(sizeof(double) * n * n);
  syrk_scaled(Z, n, q, V);
  for (int64_t i = 0; i < n; i++) V[i + i * n] += lambda;
  int64_t info = cholesky(V, n);
  if (info) {
    free(V); free(Z); free(m); free(s); free(keep); free(colmap);
    return -(1 + info);
  }
  double* v1 = (double*)malloc(sizeof(double) * n);
  double* a = (double*)malloc(sizeof(double) * n);
  for (int64_t i = 0; i < n; i++) v1[i] = 1.0;
  chol_solve(V, n, v1);
  double s11 = 0.0;
  for (int64_t i = 0; i < n; i++) s11 += v1[i];
  for (int64_t t = 0; t < nrhs; t++) {
    const double* y = Y + t * ldy;
    for (int64_t i = 0; i < n; i++) a[i] = y[i];
    chol_solve(V, n, a);
    double s1y = 0.0;
    for (int64_t i = 0; i < n; i++) s1y += a[i];
    double mu_t = s1y / s11;
    /* a = V^-1 (y - mu 1) = V^-1 y - mu V^-1 1 */
    for (int64_t i = 0; i < n; i++) a[i] -= mu_t * v1[i];
    for (int64_t i = 0; i < n; i++) y_pred[i + t * n] = mu_t + (y[i] - mu_t) - lambda * a[i];
    double* b = b_hat + t * (p + 1);
    double msum = 0.0;
    for (int64_t j = 0; j < p; j++) b[1 + j] = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : msum)
    for (int64_t k = 0; k < q; k++) {
      const double* z = Z + k * n;
      double acc = 0.0;
      for (int64_t i = 0; i < n; i++) acc += z[i] * a[i];
      int64_t j = colmap[k];
      double bj = acc / (double)q / s[j];
      b[1 + j] = bj;
      msum += m[j] * bj;
    }
    b[0] = mu_t - msum;
    if (mu) mu[t] = mu_t;
  }
  free(v1); free(a); free(V); free(Z); free(m); free(s); free(keep); free(colmap);
  return 0;
}
