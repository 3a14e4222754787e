// Device-resident genotype sessions: fold farming for cross-validation (SURVEY.md §8f row 1,
// config C5) and REML choice of λ (§8f row 2).
//
// A session uploads X once to one device (locus-major, individuals contiguous) and then fits
// GBLUP on entry subsets: the training columns are gathered on the device inside the
// standardisation pass, and the standardised training genotypes + their GRM are cached, keyed by
// the training set, so further traits, λ values or REML evaluations on the same set skip the
// SYRK. This replaces the per-fold `model(genomes=..., idx_entries=idx_training, ...)` calls of
// reference src/cross_validation.jl:159-186 (cvmultithread!), which re-extract X and rebuild
// everything per fold. One session per device; a session serialises its own calls (mutex),
// sessions on different devices run concurrently (one host thread each).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <mutex>
#include <vector>

#include "gbm_internal.h"
#include "host_util.h"

struct gbm_session {
  std::mutex mu;
  int dev = 0;
  gbm::Stream stream;
  int64_t n = 0, p = 0, npad = 0;
  gbm::DevMem Xt;  // p x npad raw genotypes
  // training-set cache (key: the entry set and the standardisation mode)
  std::vector<int64_t> key;
  int mode = -1;  // 0: GBLUP standardisation, 1: centre only (glmnet standardize=false)
  int64_t nT = 0, npadT = 0, gdimT = 0, q = 0;
  gbm::DevMem idx32, Z, mean, sd, keep, qd, Gc, wsg;
  // per-fit buffers (sized for the cached training set)
  int64_t nrhs_cap = 0;
  gbm::DevMem Gw, wss, Y, A, gebv, mu_d, info, B, msum, terms;
  // predict buffers
  gbm::DevMem bvec, part, pout;
  int64_t builds = 0, hits = 0;
  // genotypes that are diploid dosages/2 (2x ∈ {0, 1, 2} in every cell: synthetic sessions by construction,
  // others checked on the device once, when a fit first asks for it): grm_mode exact / auto
  // (gbm_session_set_grm_mode, else GBM_GRM) builds the training GRM with the exact-integer kernels
  // (grm_exact.hip) from the gathered training dosages
  bool dosage2 = false, dosage_checked = false;
  int grm_mode = GBM_GRM_DEFAULT;
  bool exact_cached = false;  // the cached training GRM is the exact one (part of the cache key)
  gbm::DevMem D8T, wsx, mean2, sd2, keep2, q2;
  int64_t d8t_bytes = 0, wsx_bytes = 0;
};

namespace gbm {

// Reference loglikreml (src/gwas.jl:450-483) with X = 1 and V = σ²_u GRM + σ²_e I, from the
// terms of one solve at λ = σ²_e/σ²_u: logdet V = n log σ²_u + logdet V_λ, yᵀPy = Q_λ/σ²_u,
// logdet XᵀV⁻¹X = log c11_λ − log σ²_u.
double reml_objective(int64_t n, double logdet, double c11, double Q, double s2u) {
  return 0.5 * ((double)n * std::log(s2u) + logdet) + Q / s2u + std::log(c11) - std::log(s2u);
}

// g(λ): the objective minimised over σ²_u inside the reference's box (σ²_e, σ²_u ∈ [eps, 1]),
// σ²_e = λσ²_u. For fixed λ the objective is a log σ + Q/σ with a = n/2 − 1 > 0: unimodal, its
// minimiser Q/a clamped to the box. t = {logdet V_λ, 1ᵀV_λ⁻¹1, 1ᵀV_λ⁻¹y, yᵀV_λ⁻¹y}.
RemlEval reml_profile(int64_t n, double lambda, const double t[4]) {
  const double logdet = t[0], c11 = t[1], c1y = t[2], yy = t[3];
  const double Q = yy - c1y * c1y / c11;
  const double eps = std::numeric_limits<double>::epsilon();
  const double lo = std::max(eps, eps / lambda), hi = std::min(1.0, 1.0 / lambda);
  const double a = 0.5 * (double)n - 1.0;
  double s2u = Q / a;
  if (!(s2u >= lo)) s2u = lo;
  if (s2u > hi) s2u = hi;
  return {reml_objective(n, logdet, c11, Q, s2u), s2u, lambda * s2u};
}

// The search of gbm_session_reml and gbm_gblup_fit_reml: a scan of log10 λ over [-6, 6] in steps of
// 0.5, then golden-section refinement on [best − 0.5, best + 0.5] (to 1e-7 in log10 λ).
int reml_search(const std::function<int(double, RemlEval&)>& eval, RemlResult& out) {
  auto g = [&](double loglam, RemlEval& e) { return eval(std::pow(10.0, loglam), e); };
  double best_x = 0.0;
  RemlEval best{std::numeric_limits<double>::infinity(), 0.0, 0.0};
  for (int k = -12; k <= 12; k++) {
    RemlEval e;
    GBM_TRY(g(0.5 * k, e));
    if (e.g < best.g) {
      best = e;
      best_x = 0.5 * k;
    }
  }
  double a = best_x - 0.5, b = best_x + 0.5;
  const double r = 0.5 * (std::sqrt(5.0) - 1.0);
  double c = b - r * (b - a), d = a + r * (b - a);
  RemlEval ec, ed;
  GBM_TRY(g(c, ec));
  GBM_TRY(g(d, ed));
  for (int it = 0; it < 60 && (b - a) > 1e-7; it++) {
    if (ec.g < ed.g) {
      b = d;
      d = c;
      ed = ec;
      c = b - r * (b - a);
      GBM_TRY(g(c, ec));
    } else {
      a = c;
      c = d;
      ec = ed;
      d = a + r * (b - a);
      GBM_TRY(g(d, ed));
    }
  }
  const RemlEval& fin = ec.g < ed.g ? ec : ed;
  const double fin_x = ec.g < ed.g ? c : d;
  if (fin.g < best.g) {
    best = fin;
    best_x = fin_x;
  }
  out = {std::pow(10.0, best_x), best.s2e, best.s2u, best.g};
  return GBM_OK;
}

// y standardised as the reference's gwasprep does before REML (src/gwas.jl:127-128; sd ddof = 1)
std::vector<double> standardise_y(const double* y, int64_t n) {
  std::vector<double> ys(y, y + n);
  double m = 0.0;
  for (double v : ys) m += v;
  m /= (double)n;
  double ss = 0.0;
  for (double v : ys) ss += (v - m) * (v - m);
  const double sdv = std::sqrt(ss / (double)(n - 1));
  for (double& v : ys) v = (v - m) / sdv;
  return ys;
}

namespace {

int session_alloc_x(gbm_session* s) {
  GBM_HIP_TRY(hipSetDevice(s->dev));
  s->stream.dev = s->dev;
  GBM_HIP_TRY(hipStreamCreateWithFlags(&s->stream.s, hipStreamNonBlocking));
  s->npad = npad_of(s->n);
  GBM_TRY(dalloc(s->Xt, s->dev, s->p * s->npad * 8));
  GBM_HIP_TRY(hipMemsetAsync(s->Xt.p, 0, (size_t)(s->p * s->npad * 8), s->stream.s));
  return GBM_OK;
}

int check_idx(const gbm_session* s, const int64_t* idx, int64_t m, const char* what) {
  if (!idx || m < 1) return fail(GBM_E_ARG, std::string(what) + ": empty entry index");
  for (int64_t i = 0; i < m; i++) {
    if (idx[i] < 0 || idx[i] >= s->n)
      return fail(GBM_E_ARG, std::string(what) + ": entry index " + std::to_string(idx[i]) + " out of range [0, " +
                                 std::to_string(s->n) + ")");
    if (i > 0 && idx[i] <= idx[i - 1])
      return fail(GBM_E_ARG, std::string(what) + ": entry indices must be strictly increasing");
  }
  return GBM_OK;
}

// Whether the session's genotypes are diploid dosages/2 (one device pass over X, the first time it is asked).
int session_dosage2(gbm_session* s, bool& out) {
  if (!s->dosage_checked) {
    GBM_TRY(dalloc(s->q2, s->dev, 8));
    GBM_HIP_TRY(hipMemsetAsync(s->q2.p, 0, 4, s->stream.s));
    GBM_TRY(launch_dosage_from_f64((const double*)s->Xt.p, s->npad, s->n, s->p, nullptr, 0, (int32_t*)s->q2.p,
                                   s->stream.s));
    int32_t bad = 0;
    GBM_HIP_TRY(hipMemcpyAsync(&bad, s->q2.p, 4, hipMemcpyDeviceToHost, s->stream.s));
    GBM_HIP_TRY(hipStreamSynchronize(s->stream.s));
    s->dosage2 = bad == 0;
    s->dosage_checked = true;
  }
  out = s->dosage2;
  return GBM_OK;
}

// Standardise (mode 0) or centre (mode 1) the training set idx and build its GRM (cached).
int ensure_training(gbm_session* s, const int64_t* idx, int64_t nT, int mode = 0) {
  GBM_TRY(check_idx(s, idx, nT, "gbm_session"));
  if (nT < 2) return fail(GBM_E_DATA, "there are less than 2 entries (reference src/prediction.jl:117-123)");
  bool exact = false;
  const int gm = resolve_grm_mode(s->grm_mode);
  if (mode == 0 && gm != GBM_GRM_FP64) {
    GBM_TRY(session_dosage2(s, exact));
    if (!exact && gm == GBM_GRM_EXACT)
      return fail(GBM_E_ARG, "grm_mode exact: the session's genotypes are not diploid dosages (2x must be exactly 0, "
                             "1 or 2 in every cell; use grm_mode auto or fp64)");
  }
  if (s->mode == mode && s->exact_cached == exact && (int64_t)s->key.size() == nT &&
      std::memcmp(s->key.data(), idx, (size_t)nT * 8) == 0) {
    s->hits++;
    return GBM_OK;
  }
  s->key.clear();
  hipStream_t st = s->stream.s;
  const int64_t npadT = npad_of(nT), gdimT = gdim_of(nT);
  if (npadT != s->npadT) {
    GBM_TRY(dalloc(s->Z, s->dev, s->p * npadT * 8));
    GBM_TRY(dalloc(s->Gc, s->dev, gdimT * gdimT * 8));
    GBM_TRY(dalloc(s->Gw, s->dev, gdimT * gdimT * 8));
    GBM_TRY(dalloc(s->wss, s->dev, gbm_dev_solve_workspace(nT, 63)));
    s->nrhs_cap = 0;
    s->npadT = npadT;
    s->gdimT = gdimT;
  }
  if (!s->mean.p) {
    GBM_TRY(dalloc(s->mean, s->dev, s->p * 8));
    GBM_TRY(dalloc(s->sd, s->dev, s->p * 8));
    GBM_TRY(dalloc(s->keep, s->dev, s->p * 4));
    GBM_TRY(dalloc(s->qd, s->dev, 8));
  }
  GBM_TRY(dalloc(s->idx32, s->dev, nT * 4));
  const int64_t wsb = gbm_dev_grm_workspace(nT, s->p);
  GBM_TRY(dalloc(s->wsg, s->dev, wsb));
  std::vector<int32_t> i32(idx, idx + nT);
  GBM_HIP_TRY(hipMemcpyAsync(s->idx32.p, i32.data(), nT * 4, hipMemcpyHostToDevice, st));
  GBM_HIP_TRY(hipMemsetAsync(s->qd.p, 0, 8, st));
  GBM_TRY(gbm_dev_standardize_gather((const double*)s->Xt.p, s->npad, s->p, (const int32_t*)s->idx32.p, nT,
                                     (double*)s->Z.p, npadT, (double*)s->mean.p, (double*)s->sd.p,
                                     (int32_t*)s->keep.p, (int64_t*)s->qd.p, mode, st));
  int64_t q = 0;
  GBM_HIP_TRY(hipMemcpyAsync(&q, s->qd.p, 8, hipMemcpyDeviceToHost, st));
  GBM_HIP_TRY(hipStreamSynchronize(st));
  if (q == 0) return fail(GBM_E_DATA, "no polymorphic locus-allele in the training set (src/gwas.jl:112-115)");
  if (exact) {
    // exact-integer GRM of the training dosages; its per-locus statistics go to scratch (Z, mean and sd
    // above are what the marker effects and predictions use; q is the same count)
    if (s->d8t_bytes < s->p * nT) {
      GBM_TRY(dalloc(s->D8T, s->dev, s->p * nT));
      s->d8t_bytes = s->p * nT;
    }
    const int64_t wsx = gbm_dev_grm_exact_workspace(nT, s->p);
    if (s->wsx_bytes < wsx) {
      GBM_TRY(dalloc(s->wsx, s->dev, wsx));
      s->wsx_bytes = wsx;
    }
    if (!s->mean2.p) {
      GBM_TRY(dalloc(s->mean2, s->dev, s->p * 8));
      GBM_TRY(dalloc(s->sd2, s->dev, s->p * 8));
      GBM_TRY(dalloc(s->keep2, s->dev, s->p * 4));
      GBM_TRY(dalloc(s->q2, s->dev, 8));
    }
    GBM_TRY(launch_gather_dosage((const double*)s->Xt.p, s->npad, s->p, (const int32_t*)s->idx32.p, nT,
                                 (int8_t*)s->D8T.p, st));
    GBM_HIP_TRY(hipMemsetAsync(s->q2.p, 0, 8, st));
    GBM_TRY(launch_grm_exact((const int8_t*)s->D8T.p, nT, s->p, nT, 2, (double*)s->Gc.p, gdimT, (double*)s->mean2.p,
                             (double*)s->sd2.p, (int32_t*)s->keep2.p, (int64_t*)s->q2.p, 0, s->wsx.p, wsx, nullptr, st));
    GBM_TRY(grm_exact_status(s->wsx.p, nT, s->p, st));
  } else {
    GBM_TRY(gbm_dev_grm((const double*)s->Z.p, npadT, s->p, nT, (double*)s->Gc.p, gdimT, s->wsg.p, wsb, st));
  }
  s->nT = nT;
  s->q = q;
  s->key.assign(idx, idx + nT);
  s->mode = mode;
  s->exact_cached = exact;
  s->builds++;
  return GBM_OK;
}

int ensure_rhs(gbm_session* s, int64_t nrhs) {
  if (nrhs <= s->nrhs_cap) return GBM_OK;
  const int64_t npadT = s->npadT;
  GBM_TRY(dalloc(s->Y, s->dev, nrhs * npadT * 8));
  GBM_TRY(dalloc(s->A, s->dev, nrhs * npadT * 8));
  GBM_TRY(dalloc(s->gebv, s->dev, nrhs * npadT * 8));
  GBM_TRY(dalloc(s->mu_d, s->dev, nrhs * 8));
  GBM_TRY(dalloc(s->info, s->dev, 4));
  GBM_TRY(dalloc(s->B, s->dev, nrhs * s->p * 8));
  GBM_TRY(dalloc(s->msum, s->dev, nrhs * 8));
  GBM_TRY(dalloc(s->terms, s->dev, (2 + 2 * nrhs) * 8));
  s->nrhs_cap = nrhs;
  return GBM_OK;
}

// Solve (G·inv_q + λI) on the cached GRM for the nrhs phenotype columns already in s->Y
// (inv_q = 1/q for GBLUP, 1 for the unscaled ridge kernel).
int solve_cached(gbm_session* s, int64_t nrhs, double lambda, double inv_q) {
  hipStream_t st = s->stream.s;
  // the solve factors in place: work on a copy of the cached GRM (rows [0, npad) are read)
  GBM_HIP_TRY(hipMemcpyAsync(s->Gw.p, s->Gc.p, (size_t)(s->npadT * s->gdimT * 8), hipMemcpyDeviceToDevice, st));
  GBM_TRY(gbm_dev_gblup_solve((double*)s->Gw.p, s->gdimT, s->nT, inv_q, nullptr, lambda,
                              (const double*)s->Y.p, s->npadT, nrhs, (double*)s->A.p, (double*)s->gebv.p, s->npadT,
                              (double*)s->mu_d.p, (int32_t*)s->info.p, s->wss.p,
                              gbm_dev_solve_workspace(s->nT, 63), st));
  int32_t info = 0;
  GBM_HIP_TRY(hipMemcpyAsync(&info, s->info.p, 4, hipMemcpyDeviceToHost, st));
  GBM_HIP_TRY(hipStreamSynchronize(st));
  if (info < 0) return fail(GBM_E_HIP, "solve: a wait between workgroups timed out (dataflow Cholesky or back substitution; the result is invalid)");
  if (info != 0)
    return fail(GBM_E_NOTPD, "G/q + lambda*I is not positive definite (pivot " + std::to_string(info) + ")");
  return GBM_OK;
}

int upload_y(gbm_session* s, const double* Y, int64_t ldy, int64_t nrhs) {
  GBM_HIP_TRY(hipMemsetAsync(s->Y.p, 0, (size_t)(nrhs * s->npadT * 8), s->stream.s));
  GBM_HIP_TRY(hipMemcpy2DAsync(s->Y.p, s->npadT * 8, Y, ldy * 8, s->nT * 8, nrhs, hipMemcpyHostToDevice, s->stream.s));
  return GBM_OK;
}

int reml_eval(gbm_session* s, double lambda, RemlEval& out) {
  GBM_TRY(solve_cached(s, 1, lambda, 1.0 / (double)s->q));
  double t[4];
  GBM_TRY(gbm_dev_gblup_terms((const double*)s->Gw.p, s->gdimT, s->nT, 1, s->wss.p, (double*)s->terms.p,
                              s->stream.s));
  GBM_HIP_TRY(hipMemcpyAsync(t, s->terms.p, 4 * 8, hipMemcpyDeviceToHost, s->stream.s));
  GBM_HIP_TRY(hipStreamSynchronize(s->stream.s));
  out = reml_profile(s->nT, lambda, t);
  return GBM_OK;
}

}  // namespace
}  // namespace gbm

using namespace gbm;

extern "C" int gbm_session_create(const double* X, int64_t n, int64_t p, int64_t ldx, int device, gbm_session** out) {
  RoctxRange r_("gbm_session_create");
  if (!out) return fail(GBM_E_ARG, "gbm_session_create: out is NULL");
  *out = nullptr;
  if (!X || n < 1 || p < 1 || ldx < n) return fail(GBM_E_ARG, "gbm_session_create: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(&device, 1, devs));
  auto s = new gbm_session();
  s->dev = devs[0];
  s->n = n;
  s->p = p;
  int rc = session_alloc_x(s);
  if (rc == GBM_OK) {
    if (hipMemcpy2DAsync(s->Xt.p, s->npad * 8, X, ldx * 8, n * 8, p, hipMemcpyHostToDevice, s->stream.s) !=
            hipSuccess ||
        hipStreamSynchronize(s->stream.s) != hipSuccess)
      rc = fail(GBM_E_HIP, "gbm_session_create: upload failed");
  }
  if (rc != GBM_OK) {
    delete s;
    return rc;
  }
  *out = s;
  return GBM_OK;
}

extern "C" int gbm_session_create_synthetic(uint64_t seed, int64_t n, int64_t p, int device, gbm_session** out) {
  RoctxRange r_("gbm_session_create_synthetic");
  if (!out) return fail(GBM_E_ARG, "gbm_session_create_synthetic: out is NULL");
  *out = nullptr;
  if (n < 1 || p < 1) return fail(GBM_E_ARG, "gbm_session_create_synthetic: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(&device, 1, devs));
  auto s = new gbm_session();
  s->dev = devs[0];
  s->n = n;
  s->p = p;
  int rc = session_alloc_x(s);
  if (rc == GBM_OK) rc = gbm_dev_synth_genotypes((double*)s->Xt.p, s->npad, p, n, seed, 0, s->stream.s);
  s->dosage2 = s->dosage_checked = true;  // X = dosage/2 (SURVEY.md §8d generator)
  if (rc == GBM_OK && hipStreamSynchronize(s->stream.s) != hipSuccess)
    rc = fail(GBM_E_HIP, "gbm_session_create_synthetic: generation failed");
  if (rc != GBM_OK) {
    delete s;
    return rc;
  }
  *out = s;
  return GBM_OK;
}

extern "C" int gbm_session_create_dosage_i8(const int8_t* D, int64_t n, int64_t p, int64_t ldd, int ploidy,
                                            int device, gbm_session** out) {
  RoctxRange r_("gbm_session_create_dosage_i8");
  if (!out) return fail(GBM_E_ARG, "gbm_session_create_dosage_i8: out is NULL");
  *out = nullptr;
  if (!D || n < 1 || p < 1 || ldd < n || ploidy < 1)
    return fail(GBM_E_ARG, "gbm_session_create_dosage_i8: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(&device, 1, devs));
  auto s = new gbm_session();
  s->dev = devs[0];
  s->n = n;
  s->p = p;
  int rc = session_alloc_x(s);
  DevMem d8;
  if (rc == GBM_OK) rc = dalloc(d8, s->dev, n * p);
  if (rc == GBM_OK && (hipMemcpy2DAsync(d8.p, n, D, ldd, n, p, hipMemcpyHostToDevice, s->stream.s) != hipSuccess))
    rc = fail(GBM_E_HIP, "gbm_session_create_dosage_i8: upload failed");
  if (rc == GBM_OK) rc = gbm_dev_expand_dosage_i8((const int8_t*)d8.p, n, n, p, ploidy, (double*)s->Xt.p, s->npad,
                                                  s->stream.s);
  if (rc == GBM_OK && hipStreamSynchronize(s->stream.s) != hipSuccess) rc = fail(GBM_E_HIP, "stream sync");
  if (rc != GBM_OK) {
    delete s;
    return rc;
  }
  *out = s;
  return GBM_OK;
}

extern "C" int gbm_session_set_grm_mode(gbm_session* s, int grm_mode) {
  if (!s) return fail(GBM_E_ARG, "gbm_session_set_grm_mode: session is NULL");
  if (grm_mode < GBM_GRM_DEFAULT || grm_mode > GBM_GRM_DROPIN)
    return fail(GBM_E_ARG, "gbm_session_set_grm_mode: grm_mode must be GBM_GRM_DEFAULT, _FP64, _EXACT, _AUTO or _DROPIN");
  std::lock_guard<std::mutex> lock(s->mu);
  s->grm_mode = grm_mode;
  return GBM_OK;
}

extern "C" int gbm_session_grm_used(gbm_session* s, int* grm_used) {
  if (!s || !grm_used) return fail(GBM_E_ARG, "gbm_session_grm_used: NULL argument");
  std::lock_guard<std::mutex> lock(s->mu);
  *grm_used = s->key.empty() ? -1 : s->exact_cached ? GBM_GRM_EXACT : GBM_GRM_FP64;
  return GBM_OK;
}

extern "C" void gbm_session_destroy(gbm_session* s) {
  if (!s) return;
  (void)hipSetDevice(s->dev);
  delete s;
}

extern "C" int gbm_session_gblup_fit(gbm_session* s, const int64_t* idx, int64_t n_train, const double* Y, int64_t ldy,
                                     int64_t nrhs, double lambda, double* b_hat_out, double* y_pred_out, double* mu_out,
                                     int64_t* q_out) {
  RoctxRange r_("gbm_session_gblup_fit");
  if (!s) return fail(GBM_E_ARG, "gbm_session_gblup_fit: session is NULL");
  if (!Y || ldy < n_train || nrhs < 1 || nrhs > 63 || !b_hat_out || !y_pred_out)
    return fail(GBM_E_ARG, "gbm_session_gblup_fit: bad arguments (ldy >= n_train, 1 <= nrhs <= 63, outputs)");
  if (!(lambda > 0.0) || !std::isfinite(lambda)) return fail(GBM_E_ARG, "gbm_session_gblup_fit: lambda must be > 0");
  std::lock_guard<std::mutex> lock(s->mu);
  GBM_HIP_TRY(hipSetDevice(s->dev));
  GBM_TRY(check_y(Y, n_train, ldy, nrhs));
  GBM_TRY(ensure_training(s, idx, n_train));
  GBM_TRY(ensure_rhs(s, nrhs));
  GBM_TRY(upload_y(s, Y, ldy, nrhs));
  GBM_TRY(solve_cached(s, nrhs, lambda, 1.0 / (double)s->q));
  hipStream_t st = s->stream.s;
  const int64_t p = s->p;
  GBM_TRY(gbm_dev_marker_effects((const double*)s->Z.p, s->npadT, p, s->nT, (const double*)s->A.p, s->npadT, nrhs,
                                 1.0 / (double)s->q, nullptr, (const double*)s->mean.p, (const double*)s->sd.p,
                                 (const int32_t*)s->keep.p, (double*)s->B.p, p, (double*)s->msum.p, st));
  std::vector<double> mu(nrhs), msum(nrhs);
  GBM_HIP_TRY(hipMemcpy2DAsync(b_hat_out + 1, (p + 1) * 8, s->B.p, p * 8, p * 8, nrhs, hipMemcpyDeviceToHost, st));
  GBM_HIP_TRY(hipMemcpy2DAsync(y_pred_out, n_train * 8, s->gebv.p, s->npadT * 8, n_train * 8, nrhs,
                               hipMemcpyDeviceToHost, st));
  GBM_HIP_TRY(hipMemcpyAsync(mu.data(), s->mu_d.p, nrhs * 8, hipMemcpyDeviceToHost, st));
  GBM_HIP_TRY(hipMemcpyAsync(msum.data(), s->msum.p, nrhs * 8, hipMemcpyDeviceToHost, st));
  GBM_HIP_TRY(hipStreamSynchronize(st));
  for (int64_t t = 0; t < nrhs; t++) {
    b_hat_out[t * (p + 1)] = mu[t] - msum[t];
    if (mu_out) mu_out[t] = mu[t];
  }
  if (q_out) *q_out = s->q;
  return GBM_OK;
}

extern "C" int gbm_session_predict(gbm_session* s, const int64_t* idx, int64_t n_val, const double* b_hat, int64_t ldb,
                                   int64_t nrhs, double* out, int64_t ldo) {
  RoctxRange r_("gbm_session_predict");
  if (!s) return fail(GBM_E_ARG, "gbm_session_predict: session is NULL");
  if (!b_hat || ldb < s->p + 1 || nrhs < 1 || !out || ldo < n_val)
    return fail(GBM_E_ARG, "gbm_session_predict: bad arguments");
  std::lock_guard<std::mutex> lock(s->mu);
  GBM_HIP_TRY(hipSetDevice(s->dev));
  GBM_TRY(check_idx(s, idx, n_val, "gbm_session_predict"));
  hipStream_t st = s->stream.s;
  const int64_t p = s->p, n = s->n, npad = s->npad;
  const int64_t nchunks = predict_chunks(n, p);
  GBM_TRY(dalloc(s->bvec, s->dev, nrhs * (p + 1) * 8));
  GBM_TRY(dalloc(s->part, s->dev, nchunks * nrhs * npad * 8));
  GBM_TRY(dalloc(s->pout, s->dev, nrhs * npad * 8));
  GBM_HIP_TRY(hipMemcpy2DAsync(s->bvec.p, (p + 1) * 8, b_hat, ldb * 8, (p + 1) * 8, nrhs, hipMemcpyHostToDevice, st));
  GBM_TRY(launch_predict((const double*)s->Xt.p, npad, p, n, (const double*)s->bvec.p, p + 1, nrhs,
                         (double*)s->part.p, nchunks, (double*)s->pout.p, npad, st));
  std::vector<double> all(nrhs * npad);
  GBM_HIP_TRY(hipMemcpyAsync(all.data(), s->pout.p, nrhs * npad * 8, hipMemcpyDeviceToHost, st));
  GBM_HIP_TRY(hipStreamSynchronize(st));
  for (int64_t t = 0; t < nrhs; t++)
    for (int64_t i = 0; i < n_val; i++) out[t * ldo + i] = all[t * npad + idx[i]];
  return GBM_OK;
}

extern "C" int gbm_session_reml_objective(gbm_session* s, const int64_t* idx, int64_t n_train, const double* y,
                                          const double* sigma2_e, const double* sigma2_u, int64_t m, double* out) {
  if (!s) return fail(GBM_E_ARG, "gbm_session_reml_objective: session is NULL");
  if (!y || !sigma2_e || !sigma2_u || m < 1 || !out) return fail(GBM_E_ARG, "gbm_session_reml_objective: bad arguments");
  std::lock_guard<std::mutex> lock(s->mu);
  GBM_HIP_TRY(hipSetDevice(s->dev));
  GBM_TRY(check_y(y, n_train, n_train, 1));
  GBM_TRY(ensure_training(s, idx, n_train));
  GBM_TRY(ensure_rhs(s, 1));
  GBM_TRY(upload_y(s, y, n_train, 1));
  for (int64_t k = 0; k < m; k++) {
    if (!(sigma2_e[k] > 0.0) || !(sigma2_u[k] > 0.0))
      return fail(GBM_E_ARG, "gbm_session_reml_objective: variance components must be > 0");
    GBM_TRY(solve_cached(s, 1, sigma2_e[k] / sigma2_u[k], 1.0 / (double)s->q));
    double t[4];
    GBM_TRY(gbm_dev_gblup_terms((const double*)s->Gw.p, s->gdimT, s->nT, 1, s->wss.p, (double*)s->terms.p,
                                s->stream.s));
    GBM_HIP_TRY(hipMemcpyAsync(t, s->terms.p, 4 * 8, hipMemcpyDeviceToHost, s->stream.s));
    GBM_HIP_TRY(hipStreamSynchronize(s->stream.s));
    const double Q = t[3] - t[2] * t[2] / t[1];
    out[k] = reml_objective(n_train, t[0], t[1], Q, sigma2_u[k]);
  }
  return GBM_OK;
}

extern "C" int gbm_session_reml(gbm_session* s, const int64_t* idx, int64_t n_train, const double* y,
                                double* lambda_out, double* sigma2_e_out, double* sigma2_u_out, double* objective_out) {
  RoctxRange r_("gbm_session_reml");
  if (!s) return fail(GBM_E_ARG, "gbm_session_reml: session is NULL");
  if (!y) return fail(GBM_E_ARG, "gbm_session_reml: y is NULL");
  std::lock_guard<std::mutex> lock(s->mu);
  GBM_HIP_TRY(hipSetDevice(s->dev));
  GBM_TRY(check_y(y, n_train, n_train, 1));
  if (n_train < 3) return fail(GBM_E_DATA, "REML needs at least 3 entries");
  GBM_TRY(ensure_training(s, idx, n_train));
  GBM_TRY(ensure_rhs(s, 1));
  const std::vector<double> ys = standardise_y(y, n_train);
  GBM_TRY(upload_y(s, ys.data(), n_train, 1));
  RemlResult res;
  GBM_TRY(reml_search([&](double lambda, RemlEval& e) { return reml_eval(s, lambda, e); }, res));
  if (lambda_out) *lambda_out = res.lambda;
  if (sigma2_e_out) *sigma2_e_out = res.s2e;
  if (sigma2_u_out) *sigma2_u_out = res.s2u;
  if (objective_out) *objective_out = res.objective;
  return GBM_OK;
}

extern "C" int gbm_session_stats(gbm_session* s, int64_t* grm_builds, int64_t* grm_hits) {
  if (!s) return fail(GBM_E_ARG, "gbm_session_stats: session is NULL");
  std::lock_guard<std::mutex> lock(s->mu);
  if (grm_builds) *grm_builds = s->builds;
  if (grm_hits) *grm_hits = s->hits;
  return GBM_OK;
}

// ---- ridge path (glmnet alpha = 0, standardize = false; reference ridge, src/linear.jl:193-203) --
// glmnet minimises (1/2n)‖y − a0 − Xb‖² + (λ/2)‖b‖² on y scaled by its population sd σ_y, with the
// user λ divided by the same σ_y (elnet: vlam = ulam/ys). On the original scale that is
// (X_cᵀX_c + (nλ/σ_y)I) b = X_cᵀ(y − ȳ): the GBLUP system on the unscaled centred-X kernel
// K = X_cX_cᵀ with λ' = nλ/σ_y, whose GLS intercept is ȳ (K1 = 0) and whose marker effects are
// b = X_cᵀa. σ_y is taken over the training rows of each call (each CV fold has its own).

extern "C" int gbm_session_ridge_lambda_max(gbm_session* s, const int64_t* idx, int64_t n_train, const double* y,
                                            double* lambda_max) {
  if (!s || !y || !lambda_max) return fail(GBM_E_ARG, "gbm_session_ridge_lambda_max: bad arguments");
  std::lock_guard<std::mutex> lock(s->mu);
  GBM_HIP_TRY(hipSetDevice(s->dev));
  GBM_TRY(check_y(y, n_train, n_train, 1));
  GBM_TRY(ensure_training(s, idx, n_train, 1));
  GBM_TRY(ensure_rhs(s, 1));
  // glmnet's first λ for alpha < 1e-3: max_j |x_cjᵀ(y − ȳ)|/n / 1e-3
  double m = 0.0;
  for (int64_t i = 0; i < n_train; i++) m += y[i];
  m /= (double)n_train;
  std::vector<double> r(s->npadT, 0.0);
  for (int64_t i = 0; i < n_train; i++) r[i] = y[i] - m;
  hipStream_t st = s->stream.s;
  GBM_HIP_TRY(hipMemcpyAsync(s->A.p, r.data(), s->npadT * 8, hipMemcpyHostToDevice, st));
  GBM_TRY(gbm_dev_marker_effects((const double*)s->Z.p, s->npadT, s->p, s->nT, (const double*)s->A.p, s->npadT, 1,
                                 1.0, nullptr, (const double*)s->mean.p, (const double*)s->sd.p,
                                 (const int32_t*)s->keep.p, (double*)s->B.p, s->p, (double*)s->msum.p, st));
  std::vector<double> g(s->p);
  GBM_HIP_TRY(hipMemcpyAsync(g.data(), s->B.p, s->p * 8, hipMemcpyDeviceToHost, st));
  GBM_HIP_TRY(hipStreamSynchronize(st));
  double gmax = 0.0;
  for (double v : g) gmax = std::max(gmax, std::fabs(v));
  *lambda_max = gmax / (double)n_train / 1e-3;
  return GBM_OK;
}

extern "C" int gbm_session_ridge_path(gbm_session* s, const int64_t* idx, int64_t n_train, const double* y,
                                      const double* lambdas, int64_t nl, double* b_path_out, const int64_t* idx_eval,
                                      int64_t n_eval, double* pred_out) {
  RoctxRange r_("gbm_session_ridge_path");
  if (!s || !y || !lambdas || nl < 1 || !b_path_out || (n_eval > 0 && (!idx_eval || !pred_out)))
    return fail(GBM_E_ARG, "gbm_session_ridge_path: bad arguments");
  for (int64_t k = 0; k < nl; k++)
    if (!(lambdas[k] > 0.0) || !std::isfinite(lambdas[k]))
      return fail(GBM_E_ARG, "gbm_session_ridge_path: lambdas must be finite and > 0");
  std::lock_guard<std::mutex> lock(s->mu);
  GBM_HIP_TRY(hipSetDevice(s->dev));
  GBM_TRY(check_y(y, n_train, n_train, 1));
  if (n_eval > 0) GBM_TRY(check_idx(s, idx_eval, n_eval, "gbm_session_ridge_path (eval)"));
  GBM_TRY(ensure_training(s, idx, n_train, 1));
  GBM_TRY(ensure_rhs(s, 1));
  GBM_TRY(upload_y(s, y, n_train, 1));
  double ym = 0.0, yss = 0.0;
  for (int64_t i = 0; i < n_train; i++) ym += y[i];
  ym /= (double)n_train;
  for (int64_t i = 0; i < n_train; i++) yss += (y[i] - ym) * (y[i] - ym);
  const double ys = std::sqrt(yss / (double)n_train);
  if (!(ys > 0.0)) return fail(GBM_E_ARG, "gbm_session_ridge_path: y has zero variance");
  hipStream_t st = s->stream.s;
  const int64_t p = s->p, n = s->n, npad = s->npad;
  const int64_t nchunks = predict_chunks(n, p);
  if (n_eval > 0) {
    GBM_TRY(dalloc(s->bvec, s->dev, (p + 1) * 8));
    GBM_TRY(dalloc(s->part, s->dev, nchunks * npad * 8));
    GBM_TRY(dalloc(s->pout, s->dev, npad * 8));
  }
  std::vector<double> all(n_eval > 0 ? npad : 0);
  for (int64_t k = 0; k < nl; k++) {
    GBM_TRY(solve_cached(s, 1, (double)n_train * lambdas[k] / ys, 1.0));
    GBM_TRY(gbm_dev_marker_effects((const double*)s->Z.p, s->npadT, p, s->nT, (const double*)s->A.p, s->npadT, 1,
                                   1.0, nullptr, (const double*)s->mean.p, (const double*)s->sd.p,
                                   (const int32_t*)s->keep.p, (double*)s->B.p, p, (double*)s->msum.p, st));
    double mu = 0.0, msum = 0.0;
    double* bk = b_path_out + k * (p + 1);
    GBM_HIP_TRY(hipMemcpyAsync(bk + 1, s->B.p, p * 8, hipMemcpyDeviceToHost, st));
    GBM_HIP_TRY(hipMemcpyAsync(&mu, s->mu_d.p, 8, hipMemcpyDeviceToHost, st));
    GBM_HIP_TRY(hipMemcpyAsync(&msum, s->msum.p, 8, hipMemcpyDeviceToHost, st));
    GBM_HIP_TRY(hipStreamSynchronize(st));
    bk[0] = mu - msum;
    if (n_eval > 0) {
      GBM_HIP_TRY(hipMemcpyAsync(s->bvec.p, bk, 8, hipMemcpyHostToDevice, st));
      GBM_HIP_TRY(hipMemcpyAsync((double*)s->bvec.p + 1, s->B.p, p * 8, hipMemcpyDeviceToDevice, st));
      GBM_TRY(launch_predict((const double*)s->Xt.p, npad, p, n, (const double*)s->bvec.p, p + 1, 1,
                             (double*)s->part.p, nchunks, (double*)s->pout.p, npad, st));
      GBM_HIP_TRY(hipMemcpyAsync(all.data(), s->pout.p, npad * 8, hipMemcpyDeviceToHost, st));
      GBM_HIP_TRY(hipStreamSynchronize(st));
      for (int64_t i = 0; i < n_eval; i++) pred_out[k * n_eval + i] = all[idx_eval[i]];
    }
  }
  return GBM_OK;
}
