// Bayesian ridge regression (BGLR model "BRR") by Gibbs sampling — SURVEY.md §8f row 3 (config
// C4); replaces the Rscript/BGLR round trip of reference src/bayes.jl:28-105,158-224.
//
// The chain is BGLR's single-site sampler (intercept, then every marker j in order with the
// residual update e += (b_old − b_new) x_j, then σ²_b and σ²_e from scaled-inverse-χ² draws;
// BGLR defaults df0 = 5, R2 = 0.5; running posterior means every `thin` iterations after
// burn-in). MI355X mapping: markers go in blocks of 64. For a block, x_jᵀe of all 64 markers
// is computed at once (one workgroup per marker), then the 64 sequential single-site steps run
// inside one wave from the block's 64x64 Gram matrix W = X_BᵀX_B (precomputed once):
// d_k = x_kᵀe is kept current by d_k += δ_j W[j][k] — exactly the residual update restricted to
// the block — and finally e += X_B δ over all individuals. Every workgroup of that last kernel
// replays the 64 steps redundantly from identical inputs (deterministic), so the block costs two
// launches and no device-wide synchronisation; one Gibbs iteration is captured as a hipGraph and
// replayed.
//
// Random numbers: a counter-based hash of (seed, stream, counter) (no sampler state), Box-Muller
// normals and Marsaglia-Tsang gammas, restated bit-for-bit in oracle/oracle.py (brr_*), so the
// device chain and the oracle's un-blocked BGLR loop follow the same sample path.
#include <cmath>
#include <vector>

#include "gbm_internal.h"
#include "host_util.h"

namespace gbm {
namespace {

constexpr int BB = 64;  // markers per block (one wave)

__device__ __forceinline__ uint64_t bmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double brr_u01(uint64_t seed, uint64_t a, uint64_t b) {
  const uint64_t h = bmix64(bmix64(seed ^ (a * 0xD1B54A32D192ED03ull)) ^ (b * 0x8CB92BA72F3D8DD7ull));
  return ((double)(h >> 11) + 0.5) * 0x1.0p-53;
}
__device__ __forceinline__ double brr_normal(uint64_t seed, uint64_t a, uint64_t b) {
  const double u1 = brr_u01(seed, a, 2 * b), u2 = brr_u01(seed, a, 2 * b + 1);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}
// χ²(df) = 2 Gamma(df/2) by Marsaglia-Tsang (df/2 >= 1); attempt t uses normal (a, 2t) and
// uniform (a, 4t + 2)
__device__ double brr_chisq(uint64_t seed, uint64_t a, double df) {
  const double d = 0.5 * df - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  for (uint64_t t = 0; t < 1000; t++) {
    const double x = brr_normal(seed, a, 2 * t);
    double v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = brr_u01(seed, a, 4 * t + 2);
    if (log(u) < 0.5 * x * x + d - d * v + d * log(v)) return 2.0 * d * v;
  }
  return df;  // unreachable in practice (acceptance ≈ 0.98 per attempt)
}

struct BrrState {
  double mu, varE, varB, S0e, S0b, df0e, df0b;
  double mubar, varEbar, varBbar;
  int64_t it, burnin, thin, nsum;
  uint64_t seed;
};

__device__ __forceinline__ bool brr_accumulate(const BrrState* st) {
  const int64_t i = st->it + 1;  // BGLR's 1-based iteration
  return (i % st->thin == 0) && (i > st->burnin);
}

template <int BS>
__device__ __forceinline__ double brr_block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < BS / 64; k++) s += red[k];
  return s;
}

// column means and Σx² of every marker (one workgroup per marker row of Xt)
__global__ void __launch_bounds__(256) brr_colstats_kernel(const double* __restrict__ Xt, int64_t ldx, int64_t p,
                                                           int64_t n, double* __restrict__ colmean,
                                                           double* __restrict__ x2) {
  __shared__ double red[4];
  for (int64_t j = blockIdx.x; j < p; j += gridDim.x) {
    const double* row = Xt + j * ldx;
    double s = 0.0, ss = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
      const double v = row[i];
      s += v;
      ss += v * v;
    }
    s = brr_block_sum<256>(s, red);
    ss = brr_block_sum<256>(ss, red);
    if (threadIdx.x == 0) {
      colmean[j] = s / (double)n;
      x2[j] = ss;
    }
  }
}

// W[blk] = X_BᵀX_B (64x64, row-major; rows/cols past p are zero), individuals in chunks of 64
// staged through LDS. One-time setup.
__global__ void __launch_bounds__(256) brr_gram_kernel(const double* __restrict__ Xt, int64_t ldx, int64_t p,
                                                       int64_t n, double* __restrict__ W) {
  __shared__ double T[BB][BB + 1];
  const int64_t j0 = (int64_t)blockIdx.x * BB;
  const int tid = threadIdx.x, a = tid >> 2, b0 = (tid & 3) * 16;
  double acc[16];
#pragma unroll
  for (int u = 0; u < 16; u++) acc[u] = 0.0;
  for (int64_t k0 = 0; k0 < n; k0 += BB) {
    for (int e = tid; e < BB * BB; e += 256) {
      const int r = e / BB, c = e % BB;
      T[r][c] = (j0 + r < p && k0 + c < n) ? Xt[(j0 + r) * ldx + k0 + c] : 0.0;
    }
    __syncthreads();
    for (int k = 0; k < BB; k++) {
      const double xa = T[a][k];
#pragma unroll
      for (int u = 0; u < 16; u++) acc[u] += xa * T[b0 + u][k];
    }
    __syncthreads();
  }
  double* out = W + (int64_t)blockIdx.x * BB * BB + a * BB + b0;
#pragma unroll
  for (int u = 0; u < 16; u++) out[u] = acc[u];
}

// intercept: BGLR adds μ back, samples μ ~ N(Σe/n, σ²_e/n), subtracts it again (one workgroup)
__global__ void __launch_bounds__(1024) brr_mu_kernel(double* __restrict__ e, int64_t n, BrrState* __restrict__ st) {
  __shared__ double red[16];
  const double mu_old = st->mu;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) s += e[i] + mu_old;
  s = brr_block_sum<1024>(s, red);
  const double varE = st->varE;
  const double mu = s / (double)n + sqrt(varE / (double)n) * brr_normal(st->seed, 4 * (uint64_t)st->it, 0xFFFFFFFFull);
  for (int64_t i = threadIdx.x; i < n; i += 1024) e[i] = (e[i] + mu_old) - mu;
  __syncthreads();
  if (threadIdx.x == 0) st->mu = mu;
}

// r[k] = x_{j0+k}ᵀ e (one workgroup per marker of the block)
__global__ void __launch_bounds__(256) brr_dots_kernel(const double* __restrict__ Xt, int64_t ldx, int64_t n,
                                                       const double* __restrict__ e, int64_t j0,
                                                       double* __restrict__ r) {
  __shared__ double red[4];
  const double* row = Xt + (j0 + blockIdx.x) * ldx;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += row[i] * e[i];
  s = brr_block_sum<256>(s, red);
  if (threadIdx.x == 0) r[blockIdx.x] = s;
}

// The block's 64 single-site steps (wave 0 of every workgroup, from identical inputs), then
// e += X_B δ for this workgroup's 256 individuals; workgroup 0 stores b and the running mean.
__global__ void __launch_bounds__(256) brr_block_kernel(const double* __restrict__ Xt, int64_t ldx, int64_t n,
                                                        const double* __restrict__ W, int64_t j0, int nb,
                                                        const double* __restrict__ r, double* __restrict__ b,
                                                        double* __restrict__ bbar, const double* __restrict__ x2,
                                                        double* __restrict__ e, const BrrState* __restrict__ st) {
  __shared__ double Ws[BB][BB + 1];
  __shared__ double delta[BB];
  const int tid = threadIdx.x, lane = tid & 63;
  const double* Wb = W + (j0 / BB) * BB * BB;
  for (int q = tid; q < BB * BB; q += 256) Ws[q / BB][q % BB] = Wb[q];
  __syncthreads();
  if (tid < 64) {
    const double varE = st->varE, varB = st->varB;
    const bool on = lane < nb;
    const int64_t j = j0 + lane;
    const double xx = on ? x2[j] : 0.0;
    const double bo = on ? b[j] : 0.0;
    // c = x2/σ²_e + 1/σ²_b; b_new = (d + x2 b)/σ²_e / c + sqrt(1/c) ξ = d α + β
    const double cinv = 1.0 / (xx / varE + 1.0 / varB);
    const double alpha = cinv / varE;
    const double xi = on ? brr_normal(st->seed, 4 * (uint64_t)st->it, (uint64_t)j) : 0.0;
    const double beta = xx * bo * alpha + sqrt(cinv) * xi;
    double d = on ? r[lane] : 0.0;
    double bn = bo;
    for (int s = 0; s < nb; s++) {
      double dl = 0.0;
      if (lane == s) {
        bn = fma(d, alpha, beta);
        dl = bo - bn;
      }
      // broadcast δ_s (v_readlane of both halves)
      union {
        double f;
        int w[2];
      } u;
      u.f = dl;
      u.w[0] = __builtin_amdgcn_readlane(u.w[0], s);
      u.w[1] = __builtin_amdgcn_readlane(u.w[1], s);
      d = fma(u.f, Ws[s][lane], d);
      if (lane == 0) delta[s] = u.f;
    }
    if (blockIdx.x == 0 && on) {
      b[j] = bn;
      if (brr_accumulate(st)) {
        const double k = (double)(st->nsum + 1);
        bbar[j] = bbar[j] * ((k - 1.0) / k) + bn / k;
      }
    }
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + tid;
  if (i < n) {
    double acc = 0.0;
    for (int s = 0; s < nb; s++) acc = fma(delta[s], Xt[(j0 + s) * ldx + i], acc);
    e[i] += acc;
  }
}

// σ²_b, σ²_e draws, running means of μ and the variances, next iteration (one workgroup)
__global__ void __launch_bounds__(1024) brr_var_kernel(const double* __restrict__ b, int64_t p,
                                                       const double* __restrict__ e, int64_t n,
                                                       BrrState* __restrict__ st) {
  __shared__ double red[16];
  double sb = 0.0, se = 0.0;
  for (int64_t j = threadIdx.x; j < p; j += 1024) sb += b[j] * b[j];
  for (int64_t i = threadIdx.x; i < n; i += 1024) se += e[i] * e[i];
  sb = brr_block_sum<1024>(sb, red);
  se = brr_block_sum<1024>(se, red);
  if (threadIdx.x == 0) {
    const uint64_t a = 4 * (uint64_t)st->it;
    st->varB = (sb + st->S0b) / brr_chisq(st->seed, a + 1, st->df0b + (double)p);
    st->varE = (se + st->S0e) / brr_chisq(st->seed, a + 2, st->df0e + (double)n);
    if (brr_accumulate(st)) {
      const double k = (double)(st->nsum + 1);
      st->mubar = st->mubar * ((k - 1.0) / k) + st->mu / k;
      st->varEbar = st->varEbar * ((k - 1.0) / k) + st->varE / k;
      st->varBbar = st->varBbar * ((k - 1.0) / k) + st->varB / k;
      st->nsum += 1;
    }
    st->it += 1;
  }
}

}  // namespace
}  // namespace gbm

using namespace gbm;

extern "C" int gbm_brr_fit(const double* X, int64_t n, int64_t p, int64_t ldx, const double* y, int64_t n_iter,
                           int64_t n_burnin, int64_t thin, double r2, double df0, uint64_t seed, int device,
                           double* b_hat_out, double* y_pred_out, double* var_out) {
  if (!X || !y || !b_hat_out || n < 3 || p < 1 || ldx < n || n_iter < 1 || n_burnin < 0 || thin < 1 ||
      !(r2 > 0.0 && r2 < 1.0) || !(df0 > 0.0))
    return fail(GBM_E_ARG, "gbm_brr_fit: bad arguments (n >= 3, p >= 1, ldx >= n, n_iter >= 1, n_burnin >= 0, "
                           "thin >= 1, 0 < r2 < 1, df0 > 0)");
  if (n_iter <= n_burnin || (n_iter / thin) <= (n_burnin / thin))
    return fail(GBM_E_ARG, "gbm_brr_fit: no post-burn-in sample (need a multiple of thin in (n_burnin, n_iter])");
  GBM_TRY(check_y(y, n, n, 1));
  std::vector<int> devs;
  GBM_TRY(check_devices(&device, 1, devs));
  const int dev = devs[0];
  GBM_HIP_TRY(hipSetDevice(dev));
  Stream stw;
  stw.dev = dev;
  GBM_HIP_TRY(hipStreamCreateWithFlags(&stw.s, hipStreamNonBlocking));
  hipStream_t s = stw.s;
  const int64_t npad = npad_of(n), nblk = (p + BB - 1) / BB;
  DevMem Xt, colmean, x2, W, e, b, bbar, r, stm, pb, part, pout;
  GBM_TRY(dalloc(Xt, dev, p * npad * 8));
  GBM_TRY(dalloc(colmean, dev, p * 8));
  GBM_TRY(dalloc(x2, dev, p * 8));
  GBM_TRY(dalloc(W, dev, nblk * BB * BB * 8));
  GBM_TRY(dalloc(e, dev, npad * 8));
  GBM_TRY(dalloc(b, dev, p * 8));
  GBM_TRY(dalloc(bbar, dev, p * 8));
  GBM_TRY(dalloc(r, dev, BB * 8));
  GBM_TRY(dalloc(stm, dev, sizeof(BrrState)));
  GBM_HIP_TRY(hipMemsetAsync(Xt.p, 0, (size_t)(p * npad * 8), s));
  GBM_HIP_TRY(hipMemcpy2DAsync(Xt.p, npad * 8, X, ldx * 8, n * 8, p, hipMemcpyHostToDevice, s));
  brr_colstats_kernel<<<(unsigned)std::min<int64_t>(p, 4096), 256, 0, s>>>((const double*)Xt.p, npad, p, n,
                                                                           (double*)colmean.p, (double*)x2.p);
  GBM_LAUNCH_CHECK();
  brr_gram_kernel<<<(unsigned)nblk, 256, 0, s>>>((const double*)Xt.p, npad, p, n, (double*)W.p);
  GBM_LAUNCH_CHECK();
  std::vector<double> cm(p), xx(p);
  GBM_HIP_TRY(hipMemcpyAsync(cm.data(), colmean.p, p * 8, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipMemcpyAsync(xx.data(), x2.p, p * 8, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  // BGLR defaults (setLT.BRR and the residual prior): var(y) with ddof 1
  double ym = 0.0;
  for (int64_t i = 0; i < n; i++) ym += y[i];
  ym /= (double)n;
  double vy = 0.0;
  for (int64_t i = 0; i < n; i++) vy += (y[i] - ym) * (y[i] - ym);
  vy /= (double)(n - 1);
  double msx = 0.0, smsq = 0.0;
  for (int64_t j = 0; j < p; j++) {
    msx += xx[j];
    smsq += cm[j] * cm[j];
  }
  msx = msx / (double)n - smsq;
  if (!(msx > 0.0)) return fail(GBM_E_DATA, "gbm_brr_fit: the markers have no variance");
  BrrState st0{};
  st0.mu = ym;
  st0.S0e = vy * (1.0 - r2) * (df0 + 2.0);
  st0.S0b = vy * r2 / msx * (df0 + 2.0);
  st0.df0e = df0;
  st0.df0b = df0;
  st0.varE = st0.S0e / (df0 + 2.0);
  st0.varB = st0.S0b / (df0 + 2.0);
  st0.burnin = n_burnin;
  st0.thin = thin;
  st0.seed = seed;
  std::vector<double> e0(npad, 0.0);
  for (int64_t i = 0; i < n; i++) e0[i] = y[i] - ym;
  GBM_HIP_TRY(hipMemcpyAsync(e.p, e0.data(), npad * 8, hipMemcpyHostToDevice, s));
  GBM_HIP_TRY(hipMemsetAsync(b.p, 0, p * 8, s));
  GBM_HIP_TRY(hipMemsetAsync(bbar.p, 0, p * 8, s));
  GBM_HIP_TRY(hipMemcpyAsync(stm.p, &st0, sizeof(BrrState), hipMemcpyHostToDevice, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  // one Gibbs iteration, captured once and replayed
  auto* stp = (BrrState*)stm.p;
  const unsigned eblocks = (unsigned)((n + 255) / 256);
  auto enqueue_iteration = [&]() -> int {
    brr_mu_kernel<<<1, 1024, 0, s>>>((double*)e.p, n, stp);
    for (int64_t k = 0; k < nblk; k++) {
      const int64_t j0 = k * BB;
      const int nb = (int)std::min<int64_t>(BB, p - j0);
      brr_dots_kernel<<<(unsigned)nb, 256, 0, s>>>((const double*)Xt.p, npad, n, (const double*)e.p, j0,
                                                   (double*)r.p);
      brr_block_kernel<<<eblocks, 256, 0, s>>>((const double*)Xt.p, npad, n, (const double*)W.p, j0, nb,
                                               (const double*)r.p, (double*)b.p, (double*)bbar.p,
                                               (const double*)x2.p, (double*)e.p, stp);
    }
    brr_var_kernel<<<1, 1024, 0, s>>>((const double*)b.p, p, (const double*)e.p, n, stp);
    return hipGetLastError() == hipSuccess ? GBM_OK : fail(GBM_E_HIP, "gbm_brr_fit: launch failed");
  };
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  int rc = GBM_OK;
  if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess) {
    rc = enqueue_iteration();
    if (hipStreamEndCapture(s, &graph) != hipSuccess || rc != GBM_OK ||
        hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess) {
      (void)hipGetLastError();
      exec = nullptr;
      rc = GBM_OK;  // fall back to direct launches (same kernels, same order)
    }
  }
  for (int64_t it = 0; it < n_iter && rc == GBM_OK; it++) {
    if (exec) {
      if (hipGraphLaunch(exec, s) != hipSuccess) rc = fail(GBM_E_HIP, "gbm_brr_fit: graph launch failed");
    } else {
      rc = enqueue_iteration();
    }
  }
  if (exec) (void)hipGraphExecDestroy(exec);
  if (graph) (void)hipGraphDestroy(graph);
  if (rc != GBM_OK) return rc;
  BrrState fin{};
  GBM_HIP_TRY(hipMemcpyAsync(&fin, stm.p, sizeof(BrrState), hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipMemcpyAsync(b_hat_out + 1, bbar.p, p * 8, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  b_hat_out[0] = fin.mubar;
  if (var_out) {
    var_out[0] = fin.varEbar;
    var_out[1] = fin.varBbar;
  }
  if (y_pred_out) {
    const int64_t nchunks = predict_chunks(n, p);
    GBM_TRY(dalloc(pb, dev, (p + 1) * 8));
    GBM_TRY(dalloc(part, dev, nchunks * npad * 8));
    GBM_TRY(dalloc(pout, dev, npad * 8));
    GBM_HIP_TRY(hipMemcpyAsync(pb.p, b_hat_out, (p + 1) * 8, hipMemcpyHostToDevice, s));
    GBM_TRY(launch_predict((const double*)Xt.p, npad, p, n, (const double*)pb.p, p + 1, 1, (double*)part.p, nchunks,
                           (double*)pout.p, npad, s));
    GBM_HIP_TRY(hipMemcpyAsync(y_pred_out, pout.p, n * 8, hipMemcpyDeviceToHost, s));
    GBM_HIP_TRY(hipStreamSynchronize(s));
  }
  return GBM_OK;
}
