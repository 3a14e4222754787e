// Host entry points of libgbm.so (include/gbm.h): argument checks, device buffers, H2D/D2H,
// SNP-column sharding over devices and the RCCL all-reduce of partial GRMs.
// Every call owns its streams and buffers (re-entrant, as cvmultithread! requires —
// reference src/cross_validation.jl:159).
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "gbm_internal.h"
#include "host_util.h"

namespace gbm {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

namespace {

// One SNP-column shard resident on one device.
struct Shard {
  int dev = 0;
  Stream stream;
  int64_t j0 = 0, p = 0;
  DevMem Xt, D8, mean, sd, keep, q, G, wsg, Y, A, gebv, mu, info, wss, B, msum;
  int64_t q_host = 0;
};

enum class Source { F64, I8, SYNTH };

struct Problem {
  Source src;
  const double* X;
  const int8_t* D;
  int ploidy;
  int64_t n, p, ld;
  uint64_t seed = 0;  // Source::SYNTH: genotypes generated on each device
};

// Upload the shard's columns and standardise them; reads back the shard's kept count.
int prepare_shard(const Problem& pr, Shard& sh) {
  const int64_t n = pr.n, npad = npad_of(n), pl = sh.p;
  GBM_HIP_TRY(hipSetDevice(sh.dev));
  sh.stream.dev = sh.dev;
  GBM_HIP_TRY(hipStreamCreateWithFlags(&sh.stream.s, hipStreamNonBlocking));
  hipStream_t s = sh.stream.s;
  GBM_TRY(dalloc(sh.Xt, sh.dev, pl * npad * 8));
  GBM_TRY(dalloc(sh.mean, sh.dev, pl * 8));
  GBM_TRY(dalloc(sh.sd, sh.dev, pl * 8));
  GBM_TRY(dalloc(sh.keep, sh.dev, pl * 4));
  GBM_TRY(dalloc(sh.q, sh.dev, 8));
  if (pr.src == Source::F64) {
    GBM_HIP_TRY(hipMemcpy2DAsync(sh.Xt.p, npad * 8, pr.X + sh.j0 * pr.ld, pr.ld * 8, n * 8, pl, hipMemcpyHostToDevice, s));
  } else if (pr.src == Source::SYNTH) {
    GBM_TRY(gbm_dev_synth_genotypes((double*)sh.Xt.p, npad, pl, n, pr.seed, sh.j0, s));
  } else {
    GBM_TRY(dalloc(sh.D8, sh.dev, pl * n));
    GBM_HIP_TRY(hipMemcpy2DAsync(sh.D8.p, n, pr.D + sh.j0 * pr.ld, pr.ld, n, pl, hipMemcpyHostToDevice, s));
    GBM_TRY(gbm_dev_expand_dosage_i8((const int8_t*)sh.D8.p, n, n, pl, pr.ploidy, (double*)sh.Xt.p, npad, s));
  }
  GBM_HIP_TRY(hipMemsetAsync(sh.q.p, 0, 8, s));
  GBM_TRY(gbm_dev_standardize((const double*)sh.Xt.p, npad, pl, n, (double*)sh.Xt.p, npad, (double*)sh.mean.p,
                              (double*)sh.sd.p,
                              (int32_t*)sh.keep.p, (int64_t*)sh.q.p, s));
  GBM_HIP_TRY(hipMemcpyAsync(&sh.q_host, sh.q.p, 8, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  return GBM_OK;
}

int grm_shard(const Problem& pr, Shard& sh) {
  const int64_t n = pr.n, npad = npad_of(n), gdim = gdim_of(n);
  GBM_HIP_TRY(hipSetDevice(sh.dev));
  GBM_TRY(dalloc(sh.G, sh.dev, gdim * gdim * 8));
  const int64_t wsb = gbm_dev_grm_workspace(n, sh.p);
  GBM_TRY(dalloc(sh.wsg, sh.dev, wsb));
  return gbm_dev_grm((const double*)sh.Xt.p, npad, sh.p, n, (double*)sh.G.p, gdim, sh.wsg.p, wsb, sh.stream.s);
}

const char* nccl_msg(ncclResult_t r) { return ncclGetErrorString(r); }

// Sum the partial GRMs across devices: the upper 128-tiles packed contiguously (half the bytes
// of G's rows), all-reduced, unpacked.
int allreduce_grm(std::vector<std::unique_ptr<Shard>>& shards, int64_t n) {
  if (shards.size() < 2) return GBM_OK;
  const int64_t gdim = gdim_of(n), psz = gbm_dev_grm_packed_size(n);
  std::vector<int> devs;
  for (auto& sh : shards) devs.push_back(sh->dev);
  std::vector<std::unique_ptr<DevMem>> packed;
  for (auto& sh : shards) {
    packed.push_back(std::make_unique<DevMem>());
    GBM_HIP_TRY(hipSetDevice(sh->dev));
    GBM_TRY(dalloc(*packed.back(), sh->dev, psz * 8));
    GBM_TRY(gbm_dev_grm_pack((const double*)sh->G.p, gdim, n, (double*)packed.back()->p, sh->stream.s));
  }
  std::vector<ncclComm_t> comms(shards.size());
  ncclResult_t r = ncclCommInitAll(comms.data(), (int)devs.size(), devs.data());
  if (r != ncclSuccess) return fail(GBM_E_RCCL, std::string("ncclCommInitAll: ") + nccl_msg(r));
  int rc = GBM_OK;
  r = ncclGroupStart();
  for (size_t k = 0; k < shards.size() && r == ncclSuccess; k++)
    r = ncclAllReduce(packed[k]->p, packed[k]->p, (size_t)psz, ncclDouble, ncclSum, comms[k], shards[k]->stream.s);
  ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    rc = fail(GBM_E_RCCL, std::string("ncclAllReduce(partial GRM): ") + nccl_msg(r != ncclSuccess ? r : r2));
  for (size_t k = 0; k < shards.size() && rc == GBM_OK; k++) {
    (void)hipSetDevice(shards[k]->dev);
    rc = gbm_dev_grm_unpack((const double*)packed[k]->p, n, (double*)shards[k]->G.p, gdim, shards[k]->stream.s);
  }
  for (auto& sh : shards) {
    (void)hipSetDevice(sh->dev);
    if (hipStreamSynchronize(sh->stream.s) != hipSuccess && rc == GBM_OK) rc = fail(GBM_E_HIP, "stream sync after all-reduce");
  }
  for (auto c : comms) (void)ncclCommDestroy(c);
  return rc;
}

int run_fit(const Problem& pr, const double* Y, int64_t ldy, int64_t nrhs, double lambda, const int* devices, int ndev,
            double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out) {
  const int64_t n = pr.n, p = pr.p;
  if (n < 2) return fail(GBM_E_DATA, "there are less than 2 entries (reference src/prediction.jl:117-123)");
  if (p < 1 || pr.ld < n || !Y || ldy < n || nrhs < 1 || nrhs > 63 || !b_hat_out || !y_pred_out)
    return fail(GBM_E_ARG, "gbm_gblup_fit: bad arguments (need p >= 1, ldx >= n, ldy >= n, 1 <= nrhs <= 63, outputs)");
  if (!(lambda > 0.0) || !std::isfinite(lambda)) return fail(GBM_E_ARG, "gbm_gblup_fit: lambda must be finite and > 0");
  GBM_TRY(check_y(Y, n, ldy, nrhs));
  std::vector<int> devs;
  GBM_TRY(check_devices(devices, ndev, devs));
  const int64_t npad = npad_of(n), gdim = gdim_of(n);
  const int nd = (int)std::min<int64_t>((int64_t)devs.size(), p);
  const int64_t per = (p + nd - 1) / nd;
  std::vector<std::unique_ptr<Shard>> shards;
  for (int k = 0; k < nd; k++) {
    auto sh = std::make_unique<Shard>();
    sh->dev = devs[k];
    sh->j0 = k * per;
    sh->p = std::min(per, p - sh->j0);
    if (sh->p <= 0) break;
    shards.push_back(std::move(sh));
  }
  int64_t q = 0;
  for (auto& sh : shards) {
    GBM_TRY(prepare_shard(pr, *sh));
    q += sh->q_host;
  }
  if (q_out) *q_out = q;
  if (q == 0) return fail(GBM_E_DATA, "no polymorphic locus-allele (all standard deviations <= eps, src/gwas.jl:112-115)");
  for (auto& sh : shards) GBM_TRY(grm_shard(pr, *sh));
  GBM_TRY(allreduce_grm(shards, n));
  const double inv_q = 1.0 / (double)q;
  std::vector<double> msum_total(nrhs, 0.0), mu(nrhs, 0.0);
  // every shard solves the (identical) n x n system redundantly, all devices at once: a is then
  // local to each shard's marker back-solve with no broadcast
  std::vector<int32_t> infos(shards.size(), 0);
  for (size_t k = 0; k < shards.size(); k++) {
    Shard& sh = *shards[k];
    GBM_HIP_TRY(hipSetDevice(sh.dev));
    hipStream_t s = sh.stream.s;
    GBM_TRY(dalloc(sh.Y, sh.dev, nrhs * npad * 8));
    GBM_TRY(dalloc(sh.A, sh.dev, nrhs * npad * 8));
    GBM_TRY(dalloc(sh.gebv, sh.dev, nrhs * npad * 8));
    GBM_TRY(dalloc(sh.mu, sh.dev, nrhs * 8));
    GBM_TRY(dalloc(sh.info, sh.dev, 4));
    const int64_t wss = gbm_dev_solve_workspace(n, nrhs);
    GBM_TRY(dalloc(sh.wss, sh.dev, wss));
    GBM_TRY(dalloc(sh.B, sh.dev, nrhs * sh.p * 8));
    GBM_TRY(dalloc(sh.msum, sh.dev, nrhs * 8));
    GBM_HIP_TRY(hipMemcpy2DAsync(sh.Y.p, npad * 8, Y, ldy * 8, n * 8, nrhs, hipMemcpyHostToDevice, s));
    GBM_TRY(gbm_dev_gblup_solve((double*)sh.G.p, gdim, n, inv_q, nullptr, lambda, (const double*)sh.Y.p, npad, nrhs,
                                (double*)sh.A.p, (double*)sh.gebv.p, npad, (double*)sh.mu.p, (int32_t*)sh.info.p,
                                sh.wss.p, wss, s));
    GBM_HIP_TRY(hipMemcpyAsync(&infos[k], sh.info.p, 4, hipMemcpyDeviceToHost, s));
  }
  std::vector<std::vector<double>> msums(shards.size(), std::vector<double>(nrhs, 0.0));
  for (size_t k = 0; k < shards.size(); k++) {
    Shard& sh = *shards[k];
    GBM_HIP_TRY(hipSetDevice(sh.dev));
    hipStream_t s = sh.stream.s;
    GBM_HIP_TRY(hipStreamSynchronize(s));
    const int32_t info = infos[k];
    if (info < 0) return fail(GBM_E_HIP, "back substitution: block synchronisation timed out");
    if (info != 0)
      return fail(GBM_E_NOTPD, "G/q + lambda*I is not positive definite (pivot " + std::to_string(info) +
                                   "); check for non-finite genotypes");
    GBM_TRY(gbm_dev_marker_effects((const double*)sh.Xt.p, npad, sh.p, n, (const double*)sh.A.p, npad, nrhs, inv_q,
                                   nullptr, (const double*)sh.mean.p, (const double*)sh.sd.p, (const int32_t*)sh.keep.p,
                                   (double*)sh.B.p, sh.p, (double*)sh.msum.p, s));
    GBM_HIP_TRY(hipMemcpy2DAsync(b_hat_out + 1 + sh.j0, (p + 1) * 8, sh.B.p, sh.p * 8, sh.p * 8, nrhs,
                                 hipMemcpyDeviceToHost, s));
    GBM_HIP_TRY(hipMemcpyAsync(msums[k].data(), sh.msum.p, nrhs * 8, hipMemcpyDeviceToHost, s));
    if (k == 0) {
      GBM_HIP_TRY(hipMemcpy2DAsync(y_pred_out, n * 8, sh.gebv.p, npad * 8, n * 8, nrhs, hipMemcpyDeviceToHost, s));
      GBM_HIP_TRY(hipMemcpyAsync(mu.data(), sh.mu.p, nrhs * 8, hipMemcpyDeviceToHost, s));
    }
  }
  for (size_t k = 0; k < shards.size(); k++) {
    GBM_HIP_TRY(hipSetDevice(shards[k]->dev));
    GBM_HIP_TRY(hipStreamSynchronize(shards[k]->stream.s));
    for (int64_t t = 0; t < nrhs; t++) msum_total[t] += msums[k][t];  // shard order: deterministic
  }
  for (int64_t t = 0; t < nrhs; t++) {
    b_hat_out[t * (p + 1)] = mu[t] - msum_total[t];
    if (mu_out) mu_out[t] = mu[t];
  }
  return GBM_OK;
}

}  // namespace
}  // namespace gbm

using namespace gbm;

extern "C" int gbm_version(void) { return GBM_VERSION; }

extern "C" const char* gbm_last_error(void) { return g_last_error.c_str(); }

extern "C" int gbm_device_count(int* count) {
  if (!count) return fail(GBM_E_ARG, "gbm_device_count: NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *count = 0;
    return e == hipErrorNoDevice ? GBM_OK : fail(GBM_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = c;
  return GBM_OK;
}

extern "C" int gbm_gblup_fit(const double* X, int64_t n, int64_t p, int64_t ldx, const double* Y, int64_t ldy,
                             int64_t nrhs, double lambda, const int* devices, int ndev, double* b_hat_out,
                             double* y_pred_out, double* mu_out, int64_t* q_out) {
  if (!X) return fail(GBM_E_ARG, "gbm_gblup_fit: X is NULL");
  Problem pr{Source::F64, X, nullptr, 1, n, p, ldx};
  return run_fit(pr, Y, ldy, nrhs, lambda, devices, ndev, b_hat_out, y_pred_out, mu_out, q_out);
}

extern "C" int gbm_gblup_fit_synthetic(uint64_t seed, int64_t n, int64_t p, const double* Y, int64_t ldy, int64_t nrhs,
                                       double lambda, const int* devices, int ndev, double* b_hat_out,
                                       double* y_pred_out, double* mu_out, int64_t* q_out) {
  if (n < 1 || p < 1) return fail(GBM_E_ARG, "gbm_gblup_fit_synthetic: bad arguments (n, p >= 1)");
  Problem pr{Source::SYNTH, nullptr, nullptr, 1, n, p, n};
  pr.seed = seed;
  return run_fit(pr, Y, ldy, nrhs, lambda, devices, ndev, b_hat_out, y_pred_out, mu_out, q_out);
}

extern "C" int gbm_gblup_fit_dosage_i8(const int8_t* D, int64_t n, int64_t p, int64_t ldd, int ploidy, const double* Y,
                                       int64_t ldy, int64_t nrhs, double lambda, const int* devices, int ndev,
                                       double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out) {
  if (!D || ploidy < 1) return fail(GBM_E_ARG, "gbm_gblup_fit_dosage_i8: D is NULL or ploidy < 1");
  Problem pr{Source::I8, nullptr, D, ploidy, n, p, ldd};
  return run_fit(pr, Y, ldy, nrhs, lambda, devices, ndev, b_hat_out, y_pred_out, mu_out, q_out);
}

extern "C" int gbm_grm(const double* X, int64_t n, int64_t p, int64_t ldx, const int* devices, int ndev, double* G_out,
                       int64_t ldg, int64_t* q_out) {
  if (!X || !G_out || n < 1 || p < 1 || ldx < n || ldg < n) return fail(GBM_E_ARG, "gbm_grm: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(devices, ndev, devs));
  Problem pr{Source::F64, X, nullptr, 1, n, p, ldx};
  const int nd = (int)std::min<int64_t>((int64_t)devs.size(), p);
  const int64_t per = (p + nd - 1) / nd;
  std::vector<std::unique_ptr<Shard>> shards;
  for (int k = 0; k < nd; k++) {
    auto sh = std::make_unique<Shard>();
    sh->dev = devs[k];
    sh->j0 = k * per;
    sh->p = std::min(per, p - sh->j0);
    if (sh->p <= 0) break;
    shards.push_back(std::move(sh));
  }
  int64_t q = 0;
  for (auto& sh : shards) {
    GBM_TRY(prepare_shard(pr, *sh));
    q += sh->q_host;
  }
  if (q_out) *q_out = q;
  if (q == 0) return fail(GBM_E_DATA, "no polymorphic locus-allele");
  for (auto& sh : shards) GBM_TRY(grm_shard(pr, *sh));
  GBM_TRY(allreduce_grm(shards, n));
  Shard& sh = *shards[0];
  GBM_HIP_TRY(hipSetDevice(sh.dev));
  DevMem out;
  GBM_TRY(dalloc(out, sh.dev, n * n * 8));
  GBM_TRY(launch_grm_export((const double*)sh.G.p, gdim_of(n), n, 1.0 / (double)q, (double*)out.p, n, sh.stream.s));
  GBM_HIP_TRY(hipMemcpy2DAsync(G_out, ldg * 8, out.p, n * 8, n * 8, n, hipMemcpyDeviceToHost, sh.stream.s));
  GBM_HIP_TRY(hipStreamSynchronize(sh.stream.s));
  return GBM_OK;
}

extern "C" int gbm_colstats(const double* X, int64_t n, int64_t p, int64_t ldx, int device, double* mean_out,
                            double* sd_out, uint8_t* keep_out, int64_t* q_out) {
  if (!X || n < 1 || p < 1 || ldx < n) return fail(GBM_E_ARG, "gbm_colstats: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(&device, 1, devs));
  Problem pr{Source::F64, X, nullptr, 1, n, p, ldx};
  Shard sh;
  sh.dev = devs[0];
  sh.j0 = 0;
  sh.p = p;
  GBM_TRY(prepare_shard(pr, sh));
  if (q_out) *q_out = sh.q_host;
  hipStream_t s = sh.stream.s;
  if (mean_out) GBM_HIP_TRY(hipMemcpyAsync(mean_out, sh.mean.p, p * 8, hipMemcpyDeviceToHost, s));
  if (sd_out) GBM_HIP_TRY(hipMemcpyAsync(sd_out, sh.sd.p, p * 8, hipMemcpyDeviceToHost, s));
  std::vector<int32_t> k32;
  if (keep_out) {
    k32.resize(p);
    GBM_HIP_TRY(hipMemcpyAsync(k32.data(), sh.keep.p, p * 4, hipMemcpyDeviceToHost, s));
  }
  GBM_HIP_TRY(hipStreamSynchronize(s));
  if (keep_out)
    for (int64_t j = 0; j < p; j++) keep_out[j] = (uint8_t)(k32[j] != 0);
  return GBM_OK;
}

extern "C" int gbm_predict(const double* X, int64_t n, int64_t p, int64_t ldx, const double* b_hat, int64_t ldb,
                           int64_t nrhs, int device, double* out, int64_t ldo) {
  if (!X || !b_hat || !out || n < 1 || p < 1 || ldx < n || ldb < p + 1 || nrhs < 1 || ldo < n)
    return fail(GBM_E_ARG, "gbm_predict: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(&device, 1, devs));
  const int dev = devs[0];
  GBM_HIP_TRY(hipSetDevice(dev));
  Stream st;
  st.dev = dev;
  GBM_HIP_TRY(hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking));
  DevMem Xt, b, part, o;
  const int64_t nchunks = predict_chunks(n, p);
  GBM_TRY(dalloc(Xt, dev, p * n * 8));
  GBM_TRY(dalloc(b, dev, nrhs * (p + 1) * 8));
  GBM_TRY(dalloc(part, dev, nchunks * nrhs * n * 8));
  GBM_TRY(dalloc(o, dev, nrhs * n * 8));
  GBM_HIP_TRY(hipMemcpy2DAsync(Xt.p, n * 8, X, ldx * 8, n * 8, p, hipMemcpyHostToDevice, st.s));
  GBM_HIP_TRY(hipMemcpy2DAsync(b.p, (p + 1) * 8, b_hat, ldb * 8, (p + 1) * 8, nrhs, hipMemcpyHostToDevice, st.s));
  GBM_TRY(launch_predict((const double*)Xt.p, n, p, n, (const double*)b.p, p + 1, nrhs, (double*)part.p, nchunks,
                         (double*)o.p, n, st.s));
  GBM_HIP_TRY(hipMemcpy2DAsync(out, ldo * 8, o.p, n * 8, n * 8, nrhs, hipMemcpyDeviceToHost, st.s));
  GBM_HIP_TRY(hipStreamSynchronize(st.s));
  return GBM_OK;
}
