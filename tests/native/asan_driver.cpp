// Host-side driver for the AddressSanitizer / UndefinedBehaviorSanitizer build of libgbm's host
// shim (capi.cpp, session.cpp and the .hip files' launchers): it calls every C-ABI entry point a
// binding uses, with bad arguments and (on a machine without a GPU) on the no-device paths, from
// one thread and from eight at once (the reference's cvmultithread! calls the model function from
// Threads.@threads), and checks return codes and the thread-local error strings. Memory errors
// and undefined behaviour abort the run (ASan/UBSan, halt_on_error). Test infrastructure only.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gbm.h"

#include "../../genomicbreedingmodels.jl_amd/csrc/gbm_internal.h"  // internal host helpers (csrc/hostpack.cpp)

static int failures = 0;
#define CHECK(cond)                                                     \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      failures++;                                                       \
    }                                                                   \
  } while (0)

static void entry_points(int seed) {
  const int64_t n = 40 + seed, p = 70;
  std::vector<double> X(n * p), Y(n), b(p + 1), yp(n), mu(1);
  for (int64_t e = 0; e < n * p; e++) X[e] = (double)((e * 2654435761u + seed) % 3) * 0.5;
  for (int64_t i = 0; i < n; i++) Y[i] = std::sin((double)(i + seed));
  int64_t q = -1;
  // NULL / shape errors: GBM_E_ARG with a message
  CHECK(gbm_gblup_fit(nullptr, n, p, n, Y.data(), n, 1, 1.0, nullptr, 0, b.data(), yp.data(), mu.data(), &q) ==
        GBM_E_ARG);
  CHECK(std::strlen(gbm_last_error()) > 0);
  CHECK(gbm_gblup_fit(X.data(), n, p, n - 1, Y.data(), n, 1, 1.0, nullptr, 0, b.data(), yp.data(), mu.data(), &q) ==
        GBM_E_ARG);
  CHECK(gbm_gblup_fit(X.data(), n, p, n, Y.data(), n, 1, 0.0, nullptr, 0, b.data(), yp.data(), mu.data(), &q) ==
        GBM_E_ARG);
  CHECK(gbm_gblup_fit(X.data(), n, p, n, Y.data(), n, 64, 1.0, nullptr, 0, b.data(), yp.data(), mu.data(), &q) ==
        GBM_E_ARG);
  CHECK(gbm_gblup_fit(X.data(), 1, p, n, Y.data(), n, 1, 1.0, nullptr, 0, b.data(), yp.data(), mu.data(), &q) ==
        GBM_E_DATA);
  std::vector<double> Ynan(Y);
  Ynan[3] = NAN;
  CHECK(gbm_gblup_fit(X.data(), n, p, n, Ynan.data(), n, 1, 1.0, nullptr, 0, b.data(), yp.data(), mu.data(), &q) !=
        GBM_OK);
  const int bad_dev[2] = {0, -3};
  CHECK(gbm_gblup_fit(X.data(), n, p, n, Y.data(), n, 1, 1.0, bad_dev, 2, b.data(), yp.data(), mu.data(), &q) !=
        GBM_OK);
  std::vector<int8_t> D(n * p, 1);
  CHECK(gbm_gblup_fit_dosage_i8(D.data(), n, p, n, 0, Y.data(), n, 1, 1.0, nullptr, 0, b.data(), yp.data(),
                                mu.data(), &q) == GBM_E_ARG);
  CHECK(gbm_gblup_fit_synthetic(1, 0, p, Y.data(), n, 1, 1.0, nullptr, 0, b.data(), yp.data(), mu.data(), &q) !=
        GBM_OK);
  std::vector<double> G(n * n);
  CHECK(gbm_grm(nullptr, n, p, n, nullptr, 0, G.data(), n, &q) == GBM_E_ARG);
  std::vector<double> m(p), s(p);
  std::vector<uint8_t> keep(p);
  CHECK(gbm_colstats(nullptr, n, p, n, 0, m.data(), s.data(), keep.data(), &q) == GBM_E_ARG);
  CHECK(gbm_predict(X.data(), n, p, n, nullptr, p + 1, 1, 0, yp.data(), n) == GBM_E_ARG);
  // the no-GPU (or bad-device) paths of a well-formed call: an error, not a crash
  int ndev = -1;
  CHECK(gbm_device_count(&ndev) == GBM_OK && ndev >= 0);
  if (ndev == 0) {
    CHECK(gbm_gblup_fit(X.data(), n, p, n, Y.data(), n, 1, 1.0, nullptr, 0, b.data(), yp.data(), mu.data(), &q) !=
          GBM_OK);
    gbm_session* sess = nullptr;
    CHECK(gbm_session_create(X.data(), n, p, n, 0, &sess) != GBM_OK && sess == nullptr);
  }
  gbm_session* sess = nullptr;
  CHECK(gbm_session_create(nullptr, n, p, n, 0, &sess) == GBM_E_ARG);
  CHECK(gbm_session_create(X.data(), n, p, n, 0, nullptr) == GBM_E_ARG);
  std::vector<int64_t> idx(n);
  for (int64_t i = 0; i < n; i++) idx[i] = i;
  CHECK(gbm_session_gblup_fit(nullptr, idx.data(), n, Y.data(), n, 1, 1.0, b.data(), yp.data(), mu.data(), &q) ==
        GBM_E_ARG);
  CHECK(gbm_session_predict(nullptr, idx.data(), n, b.data(), p + 1, 1, yp.data(), n) == GBM_E_ARG);
  gbm_session_destroy(nullptr);
  // device-level geometry helpers (host arithmetic only)
  CHECK(gbm_dev_npad(5000) == 5120 && gbm_dev_gdim(5000) == 5184);
  CHECK(gbm_dev_solve_workspace(5000, 1) > 0 && gbm_dev_grm_workspace(5000, 50000) > 0);
  CHECK(gbm_dev_chol_group_size(5000, 100000) == 0);
  CHECK(gbm_dev_chol_strip_doubles(5000, 0, 2, 0) == 0);
  CHECK(gbm_dev_gblup_solve(nullptr, 0, 0, 1.0, nullptr, 1.0, nullptr, 0, 1, nullptr, nullptr, 0, nullptr, nullptr,
                            nullptr, 0, nullptr) == GBM_E_ARG);
  CHECK(gbm_dev_grm_syrk(nullptr, 0, 0, 0, nullptr, 0, nullptr, 0, nullptr) == GBM_E_ARG);
}

// the host packer (grm_mode exact / auto on fp64 host X): 2x in {0, 1, 2} packed, anything else flagged —
// 0.25, 1.5, NaN, ±Inf, a negative dosage — in any column of a strided (ld > n) block
static void host_pack() {
  const int64_t n = 37, ld = 41, p = 5;
  std::vector<double> X(ld * p, 7.0);
  for (int64_t j = 0; j < p; j++)
    for (int64_t i = 0; i < n; i++) X[j * ld + i] = 0.5 * (double)((i * 7 + j) % 3);
  X[2 * ld + 3] = -0.0;
  std::vector<int8_t> D(n * p, -1);
  CHECK(gbm::pack_dosage_columns(X.data(), ld, n, p, D.data()));
  bool same = true;
  for (int64_t j = 0; j < p; j++)
    for (int64_t i = 0; i < n; i++) same &= D[j * n + i] == (int8_t)(2.0 * X[j * ld + i]);
  CHECK(same);
  const double bad_vals[] = {0.25, 1.5, NAN, INFINITY, -INFINITY, -0.5, 1.0000000000000002};
  for (double v : bad_vals) {
    std::vector<double> Y(X);
    Y[(p - 1) * ld + n - 1] = v;  // the last cell of the last column
    CHECK(!gbm::pack_dosage_columns(Y.data(), ld, n, p, D.data()));
  }
}

// the chunked packer: 13 chunks of a strided block through a 3-slot ring by 5 workers, each slot released after
// its chunk is consumed; then a non-dosage value in chunk 9 stops it there
static void chunk_packer() {
  const int64_t n = 53, ld = 60, p = 397, pc = 31, R = 3;
  std::vector<double> X(ld * p, 9.0);
  for (int64_t j = 0; j < p; j++)
    for (int64_t i = 0; i < n; i++) X[j * ld + i] = 0.5 * (double)((i * 5 + j * 3) % 3);
  std::vector<std::pair<int64_t, int64_t>> sched;
  for (int64_t j = 0; j < p; j += pc) sched.emplace_back(j, std::min(pc, p - j));
  std::vector<int8_t> ring(R * pc * n), out(n * p, -1);
  for (int round = 0; round < 2; round++) {
    if (round == 1) X[(9 * pc + 4) * ld + 7] = 0.75;
    gbm::ChunkPacker pk(X.data(), ld, n, sched, ring.data(), pc * n, (int)R, 5);
    int64_t k = 0;
    for (; k < (int64_t)sched.size(); k++) {
      const int8_t* src = pk.wait(k);
      if (!src) break;
      std::memcpy(out.data() + sched[k].first * n, src, sched[k].second * n);
      pk.release_upto(k + 1);
    }
    if (round == 0) {
      CHECK(k == (int64_t)sched.size());
      bool same = true;
      for (int64_t j = 0; j < p; j++)
        for (int64_t i = 0; i < n; i++) same &= out[j * n + i] == (int8_t)(2.0 * X[j * ld + i]);
      CHECK(same);
    } else {
      CHECK(k <= 9);
    }
  }
}

int main() {
  CHECK(gbm_version() == GBM_VERSION);
  host_pack();
  chunk_packer();
  entry_points(0);
  // eight threads at once: every error message stays in its own thread
  std::vector<std::thread> th;
  std::vector<int> ok(8, 0);
  for (int t = 0; t < 8; t++)
    th.emplace_back([t, &ok] {
      for (int r = 0; r < 20; r++) {
        entry_points(t);
        const std::string mine = "gbm_gblup_fit: X is NULL";
        std::vector<double> Y(10, 1.0), b(5), yp(10);
        if (gbm_gblup_fit(nullptr, 10, 4, 10, Y.data(), 10, 1, 1.0, nullptr, 0, b.data(), yp.data(), nullptr,
                          nullptr) == GBM_E_ARG &&
            mine == gbm_last_error())
          ok[t]++;
      }
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < 8; t++) CHECK(ok[t] == 20);
  // knobs (csrc/knobs.cpp): four threads change GBM_CHOL_FLOW_ORDER through gbm_debug_set while four others
  // read it on every host-side dequeue-order build; no getenv, no torn or freed value (ASan)
  CHECK(gbm_debug_set("PATH", "x") == GBM_E_ARG);
  std::vector<std::thread> kt;
  std::vector<int> kbad(8, 0);
  for (int t = 0; t < 8; t++)
    kt.emplace_back([t, &kbad] {
      static const char* vals[3] = {"4", "6", nullptr};
      for (int r = 0; r < 200; r++) {
        if (t < 4) {
          if (gbm_debug_set("GBM_CHOL_FLOW_ORDER", vals[(r + t) % 3]) != GBM_OK) kbad[t]++;
        } else {
          // one knob read per call: every variant's order is complete and deadlock-free (return 0)
          if (gbm_debug_chol_flow_order(24, nullptr, 0) != 0) kbad[t]++;
        }
      }
    });
  for (auto& x : kt) x.join();
  for (int t = 0; t < 8; t++) CHECK(kbad[t] == 0);
  CHECK(gbm_debug_set("GBM_CHOL_FLOW_ORDER", nullptr) == GBM_OK);
  std::printf("asan driver: %d failures\n", failures);
  return failures ? 1 : 0;
}
