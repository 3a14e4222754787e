// Internal helpers shared by the libgbm translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <functional>
#include <string>
#include <vector>

#include "../../include/gbm.h"

namespace gbm {

// Tile geometry (see DESIGN.md "Data layout in HBM").
constexpr int64_t kNPadTile = 128;  // individuals padded to a multiple of the GRM tile
constexpr int64_t kRhsRows = 64;    // bordered right-hand-side rows appended to V
constexpr int kCholNB = 64;         // Cholesky panel width

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
inline int64_t npad_of(int64_t n) { return round_up(n < 1 ? 1 : n, kNPadTile); }
inline int64_t gdim_of(int64_t n) { return npad_of(n) + kRhsRows; }

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

// GBM_* tuning/test knobs (knobs.cpp): the environment is read once, at the first lookup; afterwards
// values change only through gbm_debug_set. knob() returns the value (a pointer valid for the life of
// the process) or nullptr when unset; knob_i64 parses it (def when unset or empty).
const char* knob(const char* name);
int64_t knob_i64(const char* name, int64_t def);

#define GBM_HIP_TRY(expr)                                                                      \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return ::gbm::fail(GBM_E_HIP, std::string("HIP error '") + hipGetErrorString(e_) +       \
                                        "' at " __FILE__ ":" + std::to_string(__LINE__) + " (" #expr ")"); \
  } while (0)

#define GBM_LAUNCH_CHECK() GBM_HIP_TRY(hipGetLastError())

#define GBM_TRY(expr)              \
  do {                             \
    int rc_ = (expr);              \
    if (rc_ != GBM_OK) return rc_; \
  } while (0)

// Stage launchers (device pointers, stream-ordered); defined in the .hip files.
// accum = 1: G += the GRM of these loci (only where grm_can_accumulate(n, p)). err_out (device
// int32, optional): the in-order carry's error cell is copied there (< 0: a wait timed out, G
// invalid) instead of being read back with a stream sync.
int launch_grm(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
               void* ws, int64_t ws_bytes, hipStream_t s, int accum = 0, int32_t* err_out = nullptr);
bool grm_can_accumulate(int64_t n, int64_t p);
int64_t grm_workspace_bytes(int64_t n, int64_t p);
int launch_grm_export(const double* G, int64_t ldg, int64_t n, double inv_q, double* out, int64_t ldo, hipStream_t s);
int launch_predict(const double* Xt, int64_t ldx, int64_t p, int64_t n, const double* b, int64_t ldb, int64_t nrhs,
                   double* partial, int64_t nchunks, double* out, int64_t ldo, hipStream_t s);
int64_t predict_chunks(int64_t n, int64_t p);
int launch_add_inplace(double* a, const double* b, int64_t n, hipStream_t s);
// centre the columns only (Z = X − m; every column kept, sd = 1): the ploidy-aware GRM
// standardisation straight from int8 dosage rows (x = d / ploidy), out of place into Zt
int launch_standardize_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, double* Zt, int64_t ldz,
                          double* mean, double* sd, int32_t* keep, int64_t* q_dev, hipStream_t s);
// marker effects in pieces (effects.hip): B rows of fp64 standardised rows or of int8 dosage rows
// (z rebuilt bit-identically), and msum = Σ_j mean_j B[t, j] over p loci
int launch_marker_rows(const double* Zt, int64_t ldz, int64_t p, int64_t n, const double* A, int64_t lda, int64_t nrhs,
                       double inv_q, const int64_t* q_dev, const double* sd, const int32_t* keep, double* B,
                       int64_t ldb, hipStream_t s);
int launch_marker_rows_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, const double* A, int64_t lda,
                          int64_t nrhs, double inv_q, const int64_t* q_dev, const double* mean, const double* sd,
                          const int32_t* keep, double* B, int64_t ldb, hipStream_t s);
// the exact-integer GRM of diploid dosage rows (grm_exact.hip)
int launch_grm_exact(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, double* G, int64_t ldg,
                     double* mean, double* sd, int32_t* keep, int64_t* q_dev, int accum, void* ws, int64_t ws_bytes,
                     int32_t* slices_out, hipStream_t s);
// after launch_grm_exact (syncs the stream): GBM_E_HIP when a weight overflowed its digits (XgInfo bit 2)
int grm_exact_status(const void* ws, int64_t n, int64_t p, hipStream_t s);
// training-set dosages 2·Xt[j, idx[i]] (resident genotypes that are dosages/2) for the exact GRM
int launch_gather_dosage(const double* Xt, int64_t ldx, int64_t p, const int32_t* idx, int64_t nT, int8_t* D,
                         hipStream_t s);
// dosage detection (grm_mode exact / auto): D = 2·X as bytes (D may be NULL: check only), *bad = 1 when any
// 2x is not 0, 1 or 2; the same check on dosage bytes
int launch_dosage_from_f64(const double* X, int64_t ldx, int64_t n, int64_t p, int8_t* D, int64_t ldd, int32_t* bad,
                           hipStream_t s);
int launch_dosage_check_i8(const int8_t* D, int64_t ldd, int64_t n, int64_t p, int32_t* bad, hipStream_t s);
// host packing (hostpack.cpp): fp64 columns (column j at X + j·ld) → dosage bytes 2x (n per column); false when
// some 2x is not exactly 0, 1 or 2. host_pack_threads: the packing workers of one call (GBM_PACK_THREADS)
bool pack_dosage_columns(const double* X, int64_t ld, int64_t n, int64_t p, int8_t* dst);
int host_pack_threads();
// Packs the loci chunks sched[k] = (first locus, count) of fp64 columns (column j at X + j·ld) into dosage bytes,
// chunk k into ring slot k mod slots (slot_bytes each, n bytes per locus), by `threads` workers that split each
// chunk in order. wait(k): chunk k's packed bytes, or nullptr once any chunk was not dosage-valued (the workers then
// stop); release_upto(k): the slots of chunks < k may be overwritten. The destructor stops and joins the workers.
class ChunkPacker {
 public:
  ChunkPacker(const double* X, int64_t ld, int64_t n, const std::vector<std::pair<int64_t, int64_t>>& sched,
              int8_t* ring, int64_t slot_bytes, int slots, int threads);
  ~ChunkPacker();
  ChunkPacker(const ChunkPacker&) = delete;
  ChunkPacker& operator=(const ChunkPacker&) = delete;
  const int8_t* wait(int64_t k);
  void release_upto(int64_t k);

 private:
  struct Impl;
  Impl* d_;
};
// GBM_GRM_* of a call: grm_mode, or for GBM_GRM_DEFAULT the GBM_GRM environment variable, else fp64
int resolve_grm_mode(int grm_mode);
int launch_weighted_sum(const double* mean, const double* B, int64_t ldb, int64_t p, int64_t nrhs, double* msum,
                        hipStream_t s);
int launch_center_columns(const double* Xt, int64_t ldx, int64_t p, int64_t n, double* Zt, int64_t ldz, double* mean,
                          double* sd, int32_t* keep, int64_t* q_dev, hipStream_t s);


// REML choice of λ (session.cpp; reference loglikreml src/gwas.jl:450-483 with X = 1)
struct RemlEval {
  double g, s2u, s2e;  // objective, σ²_u, σ²_e at one λ (σ²_u profiled inside the box [eps, 1]²)
};
struct RemlResult {
  double lambda, s2e, s2u, objective;
};
double reml_objective(int64_t n, double logdet, double c11, double Q, double s2u);
RemlEval reml_profile(int64_t n, double lambda, const double t[4]);
int reml_search(const std::function<int(double, RemlEval&)>& eval, RemlResult& out);
std::vector<double> standardise_y(const double* y, int64_t n);
// frees the idle pooled BRR contexts (gibbs.hip; part of gbm_release_device_cache)
void brr_release_cache();

}  // namespace gbm
