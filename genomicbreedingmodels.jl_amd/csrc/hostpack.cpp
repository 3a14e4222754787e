// Host-side dosage packing for the exact-integer GRM of fp64 host genotypes (grm_mode exact / auto on the
// drop-in's allele frequencies, reference src/prediction.jl:129): X's fp64 columns are checked to be
// diploid dosages/2 (2x exactly 0, 1 or 2) and packed to bytes D = 2x on the host, by several threads,
// so that only n·p bytes cross PCIe instead of 8·n·p (C2: 250 MB instead of 2 GB). The device-side
// alternative (launch_dosage_from_f64 on uploaded fp64 chunks) is kept behind GBM_HOST_PACK=0.
#include <sched.h>

#include <algorithm>
#include <cstdint>

#include "gbm_internal.h"

namespace gbm {

namespace {

// One column: dst[i] = 2·x[i] as a byte; returns nonzero when some 2x is not exactly 0, 1 or 2 (NaN and ±Inf
// included: every comparison with them is false). Branch-free so the compiler vectorises it; an AVX2 clone is
// picked at load time where the CPU has it.
__attribute__((target_clones("avx2", "default"))) int pack_column(const double* __restrict__ x, int64_t n,
                                                                  int8_t* __restrict__ dst) {
  int bad = 0;
  for (int64_t i = 0; i < n; i++) {
    const double t = x[i] + x[i];
    const int one = t == 1.0, two = t == 2.0, zero = t == 0.0;
    bad |= !(one | two | zero);
    dst[i] = (int8_t)(one + 2 * two);
  }
  return bad;
}

}  // namespace

bool pack_dosage_columns(const double* X, int64_t ld, int64_t n, int64_t p, int8_t* dst) {
  int bad = 0;
  for (int64_t j = 0; j < p; j++) bad |= pack_column(X + j * ld, n, dst + j * n);
  return bad == 0;
}

int host_pack_threads() {
  // GBM_PACK_THREADS (tests, A/B); default the CPUs this process may run on, at most 16 (a box's share of its
  // host) and at least 1
  const int64_t forced = knob_i64("GBM_PACK_THREADS", 0);
  if (forced > 0) return (int)std::min<int64_t>(forced, 64);
  cpu_set_t set;
  int cpus = 1;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
  return std::max(1, std::min(cpus, 16));
}

}  // namespace gbm
