// Host-side dosage packing for the exact-integer GRM of fp64 host genotypes (grm_mode exact / auto on the
// drop-in's allele frequencies, reference src/prediction.jl:129): X's fp64 columns are checked to be
// diploid dosages/2 (2x exactly 0, 1 or 2) and packed to bytes D = 2x on the host, by several threads,
// so that only n·p bytes cross PCIe instead of 8·n·p (C2: 250 MB instead of 2 GB). The device-side
// alternative (launch_dosage_from_f64 on uploaded fp64 chunks) is kept behind GBM_HOST_PACK=0.
#include <sched.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

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

// ---- ChunkPacker ------------------------------------------------------------------------------------------
struct ChunkPacker::Impl {
  const double* X;
  int64_t ld, n;
  std::vector<std::pair<int64_t, int64_t>> sched;
  int8_t* ring;
  int64_t slot_bytes;
  int R, T;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<int> done;     // parts packed per chunk
  int64_t released = 0;      // chunks [0, released) have left their slots
  int64_t next_item = 0;     // (chunk, part) items handed out, chunk-major
  bool bad = false, stop = false;
  std::vector<std::thread> th;

  void work() {
    for (;;) {
      int64_t item, k;
      {
        std::unique_lock<std::mutex> lk(mu);
        if (bad || stop || next_item >= (int64_t)sched.size() * T) return;
        item = next_item++;
        k = item / T;
        cv.wait(lk, [&] { return bad || stop || k < released + R; });
        if (bad || stop) return;
      }
      const int part = (int)(item % T);
      const int64_t j = sched[k].first, pc = sched[k].second;
      const int64_t a = pc * part / T, b = pc * (part + 1) / T;  // this part's loci of the chunk
      const bool ok = b <= a || pack_dosage_columns(X + (j + a) * ld, ld, n, b - a, ring + (k % R) * slot_bytes + a * n);
      std::lock_guard<std::mutex> lk(mu);
      if (!ok) bad = true;
      else done[k]++;
      // wake the waiters only when it matters: a finished chunk (the uploader) or a stop (everyone); a worker
      // waiting for a slot is woken by release_upto
      if (!ok || done[k] == T) cv.notify_all();
      if (!ok) return;
    }
  }
};

ChunkPacker::ChunkPacker(const double* X, int64_t ld, int64_t n, const std::vector<std::pair<int64_t, int64_t>>& sched,
                         int8_t* ring, int64_t slot_bytes, int slots, int threads)
    : d_(new Impl) {
  d_->X = X;
  d_->ld = ld;
  d_->n = n;
  d_->sched = sched;
  d_->ring = ring;
  d_->slot_bytes = slot_bytes;
  d_->R = std::max(1, slots);
  d_->T = std::max(1, threads);
  d_->done.assign(sched.size(), 0);
  for (int t = 0; t < d_->T; t++) {
    try {
      d_->th.emplace_back([this] { d_->work(); });
    } catch (...) {  // no thread available: wait() packs on the calling thread
      break;
    }
  }
}

ChunkPacker::~ChunkPacker() {
  {
    std::lock_guard<std::mutex> lk(d_->mu);
    d_->stop = true;
    d_->cv.notify_all();
  }
  for (auto& t : d_->th) t.join();
  delete d_;
}

const int8_t* ChunkPacker::wait(int64_t k) {
  Impl& d = *d_;
  if (d.th.empty()) {  // no workers: pack the whole chunk here (its slot is free: the caller released k − R)
    const int64_t j = d.sched[k].first, pc = d.sched[k].second;
    if (d.bad || !pack_dosage_columns(d.X + j * d.ld, d.ld, d.n, pc, d.ring + (k % d.R) * d.slot_bytes)) {
      d.bad = true;
      return nullptr;
    }
    return d.ring + (k % d.R) * d.slot_bytes;
  }
  std::unique_lock<std::mutex> lk(d.mu);
  d.cv.wait(lk, [&] { return d.bad || d.done[k] == d.T; });
  return d.bad ? nullptr : d.ring + (k % d.R) * d.slot_bytes;
}

void ChunkPacker::release_upto(int64_t k) {
  std::lock_guard<std::mutex> lk(d_->mu);
  if (k > d_->released) {
    d_->released = k;
    d_->cv.notify_all();
  }
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
