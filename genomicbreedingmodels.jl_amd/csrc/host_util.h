// Host-side helpers shared by the libgbm entry points (capi.cpp, session.cpp): RAII device
// buffers and streams, device-list and phenotype validation. Not part of the ABI.
#pragma once
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "gbm_internal.h"

namespace gbm {

// roctx range over a host phase (rocprofv3 --marker-trace shows the fit's phases beside the
// kernel trace): an entry point, or one stage of it
struct RoctxRange {
  explicit RoctxRange(const char* name) { roctxRangePushA(name); }
  ~RoctxRange() { roctxRangePop(); }
  RoctxRange(const RoctxRange&) = delete;
  RoctxRange& operator=(const RoctxRange&) = delete;
};

// RAII device allocation on a given device
struct DevMem {
  void* p = nullptr;
  int dev = 0;
  DevMem() = default;
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  ~DevMem() { reset(); }
  void reset() {
    if (p) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(dev);
      (void)hipFree(p);
      (void)hipSetDevice(cur);
      p = nullptr;
    }
  }
};

// Device allocations made by libgbm since load (gbm_device_allocations): the pooled fit
// contexts make a repeated call allocate nothing.
inline std::atomic<int64_t>& alloc_counter() {
  static std::atomic<int64_t> c{0};
  return c;
}

// When a device allocation runs out of memory, every registered trim callback frees the idle pooled
// contexts of that device (capi.cpp: GBLUP fit contexts; gibbs.hip: BRR contexts, which also hold
// their captured graphs) and returns how many it freed; the allocation is then retried once.
using TrimFn = int64_t (*)(int dev);
struct OomTrim {
  std::mutex mu;
  std::vector<TrimFn> hooks;
  std::atomic<int64_t> retries{0}, freed{0};  // gbm_debug_oom_retries
};
inline OomTrim& oom_trim() {
  static OomTrim* t = new OomTrim;  // never destroyed (pools outlive static destruction)
  return *t;
}
inline void register_trim_hook(TrimFn f) {
  OomTrim& t = oom_trim();
  std::lock_guard<std::mutex> lock(t.mu);
  for (TrimFn g : t.hooks)
    if (g == f) return;
  t.hooks.push_back(f);
}

inline int dalloc(DevMem& m, int dev, int64_t bytes) {
  m.reset();
  m.dev = dev;
  if (bytes <= 0) bytes = 16;
  alloc_counter().fetch_add(1, std::memory_order_relaxed);
  // GBM_TEST_OOM_ONCE=1 (tests): every allocation's first attempt reports out-of-memory, so the
  // trim-and-retry path below runs
  const char* t1 = ::gbm::knob("GBM_TEST_OOM_ONCE");
  hipError_t e = (t1 && t1[0] == '1') ? hipErrorOutOfMemory : hipMalloc(&m.p, (size_t)bytes);
  if (e == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    OomTrim& t = oom_trim();
    std::vector<TrimFn> hooks;
    {
      std::lock_guard<std::mutex> lock(t.mu);
      hooks = t.hooks;
    }
    int64_t freed = 0;
    for (TrimFn f : hooks) freed += f(dev);
    t.retries.fetch_add(1, std::memory_order_relaxed);
    t.freed.fetch_add(freed, std::memory_order_relaxed);
    (void)hipSetDevice(dev);
    e = hipMalloc(&m.p, (size_t)bytes);
  }
  if (e != hipSuccess) {
    m.p = nullptr;
    (void)hipGetLastError();
    return fail(e == hipErrorOutOfMemory ? GBM_E_OOM : GBM_E_HIP,
                std::string("device allocation of ") + std::to_string(bytes) + " bytes on device " + std::to_string(dev) +
                    " failed: " + hipGetErrorString(e));
  }
  return GBM_OK;
}

// A device buffer that only grows: ensure() reallocates when the capacity is short, so a pooled
// context reused for same-sized (or smaller) problems never calls hipMalloc again.
struct DevBuf : DevMem {
  int64_t cap = 0;
};
inline int ensure(DevBuf& b, int dev, int64_t bytes) {
  if (bytes <= 0) bytes = 16;
  if (b.p && b.dev == dev && b.cap >= bytes) return GBM_OK;
  b.cap = 0;
  int rc = dalloc(b, dev, bytes);
  if (rc == GBM_OK) b.cap = bytes;
  return rc;
}

// A pinned (page-locked) host buffer that only grows (the host-pack staging ring of a pooled context).
struct HostPinned {
  void* p = nullptr;
  int64_t cap = 0;
  HostPinned() = default;
  HostPinned(const HostPinned&) = delete;
  HostPinned& operator=(const HostPinned&) = delete;
  ~HostPinned() {
    if (p) (void)hipHostFree(p);
  }
};
inline int ensure_pinned(HostPinned& b, int64_t bytes) {
  if (b.p && b.cap >= bytes) return GBM_OK;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  const hipError_t e = hipHostMalloc(&b.p, (size_t)bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    b.p = nullptr;
    return fail(GBM_E_OOM, std::string("pinned host allocation of ") + std::to_string(bytes) + " bytes failed: " +
                               hipGetErrorString(e));
  }
  b.cap = bytes;
  return GBM_OK;
}

struct Stream {
  hipStream_t s = nullptr;
  int dev = 0;
  ~Stream() {
    if (s) {
      (void)hipSetDevice(dev);
      (void)hipStreamDestroy(s);
    }
  }
};


// Device list of a call. Explicit `devices` (one SNP-column shard per entry; an ordinal may
// repeat: shards on one device are summed on that device). With none given, the calling thread
// gets ONE device, round-robin over GBM_DEVICES ("0,1,...", re-read per call; repeats allowed)
// or over all visible devices: thread k (in order of first call) -> entry k mod len. That is the
// thread -> GPU farming of SURVEY.md §8b under an unchanged cvmultithread! (reference
// src/cross_validation.jl:159, Threads.@threads over model calls that pass no devices).
inline int check_devices(const int* devices, int ndev, std::vector<int>& out) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count < 1) {
    (void)hipGetLastError();
    return fail(GBM_E_NODEV, "no HIP device available (libgbm requires an MI355X / gfx950 GPU)");
  }
  out.clear();
  if (!devices || ndev <= 0) {
    std::vector<int> pool;
    if (const char* env = ::gbm::knob("GBM_DEVICES")) {
      for (const char* q = env; *q;) {
        char* end = nullptr;
        const long v = strtol(q, &end, 10);
        if (end == q) {
          q++;
          continue;
        }
        if (v < 0 || v >= count)
          return fail(GBM_E_ARG, "GBM_DEVICES: device ordinal " + std::to_string(v) + " out of range [0, " +
                                     std::to_string(count) + ")");
        pool.push_back((int)v);
        q = end;
      }
    }
    if (pool.empty())
      for (int d = 0; d < count; d++) pool.push_back(d);
    static std::atomic<int> next_slot{0};
    thread_local int slot = -1;
    if (slot < 0) slot = next_slot.fetch_add(1, std::memory_order_relaxed);
    out.push_back(pool[(size_t)slot % pool.size()]);
  } else {
    for (int k = 0; k < ndev; k++) {
      if (devices[k] < 0 || devices[k] >= count)
        return fail(GBM_E_ARG, "device ordinal " + std::to_string(devices[k]) + " out of range [0, " +
                                   std::to_string(count) + ")");
      out.push_back(devices[k]);
    }
  }
  return GBM_OK;
}

// Phenotype checks of reference src/prediction.jl:114-127 (finite values, variance >= 1e-20).
inline int check_y(const double* Y, int64_t n, int64_t ldy, int64_t nrhs) {
  for (int64_t t = 0; t < nrhs; t++) {
    const double* y = Y + t * ldy;
    double s = 0.0;
    for (int64_t i = 0; i < n; i++) {
      if (!std::isfinite(y[i]))
        return fail(GBM_E_ARG, "phenotype " + std::to_string(t + 1) + " has a missing/NaN/Inf value at entry " +
                                   std::to_string(i + 1) + " (filter it first, reference src/prediction.jl:114-124)");
      s += y[i];
    }
    const double m = s / (double)n;
    double ss = 0.0;
    for (int64_t i = 0; i < n; i++) ss += (y[i] - m) * (y[i] - m);
    if (ss / (double)(n - 1) < 1e-20)
      return fail(GBM_E_DATA, "very low or zero variance in trait " + std::to_string(t + 1) +
                                  " (reference src/prediction.jl:125-127)");
  }
  return GBM_OK;
}

}  // namespace gbm
