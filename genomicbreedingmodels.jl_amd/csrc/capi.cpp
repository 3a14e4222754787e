// Host entry points of libgbm.so (include/gbm.h): argument checks, H2D/D2H, SNP-column sharding
// over devices and the sum of partial GRMs (device-side for shards on one device, RCCL all-reduce
// across devices).
//
// Re-entrant, as cvmultithread! requires (reference src/cross_validation.jl:159): a call leases
// one pooled fit context per shard (its own stream and buffers) and returns it afterwards; the
// contexts' buffers only grow, so repeated calls of one shape allocate no device memory. RCCL
// communicators are created once per device set and reused.
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
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

// ---- pooled fit contexts -----------------------------------------------------------------------

struct FitCtx {
  int dev = 0;
  Stream stream;
  Stream copy;                   // host -> device copies of the pipelined upload (created on first use)
  std::vector<hipEvent_t> ev;    // one per upload chunk
  DevBuf Xt, D8, mean, sd, keep, q, G, Gc, wsg, Y, A, gebv, mu, info, wss, B, msum, packed, out, part;
  DevBuf tmp, strip, gathered;   // copy exchanges; the distributed factorisation's strip all-gather
  DevBuf errs, q2;               // streamed fit: per-chunk carry error cells; scratch kept count
  DevBuf astrip, agathered;      // the distributed factorisation's area all-gather (on the copy stream)
  hipEvent_t ev_area = nullptr, ev_upd = nullptr;  // area exchange done / next area updated
  HostPinned pack;               // host-pack staging ring (fp64 host X packed to dosage bytes)
  ~FitCtx() {
    (void)hipSetDevice(dev);
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    if (ev_area) (void)hipEventDestroy(ev_area);
    if (ev_upd) (void)hipEventDestroy(ev_upd);
  }
};

class CtxPool {
 public:
  int acquire(int dev, std::unique_ptr<FitCtx>& out) {
    {
      std::lock_guard<std::mutex> lock(mu_);
      auto& v = idle_[dev];
      if (!v.empty()) {
        out = std::move(v.back());
        v.pop_back();
        return GBM_OK;
      }
    }
    auto c = std::make_unique<FitCtx>();
    c->dev = dev;
    c->stream.dev = dev;
    GBM_HIP_TRY(hipSetDevice(dev));
    GBM_HIP_TRY(hipStreamCreateWithFlags(&c->stream.s, hipStreamNonBlocking));
    out = std::move(c);
    return GBM_OK;
  }
  void release(std::unique_ptr<FitCtx> c) {
    // nothing of this call may still run on the context's stream when another call takes it
    (void)hipSetDevice(c->dev);
    if (hipStreamSynchronize(c->stream.s) != hipSuccess) {
      (void)hipGetLastError();
      return;  // a broken context is dropped (its destructor frees what it can)
    }
    std::lock_guard<std::mutex> lock(mu_);
    idle_[c->dev].push_back(std::move(c));
  }
  void clear() {
    std::map<int, std::vector<std::unique_ptr<FitCtx>>> drop;
    {
      std::lock_guard<std::mutex> lock(mu_);
      drop.swap(idle_);
    }
  }
  // drops the idle contexts of one device (their buffers are freed outside the lock); returns how many
  int64_t trim(int dev) {
    std::vector<std::unique_ptr<FitCtx>> drop;
    {
      std::lock_guard<std::mutex> lock(mu_);
      auto it = idle_.find(dev);
      if (it != idle_.end()) drop.swap(it->second);
    }
    return (int64_t)drop.size();
  }

 private:
  std::mutex mu_;
  std::map<int, std::vector<std::unique_ptr<FitCtx>>> idle_;
};

// never destroyed: pooled device memory must not be freed after the HIP runtime tears down
CtxPool& pool() {
  static CtxPool* p = [] {
    auto* cp = new CtxPool;
    // an allocation that runs out of device memory first frees the idle contexts of its device
    // (they only grow and would otherwise hold e.g. ~50 GB each at C3's shape), then retries once
    register_trim_hook([](int dev) { return pool().trim(dev); });
    return cp;
  }();
  return *p;
}

// One SNP-column shard [j0, j0 + p) on a leased context.
struct Shard {
  std::unique_ptr<FitCtx> c;
  int64_t j0 = 0, p = 0;
  int64_t q_host = 0;
  int64_t stream = 0;  // loci per chunk of the loci-streamed mode (plan_streaming); 0: resident
  bool exact = false;  // the exact-integer GRM of the resident dosages (grm_exact.hip, grm_mode exact / auto)
  bool d8_ready = false;  // fp64 X already converted into the dosage bytes D8 (dosage_upload_shard)
  int leader = -1;  // index of the shard that holds this device's summed GRM (itself if first)
  ~Shard() {
    if (c) pool().release(std::move(c));
  }
  FitCtx& x() { return *c; }
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

// GBM_SHARD_LEADERS=each (re-read per call): every shard keeps its own full G and is a rank of its
// own in the GRM sum and the distributed factorisation, its exchanges done by device copies. That
// is the one-GPU rehearsal of the multi-device path (devices = [0, 0, ...]; RCCL cannot put two
// ranks on one device). Default: one leader per device, RCCL between the leaders.
bool each_shard_leads() {
  const char* e = ::gbm::knob("GBM_SHARD_LEADERS");
  return e && strcmp(e, "each") == 0;
}

// Contiguous SNP-column blocks, one per listed device; leader = first shard on each device.
int make_shards(const std::vector<int>& devs, int64_t p, std::vector<std::unique_ptr<Shard>>& shards) {
  const int nd = (int)std::min<int64_t>((int64_t)devs.size(), p);
  const int64_t per = (p + nd - 1) / nd;
  const bool each = each_shard_leads();
  for (int k = 0; k < nd; k++) {
    const int64_t j0 = k * per;
    if (j0 >= p) break;
    auto sh = std::make_unique<Shard>();
    GBM_TRY(pool().acquire(devs[k], sh->c));
    sh->j0 = j0;
    sh->p = std::min(per, p - j0);
    for (size_t m = 0; m < shards.size() && !each; m++)
      if (shards[m]->x().dev == devs[k]) {
        sh->leader = shards[m]->leader;
        break;
      }
    if (sh->leader < 0) sh->leader = (int)shards.size();
    shards.push_back(std::move(sh));
  }
  return GBM_OK;
}

// Upload the shard's columns and standardise them in place (center_only: centre them only, the
// ploidy-aware GRM); reads back the shard's kept count (valid once the stream has synchronised:
// here with sync, else by the caller after it has queued more work behind it).
int prepare_shard(const Problem& pr, Shard& sh, bool center_only = false, bool sync = true) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, npad = npad_of(n), pl = sh.p;
  GBM_HIP_TRY(hipSetDevice(c.dev));
  hipStream_t s = c.stream.s;
  GBM_TRY(ensure(c.Xt, c.dev, pl * npad * 8));
  GBM_TRY(ensure(c.mean, c.dev, pl * 8));
  GBM_TRY(ensure(c.sd, c.dev, pl * 8));
  GBM_TRY(ensure(c.keep, c.dev, pl * 4));
  GBM_TRY(ensure(c.q, c.dev, 8));
  if (pr.src == Source::F64) {
    GBM_HIP_TRY(hipMemcpy2DAsync(c.Xt.p, npad * 8, pr.X + sh.j0 * pr.ld, pr.ld * 8, n * 8, pl, hipMemcpyHostToDevice, s));
    if (npad > n) GBM_HIP_TRY(hipMemset2DAsync((double*)c.Xt.p + n, npad * 8, 0, (npad - n) * 8, pl, s));
  } else if (pr.src == Source::SYNTH) {
    GBM_TRY(gbm_dev_synth_genotypes((double*)c.Xt.p, npad, pl, n, pr.seed, sh.j0, s));
  } else {
    GBM_TRY(ensure(c.D8, c.dev, pl * n));
    GBM_HIP_TRY(hipMemcpy2DAsync(c.D8.p, n, pr.D + sh.j0 * pr.ld, pr.ld, n, pl, hipMemcpyHostToDevice, s));
    GBM_TRY(gbm_dev_expand_dosage_i8((const int8_t*)c.D8.p, n, n, pl, pr.ploidy, (double*)c.Xt.p, npad, s));
  }
  GBM_HIP_TRY(hipMemsetAsync(c.q.p, 0, 8, s));
  if (center_only)
    GBM_TRY(launch_center_columns((const double*)c.Xt.p, npad, pl, n, (double*)c.Xt.p, npad, (double*)c.mean.p,
                                  (double*)c.sd.p, (int32_t*)c.keep.p, (int64_t*)c.q.p, s));
  else
    GBM_TRY(gbm_dev_standardize((const double*)c.Xt.p, npad, pl, n, (double*)c.Xt.p, npad, (double*)c.mean.p,
                                (double*)c.sd.p, (int32_t*)c.keep.p, (int64_t*)c.q.p, s));
  GBM_HIP_TRY(hipMemcpyAsync(&sh.q_host, c.q.p, 8, hipMemcpyDeviceToHost, s));
  if (sync) GBM_HIP_TRY(hipStreamSynchronize(s));
  return GBM_OK;
}

int grm_shard(const Problem& pr, Shard& sh);

// Upload + standardise + partial GRM of one shard, queued back to back on its stream, then one sync.
int prepare_grm_shard(const Problem& pr, Shard& sh) {
  GBM_TRY(prepare_shard(pr, sh, false, false));
  GBM_TRY(grm_shard(pr, sh));
  GBM_HIP_TRY(hipStreamSynchronize(sh.x().stream.s));
  return GBM_OK;
}

// Loci per chunk of the pipelined upload of host genotypes (0: one piece). Re-read per call:
// GBM_HOST_CHUNK = loci per chunk, 0 to disable; by default p/8 (>= 4096 loci) once p >= 16384
// (C2 host path, pageable X: 58.5 ms in one piece, 43.3 ms in 4 chunks, 40.9 ms in 8).
int64_t host_chunk(int64_t p) {
  const char* e = ::gbm::knob("GBM_HOST_CHUNK");
  int64_t c = e ? (int64_t)atoll(e) : -1;
  if (c == 0) return 0;
  if (c < 0) {
    if (p < 16384) return 0;
    c = std::max<int64_t>(4096, (p + 7) / 8);
  }
  return c >= p ? 0 : c;
}

// Chunk schedule of the pipelined upload: chunks of `chunk` loci, the last full-size piece cut
// into halving pieces (1/2, 1/4, 1/8, 1/8 of it, none below 512 loci) when `halve_tail`, so that
// the device work left after the last byte has landed is a small chunk's GRM rather than a full
// one's. That pays where the upload is copy-bound: fp64 X with n below ≈ 9 000 (PCIe ≈ 57 GB/s
// moves 8np bytes while the GRM does n²p flops at ≈ 65 TF/s; C2: 40.7 -> 39.9 ms). Where the device
// is the bound — int8 dosages (an eighth of the bytes; 25.5 -> 26.4 ms at C2) or large n (C3's
// per-GPU shape: 4.06 -> 4.10 s) — extra chunks only add launches, so by default those keep equal
// chunks. With GBM_HOST_CHUNK set, every entry halves the tail: the same partition, chunk GRMs
// summed in the same order, bit-identical fp64 and int8 results.
static std::vector<std::pair<int64_t, int64_t>> chunk_schedule(int64_t pl, int64_t chunk, bool halve_tail) {
  std::vector<std::pair<int64_t, int64_t>> cs;
  int64_t j = 0;
  while (pl - j > chunk) {
    cs.emplace_back(j, chunk);
    j += chunk;
  }
  int64_t r = pl - j;
  for (int d = 0; halve_tail && d < 3 && r / 2 >= 512; d++) {
    const int64_t h = r / 2;
    cs.emplace_back(j, r - h);
    j += r - h;
    r = h;
  }
  if (r > 0) cs.emplace_back(j, r);
  return cs;
}

// Upload, standardise and GRM of one shard with the PCIe transfer of the genotypes overlapped
// with the device work: chunk k's copy (on the context's copy stream; from pageable memory the
// call itself returns when the copy is done) runs while the compute stream standardises chunk
// k − 1 and adds its loci to G (chunk GRMs summed in chunk order: deterministic). At C2 the
// 2 GB of fp64 X take ~35 ms over PCIe and the GRM ~19 ms: pipelined, the call costs about the
// copy plus the last (small) chunk's GRM instead of their sum.
int upload_grm_pipelined(const Problem& pr, Shard& sh, int64_t chunk) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, npad = npad_of(n), gdim = gdim_of(n), pl = sh.p;
  GBM_HIP_TRY(hipSetDevice(c.dev));
  hipStream_t s = c.stream.s;
  if (!c.copy.s) {
    c.copy.dev = c.dev;
    // high priority: besides the streamed uploads it carries the distributed solve's latency-bound
    // look-ahead (area exchange, the next group's panels and row exchange) beside the trailing update
    int lo = 0, hi = 0;
    GBM_HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    GBM_HIP_TRY(hipStreamCreateWithPriority(&c.copy.s, hipStreamNonBlocking, hi));
  }
  const std::vector<std::pair<int64_t, int64_t>> sched = chunk_schedule(pl, chunk, (pr.src == Source::F64 && n <= 8192) || ::gbm::knob("GBM_HOST_CHUNK") != nullptr);
  const int64_t nch = (int64_t)sched.size();
  while ((int64_t)c.ev.size() < nch) {
    hipEvent_t e;
    GBM_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c.ev.push_back(e);
  }
  GBM_TRY(ensure(c.Xt, c.dev, pl * npad * 8));
  GBM_TRY(ensure(c.mean, c.dev, pl * 8));
  GBM_TRY(ensure(c.sd, c.dev, pl * 8));
  GBM_TRY(ensure(c.keep, c.dev, pl * 4));
  GBM_TRY(ensure(c.q, c.dev, 8));
  GBM_TRY(ensure(c.G, c.dev, gdim * gdim * 8));
  if (pr.src == Source::I8) GBM_TRY(ensure(c.D8, c.dev, pl * n));
  int64_t wsb = 0;  // the loci split (and so the workspace) is planned per chunk size
  for (const auto& jc : sched) wsb = std::max(wsb, gbm_dev_grm_workspace(n, jc.second));
  GBM_TRY(ensure(c.wsg, c.dev, wsb));
  // a second G only for chunks whose GRM cannot be added into G in place (a single loci range)
  for (int64_t k = 1; k < nch; k++)
    if (!grm_can_accumulate(n, sched[k].second)) {
      GBM_TRY(ensure(c.Gc, c.dev, gdim * gdim * 8));
      break;
    }
  GBM_HIP_TRY(hipMemsetAsync(c.q.p, 0, 8, s));
  double* Xt = (double*)c.Xt.p;
  for (int64_t k = 0; k < nch; k++) {
    const int64_t j = sched[k].first, pc = sched[k].second;
    if (pr.src == Source::F64)
      GBM_HIP_TRY(hipMemcpy2DAsync(Xt + j * npad, npad * 8, pr.X + (sh.j0 + j) * pr.ld, pr.ld * 8, n * 8, pc,
                                   hipMemcpyHostToDevice, c.copy.s));
    else
      GBM_HIP_TRY(hipMemcpy2DAsync((int8_t*)c.D8.p + j * n, n, pr.D + (sh.j0 + j) * pr.ld, pr.ld, n, pc,
                                   hipMemcpyHostToDevice, c.copy.s));
    GBM_HIP_TRY(hipEventRecord(c.ev[k], c.copy.s));
    GBM_HIP_TRY(hipStreamWaitEvent(s, c.ev[k], 0));
    if (pr.src == Source::I8) {
      // straight from the dosage bytes (no fp64 copy of X; the kernel writes Z's padding zeros)
      GBM_TRY(launch_standardize_i8((const int8_t*)c.D8.p + j * n, n, pc, n, pr.ploidy, Xt + j * npad, npad,
                                    (double*)c.mean.p + j, (double*)c.sd.p + j, (int32_t*)c.keep.p + j,
                                    (int64_t*)c.q.p, s));
    } else {
      if (npad > n) GBM_HIP_TRY(hipMemset2DAsync(Xt + j * npad + n, npad * 8, 0, (npad - n) * 8, pc, s));
      GBM_TRY(gbm_dev_standardize(Xt + j * npad, npad, pc, n, Xt + j * npad, npad, (double*)c.mean.p + j,
                                  (double*)c.sd.p + j, (int32_t*)c.keep.p + j, (int64_t*)c.q.p, s));
    }
    if (k > 0 && grm_can_accumulate(n, pc)) {
      // G += this chunk's GRM inside its reduce: with slabs G_old + ((P0 + P1) + ...), the sums of
      // G plus a separate chunk G; in the in-order carry (large n) range 0 adds G_old first,
      // ((G_old + P0) + P1) + ..., which agrees with that only to rounding (deterministic either
      // way: the mode is fixed by n and the chunk size)
      GBM_TRY(launch_grm(Xt + j * npad, npad, pc, n, (double*)c.G.p, gdim, c.wsg.p, wsb, s, 1));
    } else {
      GBM_TRY(gbm_dev_grm(Xt + j * npad, npad, pc, n, k == 0 ? (double*)c.G.p : (double*)c.Gc.p, gdim, c.wsg.p, wsb, s));
      if (k > 0) GBM_TRY(launch_add_inplace((double*)c.G.p, (const double*)c.Gc.p, gdim * gdim, s));
    }
  }
  GBM_HIP_TRY(hipMemcpyAsync(&sh.q_host, c.q.p, 8, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  return GBM_OK;
}

// ---- loci-streamed mode --------------------------------------------------------------------------
// A shard whose fp64 locus rows do not fit its device next to G (config C3 on one GPU: 600 000 loci
// x 50 048 individuals x 8 B = 240 GB beside a 20 GB G) is streamed. Its genotypes stay resident as
// int8 dosages (synthetic and int8 sources: 1 B per cell, 30 GB at C3) or stay on the host (fp64
// source), and the loci pass through one reusable fp64 chunk buffer: each chunk is standardised and
// its GRM added into G in place (chunk GRMs summed in chunk order, as the pipelined host upload
// does; same chunk partition => bit-identical G). After the solve the marker effects re-read the
// dosages with z rebuilt in registers (bit-identical to the resident kernels), or re-upload the
// fp64 chunks. Peak HBM: G + dosages + one or two chunk buffers.

int ensure_copy_stream(FitCtx& c) {
  if (!c.copy.s) {
    c.copy.dev = c.dev;
    // high priority: besides the streamed uploads it carries the distributed solve's latency-bound
    // look-ahead (area exchange, the next group's panels and row exchange) beside the trailing update
    int lo = 0, hi = 0;
    GBM_HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    GBM_HIP_TRY(hipStreamCreateWithPriority(&c.copy.s, hipStreamNonBlocking, hi));
  }
  return GBM_OK;
}

int ensure_events(FitCtx& c, int64_t k) {
  while ((int64_t)c.ev.size() < k) {
    hipEvent_t e;
    GBM_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c.ev.push_back(e);
  }
  return GBM_OK;
}

// The streamed shard's chunks: the pipelined upload's schedule rule (halving tail for copy-bound
// fp64 at n <= 8192 or when GBM_HOST_CHUNK is set), so a streamed fit and a pipelined one over the
// same chunk size sum the same chunk GRMs in the same order.
std::vector<std::pair<int64_t, int64_t>> stream_schedule(const Problem& pr, const Shard& sh) {
  return chunk_schedule(sh.p, sh.stream, (pr.src == Source::F64 && pr.n <= 8192) || ::gbm::knob("GBM_HOST_CHUNK") != nullptr);
}

// Decide, per device, whether its shards' fp64 rows fit (resident, the default) or are streamed,
// and the chunk size: GBM_STREAM_CHUNK (re-read per call) forces it (loci per chunk; 0 never
// streams); otherwise a device streams when the resident buffers of its shards exceed its free
// memory (plus what their pooled contexts already hold, minus a margin) even after its idle pooled
// contexts are freed; the chunk is then the largest equal split of the shard whose buffers fit.
int plan_streaming(const Problem& pr, std::vector<std::unique_ptr<Shard>>& shards, bool reml) {
  const int64_t forced = knob_i64("GBM_STREAM_CHUNK", -1);
  const int64_t n = pr.n, npad = npad_of(n), gdim = gdim_of(n);
  const bool bytes = pr.src != Source::F64;
  if (forced >= 0) {
    for (auto& sh : shards) sh->stream = (forced > 0 && forced < sh->p) ? forced : 0;
    return GBM_OK;
  }
  std::map<int, std::vector<Shard*>> bydev;
  for (auto& sh : shards) bydev[sh->x().dev].push_back(sh.get());
  for (auto& dv : bydev) {
    const int dev = dv.first;
    std::vector<Shard*>& v = dv.second;
    GBM_HIP_TRY(hipSetDevice(dev));
    int64_t held = 0, fixed = 0, resident = 0, dosage = 0, pmax = 0;
    for (Shard* sh : v) {
      FitCtx& c = sh->x();
      // D8 counts only where this call's path refills it (int8 or synthetic dosages); an fp64 source never reuses it
      held += c.Xt.cap + (pr.src != Source::F64 ? c.D8.cap : 0) + c.G.cap + c.Gc.cap + c.wsg.cap;
      fixed += gdim * gdim * 8 * (reml ? 2 : 1) + gbm_dev_solve_workspace(n, 63) + sh->p * 40;
      resident += sh->p * npad * 8 + (pr.src == Source::I8 ? sh->p * n : 0) + gbm_dev_grm_workspace(n, sh->p);
      dosage += bytes ? sh->p * n : 0;
      pmax = std::max(pmax, sh->p);
    }
    size_t fr = 0, tot = 0;
    GBM_HIP_TRY(hipMemGetInfo(&fr, &tot));
    const int64_t margin = ((int64_t)1 << 30) + (int64_t)tot / 50;
    if (resident + fixed + margin <= (int64_t)fr + held) continue;
    pool().trim(dev);  // idle pooled contexts of this device hold memory the fit could use
    GBM_HIP_TRY(hipMemGetInfo(&fr, &tot));
    if (resident + fixed + margin <= (int64_t)fr + held) continue;
    const int nbuf = bytes ? 1 : 2;
    int64_t budget = (int64_t)fr + held - fixed - dosage - margin;
    int64_t cmax = budget / ((int64_t)v.size() * nbuf * npad * 8);
    if (cmax >= 16) budget -= (int64_t)v.size() * gbm_dev_grm_workspace(n, std::min(cmax, pmax));  // slabs at small n
    cmax = budget / ((int64_t)v.size() * nbuf * npad * 8);
    if (cmax < 512)
      return fail(GBM_E_OOM, "device " + std::to_string(dev) + ": too little memory for a loci-streamed fit at n = " +
                                 std::to_string(n) + " (need G " + std::to_string(gdim * gdim * 8) + " B plus chunk buffers)");
    for (Shard* sh : v) {
      const int64_t nch = (sh->p + cmax - 1) / cmax;
      const int64_t chunk = round_up((sh->p + nch - 1) / nch, 16);
      sh->stream = chunk < sh->p ? chunk : 0;
    }
  }
  return GBM_OK;
}

// Upload (fp64: into its chunk buffer; int8: into the resident dosages) of chunk k on the copy
// stream, recording ev[k]. An fp64 chunk reuses buffer k % 2 after the work that read chunk k − 2
// (ev[nch + k % 2], recorded on the compute stream) is done.
int stream_upload(const Problem& pr, Shard& sh, const std::vector<std::pair<int64_t, int64_t>>& sched, int64_t k) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, npad = npad_of(n), nch = (int64_t)sched.size();
  const int64_t j = sched[k].first, pc = sched[k].second;
  if (pr.src == Source::F64) {
    if (k >= 2) GBM_HIP_TRY(hipStreamWaitEvent(c.copy.s, c.ev[nch + k % 2], 0));
    double* Zb = (double*)c.Xt.p + (k % 2) * sh.stream * npad;
    GBM_HIP_TRY(hipMemcpy2DAsync(Zb, npad * 8, pr.X + (sh.j0 + j) * pr.ld, pr.ld * 8, n * 8, pc, hipMemcpyHostToDevice,
                                 c.copy.s));
  } else if (pr.src == Source::I8) {
    GBM_HIP_TRY(hipMemcpy2DAsync((int8_t*)c.D8.p + j * n, n, pr.D + (sh.j0 + j) * pr.ld, pr.ld, n, pc,
                                 hipMemcpyHostToDevice, c.copy.s));
  }
  GBM_HIP_TRY(hipEventRecord(c.ev[k], c.copy.s));
  return GBM_OK;
}

// Chunk k's standardised rows in its chunk buffer (mean/sd/keep at the chunk's loci, kept count into
// q); returns the buffer.
int stream_standardize(const Problem& pr, Shard& sh, const std::vector<std::pair<int64_t, int64_t>>& sched, int64_t k,
                       int64_t* q, double** Zb_out) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, npad = npad_of(n);
  const int64_t j = sched[k].first, pc = sched[k].second;
  hipStream_t s = c.stream.s;
  double* Zb = (double*)c.Xt.p + (pr.src == Source::F64 ? (k % 2) * sh.stream * npad : 0);
  if (pr.src != Source::SYNTH) GBM_HIP_TRY(hipStreamWaitEvent(s, c.ev[k], 0));
  if (pr.src == Source::F64) {
    if (npad > n) GBM_HIP_TRY(hipMemset2DAsync(Zb + n, npad * 8, 0, (npad - n) * 8, pc, s));
    GBM_TRY(gbm_dev_standardize(Zb, npad, pc, n, Zb, npad, (double*)c.mean.p + j, (double*)c.sd.p + j,
                                (int32_t*)c.keep.p + j, q, s));
  } else {
    const int ploidy = pr.src == Source::SYNTH ? 2 : pr.ploidy;
    GBM_TRY(launch_standardize_i8((const int8_t*)c.D8.p + j * n, n, pc, n, ploidy, Zb, npad, (double*)c.mean.p + j,
                                  (double*)c.sd.p + j, (int32_t*)c.keep.p + j, q, s));
  }
  *Zb_out = Zb;
  return GBM_OK;
}

// Standardise + GRM of a streamed shard: every chunk's GRM added into G (a chunk planned as a single
// loci range goes through Gc), the copy of chunk k + 1 overlapping chunk k's GRM.
int stream_grm_shard(const Problem& pr, Shard& sh) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, npad = npad_of(n), gdim = gdim_of(n), pl = sh.p;
  GBM_HIP_TRY(hipSetDevice(c.dev));
  hipStream_t s = c.stream.s;
  const auto sched = stream_schedule(pr, sh);
  const int64_t nch = (int64_t)sched.size();
  const bool bytes = pr.src != Source::F64;
  if (pr.src != Source::SYNTH) GBM_TRY(ensure_copy_stream(c));
  GBM_TRY(ensure_events(c, nch + 2));
  GBM_TRY(ensure(c.Xt, c.dev, (bytes ? 1 : 2) * sh.stream * npad * 8));
  GBM_TRY(ensure(c.mean, c.dev, pl * 8));
  GBM_TRY(ensure(c.sd, c.dev, pl * 8));
  GBM_TRY(ensure(c.keep, c.dev, pl * 4));
  GBM_TRY(ensure(c.q, c.dev, 8));
  GBM_TRY(ensure(c.errs, c.dev, nch * 4));
  GBM_TRY(ensure(c.G, c.dev, gdim * gdim * 8));
  if (bytes) GBM_TRY(ensure(c.D8, c.dev, pl * n));
  int64_t wsb = 0;
  for (const auto& jc : sched) wsb = std::max(wsb, gbm_dev_grm_workspace(n, jc.second));
  GBM_TRY(ensure(c.wsg, c.dev, wsb));
  for (int64_t k = 1; k < nch; k++)
    if (!grm_can_accumulate(n, sched[k].second)) {
      GBM_TRY(ensure(c.Gc, c.dev, gdim * gdim * 8));
      break;
    }
  GBM_HIP_TRY(hipMemsetAsync(c.q.p, 0, 8, s));
  GBM_HIP_TRY(hipMemsetAsync(c.errs.p, 0, nch * 4, s));
  if (pr.src == Source::SYNTH)
    GBM_TRY(gbm_dev_synth_dosage_i8((int8_t*)c.D8.p, n, pl, n, pr.seed, sh.j0, s));
  else
    GBM_TRY(stream_upload(pr, sh, sched, 0));
  for (int64_t k = 0; k < nch; k++) {
    const int64_t pc = sched[k].second;
    double* Zb = nullptr;
    GBM_TRY(stream_standardize(pr, sh, sched, k, (int64_t*)c.q.p, &Zb));
    int32_t* err = (int32_t*)c.errs.p + k;
    if (k > 0 && grm_can_accumulate(n, pc)) {
      GBM_TRY(launch_grm(Zb, npad, pc, n, (double*)c.G.p, gdim, c.wsg.p, wsb, s, 1, err));
    } else {
      GBM_TRY(launch_grm(Zb, npad, pc, n, k == 0 ? (double*)c.G.p : (double*)c.Gc.p, gdim, c.wsg.p, wsb, s, 0, err));
      if (k > 0) GBM_TRY(launch_add_inplace((double*)c.G.p, (const double*)c.Gc.p, gdim * gdim, s));
    }
    if (pr.src == Source::F64) GBM_HIP_TRY(hipEventRecord(c.ev[nch + k % 2], s));
    // queued behind chunk k's work (a pageable copy blocks this thread while the device computes)
    if (pr.src != Source::SYNTH && k + 1 < nch) GBM_TRY(stream_upload(pr, sh, sched, k + 1));
  }
  std::vector<int32_t> errs(nch, 0);
  GBM_HIP_TRY(hipMemcpyAsync(errs.data(), c.errs.p, nch * 4, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipMemcpyAsync(&sh.q_host, c.q.p, 8, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  for (int64_t k = 0; k < nch; k++)
    if (errs[k] < 0)
      return fail(GBM_E_HIP, "GRM in-order carry accumulation (streamed chunk " + std::to_string(k) +
                                 "): an inter-workgroup wait timed out (G is invalid)");
  return GBM_OK;
}

// ---- GRM mode of a call (include/gbm.h GBM_GRM_*) -------------------------------------------------------
// The exact-integer GRM (grm_exact.hip) of a dosage shard: the dosages stay resident as
// bytes (uploaded, converted from fp64 X on the device, or generated there), their GRM is computed exactly by
// int8 digit GEMMs, and the marker effects re-read them (stream_effects_shard). No fp64 genotype rows are
// formed. grm_mode exact / auto picks it per call; GBM_GRM (fp64 | exact | auto) only supplies the mode of
// calls that pass GBM_GRM_DEFAULT.
constexpr int kNotDosage = 1;  // internal: the genotypes are not diploid dosages (auto falls back to fp64)

}  // namespace

int resolve_grm_mode(int grm_mode) {
  if (grm_mode != GBM_GRM_DEFAULT && grm_mode != GBM_GRM_DROPIN) return grm_mode;
  const char* e = ::gbm::knob("GBM_GRM");
  if (e && strcmp(e, "exact") == 0) return GBM_GRM_EXACT;
  if (e && strcmp(e, "auto") == 0) return GBM_GRM_AUTO;
  if (e && strcmp(e, "fp64") == 0) return GBM_GRM_FP64;
  return grm_mode == GBM_GRM_DROPIN ? GBM_GRM_AUTO : GBM_GRM_FP64;
}

namespace {

// fp64 host X of a shard → dosage bytes D8 = 2x on the device (chunks of loci through two fp64 staging
// buffers, the upload of chunk k + 1 beside the conversion of chunk k). Returns kNotDosage when some 2x is not
// exactly 0, 1 or 2 — with early_exit (grm_mode auto) already after the first chunk, so data that is not
// dosage-valued costs one chunk's upload before the fp64 path takes over.
int dosage_upload_shard(const Problem& pr, Shard& sh, bool early_exit) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, pl = sh.p;
  GBM_HIP_TRY(hipSetDevice(c.dev));
  hipStream_t s = c.stream.s;
  GBM_TRY(ensure_copy_stream(c));
  const int64_t chunk = std::max<int64_t>(256, std::min<int64_t>((pl + 7) / 8, ((int64_t)1 << 30) / (n * 8)));
  const auto sched = chunk_schedule(pl, std::min(chunk, pl), false);
  const int64_t nch = (int64_t)sched.size();
  GBM_TRY(ensure_events(c, nch + 2));
  GBM_TRY(ensure(c.Xt, c.dev, 2 * std::min(chunk, pl) * n * 8));
  GBM_TRY(ensure(c.D8, c.dev, pl * n));
  GBM_TRY(ensure(c.errs, c.dev, 4));
  GBM_HIP_TRY(hipMemsetAsync(c.errs.p, 0, 4, s));
  int32_t bad = 0;
  for (int64_t k = 0; k < nch; k++) {
    const int64_t j = sched[k].first, pc = sched[k].second;
    double* buf = (double*)c.Xt.p + (k % 2) * std::min(chunk, pl) * n;
    if (k >= 2) GBM_HIP_TRY(hipStreamWaitEvent(c.copy.s, c.ev[nch + k % 2], 0));
    GBM_HIP_TRY(hipMemcpy2DAsync(buf, n * 8, pr.X + (sh.j0 + j) * pr.ld, pr.ld * 8, n * 8, pc, hipMemcpyHostToDevice,
                                 c.copy.s));
    GBM_HIP_TRY(hipEventRecord(c.ev[k], c.copy.s));
    GBM_HIP_TRY(hipStreamWaitEvent(s, c.ev[k], 0));
    GBM_TRY(launch_dosage_from_f64(buf, n, n, pc, (int8_t*)c.D8.p + j * n, n, (int32_t*)c.errs.p, s));
    GBM_HIP_TRY(hipEventRecord(c.ev[nch + k % 2], s));
    if (k == 0 && early_exit && nch > 1) {
      GBM_HIP_TRY(hipMemcpyAsync(&bad, c.errs.p, 4, hipMemcpyDeviceToHost, s));
      GBM_HIP_TRY(hipStreamSynchronize(s));
      if (bad) break;
    }
  }
  GBM_HIP_TRY(hipMemcpyAsync(&bad, c.errs.p, 4, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  GBM_HIP_TRY(hipStreamSynchronize(c.copy.s));  // no upload still writes a staging buffer
  if (bad) return kNotDosage;
  sh.d8_ready = true;
  return GBM_OK;
}

// fp64 host X of a shard → dosage bytes D8 = 2x, packed on the HOST (GBM_HOST_PACK, default 1): `threads` workers
// check and pack chunks of loci (≈ 16 MB of bytes each, GBM_PACK_CHUNK loci for tests) into a ring of pinned
// staging slots (ChunkPacker, hostpack.cpp), and this thread uploads each chunk as soon as it is packed (the copy
// stream); a slot is reused only after its previous chunk's copy has landed. Only n·p bytes cross PCIe (C2: 250 MB
// instead of 2 GB of fp64). Returns kNotDosage as soon as any worker meets a 2x that is not exactly 0, 1 or 2.
int host_pack_upload_shard(const Problem& pr, Shard& sh, int threads) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, pl = sh.p;
  GBM_HIP_TRY(hipSetDevice(c.dev));
  GBM_TRY(ensure_copy_stream(c));
  const int64_t pc = std::max<int64_t>(1, std::min<int64_t>(pl, knob_i64("GBM_PACK_CHUNK", ((int64_t)16 << 20) / n)));
  const auto sched = chunk_schedule(pl, pc, false);
  constexpr int R = 4;
  GBM_TRY(ensure(c.D8, c.dev, pl * n));
  GBM_TRY(ensure_pinned(c.pack, R * pc * n));
  GBM_TRY(ensure_events(c, R));
  int rc = GBM_OK;
  bool bad = false;
  {
    ChunkPacker packer(pr.X + sh.j0 * pr.ld, pr.ld, n, sched, static_cast<int8_t*>(c.pack.p), pc * n, R, threads);
    for (int64_t k = 0; k < (int64_t)sched.size(); k++) {
      const int8_t* src = packer.wait(k);
      if (!src) {
        bad = true;
        break;
      }
      const int64_t j = sched[k].first, cnt = sched[k].second;
      hipError_t e = hipMemcpyAsync((int8_t*)c.D8.p + j * n, src, cnt * n, hipMemcpyHostToDevice, c.copy.s);
      if (e == hipSuccess) e = hipEventRecord(c.ev[k % R], c.copy.s);
      // the previous chunk has landed: its slot (and every earlier one) goes back to the packer
      if (e == hipSuccess && k >= 1) e = hipEventSynchronize(c.ev[(k - 1) % R]);
      if (e != hipSuccess) {
        rc = fail(GBM_E_HIP, std::string("host-pack upload: HIP error '") + hipGetErrorString(e) + "'");
        break;
      }
      packer.release_upto(k);
    }
  }  // (the packer's workers have stopped)
  GBM_HIP_TRY(hipStreamSynchronize(c.copy.s));  // no copy still reads a staging slot
  GBM_TRY(rc);
  if (bad) return kNotDosage;
  sh.d8_ready = true;
  return GBM_OK;
}

// The pipelined fp64 upload + GRM (upload_grm_pipelined) of fp64 host X whose values are dosages/2, through the
// host packer (grm_mode fp64, GBM_HOST_PACK): each pipeline chunk (the fp64 schedule, so the chunk GRMs are summed
// exactly as there) is packed to bytes by the host workers into a pinned slot, uploaded at 1 B per cell and
// standardised straight from the bytes (launch_standardize_i8: the same Z bits as the fp64 standardisation of
// d/2), then its GRM added into G as in the fp64 path. Returns kNotDosage (G untouched by later chunks) when a
// chunk is not dosage-valued: the caller then runs the plain fp64 upload for the shard.
int upload_grm_pipelined_packed(const Problem& pr, Shard& sh, int64_t chunk, int threads) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, npad = npad_of(n), gdim = gdim_of(n), pl = sh.p;
  GBM_HIP_TRY(hipSetDevice(c.dev));
  hipStream_t s = c.stream.s;
  GBM_TRY(ensure_copy_stream(c));
  const auto sched = chunk_schedule(pl, chunk, n <= 8192 || ::gbm::knob("GBM_HOST_CHUNK") != nullptr);
  const int64_t nch = (int64_t)sched.size();
  int64_t pmax = 0;
  for (const auto& jc : sched) pmax = std::max(pmax, jc.second);
  constexpr int R = 3;
  GBM_TRY(ensure_events(c, nch));
  GBM_TRY(ensure(c.Xt, c.dev, pl * npad * 8));
  GBM_TRY(ensure(c.D8, c.dev, pl * n));
  GBM_TRY(ensure(c.mean, c.dev, pl * 8));
  GBM_TRY(ensure(c.sd, c.dev, pl * 8));
  GBM_TRY(ensure(c.keep, c.dev, pl * 4));
  GBM_TRY(ensure(c.q, c.dev, 8));
  GBM_TRY(ensure(c.G, c.dev, gdim * gdim * 8));
  GBM_TRY(ensure_pinned(c.pack, R * pmax * n));
  int64_t wsb = 0;
  for (const auto& jc : sched) wsb = std::max(wsb, gbm_dev_grm_workspace(n, jc.second));
  GBM_TRY(ensure(c.wsg, c.dev, wsb));
  for (int64_t k = 1; k < nch; k++)
    if (!grm_can_accumulate(n, sched[k].second)) {
      GBM_TRY(ensure(c.Gc, c.dev, gdim * gdim * 8));
      break;
    }
  GBM_HIP_TRY(hipMemsetAsync(c.q.p, 0, 8, s));
  double* Xt = (double*)c.Xt.p;
  int rc = GBM_OK;
  bool bad = false;
  {
    ChunkPacker packer(pr.X + sh.j0 * pr.ld, pr.ld, n, sched, static_cast<int8_t*>(c.pack.p), pmax * n, R, threads);
    for (int64_t k = 0; k < nch && rc == GBM_OK; k++) {
      const int8_t* src = packer.wait(k);
      if (!src) {
        bad = true;
        break;
      }
      const int64_t j = sched[k].first, pc = sched[k].second;
      hipError_t e = hipMemcpyAsync((int8_t*)c.D8.p + j * n, src, pc * n, hipMemcpyHostToDevice, c.copy.s);
      if (e == hipSuccess) e = hipEventRecord(c.ev[k], c.copy.s);
      if (e == hipSuccess) e = hipStreamWaitEvent(s, c.ev[k], 0);
      if (e != hipSuccess) {
        rc = fail(GBM_E_HIP, std::string("host-pack upload: HIP error '") + hipGetErrorString(e) + "'");
        break;
      }
      rc = launch_standardize_i8((const int8_t*)c.D8.p + j * n, n, pc, n, 2, Xt + j * npad, npad, (double*)c.mean.p + j,
                                 (double*)c.sd.p + j, (int32_t*)c.keep.p + j, (int64_t*)c.q.p, s);
      if (rc == GBM_OK) {
        if (k > 0 && grm_can_accumulate(n, pc)) {
          rc = launch_grm(Xt + j * npad, npad, pc, n, (double*)c.G.p, gdim, c.wsg.p, wsb, s, 1);
        } else {
          rc = gbm_dev_grm(Xt + j * npad, npad, pc, n, k == 0 ? (double*)c.G.p : (double*)c.Gc.p, gdim, c.wsg.p, wsb, s);
          if (rc == GBM_OK && k > 0) rc = launch_add_inplace((double*)c.G.p, (const double*)c.Gc.p, gdim * gdim, s);
        }
      }
      // the previous chunk's copy has landed: its slot goes back to the packer
      if (rc == GBM_OK && k >= 1) {
        e = hipEventSynchronize(c.ev[k - 1]);
        if (e != hipSuccess) rc = fail(GBM_E_HIP, std::string("host-pack upload: HIP error '") + hipGetErrorString(e) + "'");
      }
      if (rc == GBM_OK) packer.release_upto(k);  // (after a failure no slot is handed back: a copy may still read it)
    }
  }
  GBM_HIP_TRY(hipStreamSynchronize(c.copy.s));
  GBM_TRY(rc);
  if (bad) {
    GBM_HIP_TRY(hipStreamSynchronize(s));  // the chunks already queued are done before the fp64 path reuses G
    return kNotDosage;
  }
  GBM_HIP_TRY(hipMemcpyAsync(&sh.q_host, c.q.p, 8, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  return GBM_OK;
}

// check_bytes (grm_mode auto on int8 input): bytes outside {0, 1, 2} return kNotDosage instead of the
// exact kernels' GBM_E_ARG, so that the call falls back to the fp64 path
int exact_grm_shard(const Problem& pr, Shard& sh, bool check_bytes = false) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, gdim = gdim_of(n), pl = sh.p;
  GBM_HIP_TRY(hipSetDevice(c.dev));
  hipStream_t s = c.stream.s;
  GBM_TRY(ensure(c.D8, c.dev, pl * n));
  GBM_TRY(ensure(c.mean, c.dev, pl * 8));
  GBM_TRY(ensure(c.sd, c.dev, pl * 8));
  GBM_TRY(ensure(c.keep, c.dev, pl * 4));
  GBM_TRY(ensure(c.q, c.dev, 8));
  GBM_TRY(ensure(c.G, c.dev, gdim * gdim * 8));
  const int64_t wsb = gbm_dev_grm_exact_workspace(n, pl);
  GBM_TRY(ensure(c.wsg, c.dev, wsb));
  if (!sh.d8_ready) {
    if (pr.src == Source::SYNTH)
      GBM_TRY(gbm_dev_synth_dosage_i8((int8_t*)c.D8.p, n, pl, n, pr.seed, sh.j0, s));
    else if (pr.src == Source::I8)
      GBM_HIP_TRY(hipMemcpy2DAsync(c.D8.p, n, pr.D + sh.j0 * pr.ld, pr.ld, n, pl, hipMemcpyHostToDevice, s));
    else
      return fail(GBM_E_ARG, "exact GRM: fp64 genotypes not converted to dosages");
  }
  if (check_bytes) {
    int32_t bad = 0;
    GBM_TRY(ensure(c.errs, c.dev, 4));
    GBM_HIP_TRY(hipMemsetAsync(c.errs.p, 0, 4, s));
    GBM_TRY(launch_dosage_check_i8((const int8_t*)c.D8.p, n, n, pl, (int32_t*)c.errs.p, s));
    GBM_HIP_TRY(hipMemcpyAsync(&bad, c.errs.p, 4, hipMemcpyDeviceToHost, s));
    GBM_HIP_TRY(hipStreamSynchronize(s));
    if (bad) return kNotDosage;
  }
  GBM_HIP_TRY(hipMemsetAsync(c.q.p, 0, 8, s));
  GBM_TRY(launch_grm_exact((const int8_t*)c.D8.p, n, pl, n, 2, (double*)c.G.p, gdim, (double*)c.mean.p,
                           (double*)c.sd.p, (int32_t*)c.keep.p, (int64_t*)c.q.p, 0, c.wsg.p, wsb, nullptr, s));
  GBM_HIP_TRY(hipMemcpyAsync(&sh.q_host, c.q.p, 8, hipMemcpyDeviceToHost, s));
  return grm_exact_status(c.wsg.p, n, pl, s);  // syncs the stream
}

// Marker effects of a streamed shard into B (nt x p) and msum: from the resident dosages in one
// pass (z rebuilt in registers), or chunk by chunk from re-uploaded fp64 rows (standardised again:
// the same bits; kept count into a scratch cell).
int stream_effects_shard(const Problem& pr, Shard& sh, int64_t nt, double inv_q) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, npad = npad_of(n), pl = sh.p;
  hipStream_t s = c.stream.s;
  if (pr.src != Source::F64 || sh.exact) {  // resident dosage bytes (an exact shard of fp64 X holds D8 = 2x)
    const int ploidy = pr.src == Source::I8 ? pr.ploidy : 2;
    GBM_TRY(launch_marker_rows_i8((const int8_t*)c.D8.p, n, pl, n, ploidy, (const double*)c.A.p, npad, nt, inv_q,
                                  nullptr, (const double*)c.mean.p, (const double*)c.sd.p, (const int32_t*)c.keep.p,
                                  (double*)c.B.p, pl, s));
  } else {
    const auto sched = stream_schedule(pr, sh);
    const int64_t nch = (int64_t)sched.size();
    GBM_TRY(ensure(c.q2, c.dev, 8));
    GBM_TRY(stream_upload(pr, sh, sched, 0));
    for (int64_t k = 0; k < nch; k++) {
      const int64_t j = sched[k].first, pc = sched[k].second;
      double* Zb = nullptr;
      GBM_TRY(stream_standardize(pr, sh, sched, k, (int64_t*)c.q2.p, &Zb));
      GBM_TRY(launch_marker_rows(Zb, npad, pc, n, (const double*)c.A.p, npad, nt, inv_q, nullptr,
                                 (const double*)c.sd.p + j, (const int32_t*)c.keep.p + j, (double*)c.B.p + j, pl, s));
      GBM_HIP_TRY(hipEventRecord(c.ev[nch + k % 2], s));
      if (k + 1 < nch) GBM_TRY(stream_upload(pr, sh, sched, k + 1));
    }
  }
  return launch_weighted_sum((const double*)c.mean.p, (const double*)c.B.p, pl, pl, nt, (double*)c.msum.p, s);
}

int grm_shard(const Problem& pr, Shard& sh) {
  FitCtx& c = sh.x();
  const int64_t n = pr.n, npad = npad_of(n), gdim = gdim_of(n);
  GBM_HIP_TRY(hipSetDevice(c.dev));
  GBM_TRY(ensure(c.G, c.dev, gdim * gdim * 8));
  const int64_t wsb = gbm_dev_grm_workspace(n, sh.p);
  GBM_TRY(ensure(c.wsg, c.dev, wsb));
  return gbm_dev_grm((const double*)c.Xt.p, npad, sh.p, n, (double*)c.G.p, gdim, c.wsg.p, wsb, c.stream.s);
}

// Runs fn(shard) for every shard at once, one host thread per shard (shard 0 on the calling
// thread): each device (and each shard sharing a device) uploads, standardises and builds its
// partial GRM side by side with the others. A pageable hipMemcpy blocks its calling thread until
// the copy is done, and each shard's final stream sync waits only for its own work, so driving the
// shards from one thread would run them back to back. Every shard's device work is the same as
// when run alone (fixed summation orders), so results do not depend on the interleaving. The
// lowest-numbered failing shard's code and message become the call's (the thread-local error of
// the worker is carried over to the caller).
template <class Fn>
int parallel_shards(std::vector<std::unique_ptr<Shard>>& shards, Fn&& fn) {
  const size_t m = shards.size();
  const char* e = ::gbm::knob("GBM_SHARD_THREADS");  // "0": one shard after the other (A/B, tests)
  if (m == 1 || (e && strcmp(e, "0") == 0)) {
    for (size_t k = 0; k < m; k++) GBM_TRY(fn(k, *shards[k]));
    return GBM_OK;
  }
  std::vector<int> rc(m, GBM_OK);
  std::vector<std::string> msg(m);
  auto run = [&](size_t k) {
    rc[k] = fn(k, *shards[k]);
    if (rc[k] != GBM_OK) msg[k] = g_last_error;
  };
  std::vector<std::thread> th;
  th.reserve(m - 1);
  for (size_t k = 1; k < m; k++) {
    try {
      th.emplace_back(run, k);
    } catch (...) {  // no thread available: run this shard on the calling thread
      run(k);
    }
  }
  run(0);
  for (auto& t : th) t.join();
  // a real error (negative code) of any shard takes priority over an internal status (kNotDosage > 0) of a
  // lower-numbered one: a fall-back must never hide a HIP/RCCL/OOM failure
  for (size_t k = 0; k < m; k++)
    if (rc[k] < 0) return fail(rc[k], msg[k]);
  for (size_t k = 0; k < m; k++)
    if (rc[k] != GBM_OK) return fail(rc[k], msg[k]);
  return GBM_OK;
}

// ---- RCCL communicators, one set per distinct device list, created once ----------------------

// successful RCCL collectives so far (gbm_debug_rccl_calls: tests check that the RCCL path ran)
std::atomic<int64_t> g_rccl_allreduce{0}, g_rccl_allgather{0};

struct CommSet {
  std::vector<ncclComm_t> comms;
  std::mutex mu;  // one collective at a time on a communicator (same op order on every device)
};

int comm_set(const std::vector<int>& devs, CommSet** out) {
  static std::mutex mu;
  static auto* cache = new std::map<std::vector<int>, std::unique_ptr<CommSet>>;  // never destroyed
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache->find(devs);
  if (it == cache->end()) {
    auto cs = std::make_unique<CommSet>();
    cs->comms.resize(devs.size());
    ncclResult_t r = ncclCommInitAll(cs->comms.data(), (int)devs.size(), devs.data());
    if (r != ncclSuccess) return fail(GBM_E_RCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    it = cache->emplace(devs, std::move(cs)).first;
  }
  *out = it->second.get();
  return GBM_OK;
}

// Copy bytes from one context's buffer to another's on dst's stream (same device or peer).
int copy_dd(FitCtx& dst, void* d, const FitCtx& src, const void* s, int64_t bytes, hipStream_t on = nullptr) {
  GBM_HIP_TRY(hipSetDevice(dst.dev));
  if (!on) on = dst.stream.s;
  if (dst.dev == src.dev)
    GBM_HIP_TRY(hipMemcpyAsync(d, s, (size_t)bytes, hipMemcpyDeviceToDevice, on));
  else
    GBM_HIP_TRY(hipMemcpyPeerAsync(d, dst.dev, s, src.dev, (size_t)bytes, on));
  return GBM_OK;
}

// copy = true: the contexts' copy streams (the distributed factorisation's area exchange)
int sync_all(std::vector<std::unique_ptr<Shard>>& shards, const std::vector<int>& which, bool copy = false) {
  for (int k : which) {
    FitCtx& c = shards[k]->x();
    GBM_HIP_TRY(hipSetDevice(c.dev));
    GBM_HIP_TRY(hipStreamSynchronize(copy ? c.copy.s : c.stream.s));
  }
  return GBM_OK;
}

// All-reduce by copies (leaders sharing a device, GBM_SHARD_LEADERS=each): the packed partials
// summed in leader order on the first leader (the order of the same-device sum), then copied back.
int copy_allreduce(std::vector<std::unique_ptr<Shard>>& shards, const std::vector<int>& leaders, int64_t psz) {
  GBM_TRY(sync_all(shards, leaders));
  FitCtx& c0 = shards[leaders[0]]->x();
  GBM_HIP_TRY(hipSetDevice(c0.dev));
  GBM_TRY(ensure(c0.tmp, c0.dev, psz * 8));
  for (size_t k = 1; k < leaders.size(); k++) {
    FitCtx& ck = shards[leaders[k]]->x();
    GBM_TRY(copy_dd(c0, c0.tmp.p, ck, ck.packed.p, psz * 8));
    GBM_TRY(launch_add_inplace((double*)c0.packed.p, (const double*)c0.tmp.p, psz, c0.stream.s));
  }
  GBM_TRY(sync_all(shards, {leaders[0]}));
  for (size_t k = 1; k < leaders.size(); k++) {
    FitCtx& ck = shards[leaders[k]]->x();
    GBM_TRY(copy_dd(ck, ck.packed.p, c0, c0.packed.p, psz * 8));
  }
  return GBM_OK;
}

// GBM_FORCE_RCCL=1 (re-read per call; a test hook): the collectives of a fit run even with one device
// leader — the partial-GRM all-reduce and the Cholesky strip all-gathers (from n >= GBM_DIST_SOLVE_MIN_N)
// execute on a 1-rank RCCL communicator (ncclCommInitAll over the one device) with the real payloads,
// so the RCCL path runs on a one-GPU box. A sum or gather over one rank is the identity: same bits.
bool force_rccl() { return knob_i64("GBM_FORCE_RCCL", 0) != 0; }

// Sum the partial GRMs of all shards into each device leader's G: the upper 128-tiles packed
// contiguously (half the bytes of G's rows); shards on one device added there in shard order,
// then the leaders all-reduced over RCCL (xGMI), then unpacked.
int allreduce_grm(std::vector<std::unique_ptr<Shard>>& shards, int64_t n) {
  const bool force = force_rccl();
  if (shards.size() < 2 && !force) return GBM_OK;
  const int64_t gdim = gdim_of(n), psz = gbm_dev_grm_packed_size(n);
  for (auto& sh : shards) {
    FitCtx& c = sh->x();
    GBM_HIP_TRY(hipSetDevice(c.dev));
    GBM_TRY(ensure(c.packed, c.dev, psz * 8));
    GBM_TRY(gbm_dev_grm_pack((const double*)c.G.p, gdim, n, (double*)c.packed.p, c.stream.s));
  }
  std::vector<int> leaders, devs;
  for (size_t k = 0; k < shards.size(); k++) {
    Shard& sh = *shards[k];
    if (sh.leader == (int)k) {
      leaders.push_back((int)k);
      devs.push_back(sh.x().dev);
      continue;
    }
    FitCtx& lc = shards[sh.leader]->x();
    GBM_HIP_TRY(hipSetDevice(lc.dev));
    GBM_HIP_TRY(hipStreamSynchronize(sh.x().stream.s));
    GBM_TRY(launch_add_inplace((double*)lc.packed.p, (const double*)sh.x().packed.p, psz, lc.stream.s));
  }
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool shared_dev = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
  if (leaders.size() > 1 && shared_dev) {
    GBM_TRY(copy_allreduce(shards, leaders, psz));
  } else if (leaders.size() > 1 || force) {
    CommSet* cs = nullptr;
    GBM_TRY(comm_set(devs, &cs));
    std::lock_guard<std::mutex> lock(cs->mu);
    int rc = GBM_OK;
    ncclResult_t r = ncclGroupStart();
    for (size_t k = 0; k < leaders.size() && r == ncclSuccess; k++) {
      FitCtx& c = shards[leaders[k]]->x();
      r = ncclAllReduce(c.packed.p, c.packed.p, (size_t)psz, ncclDouble, ncclSum, cs->comms[k], c.stream.s);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      rc = fail(GBM_E_RCCL, std::string("ncclAllReduce(partial GRM): ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    else
      g_rccl_allreduce.fetch_add(1);
    for (int k : leaders) {  // complete the collective while holding the communicator
      FitCtx& c = shards[k]->x();
      (void)hipSetDevice(c.dev);
      if (hipStreamSynchronize(c.stream.s) != hipSuccess && rc == GBM_OK) rc = fail(GBM_E_HIP, "stream sync after all-reduce");
    }
    if (rc != GBM_OK) return rc;
  }
  for (int k : leaders) {
    FitCtx& c = shards[k]->x();
    GBM_HIP_TRY(hipSetDevice(c.dev));
    GBM_TRY(gbm_dev_grm_unpack((const double*)c.packed.p, n, (double*)c.G.p, gdim, c.stream.s));
  }
  return GBM_OK;
}

// All-gather of the leaders' strip packs (cnt doubles each) into every leader's `gathered`, in
// leader (= rank) order: RCCL across distinct devices, device copies when leaders share one.
// area = true: the area buffers (astrip -> agathered) on the copy streams.
// on_copy: the strip buffers on the copy streams (the look-ahead's row exchange).
int allgather_strips(std::vector<std::unique_ptr<Shard>>& shards, const std::vector<int>& leaders, CommSet* cs,
                     int64_t cnt, bool area = false, bool on_copy = false) {
  auto src = [&](FitCtx& c) { return area ? c.astrip.p : c.strip.p; };
  auto dst = [&](FitCtx& c) { return (double*)(area ? c.agathered.p : c.gathered.p); };
  const bool cp = area || on_copy;
  if (cs) {
    ncclResult_t r = ncclGroupStart();
    for (size_t k = 0; k < leaders.size() && r == ncclSuccess; k++) {
      FitCtx& c = shards[leaders[k]]->x();
      r = ncclAllGather(src(c), dst(c), (size_t)cnt, ncclDouble, cs->comms[k], cp ? c.copy.s : c.stream.s);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return fail(GBM_E_RCCL, std::string("ncclAllGather(Cholesky strip): ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    g_rccl_allgather.fetch_add(1);
    return GBM_OK;
  }
  GBM_TRY(sync_all(shards, leaders, cp));  // every pack is complete
  for (int d : leaders) {
    FitCtx& cd = shards[d]->x();
    for (size_t r = 0; r < leaders.size(); r++) {
      FitCtx& cr = shards[leaders[r]]->x();
      GBM_TRY(copy_dd(cd, dst(cd) + r * cnt, cr, src(cr), cnt * 8, cp ? cd.copy.s : cd.stream.s));
    }
  }
  return sync_all(shards, leaders, cp);  // no copy still reads a pack the next step overwrites
}

// GBLUP solve of V = G/q + λI factored across the device leaders (each holding the summed G): the
// C-ABI counterpart of gbm.sharded.chol_distributed. Per panel group, the leaders
// all-gather the group's diagonal area (after an earlier distributed group: its columns were updated
// by their owners) and factor its first block, every leader runs the group's panels and row updates
// on its own 128-column tiles (plus the area and the right-hand sides), the group's solved rows are
// all-gathered (each leader then holds them at every column, with their lower copy), and the
// trailing update runs on the leader's own tiles and the right-hand sides. Once the
// trailing matrix is small (GBM_DIST_TAIL_ROWS, default 8192) every remaining row is gathered once
// and the tail and the back substitution run on every leader. Bit-identical to the redundant
// launch-per-panel solve (the same kernels compute every tile from the same operands). Replaces the
// per-device pinv/Cholesky of V (reference src/gwas.jl:472,595) at multi-GPU scale.
int solve_distributed(std::vector<std::unique_ptr<Shard>>& shards, const std::vector<int>& leaders,
                      const std::vector<int>& ldevs, int64_t n, double inv_q, double lambda, int64_t nrhs) {
  const int64_t npad = npad_of(n), gdim = gdim_of(n), nb = npad / kCholNB;
  const int R = (int)leaders.size();
  const int64_t tail_rows = knob_i64("GBM_DIST_TAIL_ROWS", 8192);
  std::vector<int> sorted = ldevs;
  std::sort(sorted.begin(), sorted.end());
  CommSet* cs = nullptr;
  if (std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end()) GBM_TRY(comm_set(ldevs, &cs));
  std::unique_lock<std::mutex> lock;
  if (cs) lock = std::unique_lock<std::mutex>(cs->mu);  // this solve's collectives in one order on every device
  auto each = [&](auto&& fn) -> int {
    for (int r = 0; r < R; r++) {
      FitCtx& c = shards[leaders[r]]->x();
      GBM_HIP_TRY(hipSetDevice(c.dev));
      GBM_TRY(fn(r, c));
    }
    return GBM_OK;
  };
  auto distributable = [&](int64_t kb) {  // (a group reaching the end is the dataflow tail, GBM_CHOL_TAIL_FLOW)
    const int64_t g = gbm_dev_chol_group_size(n, kb);
    return gdim - kCholNB * kb > tail_rows && g >= 2 && g < nb - kb && (kCholNB * kb) % 128 == 0;
  };
  // rows [64 kb, 64 (kb + rows64)) of every leader's own tiles, all-gathered. kRows: final U rows
  // (their lower copy completed too); kRest: the trailing matrix's remaining rows (the tail switch);
  // kArea: the square diagonal area of a group only
  enum { kRows, kRest, kArea };
  // on_copy (kRows only): on the copy streams — the look-ahead's row exchange of the next group, beside the
  // trailing update on the main streams (the strip buffers are then free of main-stream work: the sizes
  // do not grow from group to group, and the tail's kRest exchange comes after a join)
  auto exchange = [&](int64_t kb, int64_t rows64, int what, bool on_copy = false) -> int {
    const int64_t cnt = what == kArea ? gbm_dev_chol_area_doubles(n, kb, rows64, R)
                                      : gbm_dev_chol_strip_doubles(n, kb, rows64, R);
    GBM_TRY(each([&](int r, FitCtx& c) {
      GBM_TRY(ensure(c.strip, c.dev, cnt * 8));
      GBM_TRY(ensure(c.gathered, c.dev, R * cnt * 8));
      const hipStream_t s = on_copy ? c.copy.s : c.stream.s;
      if (what == kArea)
        return gbm_dev_chol_area_pack((const double*)c.G.p, gdim, n, kb, rows64, r, R, (double*)c.strip.p, s);
      return gbm_dev_chol_strip_pack((const double*)c.G.p, gdim, n, kb, rows64, r, R, (double*)c.strip.p, s);
    }));
    GBM_TRY(allgather_strips(shards, leaders, cs, cnt, false, on_copy));
    return each([&](int r, FitCtx& c) {
      const double* gathered = (const double*)c.gathered.p;
      if (what == kRows)
        return gbm_dev_chol_strip_unpack_rows((double*)c.G.p, gdim, n, kb, rows64, r, R, gathered,
                                              on_copy ? c.copy.s : c.stream.s);
      if (what == kArea) {
        GBM_TRY(gbm_dev_chol_area_unpack((double*)c.G.p, gdim, n, kb, rows64, R, gathered, c.stream.s));
      } else {
        GBM_TRY(gbm_dev_chol_strip_unpack((double*)c.G.p, gdim, n, kb, rows64, R, gathered, c.stream.s));
      }
      return gbm_dev_chol_factor_diag((double*)c.G.p, gdim, n, kb, (int32_t*)c.info.p, c.wss.p, c.wss.cap, c.stream.s);
    });
  };
  // V only on the columns each leader reads before an exchange overwrites them, when the factorisation
  // distributes from the first group on
  const bool dist0 = R > 1 && distributable(0);
  GBM_TRY(each([&](int r, FitCtx& c) {
    return gbm_dev_chol_prepare_cols((double*)c.G.p, gdim, n, inv_q, nullptr, lambda, (const double*)c.Y.p, npad,
                                     nrhs, dist0 ? r : 0, dist0 ? R : 1, (int32_t*)c.info.p, c.wss.p, c.wss.cap,
                                     c.stream.s);
  }));
  if (R == 1) {
    // one leader (GBM_FORCE_RCCL): the redundant solve, each distributable group's final rows passed
    // through the 1-rank all-gather between its panels and its trailing update (an identity exchange
    // with the real payload; same bits as gbm_dev_gblup_solve's launch-per-panel path)
    FitCtx& c = shards[leaders[0]]->x();
    for (int64_t kb = 0; kb < nb;) {
      const int64_t g = gbm_dev_chol_group_size(n, kb);
      if (distributable(kb)) {
        GBM_TRY(gbm_dev_chol_group_panels((double*)c.G.p, gdim, n, kb, 0, 1, (int32_t*)c.info.p, c.wss.p, c.wss.cap,
                                          c.stream.s));
        GBM_TRY(exchange(kb, g, kRows));
        GBM_TRY(gbm_dev_chol_group_update((double*)c.G.p, gdim, n, kb, 0, 1, (int32_t*)c.info.p, c.wss.p, c.wss.cap,
                                          c.stream.s));
      } else {
        GBM_TRY(gbm_dev_chol_group((double*)c.G.p, gdim, n, kb, 0, 1, (int32_t*)c.info.p, c.wss.p, c.wss.cap, c.stream.s));
      }
      kb += g;
    }
    GBM_TRY(gbm_dev_chol_finish((double*)c.G.p, gdim, n, (const double*)c.Y.p, npad, nrhs, lambda, (double*)c.A.p,
                                (double*)c.gebv.p, npad, (double*)c.mu.p, (int32_t*)c.info.p, c.wss.p, c.wss.cap,
                                c.stream.s));
    return cs ? sync_all(shards, leaders) : GBM_OK;
  }
  // GBM_DIST_OVERLAP (default 1): the next group's area is updated and all-gathered on the copy streams
  // while the rest of the trailing update runs (same kernels, same tiles: same bits)
  const bool overlap = knob_i64("GBM_DIST_OVERLAP", 1) != 0;
  // GBM_DIST_LOOKAHEAD (with overlap): the next group's rows are updated first, then its panels and row
  // exchange run on the copy streams beside the rest of the trailing update. Default 1 for the device-copy
  // exchanges (the one-GPU rehearsal, tested bit-identical); default 0 over real RCCL (cs != nullptr) until a
  // multi-GPU run has shown the look-ahead's stream/communicator interleaving bit-identical there
  const bool lookahead = overlap && knob_i64("GBM_DIST_LOOKAHEAD", cs ? 0 : 1) != 0;
  if (overlap)
    GBM_TRY(each([&](int, FitCtx& c) -> int {
      GBM_TRY(ensure_copy_stream(c));
      if (!c.ev_area) GBM_HIP_TRY(hipEventCreateWithFlags(&c.ev_area, hipEventDisableTiming));
      if (!c.ev_upd) GBM_HIP_TRY(hipEventCreateWithFlags(&c.ev_upd, hipEventDisableTiming));
      return GBM_OK;
    }));
  auto update = [&](int64_t kb, int64_t lo, int64_t hi) {
    return each([&](int r, FitCtx& c) {
      return gbm_dev_chol_group_update_cols((double*)c.G.p, gdim, n, kb, r, R, lo, hi, (int32_t*)c.info.p, c.wss.p,
                                            c.wss.cap, c.stream.s);
    });
  };
  // the update of the columns [lo, hi) (the next group's area: about one tile column per rank, a few
  // workgroups one K = 64 g tile long) on the copy streams, beside the rest of the update on the main ones
  auto area_update_async = [&](int64_t kb, int64_t lo, int64_t hi) {
    return each([&](int r, FitCtx& c) -> int {
      GBM_HIP_TRY(hipEventRecord(c.ev_upd, c.stream.s));  // after the group's rows arrived
      GBM_HIP_TRY(hipStreamWaitEvent(c.copy.s, c.ev_upd, 0));
      return gbm_dev_chol_group_update_cols((double*)c.G.p, gdim, n, kb, r, R, lo, hi, (int32_t*)c.info.p, c.wss.p,
                                            c.wss.cap, c.copy.s);
    });
  };
  // the area exchange of the group at kb on the copy streams (after area_update_async); ends with ev_area,
  // which the group's panels wait for
  auto area_async = [&](int64_t kb, int64_t g) -> int {
    const int64_t cnt = gbm_dev_chol_area_doubles(n, kb, g, R);  // non-increasing over the groups
    GBM_TRY(each([&](int r, FitCtx& c) -> int {
      GBM_TRY(ensure(c.astrip, c.dev, cnt * 8));
      GBM_TRY(ensure(c.agathered, c.dev, R * cnt * 8));
      return gbm_dev_chol_area_pack((const double*)c.G.p, gdim, n, kb, g, r, R, (double*)c.astrip.p, c.copy.s);
    }));
    GBM_TRY(allgather_strips(shards, leaders, cs, cnt, true));
    return each([&](int, FitCtx& c) -> int {
      GBM_TRY(gbm_dev_chol_area_unpack((double*)c.G.p, gdim, n, kb, g, R, (const double*)c.agathered.p, c.copy.s));
      GBM_TRY(gbm_dev_chol_factor_diag((double*)c.G.p, gdim, n, kb, (int32_t*)c.info.p, c.wss.p, c.wss.cap, c.copy.s));
      GBM_HIP_TRY(hipEventRecord(c.ev_area, c.copy.s));
      return GBM_OK;
    });
  };
  bool dist = R > 1 && distributable(0), stale = false;  // stale: a distributed update skipped other ranks' tiles
  bool area_pending = false;                    // the current group's area is being exchanged (overlap)
  bool ahead = false;                           // (look-ahead) the current group's panels and rows: copy streams
  for (int64_t kb = 0; kb < nb;) {
    const int64_t g = gbm_dev_chol_group_size(n, kb);
    if (!dist) {
      GBM_TRY(each([&](int, FitCtx& c) {
        return gbm_dev_chol_group((double*)c.G.p, gdim, n, kb, 0, 1, (int32_t*)c.info.p, c.wss.p, c.wss.cap, c.stream.s);
      }));
      kb += g;
      continue;
    }
    if (area_pending) {
      GBM_TRY(each([&](int, FitCtx& c) -> int {
        GBM_HIP_TRY(hipStreamWaitEvent(c.stream.s, c.ev_area, 0));
        return GBM_OK;
      }));
      area_pending = false;
    } else if (stale) {
      GBM_TRY(exchange(kb, g, kArea));
    }
    auto panels = [&](int64_t k, bool on_copy) {
      return each([&](int r, FitCtx& c) {
        return gbm_dev_chol_group_panels((double*)c.G.p, gdim, n, k, r, R, (int32_t*)c.info.p, c.wss.p, c.wss.cap,
                                         on_copy ? c.copy.s : c.stream.s);
      });
    };
    if (!ahead) {
      GBM_TRY(panels(kb, false));
      GBM_TRY(exchange(kb, g, kRows));
    }
    ahead = false;
    const int64_t k1 = kb + g;
    const bool next_dist = k1 < nb && distributable(k1);
    if (overlap && next_dist) {
      const int64_t g1 = gbm_dev_chol_group_size(n, k1);
      const int64_t area_hi = kCholNB * (k1 + g1);
      if (lookahead) {
        // on the copy streams: the next group's rows of every kept column (its area among them: one launch),
        // the area exchange, the next group's panels and row exchange — beside the rest of the update on
        // the main streams (the rows from area_hi on: disjoint tiles)
        auto tiles = [&](int64_t r_lo, int64_t r_hi, int64_t c_lo, bool on_copy) {
          return each([&](int r, FitCtx& c) -> int {
            if (on_copy) {
              GBM_HIP_TRY(hipEventRecord(c.ev_upd, c.stream.s));  // after the group's rows arrived
              GBM_HIP_TRY(hipStreamWaitEvent(c.copy.s, c.ev_upd, 0));
            }
            return gbm_dev_chol_group_update_tiles((double*)c.G.p, gdim, n, kb, r, R, r_lo, r_hi, c_lo, gdim,
                                                   (int32_t*)c.info.p, c.wss.p, c.wss.cap,
                                                   on_copy ? c.copy.s : c.stream.s);
          });
        };
        GBM_TRY(tiles(kCholNB * k1, area_hi, kCholNB * k1, true));
        GBM_TRY(area_async(k1, g1));
        GBM_TRY(panels(k1, true));
        GBM_TRY(exchange(k1, g1, kRows, true));
        GBM_TRY(each([&](int, FitCtx& c) -> int {
          GBM_HIP_TRY(hipEventRecord(c.ev_area, c.copy.s));  // the next group waits for all of it
          return GBM_OK;
        }));
        GBM_TRY(tiles(area_hi, gdim, area_hi, false));
        ahead = true;
      } else {
        GBM_TRY(area_update_async(kb, kCholNB * k1, area_hi));  // the next group's area, on the copy streams
        GBM_TRY(update(kb, area_hi, gdim));  // the rest (and the right-hand sides) beside it and its exchange
        GBM_TRY(area_async(k1, g1));
      }
      area_pending = true;
    } else {
      GBM_TRY(update(kb, kCholNB * k1, gdim));
    }
    stale = true;
    kb = k1;
    if (kb >= nb) break;
    dist = next_dist;
    if (!dist) GBM_TRY(exchange(kb, nb - kb, kRest));  // the tail: every remaining row, once
  }
  GBM_TRY(each([&](int, FitCtx& c) {
    return gbm_dev_chol_finish((double*)c.G.p, gdim, n, (const double*)c.Y.p, npad, nrhs, lambda, (double*)c.A.p,
                               (double*)c.gebv.p, npad, (double*)c.mu.p, (int32_t*)c.info.p, c.wss.p, c.wss.cap,
                               c.stream.s);
  }));
  // the solve's collectives complete while this call still holds the communicators (as in
  // allreduce_grm): another call's collectives on the same device set come strictly after
  return cs ? sync_all(shards, leaders) : GBM_OK;
}

// Solve + marker effects for the traits [t0, t0 + nt) of Y at one λ on the summed G of every device
// leader (factored in place), into the caller's output columns of those traits.
int solve_effects(const Problem& pr, std::vector<std::unique_ptr<Shard>>& shards, const std::vector<int>& leaders,
                  const std::vector<int>& ldevs, int64_t q, const double* Y, int64_t ldy, int64_t t0, int64_t nt,
                  double lambda, double* b_hat_out, double* y_pred_out, double* mu_out) {
  const int64_t n = pr.n, p = pr.p, npad = npad_of(n), gdim = gdim_of(n);
  const double inv_q = 1.0 / (double)q;
  // Below GBM_DIST_SOLVE_MIN_N individuals (default 16384, re-read per call; the knob of
  // gbm.sharded.dist_solve_min_n) each device leader solves the (identical) n x n system, all
  // devices at once; from there the leaders factor it together (solve_distributed). Either way a
  // ends up on every leader for the marker back-solve (same-device shards copy it from theirs).
  const bool distributed = (leaders.size() > 1 || force_rccl()) && n >= knob_i64("GBM_DIST_SOLVE_MIN_N", 16384);
  std::vector<int32_t> infos(shards.size(), 0);
  {
    RoctxRange rsolve(distributed ? "gbm: distributed solve" : "gbm: solve");
    for (size_t k = 0; k < shards.size(); k++) {
      Shard& sh = *shards[k];
      FitCtx& c = sh.x();
      GBM_HIP_TRY(hipSetDevice(c.dev));
      hipStream_t s = c.stream.s;
      GBM_TRY(ensure(c.A, c.dev, nt * npad * 8));
      GBM_TRY(ensure(c.B, c.dev, nt * sh.p * 8));
      GBM_TRY(ensure(c.msum, c.dev, nt * 8));
      if (sh.leader != (int)k) continue;
      GBM_TRY(ensure(c.Y, c.dev, nt * npad * 8));
      GBM_TRY(ensure(c.gebv, c.dev, nt * npad * 8));
      GBM_TRY(ensure(c.mu, c.dev, nt * 8));
      GBM_TRY(ensure(c.info, c.dev, 4));
      const int64_t wss = gbm_dev_solve_workspace(n, nt);
      GBM_TRY(ensure(c.wss, c.dev, wss));
      GBM_HIP_TRY(hipMemcpy2DAsync(c.Y.p, npad * 8, Y + t0 * ldy, ldy * 8, n * 8, nt, hipMemcpyHostToDevice, s));
      if (!distributed)
        GBM_TRY(gbm_dev_gblup_solve((double*)c.G.p, gdim, n, inv_q, nullptr, lambda, (const double*)c.Y.p, npad, nt,
                                    (double*)c.A.p, (double*)c.gebv.p, npad, (double*)c.mu.p, (int32_t*)c.info.p,
                                    c.wss.p, wss, s));
    }
    if (distributed) GBM_TRY(solve_distributed(shards, leaders, ldevs, n, inv_q, lambda, nt));
    for (int k : leaders) {
      FitCtx& c = shards[k]->x();
      GBM_HIP_TRY(hipSetDevice(c.dev));
      GBM_HIP_TRY(hipMemcpyAsync(&infos[k], c.info.p, 4, hipMemcpyDeviceToHost, c.stream.s));
    }
    for (int k : leaders) {
      FitCtx& c = shards[k]->x();
      GBM_HIP_TRY(hipSetDevice(c.dev));
      GBM_HIP_TRY(hipStreamSynchronize(c.stream.s));
      const int32_t info = infos[k];
      if (info < 0) return fail(GBM_E_HIP, "solve: a wait between workgroups timed out (dataflow Cholesky or back substitution; the result is invalid)");
      if (info != 0)
        return fail(GBM_E_NOTPD, "G/q + lambda*I is not positive definite (pivot " + std::to_string(info) +
                                     "); check for non-finite genotypes");
    }
  }
  RoctxRange reff("gbm: marker effects + download");
  std::vector<std::vector<double>> msums(shards.size(), std::vector<double>(nt, 0.0));
  std::vector<double> mu(nt, 0.0);
  double* bo = b_hat_out + t0 * (p + 1);
  for (size_t k = 0; k < shards.size(); k++) {
    Shard& sh = *shards[k];
    FitCtx& c = sh.x();
    GBM_HIP_TRY(hipSetDevice(c.dev));
    hipStream_t s = c.stream.s;
    if (sh.leader != (int)k)
      GBM_HIP_TRY(hipMemcpyAsync(c.A.p, shards[sh.leader]->x().A.p, nt * npad * 8, hipMemcpyDeviceToDevice, s));
    if (sh.stream || sh.exact)
      GBM_TRY(stream_effects_shard(pr, sh, nt, inv_q));
    else
      GBM_TRY(gbm_dev_marker_effects((const double*)c.Xt.p, npad, sh.p, n, (const double*)c.A.p, npad, nt, inv_q,
                                     nullptr, (const double*)c.mean.p, (const double*)c.sd.p, (const int32_t*)c.keep.p,
                                     (double*)c.B.p, sh.p, (double*)c.msum.p, s));
    GBM_HIP_TRY(hipMemcpy2DAsync(bo + 1 + sh.j0, (p + 1) * 8, c.B.p, sh.p * 8, sh.p * 8, nt, hipMemcpyDeviceToHost, s));
    GBM_HIP_TRY(hipMemcpyAsync(msums[k].data(), c.msum.p, nt * 8, hipMemcpyDeviceToHost, s));
    if (k == 0) {
      GBM_HIP_TRY(hipMemcpy2DAsync(y_pred_out + t0 * n, n * 8, c.gebv.p, npad * 8, n * 8, nt, hipMemcpyDeviceToHost, s));
      GBM_HIP_TRY(hipMemcpyAsync(mu.data(), c.mu.p, nt * 8, hipMemcpyDeviceToHost, s));
    }
  }
  std::vector<double> msum_total(nt, 0.0);
  for (size_t k = 0; k < shards.size(); k++) {
    GBM_HIP_TRY(hipSetDevice(shards[k]->x().dev));
    GBM_HIP_TRY(hipStreamSynchronize(shards[k]->x().stream.s));
    for (int64_t t = 0; t < nt; t++) msum_total[t] += msums[k][t];  // shard order: deterministic
  }
  for (int64_t t = 0; t < nt; t++) {
    bo[t * (p + 1)] = mu[t] - msum_total[t];
    if (mu_out) mu_out[t0 + t] = mu[t];
  }
  return GBM_OK;
}

// REML outputs of gbm_gblup_fit_reml (per trait; any may be NULL)
struct RemlOut {
  double* lambda;
  double* s2e;
  double* s2u;
};

// REML λ of trait column y on device leader `c`: each evaluation restores the summed G from its
// pristine copy Gc, solves at λ for the standardised y (one right-hand side) and reads the
// loglikreml terms off the bordered factorisation (as gbm_session_reml does on its cached GRM).
int reml_lambda(FitCtx& c, int64_t n, int64_t q, const double* y, RemlResult& res) {
  const int64_t npad = npad_of(n), gdim = gdim_of(n);
  GBM_HIP_TRY(hipSetDevice(c.dev));
  hipStream_t s = c.stream.s;
  const int64_t wss = gbm_dev_solve_workspace(n, 1);
  GBM_TRY(ensure(c.Y, c.dev, npad * 8));
  GBM_TRY(ensure(c.A, c.dev, npad * 8));
  GBM_TRY(ensure(c.gebv, c.dev, npad * 8));
  GBM_TRY(ensure(c.mu, c.dev, 8));
  GBM_TRY(ensure(c.info, c.dev, 4));
  GBM_TRY(ensure(c.wss, c.dev, wss));
  GBM_TRY(ensure(c.tmp, c.dev, 4 * 8));
  const std::vector<double> ys = standardise_y(y, n);
  GBM_HIP_TRY(hipMemsetAsync(c.Y.p, 0, (size_t)(npad * 8), s));
  GBM_HIP_TRY(hipMemcpyAsync(c.Y.p, ys.data(), n * 8, hipMemcpyHostToDevice, s));
  auto eval = [&](double lambda, RemlEval& e) -> int {
    GBM_HIP_TRY(hipMemcpyAsync(c.G.p, c.Gc.p, (size_t)(npad * gdim * 8), hipMemcpyDeviceToDevice, s));
    GBM_TRY(gbm_dev_gblup_solve((double*)c.G.p, gdim, n, 1.0 / (double)q, nullptr, lambda, (const double*)c.Y.p, npad,
                                1, (double*)c.A.p, (double*)c.gebv.p, npad, (double*)c.mu.p, (int32_t*)c.info.p, c.wss.p,
                                wss, s));
    GBM_TRY(gbm_dev_gblup_terms((const double*)c.G.p, gdim, n, 1, c.wss.p, (double*)c.tmp.p, s));
    double t[4];
    int32_t info = 0;
    GBM_HIP_TRY(hipMemcpyAsync(t, c.tmp.p, 4 * 8, hipMemcpyDeviceToHost, s));
    GBM_HIP_TRY(hipMemcpyAsync(&info, c.info.p, 4, hipMemcpyDeviceToHost, s));
    GBM_HIP_TRY(hipStreamSynchronize(s));
    if (info < 0) return fail(GBM_E_HIP, "solve: a wait between workgroups timed out (dataflow Cholesky or back substitution; the result is invalid)");
    if (info != 0) return fail(GBM_E_NOTPD, "REML: G/q + lambda*I is not positive definite (pivot " + std::to_string(info) + ")");
    e = reml_profile(n, lambda, t);
    return GBM_OK;
  };
  return reml_search(eval, res);
}

int run_fit(const Problem& pr, const double* Y, int64_t ldy, int64_t nrhs, double lambda, const int* devices, int ndev,
            double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out, const RemlOut* reml = nullptr,
            int grm_mode = GBM_GRM_DEFAULT, int* grm_used_out = nullptr) {
  const int64_t n = pr.n, p = pr.p;
  if (n < 2) return fail(GBM_E_DATA, "there are less than 2 entries (reference src/prediction.jl:117-123)");
  if (p < 1 || pr.ld < n || !Y || ldy < n || nrhs < 1 || nrhs > 63 || !b_hat_out || !y_pred_out)
    return fail(GBM_E_ARG, "gbm_gblup_fit: bad arguments (need p >= 1, ldx >= n, ldy >= n, 1 <= nrhs <= 63, outputs)");
  if (!reml && (!(lambda > 0.0) || !std::isfinite(lambda)))
    return fail(GBM_E_ARG, "gbm_gblup_fit: lambda must be finite and > 0");
  if (reml && n < 3) return fail(GBM_E_DATA, "REML needs at least 3 entries");
  GBM_TRY(check_y(Y, n, ldy, nrhs));
  const int mode = resolve_grm_mode(grm_mode);
  if (mode != GBM_GRM_FP64 && mode != GBM_GRM_EXACT && mode != GBM_GRM_AUTO)
    return fail(GBM_E_ARG, "grm_mode must be GBM_GRM_DEFAULT, GBM_GRM_FP64, GBM_GRM_EXACT or GBM_GRM_AUTO (GBM_GRM: fp64 | exact | auto)");
  if (mode == GBM_GRM_EXACT && pr.src == Source::I8 && pr.ploidy != 2)
    return fail(GBM_E_ARG, "grm_mode exact: the exact-integer GRM needs diploid dosages (ploidy 2)");
  std::vector<int> devs;
  GBM_TRY(check_devices(devices, ndev, devs));
  const int64_t npad = npad_of(n), gdim = gdim_of(n);
  std::vector<std::unique_ptr<Shard>> shards;
  GBM_TRY(make_shards(devs, p, shards));
  int64_t q = 0;
  int64_t pmax = 0;
  for (auto& sh : shards) pmax = std::max(pmax, sh->p);
  const int64_t chunk = pr.src == Source::SYNTH ? 0 : host_chunk(pmax);
  // exact: every shard's dosages resident as bytes, nothing to stream; auto: the same unless the genotypes
  // turn out not to be diploid dosages (2x outside {0, 1, 2}, int8 ploidy != 2), then the fp64 path
  bool exact = mode != GBM_GRM_FP64 && !(pr.src == Source::I8 && pr.ploidy != 2);
  auto fp64_grm = [&]() -> int {
    GBM_TRY(plan_streaming(pr, shards, reml != nullptr));
    // each shard's GRM is launched behind its own standardisation (a shard without polymorphic
    // loci contributes a zero partial; q == 0 over all shards fails below): streamed when its
    // rows do not fit, else resident (host chunks pipelined with the GRM, or in one piece)
    // fp64 host X with grm_mode fp64: tried as dosages packed on the host first (GBM_HOST_PACK), 1 B per cell over
    // PCIe; X that is not dosage-valued falls back to the fp64 upload at its first non-dosage chunk
    const bool pack = mode == GBM_GRM_FP64 && pr.src == Source::F64 && knob_i64("GBM_HOST_PACK", 1) != 0;
    const int pthreads = std::max(1, host_pack_threads() / (int)shards.size());
    return parallel_shards(shards, [&](size_t, Shard& sh) {
      if (sh.stream) return stream_grm_shard(pr, sh);
      if (chunk > 0) {
        if (pack) {
          const int rc = upload_grm_pipelined_packed(pr, sh, chunk, pthreads);
          if (rc != kNotDosage) return rc;
        }
        return upload_grm_pipelined(pr, sh, chunk);
      }
      return prepare_grm_shard(pr, sh);
    });
  };
  {
    RoctxRange r("gbm: upload + standardise + GRM");
    if (exact) {
      for (auto& sh : shards) sh->exact = true;
      // fp64 host X: packed to dosage bytes on the host (GBM_HOST_PACK=1, default) or converted on the device from
      // uploaded fp64 chunks (0); the host threads are shared among the call's shards
      const bool host_pack = knob_i64("GBM_HOST_PACK", 1) != 0;
      const int pack_threads = std::max(1, host_pack_threads() / (int)shards.size());
      const int rc = parallel_shards(shards, [&](size_t, Shard& sh) {
        if (pr.src == Source::F64) {
          if (host_pack)
            GBM_TRY(host_pack_upload_shard(pr, sh, pack_threads));
          else
            GBM_TRY(dosage_upload_shard(pr, sh, mode == GBM_GRM_AUTO));
        }
        return exact_grm_shard(pr, sh, mode == GBM_GRM_AUTO && pr.src == Source::I8);
      });
      if (rc == kNotDosage && mode == GBM_GRM_EXACT)
        return fail(GBM_E_ARG, "grm_mode exact: the genotypes are not diploid dosages (2x must be exactly 0, 1 or 2 "
                               "in every cell; use grm_mode auto or fp64)");
      // auto: data that is not dosage-valued, and the exact path's own limits (out of memory for the resident
      // bytes and staging, the 128-bit bracket's range: GBM_E_OOM / GBM_E_ARG), fall back to the fp64 path
      const bool fallback = mode == GBM_GRM_AUTO && (rc == kNotDosage || rc == GBM_E_OOM || rc == GBM_E_ARG);
      if (fallback) {
        exact = false;
        for (auto& sh : shards) {
          sh->exact = sh->d8_ready = false;
          // the fp64 path of fp64 genotypes never reads D8: free it, so plan_streaming sees the memory (a
          // dosage source keeps it: its fp64 path refills D8)
          FitCtx& c = sh->x();
          if (pr.src == Source::F64 && c.D8.p) {
            (void)hipSetDevice(c.dev);
            c.D8.reset();
            c.D8.cap = 0;
          }
        }
        set_error("");
      } else {
        GBM_TRY(rc);
      }
    }
    if (!exact) GBM_TRY(fp64_grm());
  }
  if (grm_used_out) *grm_used_out = exact ? GBM_GRM_EXACT : GBM_GRM_FP64;
  for (auto& sh : shards) q += sh->q_host;
  if (q_out) *q_out = q;
  if (q == 0) return fail(GBM_E_DATA, "no polymorphic locus-allele (all standard deviations <= eps, src/gwas.jl:112-115)");
  {
    RoctxRange r("gbm: partial-GRM all-reduce");
    GBM_TRY(allreduce_grm(shards, n));
  }
  std::vector<int> leaders, ldevs;
  for (size_t k = 0; k < shards.size(); k++)
    if (shards[k]->leader == (int)k) {
      leaders.push_back((int)k);
      ldevs.push_back(shards[k]->x().dev);
    }
  if (!reml) return solve_effects(pr, shards, leaders, ldevs, q, Y, ldy, 0, nrhs, lambda, b_hat_out, y_pred_out, mu_out);
  // REML (gbm_gblup_fit_reml): λ per trait chosen on the first leader's summed G, kept pristine in
  // that leader's Gc only (each solve factors G in place; every leader restores its G from it:
  // one extra n x n buffer per call, not per leader — 20 GB per device at C3); then one solve +
  // effects per trait at its λ.
  const int64_t vbytes = npad * gdim * 8;  // rows [0, npad) of G: everything a solve reads of it
  FitCtx& c0 = shards[leaders[0]]->x();
  GBM_HIP_TRY(hipSetDevice(c0.dev));
  GBM_TRY(ensure(c0.Gc, c0.dev, gdim * gdim * 8));
  GBM_HIP_TRY(hipMemcpyAsync(c0.Gc.p, c0.G.p, (size_t)vbytes, hipMemcpyDeviceToDevice, c0.stream.s));
  std::vector<double> lam(nrhs);
  {
    RoctxRange r("gbm: REML lambda");
    for (int64_t t = 0; t < nrhs; t++) {
      RemlResult res;
      GBM_TRY(reml_lambda(shards[leaders[0]]->x(), n, q, Y + t * ldy, res));
      lam[t] = res.lambda;
      if (reml->lambda) reml->lambda[t] = res.lambda;
      if (reml->s2e) reml->s2e[t] = res.s2e;
      if (reml->s2u) reml->s2u[t] = res.s2u;
    }
  }
  GBM_HIP_TRY(hipSetDevice(c0.dev));
  GBM_HIP_TRY(hipStreamSynchronize(c0.stream.s));  // Gc complete before other leaders' streams read it
  for (int64_t t = 0; t < nrhs; t++) {
    for (int k : leaders) {
      FitCtx& c = shards[k]->x();
      GBM_TRY(copy_dd(c, c.G.p, c0, c0.Gc.p, vbytes));
    }
    GBM_TRY(solve_effects(pr, shards, leaders, ldevs, q, Y, ldy, t, 1, lam[t], b_hat_out, y_pred_out, mu_out));
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

extern "C" int64_t gbm_device_allocations(void) { return alloc_counter().load(std::memory_order_relaxed); }

extern "C" int gbm_debug_oom_retries(int64_t* retries, int64_t* contexts_freed) {
  if (retries) *retries = oom_trim().retries.load();
  if (contexts_freed) *contexts_freed = oom_trim().freed.load();
  return GBM_OK;
}

extern "C" int gbm_release_device_cache(void) {
  pool().clear();
  brr_release_cache();
  return GBM_OK;
}

extern "C" int gbm_gblup_fit_ex(const double* X, int64_t n, int64_t p, int64_t ldx, const double* Y, int64_t ldy,
                                int64_t nrhs, double lambda, const int* devices, int ndev, int grm_mode,
                                double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out,
                                int* grm_used_out) {
  RoctxRange r_("gbm_gblup_fit");
  if (!X) return fail(GBM_E_ARG, "gbm_gblup_fit: X is NULL");
  Problem pr{Source::F64, X, nullptr, 1, n, p, ldx};
  return run_fit(pr, Y, ldy, nrhs, lambda, devices, ndev, b_hat_out, y_pred_out, mu_out, q_out, nullptr, grm_mode,
                 grm_used_out);
}

extern "C" int gbm_gblup_fit(const double* X, int64_t n, int64_t p, int64_t ldx, const double* Y, int64_t ldy,
                             int64_t nrhs, double lambda, const int* devices, int ndev, double* b_hat_out,
                             double* y_pred_out, double* mu_out, int64_t* q_out) {
  return gbm_gblup_fit_ex(X, n, p, ldx, Y, ldy, nrhs, lambda, devices, ndev, GBM_GRM_DEFAULT, b_hat_out, y_pred_out,
                          mu_out, q_out, nullptr);
}

extern "C" int gbm_gblup_fit_reml_ex(const double* X, int64_t n, int64_t p, int64_t ldx, const double* Y, int64_t ldy,
                                     int64_t nrhs, const int* devices, int ndev, int grm_mode, double* b_hat_out,
                                     double* y_pred_out, double* mu_out, int64_t* q_out, double* lambda_out,
                                     double* sigma2_e_out, double* sigma2_u_out, int* grm_used_out) {
  RoctxRange r_("gbm_gblup_fit_reml");
  if (!X) return fail(GBM_E_ARG, "gbm_gblup_fit_reml: X is NULL");
  Problem pr{Source::F64, X, nullptr, 1, n, p, ldx};
  const RemlOut ro{lambda_out, sigma2_e_out, sigma2_u_out};
  return run_fit(pr, Y, ldy, nrhs, 0.0, devices, ndev, b_hat_out, y_pred_out, mu_out, q_out, &ro, grm_mode,
                 grm_used_out);
}

extern "C" int gbm_gblup_fit_reml(const double* X, int64_t n, int64_t p, int64_t ldx, const double* Y, int64_t ldy,
                                  int64_t nrhs, const int* devices, int ndev, double* b_hat_out, double* y_pred_out,
                                  double* mu_out, int64_t* q_out, double* lambda_out, double* sigma2_e_out,
                                  double* sigma2_u_out) {
  return gbm_gblup_fit_reml_ex(X, n, p, ldx, Y, ldy, nrhs, devices, ndev, GBM_GRM_DEFAULT, b_hat_out, y_pred_out,
                               mu_out, q_out, lambda_out, sigma2_e_out, sigma2_u_out, nullptr);
}

extern "C" int gbm_gblup_fit_synthetic_ex(uint64_t seed, int64_t n, int64_t p, const double* Y, int64_t ldy,
                                          int64_t nrhs, double lambda, const int* devices, int ndev, int grm_mode,
                                          double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out,
                                          int* grm_used_out) {
  RoctxRange r_("gbm_gblup_fit_synthetic");
  if (n < 1 || p < 1) return fail(GBM_E_ARG, "gbm_gblup_fit_synthetic: bad arguments (n, p >= 1)");
  Problem pr{Source::SYNTH, nullptr, nullptr, 1, n, p, n};
  pr.seed = seed;
  return run_fit(pr, Y, ldy, nrhs, lambda, devices, ndev, b_hat_out, y_pred_out, mu_out, q_out, nullptr, grm_mode,
                 grm_used_out);
}

extern "C" int gbm_gblup_fit_synthetic(uint64_t seed, int64_t n, int64_t p, const double* Y, int64_t ldy, int64_t nrhs,
                                       double lambda, const int* devices, int ndev, double* b_hat_out,
                                       double* y_pred_out, double* mu_out, int64_t* q_out) {
  return gbm_gblup_fit_synthetic_ex(seed, n, p, Y, ldy, nrhs, lambda, devices, ndev, GBM_GRM_DEFAULT, b_hat_out,
                                    y_pred_out, mu_out, q_out, nullptr);
}

extern "C" int gbm_gblup_fit_dosage_i8_ex(const int8_t* D, int64_t n, int64_t p, int64_t ldd, int ploidy,
                                          const double* Y, int64_t ldy, int64_t nrhs, double lambda, const int* devices,
                                          int ndev, int grm_mode, double* b_hat_out, double* y_pred_out,
                                          double* mu_out, int64_t* q_out, int* grm_used_out) {
  RoctxRange r_("gbm_gblup_fit_dosage_i8");
  if (!D || ploidy < 1) return fail(GBM_E_ARG, "gbm_gblup_fit_dosage_i8: D is NULL or ploidy < 1");
  Problem pr{Source::I8, nullptr, D, ploidy, n, p, ldd};
  return run_fit(pr, Y, ldy, nrhs, lambda, devices, ndev, b_hat_out, y_pred_out, mu_out, q_out, nullptr, grm_mode,
                 grm_used_out);
}

extern "C" int gbm_gblup_fit_dosage_i8(const int8_t* D, int64_t n, int64_t p, int64_t ldd, int ploidy, const double* Y,
                                       int64_t ldy, int64_t nrhs, double lambda, const int* devices, int ndev,
                                       double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out) {
  return gbm_gblup_fit_dosage_i8_ex(D, n, p, ldd, ploidy, Y, ldy, nrhs, lambda, devices, ndev, GBM_GRM_DEFAULT,
                                    b_hat_out, y_pred_out, mu_out, q_out, nullptr);
}

extern "C" int gbm_debug_rccl_calls(int64_t* allreduce, int64_t* allgather) {
  if (allreduce) *allreduce = g_rccl_allreduce.load();
  if (allgather) *allgather = g_rccl_allgather.load();
  return GBM_OK;
}

extern "C" int gbm_grm(const double* X, int64_t n, int64_t p, int64_t ldx, const int* devices, int ndev, double* G_out,
                       int64_t ldg, int64_t* q_out) {
  RoctxRange r_("gbm_grm");
  if (!X || !G_out || n < 1 || p < 1 || ldx < n || ldg < n) return fail(GBM_E_ARG, "gbm_grm: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(devices, ndev, devs));
  Problem pr{Source::F64, X, nullptr, 1, n, p, ldx};
  std::vector<std::unique_ptr<Shard>> shards;
  GBM_TRY(make_shards(devs, p, shards));
  int64_t q = 0;
  {
    RoctxRange r("gbm: upload + standardise + GRM");
    GBM_TRY(parallel_shards(shards, [&](size_t, Shard& sh) { return prepare_grm_shard(pr, sh); }));
  }
  for (auto& sh : shards) q += sh->q_host;
  if (q_out) *q_out = q;
  if (q == 0) return fail(GBM_E_DATA, "no polymorphic locus-allele");
  {
    RoctxRange r("gbm: partial-GRM all-reduce");
    GBM_TRY(allreduce_grm(shards, n));
  }
  FitCtx& c = shards[0]->x();
  GBM_HIP_TRY(hipSetDevice(c.dev));
  GBM_TRY(ensure(c.out, c.dev, n * n * 8));
  GBM_TRY(launch_grm_export((const double*)c.G.p, gdim_of(n), n, 1.0 / (double)q, (double*)c.out.p, n, c.stream.s));
  GBM_HIP_TRY(hipMemcpy2DAsync(G_out, ldg * 8, c.out.p, n * 8, n * 8, n, hipMemcpyDeviceToHost, c.stream.s));
  GBM_HIP_TRY(hipStreamSynchronize(c.stream.s));
  return GBM_OK;
}

extern "C" int gbm_grm_ploidy_aware(const double* X, int64_t n, int64_t p, int64_t ldx, int ploidy, const int* devices,
                                    int ndev, double* G_out, int64_t ldg, double* denom_out) {
  RoctxRange r_("gbm_grm_ploidy_aware");
  if (!X || !G_out || n < 1 || p < 1 || ldx < n || ldg < n || ploidy < 1)
    return fail(GBM_E_ARG, "gbm_grm_ploidy_aware: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(devices, ndev, devs));
  Problem pr{Source::F64, X, nullptr, 1, n, p, ldx};
  std::vector<std::unique_ptr<Shard>> shards;
  GBM_TRY(make_shards(devs, p, shards));
  // X_c = X − 1 fᵀ (f_j = column mean = allele frequency); denominator Σ_j f_j (1 − f_j) in locus
  // order over the shards (host, from the device means)
  double den = 0.0;
  {
    RoctxRange r("gbm: upload + centre + GRM");
    std::vector<std::vector<double>> f(shards.size());
    GBM_TRY(parallel_shards(shards, [&](size_t k, Shard& sh) {
      GBM_TRY(prepare_shard(pr, sh, true, false));
      FitCtx& c = sh.x();
      f[k].resize(sh.p);
      GBM_HIP_TRY(hipMemcpyAsync(f[k].data(), c.mean.p, sh.p * 8, hipMemcpyDeviceToHost, c.stream.s));
      GBM_TRY(grm_shard(pr, sh));
      GBM_HIP_TRY(hipStreamSynchronize(c.stream.s));
      return GBM_OK;
    }));
    for (const auto& fk : f)
      for (double v : fk) den += v * (1.0 - v);  // locus order over the shards, as before
  }
  if (denom_out) *denom_out = den;
  if (!(den > 0.0) || !std::isfinite(den)) return fail(GBM_E_DATA, "gbm_grm_ploidy_aware: no polymorphic locus-allele");
  {
    RoctxRange r("gbm: partial-GRM all-reduce");
    GBM_TRY(allreduce_grm(shards, n));
  }
  FitCtx& c = shards[0]->x();
  GBM_HIP_TRY(hipSetDevice(c.dev));
  GBM_TRY(ensure(c.out, c.dev, n * n * 8));
  GBM_TRY(launch_grm_export((const double*)c.G.p, gdim_of(n), n, (double)ploidy / den, (double*)c.out.p, n, c.stream.s));
  GBM_HIP_TRY(hipMemcpy2DAsync(G_out, ldg * 8, c.out.p, n * 8, n * 8, n, hipMemcpyDeviceToHost, c.stream.s));
  GBM_HIP_TRY(hipStreamSynchronize(c.stream.s));
  return GBM_OK;
}

extern "C" int gbm_colstats(const double* X, int64_t n, int64_t p, int64_t ldx, int device, double* mean_out,
                            double* sd_out, uint8_t* keep_out, int64_t* q_out) {
  if (!X || n < 1 || p < 1 || ldx < n) return fail(GBM_E_ARG, "gbm_colstats: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(&device, 1, devs));
  Problem pr{Source::F64, X, nullptr, 1, n, p, ldx};
  std::vector<std::unique_ptr<Shard>> shards;
  GBM_TRY(make_shards(devs, p, shards));
  Shard& sh = *shards[0];
  GBM_TRY(prepare_shard(pr, sh));
  if (q_out) *q_out = sh.q_host;
  FitCtx& c = sh.x();
  hipStream_t s = c.stream.s;
  if (mean_out) GBM_HIP_TRY(hipMemcpyAsync(mean_out, c.mean.p, p * 8, hipMemcpyDeviceToHost, s));
  if (sd_out) GBM_HIP_TRY(hipMemcpyAsync(sd_out, c.sd.p, p * 8, hipMemcpyDeviceToHost, s));
  std::vector<int32_t> k32;
  if (keep_out) {
    k32.resize(p);
    GBM_HIP_TRY(hipMemcpyAsync(k32.data(), c.keep.p, p * 4, hipMemcpyDeviceToHost, s));
  }
  GBM_HIP_TRY(hipStreamSynchronize(s));
  if (keep_out)
    for (int64_t j = 0; j < p; j++) keep_out[j] = (uint8_t)(k32[j] != 0);
  return GBM_OK;
}

extern "C" int gbm_predict(const double* X, int64_t n, int64_t p, int64_t ldx, const double* b_hat, int64_t ldb,
                           int64_t nrhs, int device, double* out, int64_t ldo) {
  RoctxRange r_("gbm_predict");
  if (!X || !b_hat || !out || n < 1 || p < 1 || ldx < n || ldb < p + 1 || nrhs < 1 || ldo < n)
    return fail(GBM_E_ARG, "gbm_predict: bad arguments");
  std::vector<int> devs;
  GBM_TRY(check_devices(&device, 1, devs));
  std::unique_ptr<FitCtx> lease;
  GBM_TRY(pool().acquire(devs[0], lease));
  struct Release {
    std::unique_ptr<FitCtx>& c;
    ~Release() { pool().release(std::move(c)); }
  } release{lease};
  FitCtx& c = *lease;
  GBM_HIP_TRY(hipSetDevice(c.dev));
  hipStream_t s = c.stream.s;
  const int64_t nchunks = predict_chunks(n, p);
  GBM_TRY(ensure(c.Xt, c.dev, p * n * 8));
  GBM_TRY(ensure(c.B, c.dev, nrhs * (p + 1) * 8));
  GBM_TRY(ensure(c.part, c.dev, nchunks * nrhs * n * 8));
  GBM_TRY(ensure(c.out, c.dev, nrhs * n * 8));
  GBM_HIP_TRY(hipMemcpy2DAsync(c.Xt.p, n * 8, X, ldx * 8, n * 8, p, hipMemcpyHostToDevice, s));
  GBM_HIP_TRY(hipMemcpy2DAsync(c.B.p, (p + 1) * 8, b_hat, ldb * 8, (p + 1) * 8, nrhs, hipMemcpyHostToDevice, s));
  GBM_TRY(launch_predict((const double*)c.Xt.p, n, p, n, (const double*)c.B.p, p + 1, nrhs, (double*)c.part.p, nchunks,
                         (double*)c.out.p, n, s));
  GBM_HIP_TRY(hipMemcpy2DAsync(out, ldo * 8, c.out.p, n * 8, n * 8, nrhs, hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  return GBM_OK;
}
