// Dataflow factorisation of the bordered GBLUP matrix in ONE persistent launch (single device,
// n up to a few ten thousand). It replaces, for gbm_dev_gblup_solve, the chain of ~3 launches per
// 64-row panel (panel solve, row update, trailing update) whose latency bounded the C2 solve.
//
// Same factorisation as chol.hip — V = UᵀU on the upper triangle, the R = [1, y…] columns
// bordered so that the forward substitution W = U⁻ᵀR is part of it and the Schur block ends as
// −WᵀW — but LEFT-looking per 64x64 tile (i, j), i <= j, of the nbc x nbc tile grid
// (nbc = gdim / 64; tile column nbc − 1 holds R, tile (nbc − 1, nbc − 1) the Schur block):
//
//   A_ij −= Σ_{k<i} U_kiᵀ U_kj     in MFMA accumulators, step k as soon as U_ki and U_kj are final
//   i == j  : U_ii = chol(A_ii)     (factor_diag_block) → Ld, Dinv (16x16 diagonal inverses)
//   i <  j  : U_ij = U_ii⁻ᵀ A_ij    (block forward substitution, all MFMA) → G upper + the
//                                    transposed lower copy that the back substitution reads
//
// The C tile is read once and written once (the right-looking trailing updates re-read and
// re-write the whole trailing matrix at every panel group, which made them HBM/MALL-bound).
//
// Scheduling (round 3). Workgroup 0 is the chain: it factors the diagonal tiles one after the
// other, solves each right neighbour and applies the next diagonal tile's last update from LDS,
// so the chain pays no hand-off of its own (chol_flow_kernel below). The other workgroups (one per
// CU) take the remaining tiles from one atomic counter in row-major order (a row's right neighbour
// before its diagonal tile); a diagonal or neighbour task hands the chain its accumulated partial.
// A worker waits only for tiles of earlier rows or for the chain's step of its row; the chain's
// step i waits only for the partials of (i, i + 1) and (i + 1, i + 1), which wait only for rows < i
// and are dequeued first in row i: the launch completes with the chain and one resident worker. Waits are bounded (~1 s,
// info = −1, as in chol_device.h). Round 4: workgroup 1 is the ASSISTANT — it applies each right
// neighbour's last k-step (k = i − 1) to the worker's partial, so the chain's input no longer waits
// for a worker's whole epilogue after the chain's own previous step.
//
// Hand-off between workgroups (MI355X: per-XCD L2s are not coherent): every byte another
// workgroup of this launch reads — U tiles in G, Ld, Dinv — is stored write-through (`sc1`
// buffer stores), every storing wave drains (`s_waitcnt vmcnt(0)`), a workgroup barrier, then one
// lane stores the tile's flag (relaxed agent-scope = `sc1`). Consumers poll the flag (one lane per
// wave, relaxed), and read the payload ONLY through `sc1` buffer loads into registers — so no
// agent acquire (an L1 invalidate, ≈1.7 µs) per hand-off. The transposed lower copy and the
// Schur block are read only by later kernels: plain stores.
#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "chol_device.h"

namespace gbm {

namespace {

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef unsigned int u2 __attribute__((ext_vector_type(2)));
constexpr int FT = 64;         // tile edge
constexpr int32_t kPairBit = 0x8000;
constexpr int kTraceRec = 32;  // int64 per trace record (timing tool only)  // dequeue-order entry (i << 16) | j | kPairBit: the tiles (i, j) and (i, j + 1)
constexpr int kSc1 = 16;       // buffer instruction aux bits: sc1 (write-through store / L1-bypassing load)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ dbl2 ld2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(dbl2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, kSc1));
}
__device__ __forceinline__ double ld1(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, 0, kSc1));
}
__device__ __forceinline__ void st2(__amdgpu_buffer_rsrc_t r, uint32_t voff, dbl2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, (int)voff, 0, kSc1);
}
__device__ __forceinline__ void st1(__amdgpu_buffer_rsrc_t r, uint32_t voff, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, (int)voff, 0, kSc1);
}

// chain tuning (compile time; tools/build_flow_variants.sh builds timing variants): the leaf owner
// publishes its row count every GBM_FLOW_POST_EVERY steps — the followers consume four rows at a
// time, and a post per step (an exec-masked LDS store on the pivot chain) made each 16-pivot leaf
// 1.93 instead of 1.58 µs; LDS polls sleep GBM_FLOW_POLL_SLEEP x 64 cycles between reads
#ifndef GBM_FLOW_POST_EVERY
#define GBM_FLOW_POST_EVERY 4
#endif
// the register k-loop's pipeline: stages per 64-deep step (2 = round 4's two halves)
#ifndef GBM_FLOW_STAGES
#define GBM_FLOW_STAGES 8
#endif
#ifndef GBM_FLOW_POLL_SLEEP
#define GBM_FLOW_POLL_SLEEP 4
#endif

// (lds_sync, chol_device.h: a workgroup barrier for LDS data only — __syncthreads also waits for every
// outstanding global load and store of the calling wave, and the write-through stores of a hand-off
// would sit on the chain)

// tile flags (monotonic): kPartial = the accumulated (not yet solved) partial of a right neighbour or
// a diagonal tile, handed on; kAssisted = a right neighbour's partial with its last k-step applied
// by the assistant workgroup (the chain's input); kFinal = the tile's U (or, on the diagonal, Ld +
// Dinv) is stored
constexpr int32_t kPartial = 1, kAssisted = 2, kFinal = 3;
__device__ __forceinline__ bool flag_at_least(const int32_t* f, int32_t v) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= v;
}
__device__ __forceinline__ bool flag_set(const int32_t* f) { return flag_at_least(f, kFinal); }
// one lane: spin until both flags are set; false (info = −1) after ~1 s or when another waiter
// already gave up
__device__ __noinline__ bool poll2(const int32_t* fa, const int32_t* fb, int32_t* info, int32_t v = kFinal) {
  for (int64_t it = 0;; it++) {
    if (flag_at_least(fa, v) && flag_at_least(fb, v)) return true;
    if ((it & 255) == 255) {
      if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0) return false;
      if (it > ((int64_t)1 << 22)) {
        __hip_atomic_store(info, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// every lane of the calling wave: wait (one lane polls) for both flags
__device__ __forceinline__ void wave_wait2(const int32_t* fa, const int32_t* fb, int32_t* info, int lane,
                                           int32_t v = kFinal) {
  int ok = 1;
  if (lane == 0) ok = poll2(fa, fb, info, v) ? 1 : 0;
  (void)__builtin_amdgcn_readfirstlane(ok);
  // payload loads after this point are sc1 loads: nothing to invalidate, only keep the
  // compiler from hoisting them above the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// every lane of the calling wave: wait (one lane polls, bounded as poll2) until *f has every bit of mask
__device__ __noinline__ bool poll_bits(const int32_t* f, int32_t mask, int32_t* info) {
  for (int64_t it = 0;; it++) {
    if ((__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & mask) == mask) return true;
    if ((it & 255) == 255) {
      if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0) return false;
      if (it > ((int64_t)1 << 22)) {
        __hip_atomic_store(info, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ void wave_wait_bits(const int32_t* f, int32_t mask, int32_t* info, int lane) {
  int ok = 1;
  if (lane == 0) ok = poll_bits(f, mask, info) ? 1 : 0;
  (void)__builtin_amdgcn_readfirstlane(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ bool wave_ready2(const int32_t* fa, const int32_t* fb, int lane) {
  int r = 0;
  if (lane == 0) r = (flag_set(fa) && flag_set(fb)) ? 1 : 0;
  return __builtin_amdgcn_readfirstlane(r) != 0;
}

// LDS words the chain's four waves synchronise on inside a factor (monotonic over the steps, so
// nothing is reset between steps)
struct ChainSync {
  int rows;    // 64 * step + the rows of U_ii final in X
  int b12;     // step + 1 once block (1, 2) of the previous step's last update is in X (wave 2)
  int b13;     // step + 1 once block (1, 3) of the previous step's last update is in X (wave 3)
  int pro;     // 3 per step: waves 1-3 have finished reading X2 for that last update
  int x2;      // step + 1 once X2 holds the right neighbour's partial A_i,i+1
  int dl;      // 4 * step + leaves whose inverse is in Dl
  int64_t tt[4];  // trace: leaf ends
  int64_t ts[4];  // trace: own-leaf starts (after following the earlier leaves)
  int64_t th[5];  // trace: X2 fetched, Xn fetched, helper waves 0, 1 and 2 done
  int64_t tw[4];  // trace: wave 1 before its (1, 2) / (1, 3) waits, after them, last group's MFMAs issued, rows read back
};
__device__ __forceinline__ int lds_poll(int* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_post(int* p, int v, int lane) {
  if (lane == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// every lane of the calling wave: spin on an LDS word of this workgroup until it reaches v (bounded: the
// writers never wait on anything outside the workgroup, so the bound only guards a bug). Once any wait of
// the factorisation has given up (info < 0) every later wait returns at once: the run then ends quickly
// over stale tiles and the host reports info < 0, instead of each wait spinning out its own bound.
__device__ __forceinline__ int lds_wait(int* p, int v, int32_t* info, int lane) {
  int s = lds_poll(p);
  for (int it = 0; s < v; it++) {
    __builtin_amdgcn_s_sleep(GBM_FLOW_POLL_SLEEP);  // the spin shares the LDS pipe with the leaf owner
    s = lds_poll(p);
    if ((it & 255) == 255 &&
        __builtin_amdgcn_readfirstlane(__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < 0)
      return v;
    if (it > (1 << 22)) {
      if (lane == 0) atomicCAS(info, 0, -1);
      return v;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // no LDS read of the payload above the poll
  return s;
}

// Wave W (1..3) of the chain before its own leaf: the update of its rows 16W..16W+15 (column blocks
// W..3) by every earlier row of U_ii, accumulated by MFMA in registers four rows at a time as the
// owners publish them (sy->rows), then subtracted from the rows (x, lane = column 16W + lane) once. With prev, the accumulators start
// with the previous step's last update (k = i − 1, from U_i−1,i in X2) of the same blocks; blocks
// (1, 2) and (1, 3) of it are waves 2 and 3's (applied to X first, then sy->b12 / b13), so that
// wave 1, whose rows are needed first, has one block of it instead of three. Four rows per MFMA group: five LDS reads per group
// instead of a broadcast read per row and element (the LDS pipe is shared with the owner).
template <int W>
__device__ __forceinline__ void follow_leaves(double* X, const double* X2, bool prev, ChainSync* sy, int step,
                                              int32_t* info, int lane, double (&x)[16], bool tr) {
  auto tw = [&](int e) {
    if (W == 1 && tr && lane == 0) sy->tw[e] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  constexpr int NB = 4 - W;
  const int fr = lane >> 4, fc = lane & 15;
  const int base = 64 * step;
  d4 acc[NB];
#pragma unroll
  for (int b = 0; b < NB; b++) acc[b] = (d4){0.0, 0.0, 0.0, 0.0};
  if (prev) {
    if (W >= 2) {
      // first, block (1, W) of wave 1's rows (wave 1, whose leaf comes first, keeps only (1, 1))
      // every operand read first (pinned ahead of the MFMAs): read beside each MFMA, the 16 dependent MFMAs
      // paid an LDS round trip each and wave 1 waited ≈ 1 µs for this block (round-5 trace)
      d4 t1 = (d4){0.0, 0.0, 0.0, 0.0};
      double ta[16], tb[16];
#pragma unroll
      for (int ks = 0; ks < 16; ks++) {
        const double* r = X2 + (ks * 4 + fr) * PS;
        ta[ks] = r[16 + fc];
        tb[ks] = r[16 * W + fc];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 16; ks++) t1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ta[ks], tb[ks], t1, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; r++) X[(16 + fr + 4 * r) * PS + 16 * W + fc] -= t1[r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lds_post(W == 2 ? &sy->b12 : &sy->b13, step + 1, lane);
    }
    // (the same for the blocks this wave keeps, eight k-steps of operands at a time)
    constexpr int NK = W == 1 ? 1 : NB;  // blocks of the last update this wave applies
#pragma unroll
    for (int h = 0; h < 2; h++) {
      double pa[8], pb[8][NK];
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const double* r = X2 + ((8 * h + e) * 4 + fr) * PS;
        pa[e] = r[16 * W + fc];
#pragma unroll
        for (int b = 0; b < NK; b++) pb[e][b] = r[16 * (W + b) + fc];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < 8; e++)
#pragma unroll
        for (int b = 0; b < NK; b++) acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[e], pb[e][b], acc[b], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // X2 read
  if (lane == 0) __hip_atomic_fetch_add(&sy->pro, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  // the rows' current values (wave 1: with waves 2 and 3's blocks (1, 2) and (1, 3) of the last update)
  tw(0);
  if (W == 1 && prev) {
    lds_wait(&sy->b12, step + 1, info, lane);
    lds_wait(&sy->b13, step + 1, info, lane);
  }
  tw(1);
  const int cc = 16 * W + (lane < 64 - 16 * W ? lane : 0);
#pragma unroll
  for (int t = 0; t < 16; t++) x[t] = X[(16 * W + t) * PS + cc];
  int seen = 0;
#pragma unroll 1
  for (int g = 0; g < 4 * W; g++) {
    if (seen < 4 * g + 4) seen = lds_wait(&sy->rows, base + 4 * g + 4, info, lane) - base;
    const double* r = X + (4 * g + fr) * PS;
    const double a = r[16 * W + fc];
#pragma unroll
    for (int b = 0; b < NB; b++) acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, r[16 * (W + b) + fc], acc[b], 0, 0, 0);
  }
  tw(2);
  // the accumulated update, transposed to the leaf layout (lane = column) through the rows' place in X
  // (the previous leaf's last four rows applied one by one as rank-1 updates in the leaf layout
  // instead measured slower: hand-over 0.65 -> 0.9-1.4 µs)
#pragma unroll
  for (int b = 0; b < NB; b++)
#pragma unroll
    for (int r = 0; r < 4; r++) X[(16 * W + fr + 4 * r) * PS + 16 * (W + b) + fc] = acc[b][r];
  // (gfx950 does not order a wave's ds_read after its own ds_write)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int t = 0; t < 16; t++) x[t] -= X[(16 * W + t) * PS + cc];
  tw(3);
}

// Block row RB, column block cb of the right neighbour U_i,i+1 = U_ii⁻ᵀ A_i,i+1 (in X2, pitch PS), one
// wave: X2_RB,cb <- (D_RB⁻¹)ᵀ (X2_RB,cb − U[0:16 RB, RB]ᵀ X2[0:16 RB, cb]). All operand reads are issued
// before the first MFMA; the updated block is already in the B-operand layout of the D⁻¹ product
// (lane (fr, fc) holds rows fr + 4r = the k-step r operand), so it needs no LDS round trip.
// emit(row, v): the final value of row `row` (0..63), column 16 cb + (lane & 15).
template <int RB, typename Emit>
__device__ __forceinline__ void nbr_block(double* X2, const double* Xa, const double* Dl, int cb, int lane,
                                          Emit&& emit) {
  const int fr = lane >> 4, fc = lane & 15;
  constexpr int KS = RB > 0 ? 4 * RB : 1;
  double a[KS], b[KS], c[4];
#pragma unroll
  for (int r = 0; r < 4; r++) c[r] = X2[(16 * RB + fr + 4 * r) * PS + 16 * cb + fc];
  if (RB > 0) {
#pragma unroll
    for (int ks = 0; ks < 4 * RB; ks++) {
      a[ks] = Xa[(ks * 4 + fr) * PS + 16 * RB + fc];
      b[ks] = X2[(ks * 4 + fr) * PS + 16 * cb + fc];
    }
    d4 sacc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 4 * RB; ks++) sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], b[ks], sacc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; r++) c[r] -= sacc[r];
  }
  d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 4; ks++)
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Dl[RB * 256 + (ks * 4 + fr) * 16 + fc], c[ks], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int row = 16 * RB + fr + 4 * r;
    X2[row * PS + 16 * cb + fc] = acc[r];
    emit(row, acc[r]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Upper Cholesky of the 64x64 block in X (LDS, pitch PS) by the chain's 256 threads, with the inverses
// of its four 16x16 diagonal blocks. Wave w owns leaf w (rows 16w..16w+15). While the earlier leaves
// are factored it FOLLOWS them (follow_leaves: their final rows applied to its rows by MFMA, four at a
// time, as the owners publish them), so when its own leaf begins its rows are up to date — no
// workgroup barrier and no separate leaf update between leaves. The owner's 16-step loop (lane l =
// column 16w + l): the pivot chain (readlane → rsqrt + Newton → scale) with rows c + 1, c + 2 updated
// from v_readlane of U[c][c+1..c+2] and the rows beyond from the LDS row written the step before,
// applied two steps behind; lanes 0..15 carry identity columns through the same eliminations, so
// column l of U_leaf⁻ᵀ (= row l of U_leaf⁻¹, the Dinv layout) comes out beside the factor. Each
// final row goes to X as soon as it is computed, and the row count to sy->rows one step later.
// prev: the step's last update k = i − 1 of rows 16.. (from U_i−1,i in X2) is still to be applied
// (row block 0 was, at the end of the previous step); the followers fold it into their accumulators.
// Each owner stores its leaf's rows to Ld (rLd, write-through) and its Dinv block, then sets bit w
// of leaf_bits; after_own(w) runs on wave w once its leaf is done. Returns the first failing column
// or −1.
template <typename AfterOwn>
__device__ __forceinline__ int factor_block_pipe(double* X, const double* X2, bool prev, double* Dl, int tid,
                                                 __amdgpu_buffer_rsrc_t rDi, uint32_t dinv_base,
                                                 __amdgpu_buffer_rsrc_t rLd, int64_t i0, ChainSync* sy, int step,
                                                 int32_t* info, int32_t* leaf_bits, AfterOwn&& after_own, bool tr = false) {
  const int lane = tid & 63, w = tid >> 6;
  const int o = 16 * w, base = 64 * step;
  const int ncols = CNB - o;
  const int cc = o + (lane < ncols ? lane : 0);
  // row writes: lanes beyond the block go to the pitch padding (never read), so the store needs no
  // exec mask; nothing reads X below the diagonal of a factored block, so no zeros are written there
  const int cw = lane < ncols ? o + lane : CNB + (lane & 15);
  double x[16], y[16];
  if (w == 1) follow_leaves<1>(X, X2, prev, sy, step, info, lane, x, tr);
  else if (w == 2) follow_leaves<2>(X, X2, prev, sy, step, info, lane, x, tr);
  else if (w == 3) follow_leaves<3>(X, X2, prev, sy, step, info, lane, x, tr);
  else {
#pragma unroll
    for (int t = 0; t < 16; t++) x[t] = X[(o + t) * PS + cc];
  }
  // ---- own leaf w
  if (lane == 0) sy->ts[w] = (int64_t)__builtin_amdgcn_s_memrealtime();
  double b1[16], b2[16];
#pragma unroll
  for (int t = 0; t < 16; t++) {
    y[t] = t == lane ? 1.0 : 0.0;
    b1[t] = 0.0;
    b2[t] = 0.0;
  }
  double l1 = 0.0, m1 = 0.0, l2 = 0.0, m2 = 0.0;  // multipliers of steps c − 1 and c − 2
#pragma unroll
  for (int c = 0; c < 16; c++) {
    // chain: pivot -> multipliers -> rows c + 1 and c + 2 (from v_readlane of U[c][c+1..c+2])
    const double r = rsqrt_nr(readlane_d(x[c], c));  // a non-positive pivot propagates NaN
    const double lc = x[c] * r, yc = y[c] * r;
    x[c] = lc;
    y[c] = yc;
#pragma unroll
    for (int d = 1; d <= 2; d++)
      if (c + d < 16) {
        const double u = readlane_d(lc, c + d);  // U[o + c][o + c + d]
        x[c + d] = fma(-lc, u, x[c + d]);
#ifndef GBM_FLOW_TIMING_NOY
        y[c + d] = fma(-yc, u, y[c + d]);
#endif
      }
    __builtin_amdgcn_sched_barrier(0);
    // row c − 1 (written last step) is in X: publish it to the followers, read U[c − 1][·] -> b1;
    // this step's final row -> X
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    if (c >= 1 && c % GBM_FLOW_POST_EVERY == 0) lds_post(&sy->rows, base + o + c, lane);
    X[(o + c) * PS + cw] = lc;
    if (c >= 1 && c + 2 < 16) {
#pragma unroll
      for (int t = c + 2; t < 16; t++) b1[t] = X[(o + c - 1) * PS + o + t];
    }
    // step c − 2's updates of rows c + 1.. (rows c − 1 and c were its chain part)
    if (c >= 2) {
#pragma unroll
      for (int t = c + 1; t < 16; t++) {
        x[t] = fma(-l2, b2[t], x[t]);
#ifndef GBM_FLOW_TIMING_NOY  // (timing variant: the identity columns' eliminations left out; Dinv wrong)
        y[t] = fma(-m2, b2[t], y[t]);
#endif
      }
    }
    // y[c] is final here: pinned, so that LLVM cannot sink the identity columns' eliminations out of
    // the loop (it did: a serial chain of ~200 dependent fp64 ops after every leaf)
    asm volatile("" : "+v"(y[c]));
    __builtin_amdgcn_sched_barrier(0);
    l2 = l1;
    m2 = m1;
    l1 = lc;
    m1 = yc;
#pragma unroll
    for (int t = 0; t < 16; t++) b2[t] = b1[t];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_post(&sy->rows, base + o + 16, lane);  // the next leaf's owner goes on from here
  if (lane == 0) sy->tt[w] = (int64_t)__builtin_amdgcn_s_memrealtime();
  // ---- off the chain: this leaf's rows -> Ld, its inverse -> Dl and Dinv (write-through)
  if (lane < ncols) {
#pragma unroll
    for (int t = 0; t < 16; t++) st1(rLd, (uint32_t)(((i0 + o + t) * CNB + cc) * 8), (lane < 16 && t > lane) ? 0.0 : x[t]);
  }
  if (lane < 16) {
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      dbl2 v;
      v.x = y[e];
      v.y = y[e + 1];
      *reinterpret_cast<dbl2*>(&Dl[w * 256 + lane * 16 + e]) = v;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (w > 0) lds_wait(&sy->dl, 4 * step + w, info, lane);  // keep sy->dl in leaf order
  lds_post(&sy->dl, 4 * step + w + 1, lane);
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int e = (q * 64 + lane) * 2;
    st2(rDi, dinv_base + (uint32_t)((w * 256 + e) * 8), *reinterpret_cast<const dbl2*>(&Dl[w * 256 + e]));
  }
  // workers solving this row's tiles go on leaf by leaf: one bit per leaf once its Ld rows and Dinv
  // block are stored (drained write-through stores, then a relaxed agent-scope atomic)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_or(leaf_bits, 1 << w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  after_own(w);
  lds_sync();
  const double dg = X[lane * PS + lane];
  const unsigned long long bm = __ballot(!(dg > 0.0) || !isfinite(dg));
  return bm ? (int)__builtin_ctzll(bm) : -1;
}

// The workers' dequeue order (a table t -> (i, j) built on the host, flow_order below): row-major over the
// upper tile triangle, except that the tiles the chain's step i waits for come early —
//  - the right neighbour (r, r + 1) of row r >= 2 is dequeued in row r − 2, right after (r − 2, r + 1) (round 4):
//    its k-loop stops at k = r − 2 (the assistant adds k = r − 1), so everything it waits for comes before it;
//  - the diagonal partial (d, d) of row d >= 2 is dequeued in row d − 2, right after (d − 2, d), its last
//    operand (round 5; round 4 dequeued it in row d − 1): its k-loop (k < d − 1, d − 1 steps of ≈ 2.4 µs on
//    one workgroup) then starts a chain step earlier — in the middle third of the C2 factorisation it used to
//    reach the chain's LDS 5–10 µs after the step needed it (profiles/r05_chol_flow_per_step.txt);
//  - row 0 starts with (0, 1) and (1, 1); the Schur block (nb, nb) is last. A_00 needs no task.
// Every task follows all the tasks it waits for, and the chain's step i waits only for tasks of rows < i, so the
// launch completes with the chain, the assistant and ONE resident worker (flow_order_check on the host).

// kTrace: per-task timestamps (s_memrealtime, 100 MHz) into trace[t * kTraceRec ...] for the timeline tool;
// the chain workgroup's steps at trace[(ntasks + i) * kTraceRec ...]
//
// Workgroup 0 is the CHAIN: it factors every diagonal tile in turn and keeps the chain's data in LDS.
// Step i: U_ii = chol(A_ii) with its 16x16 inverses (Ld, Dinv); meanwhile its idle waves fetch the
// right neighbour's partial A_i,i+1 (all updates k < i) and the next diagonal tile's partial
// A_i+1,i+1 (all updates k < i); U_i,i+1 = U_ii⁻ᵀ A_i,i+1 (all MFMA, in LDS), stored and published
// with (i, i); then the next diagonal tile's last update A_i+1,i+1 −= U_i,i+1ᵀ U_i,i+1 straight
// from LDS — so the chain never waits for its own hand-off. The other workgroups take tasks from
// the queue (row-major; row i's right neighbour and row i + 1's diagonal tile first, task_tile):
//   diagonal (i == j < nb, i >= 1): k-loop over k < i − 1, stored as a partial for the chain;
//   right neighbour (j == i + 1): k-loop over k < i − 1 (k < i for i = 0), stored as a partial for
//   the assistant (workgroup 1), which adds the last k-step and hands it to the chain;
//   other (j > i + 1): k-loop; once (i, i) is final, U_ij = U_ii⁻ᵀ A_ij;
//   Schur (i == j == nb): k-loop; −WᵀW for the later kernels.
// Deadlock freedom: the chain's step i waits only for the assisted partial of (i, i + 1) and the
// partial of (i + 1, i + 1). The assistant's step i waits for the partial of (i, i + 1), the tile
// (i − 1, i + 1) of the previous row and the chain's step i − 1; the partials wait only for tiles of
// rows < i and are dequeued before every other tile of row i; every worker wait targets the chain's
// earlier steps or a task dequeued earlier. So the launch completes with the chain, the assistant
// and ONE resident worker.
template <bool kTrace>
__global__ void __launch_bounds__(256, 1)
chol_flow_kernel(double* __restrict__ G, int64_t ld, int nbc, double* __restrict__ Ld, double* __restrict__ Dinv,
                 int32_t* __restrict__ queue, int32_t* __restrict__ flags, int32_t* __restrict__ info,
                 const int32_t* __restrict__ order, int nwork, int xn_defer, int64_t* __restrict__ trace,
                 int trace_roles) {
  // ≈ 130 KB: one workgroup per CU (the chain's serial steps then share no SIMD with other tiles)
  __shared__ __attribute__((aligned(16))) double X[FT * PS];
  __shared__ __attribute__((aligned(16))) double X2[FT * PS];
  __shared__ __attribute__((aligned(16))) double X3[FT * PS];
  __shared__ __attribute__((aligned(16))) double Dl[4 * 256];
  __shared__ ChainSync sy;
  __shared__ int s_task;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int fr = lane >> 4, fc = lane & 15;
  const int nb = nbc - 1;  // diagonal tiles with a factor; tile (nb, nb) is the Schur block
  const int ntasks = nbc * (nbc + 1) / 2;  // trace records (one more than the tasks: A_00 has none)
  const int64_t gbytes_rowblk = (int64_t)FT * ld * 8;
  const __amdgpu_buffer_rsrc_t rLd = rsrc(Ld, (int64_t)nb * FT * CNB * 8);
  const __amdgpu_buffer_rsrc_t rDi = rsrc(Dinv, (int64_t)nb * FT * 16 * 8);

  // a solved tile's transposed copy -> G lower (rows j0.., columns i0..; read only by the back
  // substitution / μ̂ kernels after this launch, so stored after the tile's flag)
  // (wave = quarter, lane = row: a wave's LDS reads walk one source row, conflict-free; with four lanes per row and
  // the quarters in the same 32-lane half, the four quarters' rows 16 apart hit the same banks: 4-way)
  auto store_lower = [&](const double* Xs, int64_t i0, int64_t j0) {
    const int row = tid & 63, quarter = tid >> 6;
    double* dl = G + (j0 + row) * ld + i0 + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      dbl2 v;
      v.x = Xs[(quarter * 16 + e) * PS + row];
      v.y = Xs[(quarter * 16 + e + 1) * PS + row];
      *reinterpret_cast<dbl2*>(dl + e) = v;
    }
  };

  if (blockIdx.x == 0) {
    // ================================ the chain ================================
    if (tid == 0) {
      sy.rows = sy.b12 = sy.b13 = sy.pro = sy.x2 = sy.dl = 0;
    }
    // A_00 has no update: straight from G (written before this launch)
    for (int e = tid; e < FT * FT / 2; e += 256) {
      const int r = e >> 5, c2 = (e & 31) * 2;
      *reinterpret_cast<dbl2*>(&X[r * PS + c2]) = *reinterpret_cast<const dbl2*>(G + (int64_t)r * ld + c2);
    }
    lds_sync();
    double* Xa = X;   // A_ii, then U_ii
    double* Xn = X3;  // the next diagonal tile
    for (int i = 0; i < nb; i++) {
      const int64_t i0 = (int64_t)i * FT, j0 = i0 + FT;
      const bool next_diag = i + 1 < nb;
      // trace: 0 start, 1-4 leaf ends, 5-7 own starts of leaves 1-3, 8 factored, 9 X2 fetched,
      // 10 neighbour solved and published, 11 next tile updated, 12 step end, 13 own start of leaf 0,
      // 14 Xn fetched, 15 helpers done
      // trace: one lane stores each timestamp as it is taken (holding them in registers until the step's
      // end raised the traced kernel's register pressure past what it could run with)
      int64_t* const crec = kTrace && (trace_roles & 1) ? trace + (int64_t)(ntasks + i) * kTraceRec : nullptr;
      auto cstamp = [&](int e, int64_t v) {
        if (kTrace && crec && tid == 0) crec[3 + e] = v;
      };
      cstamp(0, (int64_t)__builtin_amdgcn_s_memrealtime());
      __builtin_amdgcn_s_setprio(2);
      // one wave: a partial tile of G (rows r0.., columns j0..; another workgroup's sc1 stores, seen
      // through its flag) -> dst in LDS, all 32 pieces of 16 bytes per lane in flight at once; the LDS
      // writes only after `gate` (the previous contents are no longer read)
      auto fetch_tile = [&](double* dst, int64_t r0, const int32_t* f, int32_t ready, auto&& gate) {
        const __amdgpu_buffer_rsrc_t rG = rsrc(G + r0 * ld, gbytes_rowblk);
        wave_wait2(f, f, info, lane, ready);
        dbl2 v[32];
#pragma unroll
        for (int q = 0; q < 32; q++) {
          const int e = lane + q * 64;
          v[q] = ld2(rG, (uint32_t)(((int64_t)(e >> 5) * ld + j0 + 2 * (e & 31)) * 8), 0);
        }
        gate();
#pragma unroll
        for (int q = 0; q < 32; q++) {
          const int e = lane + q * 64;
          *reinterpret_cast<dbl2*>(&dst[(e >> 5) * PS + 2 * (e & 31)]) = v[q];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      };
      // the neighbour's blocks, stored write-through to G as soon as they are final
      const __amdgpu_buffer_rsrc_t rN = rsrc(G + i0 * ld, gbytes_rowblk);
      auto nbr_item = [&](int rb, int cb) {
        auto emit = [&](int row, double v) { st1(rN, (uint32_t)(((int64_t)row * ld + j0 + 16 * cb + fc) * 8), v); };
        if (rb == 0) nbr_block<0>(X2, Xa, Dl, cb, lane, emit);
        else if (rb == 1) nbr_block<1>(X2, Xa, Dl, cb, lane, emit);
        else if (rb == 2) nbr_block<2>(X2, Xa, Dl, cb, lane, emit);
        else nbr_block<3>(X2, Xa, Dl, cb, lane, emit);
      };
      // wave w once leaf w is factored (beside the later leaves):
      //   wave 0: the previous step's transposed copy of U_i−1,i (X2) below the diagonal of G (read
      //   only by later kernels), then the neighbour's partial A_i,i+1 -> X2 (once waves 1-3 have read
      //   X2 for this step's last update);
      //   wave 1: the next diagonal tile's partial A_i+1,i+1 -> Xn (needed at the step's end);
      //   waves 0-2: the neighbour solve's block rows 0-2, column block by column block (block row rb
      //   once leaf rb is factored).
      auto after_own = [&](int w) {
        if (w == 0) {
          if (i > 0) {
            // 64 rows x 8 pieces of 8 doubles, lane = row (conflict-free LDS reads: the former 8 pieces per row in
            // one 32-lane half read rows 8 apart, the same banks: 8-way)
            for (int piece = 0; piece < 8; piece++) {
              const int row = lane;
              double* dl = G + (i0 + row) * ld + (i0 - FT) + piece * 8;
#pragma unroll
              for (int u = 0; u < 8; u += 2) {
                dbl2 v;
                v.x = X2[(piece * 8 + u) * PS + row];
                v.y = X2[(piece * 8 + u + 1) * PS + row];
                *reinterpret_cast<dbl2*>(dl + u) = v;
              }
            }
          }
          fetch_tile(X2, i0, flags + (int64_t)i * nbc + i + 1, i > 0 ? kAssisted : kPartial,
                     [&]() { lds_wait(&sy.pro, 3 * (i + 1), info, lane); });
          lds_post(&sy.x2, i + 1, lane);
          if (kTrace && lane == 0) sy.th[0] = (int64_t)__builtin_amdgcn_s_memrealtime();
        }
        // wave 1 fetches the next diagonal partial (needed at the step's end) now if it is there, else after
        // its neighbour items, so that a late partial does not hold up the neighbour solve
        const int32_t* fxn = flags + (int64_t)(i + 1) * nbc + i + 1;
        bool xn_late = false;
        if (w == 1 && next_diag) {
          int rdy = 0;
          if (lane == 0) rdy = flag_at_least(fxn, kPartial) ? 1 : 0;
          xn_late = xn_defer && __builtin_amdgcn_readfirstlane(rdy) == 0;
          if (!xn_late) {
            fetch_tile(Xn, j0, fxn, kPartial, []() {});
            if (kTrace && lane == 0) sy.th[1] = (int64_t)__builtin_amdgcn_s_memrealtime();
          }
        }
        if (w <= 2) {
          // column blocks: wave 0 takes 0 and 3, waves 1 and 2 their own; a column's block rows run in
          // order on one wave, so only the leaf (sy.dl) and X2 (sy.x2) are waited for. (Round 4: moving
          // column block 3's rows to the wave of the same index balanced the items but was not faster:
          // wave 2, whose own leaf ends last, then finished last.)
#pragma unroll 1
          for (int rb = 0; rb < 3; rb++) {
            lds_wait(&sy.x2, i + 1, info, lane);
            lds_wait(&sy.dl, 4 * i + rb + 1, info, lane);
            nbr_item(rb, w);
            if (w == 0) nbr_item(rb, 3);
          }
          if (kTrace && lane == 0) sy.th[2 + w] = (int64_t)__builtin_amdgcn_s_memrealtime();
        }
        if (xn_late) {
          fetch_tile(Xn, j0, fxn, kPartial, []() {});
          if (kTrace && lane == 0) sy.th[1] = (int64_t)__builtin_amdgcn_s_memrealtime();
        }
      };
      // ---- U_ii = chol(A_ii) -> Ld, its 16x16 diagonal inverses -> Dinv (and Dl)
      const int bad = factor_block_pipe(Xa, X2, i > 0, Dl, tid, rDi, (uint32_t)((i0 / 16) * 256 * 8), rLd, i0, &sy, i,
                                        info, flags + (int64_t)(i + 1) * nbc + i, after_own, kTrace && crec);
      if (tid == 0 && bad >= 0) atomicCAS(info, 0, (int32_t)(i0 + bad + 1));
      if (kTrace && crec && tid == 0) {
#pragma unroll
        for (int kb = 0; kb < 4; kb++) crec[3 + 1 + kb] = sy.tt[kb];
#pragma unroll
        for (int kb = 0; kb < 3; kb++) crec[3 + 5 + kb] = sy.ts[kb + 1];  // the next leaf's own start
        crec[3 + 13] = sy.ts[0];
        crec[3 + 9] = sy.th[0];
        crec[3 + 14] = sy.th[1];
        const int64_t h = sy.th[2] > sy.th[3] ? sy.th[2] : sy.th[3];
        crec[3 + 15] = h > sy.th[4] ? h : sy.th[4];
      }
      cstamp(8, (int64_t)__builtin_amdgcn_s_memrealtime());
      // ---- the neighbour's last block row (wave w: column block w); its earlier rows were solved
      // beside the factor
      nbr_item(3, wave);
      lds_sync();
      cstamp(10, (int64_t)__builtin_amdgcn_s_memrealtime());
      // ---- the next diagonal tile's last update, k = i, from LDS: on the chain only its first 16
      // rows (block (0, w) on wave w), which the next factor's first leaf needs; the other six
      // upper blocks are folded into the followers' accumulators of the next factor
      if (next_diag) mfma_tile_sub_t(Xn, 0, wave * 16, X2, 0, X2, wave * 16, 0, 16, lane);
      // ---- publish (i, i) and (i, i + 1): every storing wave drains its write-through stores (Ld and
      // Dinv during the factor, U_i,i+1 block by block), then one flag store each
      cstamp(11, (int64_t)__builtin_amdgcn_s_memrealtime());
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // a wait timed out somewhere in the launch (info = −1; a bug guard): the chain stops here,
      // before publishing tiles built from stale operands (read by every wave after the barrier)
      if (tid == 0) s_task = __hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0 ? 1 : 0;
      lds_sync();
      if (s_task) return;
      if (tid == 0) {
        __hip_atomic_store(flags + (int64_t)i * nbc + i, kFinal, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(flags + (int64_t)i * nbc + i + 1, kFinal, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      cstamp(12, (int64_t)__builtin_amdgcn_s_memrealtime());
      if (i + 1 == nb) store_lower(X2, i0, j0);  // no next step to store it beside
      __builtin_amdgcn_s_setprio(0);
      if (kTrace && crec && tid == 0) {
        crec[0] = i;
        crec[1] = i;
        crec[2] = -1;
        crec[22] = sy.th[2];  // helper wave 0 (column blocks 0 and 3) done
        crec[23] = sy.th[4];  // helper wave 2 done
#pragma unroll
        for (int e = 0; e < 4; e++) crec[24 + e] = sy.tw[e];  // wave 1's hand-over into leaf 1
      }
      double* t = Xa;
      Xa = Xn;
      Xn = t;
    }
    return;
  }

  if (blockIdx.x == 1) {
    // ================================ the assistant ================================
    // The right neighbour's last k-step, A_i,i+1 −= U_i−1,iᵀ U_i−1,i+1, off the chain's workers: the
    // worker's partial (k < i − 1) and U_i−1,i+1 are final about a step ahead, so only U_i−1,i (the
    // chain's previous step) is waited for at the step's start; the chain's input then arrives
    // ≈ 5 µs earlier than from a worker that first waits for U_i−1,i and then runs its whole
    // epilogue. Waits: a partial and tiles of row i − 1 (dequeued earlier) and the chain's step i − 1.
    const int64_t kstep = 4 * ld * 8;
    for (int i = 1; i < nb; i++) {
      const int64_t i0 = (int64_t)i * FT, j0 = i0 + FT, k0 = i0 - FT;
      const __amdgpu_buffer_rsrc_t rT = rsrc(G + i0 * ld, gbytes_rowblk);
      const __amdgpu_buffer_rsrc_t rK = rsrc(G + k0 * ld, gbytes_rowblk);
      const int32_t* fP = flags + (int64_t)i * nbc + i + 1;        // the worker's partial
      const int32_t* fB = flags + (int64_t)(i - 1) * nbc + i + 1;  // U_i−1,i+1
      const int32_t* fA = flags + (int64_t)(i - 1) * nbc + i;      // U_i−1,i (the chain)
      wave_wait2(fP, fB, info, lane, kPartial);
      wave_wait2(fB, fB, info, lane, kFinal);
      int64_t* const arec = kTrace && (trace_roles & 2) ? trace + (int64_t)(ntasks + i) * kTraceRec : nullptr;  // slots 19-21 of step i
      if (kTrace && arec && tid == 0) arec[19] = (int64_t)__builtin_amdgcn_s_memrealtime();
      // the chain's U_i−1,i: its flag is loaded BEFORE the operands below, so (vmcnt being in order)
      // checking it leaves those loads in flight; a poll (a call, which drains loads in flight) only
      // if it is not set yet
      int a_ready = 0;
      if (lane == 0) a_ready = flag_at_least(fA, kFinal) ? 1 : 0;
      asm volatile("" ::: "memory");  // (the flag load stays ahead of the operand loads)
      d4 acc[2][2];
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = 32 * wr + 2 * (fr + 4 * r) + m;
          const dbl2 v = ld2(rT, (uint32_t)((row * ld + j0 + 32 * wc + 2 * fc) * 8), 0);
          acc[m][0][r] = v.x;
          acc[m][1][r] = v.y;
        }
      const uint32_t offA = (uint32_t)(((int64_t)fr * ld + i0 + 32 * wr + 2 * fc) * 8);
      const uint32_t offB = (uint32_t)(((int64_t)fr * ld + j0 + 32 * wc + 2 * fc) * 8);
      dbl2 a[16], b[16];
#pragma unroll
      for (int ks = 0; ks < 16; ks++) b[ks] = ld2(rK, offB, (uint32_t)(ks * kstep));
      if (!__builtin_amdgcn_readfirstlane(a_ready)) wave_wait2(fA, fA, info, lane, kFinal);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (kTrace && arec && tid == 0) arec[20] = (int64_t)__builtin_amdgcn_s_memrealtime();
#pragma unroll
      for (int ks = 0; ks < 16; ks++) a[ks] = ld2(rK, offA, (uint32_t)(ks * kstep));
#pragma unroll
      for (int ks = 0; ks < 16; ks++) {
        const double na0 = -a[ks].x, na1 = -a[ks].y;
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(na0, b[ks].x, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(na0, b[ks].y, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(na1, b[ks].x, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(na1, b[ks].y, acc[1][1], 0, 0, 0);
      }
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = 32 * wr + 2 * (fr + 4 * r) + m;
          dbl2 v;
          v.x = acc[m][0][r];
          v.y = acc[m][1][r];
          st2(rT, (uint32_t)((row * ld + j0 + 32 * wc + 2 * fc) * 8), v);
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // a wait timed out somewhere (info = −1): stop before handing on a partial built from stale
      // operands (the chain then stops at its next publish)
      if (tid == 0) s_task = __hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0 ? 1 : 0;
      __syncthreads();
      if (s_task) return;
      if (tid == 0) __hip_atomic_store(flags + (int64_t)i * nbc + i + 1, kAssisted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (kTrace && arec && tid == 0) arec[21] = (int64_t)__builtin_amdgcn_s_memrealtime();
      __syncthreads();  // s_task is rewritten next step
    }
    return;
  }

  // ================================ the workers ================================
  // One task: tile (i, j), or with NT = 2 the pair (i, j), (i, j + 1) (both "other" tiles, j >= i + 3,
  // flow_order): one k-loop loads U_ki once for both tiles, so a pair moves 48 instead of 64 KB per tile
  // and 64-deep step. The workers' k-loops are bound by those bytes, not by their MFMAs: with every CU
  // loading, one tile's 64-deep step took 2.6 µs against 1.75 µs of MFMA issue whatever the pipeline
  // depth (C2 trace, round 5: the operands come from the Infinity Cache / HBM, the L2 re-use being nil).
  auto worker_task = [&](auto nt, int t, int i, int j) {
    constexpr int NT = decltype(nt)::value;
    const bool diag = i == j;
    const bool nbr = j == i + 1;
    // the chain waits for the diagonal tiles and right neighbours, which wait for the (i, i + 2) tiles
    if ((diag && i < nb) || nbr || j == i + 2) __builtin_amdgcn_s_setprio(2);
    const int64_t i0 = (int64_t)i * FT, j0 = (int64_t)j * FT;
    // a diagonal tile's last update (k = i − 1) is the chain's, a right neighbour's the assistant's
    const int kend = ((diag && i < nb) || (nbr && i >= 1)) ? i - 1 : i;
    int64_t* const wrec = kTrace && (trace_roles & 4) ? trace + (int64_t)t * kTraceRec : nullptr;
    auto wstamp = [&](int e) {
      if (kTrace && wrec && tid == 0) wrec[3 + e] = (int64_t)__builtin_amdgcn_s_memrealtime();
    };
    wstamp(0);

    // ---- accumulators = A_ij (interleaved wave tile: MFMA tile m holds rows 32wr + 2ρ + m,
    // tile q columns 32wc + 2γ + q, so a lane's two A (B) operands are one 16-byte load)
    d4 acc[NT][2][2];
#pragma unroll
    for (int q = 0; q < NT; q++)
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = i0 + 32 * wr + 2 * (fr + 4 * r) + m;
          const dbl2 v = *reinterpret_cast<const dbl2*>(G + row * ld + j0 + q * FT + 32 * wc + 2 * fc);
          acc[q][m][0][r] = v.x;
          acc[q][m][1][r] = v.y;
        }

    // ---- A_ij −= Σ_k U_kiᵀ U_kj, the 64-deep steps' 16 MFMA k-steps of 4 run through a ring of NS stages
    // of SD k-steps (one 64-deep step of operands): while one stage's MFMAs run, the other stages' loads
    // are in flight (round 4: two 32-deep halves). A half-step ring for pairs (fewer registers) made the
    // compiler wait for every load at the top of each pass. The summation order is the same for every tile
    // and pipeline shape. The lower quadrant of a diagonal (or Schur) tile is never read: that wave skips
    // the loop.
    // k-steps known to be final: U_ki and U_kj (.. U_k,j+NT−1) for k < kr. One vector load checks the
    // flags of the next GS steps (lane group g: column i, then the task's tiles), so a worker catching up
    // to the chain polls once per GS steps: a poll per step (dependent flag loads, which drain the
    // operand loads in flight) made the k-loop ≈ 2.8 µs per step, and the chain's neighbour partial
    // (i − 1 steps) late. Bounded like poll2.
    constexpr int GS = NT == 1 ? 32 : 21;
    constexpr unsigned long long GM = (1ull << GS) - 1;
    int kr = 0;
    bool gave_up = false;  // a wait timed out or another waiter gave up (info = −1): drain, no more waits
    auto ready_upto = [&](int k) {
      for (int64_t it = 0; k >= kr && !gave_up; it++) {
        const int g = lane / GS, kk = kr + lane % GS;
        int ok = 1;
        if (g <= NT && kk < kend) ok = flag_at_least(flags + (int64_t)kk * nbc + (g == 0 ? i : j + g - 1), kFinal) ? 1 : 0;
        const unsigned long long bm = __ballot(ok);
        unsigned long long all = bm & GM;
#pragma unroll
        for (int q = 1; q <= NT; q++) all &= (bm >> (q * GS)) & GM;
        kr += all == GM ? GS : __builtin_ctzll(~all);
        if (k < kr) break;
        if ((it & 255) == 255) {
          gave_up = __hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0;
          if (!gave_up && it > ((int64_t)1 << 22)) {
            if (lane == 0) __hip_atomic_store(info, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            gave_up = true;
          }
          gave_up = __builtin_amdgcn_readfirstlane((int)gave_up) != 0;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    if (kend > 0 && !(diag && wr == 1 && wc == 0)) {
      const uint32_t offA = (uint32_t)(((int64_t)fr * ld + i0 + 32 * wr + 2 * fc) * 8);
      const uint32_t offB = (uint32_t)(((int64_t)fr * ld + j0 + 32 * wc + 2 * fc) * 8);
      const uint32_t kstep = (uint32_t)(4 * ld * 8);
      constexpr int NS = GBM_FLOW_STAGES, SD = 16 / NS, R = NS * SD;
      static_assert(16 % R == 0 && R % SD == 0, "the ring must tile a 64-deep step");
      dbl2 A[NS][SD], B[NT][NS][SD];
#ifdef GBM_FLOW_TIMING_NOLOAD
      const dbl2 zop = acc[0][0][0][0] * 0.0 == 1.0 ? (dbl2){1.0, 1.0} : (dbl2){0.0, 0.0};
#endif
      auto issue = [&](int pass, int st) {
        const int q0 = pass * R + st * SD;  // first MFMA k-step of the stage
        const __amdgpu_buffer_rsrc_t r = rsrc(G + (int64_t)(q0 >> 4) * FT * ld, gbytes_rowblk);
#pragma unroll
        for (int e = 0; e < SD; e++) {
          const uint32_t so = (uint32_t)((q0 & 15) + e) * kstep;
#ifdef GBM_FLOW_TIMING_NOLOAD
          // timing variant only (tools/build_flow_variants.sh): zero operands, no loads
          A[st][e] = zop;
#pragma unroll
          for (int q = 0; q < NT; q++) B[q][st][e] = zop;
#else
          A[st][e] = ld2(r, offA, so);
#pragma unroll
          for (int q = 0; q < NT; q++) B[q][st][e] = ld2(r, offB + (uint32_t)(q * FT * 8), so);
#endif
        }
      };
      auto mfma = [&](int st) {
#ifdef GBM_FLOW_TIMING_NOMFMA
        // timing variant only: the operands are waited for and compared, no MFMA
#pragma unroll
        for (int e = 0; e < SD; e++)
          if (A[st][e].x == 1234.5 && B[0][st][e].y == 1234.5) acc[0][0][0][0] += 1.0;
        return;
#endif
#pragma unroll
        for (int e = 0; e < SD; e++) {
          const double na0 = -A[st][e].x, na1 = -A[st][e].y;
#pragma unroll
          for (int q = 0; q < NT; q++) {
            acc[q][0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(na0, B[q][st][e].x, acc[q][0][0], 0, 0, 0);
            acc[q][0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(na0, B[q][st][e].y, acc[q][0][1], 0, 0, 0);
            acc[q][1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(na1, B[q][st][e].x, acc[q][1][0], 0, 0, 0);
            acc[q][1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(na1, B[q][st][e].y, acc[q][1][1], 0, 0, 0);
          }
        }
      };
      // one flag check per pass, ahead of its loads of the next pass (whose stages all lie in one 64-deep
      // step), and no branch between the stages: a conditional inside the ring made the compiler wait for
      // every load in flight at the top of each pass (s_waitcnt vmcnt(0)), 4.9 µs per 64-deep step
      const int passes = kend * (16 / R);
      ready_upto(0);
#pragma unroll
      for (int st = 0; st < NS; st++) issue(0, st);
      for (int p = 0; p + 1 < passes; p++) {
        ready_upto(((p + 1) * R) >> 4);
#pragma unroll
        for (int st = 0; st < NS; st++) {
          mfma(st);
          issue(p + 1, st);
        }
      }
#pragma unroll
      for (int st = 0; st < NS; st++) mfma(st);
    }
    wstamp(1);

    int32_t publish = kFinal;
    bool solved = false;  // solved tiles whose lower copies are still to be stored
    if (NT == 1 && ((nbr && i < nb) || (diag && i < nb))) {
      // ---- a partial for the chain (right neighbour: all k < i; diagonal: all k < i − 1), sc1,
      // straight from the accumulators into the tile's place in G (the chain stores U over it)
      const __amdgpu_buffer_rsrc_t rG = rsrc(G + i0 * ld, gbytes_rowblk);
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = 32 * wr + 2 * (fr + 4 * r) + m;
          dbl2 v;
          v.x = acc[0][m][0][r];
          v.y = acc[0][m][1][r];
          st2(rG, (uint32_t)((row * ld + j0 + 32 * wc + 2 * fc) * 8), v);
        }
      publish = kPartial;
    } else {
      // ---- accumulators -> X (and X2 for the pair's second tile; natural layout)
      double* const Xq[2] = {X, X2};
#pragma unroll
      for (int q = 0; q < NT; q++)
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int row = 32 * wr + 2 * (fr + 4 * r) + m;
            dbl2 v;
            v.x = acc[q][m][0][r];
            v.y = acc[q][m][1][r];
            *reinterpret_cast<dbl2*>(&Xq[q][row * PS + 32 * wc + 2 * fc]) = v;
          }
      __syncthreads();
      wstamp(2);
      if (!diag) {
        // ---- U_ij = U_ii⁻ᵀ A_ij once U_ii is final. Operands of U_ii and its 16x16 inverses come
        // straight from the sc1-stored Ld / Dinv into registers (once for both tiles of a pair); X (LDS)
        // is solved in place:
        //   X_rb <- (D_rb⁻¹)ᵀ (X_rb − U[0:o, rb]ᵀ X[0:o]),  rb = 0..3, wave w on columns 16w..16w+15
        // block row rb needs Dinv_rb (leaf rb of U_ii) and U[0:16 rb, rb] (leaves < rb): the chain
        // sets one bit per stored leaf, so the solve runs leaf by leaf beside the factor and only the
        // last block row is left once U_ii is final
        const int32_t* fl = flags + (int64_t)(i + 1) * nbc + i;
        const __amdgpu_buffer_rsrc_t rU = rsrc(G + i0 * ld, gbytes_rowblk);
        double u[24], di[4];
        const int cw = wave * 16;
        int c = 0;
#pragma unroll
        for (int rb = 0; rb < 4; rb++) {
          const int o = rb * 16;
          wave_wait_bits(fl, (2 << rb) - 1, info, lane);
          if (rb == 3) wstamp(3);
#pragma unroll
          for (int ks = 0; ks < 4; ks++)
            di[ks] = ld1(rDi, (uint32_t)(((i0 / 16) * 256 + rb * 256 + (ks * 4 + fr) * 16 + fc) * 8));
          if (rb + 1 < 4) {  // the next block row's U operands (rows of leaves <= rb)
#pragma unroll
            for (int ks = 0; ks < 4 * (rb + 1); ks++)
              u[c + 4 * rb + ks] = ld1(rLd, (uint32_t)(((i0 + ks * 4 + fr) * CNB + (rb + 1) * 16 + fc) * 8));
          }
#pragma unroll
          for (int q = 0; q < NT; q++) {
            double* const Y = Xq[q];
            if (rb > 0) {
              d4 sacc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
              for (int ks = 0; ks < 4 * rb; ks++)
                sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(u[c + ks], Y[(ks * 4 + fr) * PS + cw + fc], sacc, 0, 0, 0);
#pragma unroll
              for (int r = 0; r < 4; r++) Y[(o + fr + 4 * r) * PS + cw + fc] -= sacc[r];
            }
            d4 sacc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int ks = 0; ks < 4; ks++)
              sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(di[ks], Y[(o + ks * 4 + fr) * PS + cw + fc], sacc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; r++) {
              Y[(o + fr + 4 * r) * PS + cw + fc] = sacc[r];
              // each final 16x16 block goes out at once (write-through): the drain before the flag then
              // waits for the last block row only
              st1(rU, (uint32_t)(((int64_t)(o + fr + 4 * r) * ld + j0 + q * FT + cw + fc) * 8), sacc[r]);
            }
          }
          if (rb > 0) c += 4 * rb;
        }
        __syncthreads();
        solved = true;
      } else {
        // ---- the Schur block −WᵀW (read by later kernels only)
        const int row = tid >> 2, quarter = tid & 3;
        double* d = G + (i0 + row) * ld + j0 + quarter * 16;
#pragma unroll
        for (int e = 0; e < 16; e += 2)
          *reinterpret_cast<dbl2*>(d + e) = *reinterpret_cast<const dbl2*>(&X[row * PS + quarter * 16 + e]);
      }
    }
    // ---- publish: every storing wave drains its write-through stores, then one flag store per tile
    wstamp(4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
#pragma unroll
      for (int q = 0; q < NT; q++)
        __hip_atomic_store(flags + (int64_t)i * nbc + j + q, publish, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (solved) {
      store_lower(X, i0, j0);
      if (NT == 2) store_lower(X2, i0, j0 + FT);
    }
    __builtin_amdgcn_s_setprio(0);
    wstamp(5);
    if (kTrace && wrec && tid == 0) {
      wrec[0] = i;
      wrec[1] = j | (NT == 2 ? kPairBit : 0);
      wrec[2] = (int64_t)(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) & 7) /* XCC_ID */ * 1000 +
                (int64_t)blockIdx.x;
    }
  };

  for (;;) {
    // no new task once a wait has timed out (info = −1): the launch drains instead of computing on
    // tiles that will never be final
    if (tid == 0)
      s_task = __hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0 ? nwork : atomicAdd(queue, 1);
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    if (t >= nwork) return;
    const int32_t ij = __builtin_amdgcn_readfirstlane(order[t]);
    const int i = ij >> 16, j = ij & 0x7fff;
    if (ij & kPairBit) worker_task(std::integral_constant<int, 2>{}, t, i, j);
    else worker_task(std::integral_constant<int, 1>{}, t, i, j);
  }
}

int flow_cus() {
  static std::atomic<int> cached[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int v = cached[dev].load(std::memory_order_relaxed);
  if (v <= 0) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cached[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

int64_t* g_trace = nullptr;
int64_t g_trace_cap = 0, g_trace_n = 0;

}  // namespace

// The workers' dequeue order (see above the kernel): (i << 16) | j per task, | kPairBit for the pair (i, j),
// (i, j + 1). variant 5 (default): every tile alone; 6 (GBM_CHOL_FLOW_ORDER=6): the "other" tiles j >= r + 3
// of row r in pairs (a last odd one alone) — 48 instead of 64 KB per tile and 64-deep step, but 1.48 against
// 1.33 ms for the C2 solve (round 5: a pair holds its CU twice as long and every k-step ran slower); 4:
// round 4's order, every tile alone and the diagonal partial (d, d) in row d − 1. (A/B timing only.)
std::vector<int32_t> flow_order(int nbc, int variant) {
  const int nb = nbc - 1;
  std::vector<int32_t> o;
  o.reserve((size_t)nbc * (nbc + 1) / 2);
  auto add = [&](int i, int j) { o.push_back((i << 16) | j); };
  const bool r4 = variant == 4, pairs = variant == 6;
  for (int r = 0; r <= nb; r++) {
    if (r == 0 && nb >= 1) {
      add(0, 1);
      if (nb > 1) add(1, 1);
    }
    if (r == 1 && nb >= 2) add(1, 2);
    if (r4 && r >= 1 && r + 1 < nb) add(r + 1, r + 1);
    for (int j = r + 2; j < nbc;) {
      // (r, r + 2) stays alone: the assistant's step r + 1 waits for it
      const bool pr = pairs && j >= r + 3 && j + 1 < nbc;
      o.push_back((r << 16) | j | (pr ? kPairBit : 0));
      if (!r4 && j == r + 2 && r + 2 <= nb - 1) add(r + 2, r + 2);  // the diagonal partial two rows early
      if (j == r + 3 && r + 3 <= nb) add(r + 2, r + 3);             // the right neighbour two rows early
      j += pr ? 2 : 1;
    }
    if (r == nb) add(nb, nb);  // the Schur block
  }
  return o;
}

int flow_order_variant() {
  const char* ev = ::gbm::knob("GBM_CHOL_FLOW_ORDER");
  const int v = ev ? atoi(ev) : 5;
  return v == 4 || v == 6 ? v : 5;
}

std::vector<int32_t> flow_order(int nbc) { return flow_order(nbc, flow_order_variant()); }

// 0 when `order` (m entries) is a valid dequeue order for nbc: every tile (i, j), i <= j <= nb, except (0, 0)
// exactly once (a pair entry covers (i, j) and (i, j + 1), both "other" tiles, j >= i + 2), and every task after
// the tasks it waits for (its tiles' k-loop operands (k, i), (k, j) for k < their last step, and for the chain's
// step i (the tiles (i, j > i + 1) and every tile whose operands need it) after the chain's inputs of steps <= i:
// (s, s + 1), (s + 1, s + 1), and the assistant's (s − 1, s + 1)); else the first failing position + 1.
int64_t flow_order_check(int nbc, const int32_t* order, int64_t m) {
  const int nb = nbc - 1;
  std::vector<int64_t> pos((size_t)nbc * nbc, -1);
  int64_t tiles = 0;
  for (int64_t t = 0; t < m; t++) {
    const int i = order[t] >> 16, j = order[t] & 0x7fff, nt = (order[t] & kPairBit) ? 2 : 1;
    if (i < 0 || j < i || j + nt - 1 > nb || (i == 0 && j == 0) || (nt == 2 && j < i + 2)) return t + 1;
    for (int q = 0; q < nt; q++) {
      if (pos[(size_t)i * nbc + j + q] >= 0) return t + 1;
      pos[(size_t)i * nbc + j + q] = t;
      tiles++;
    }
  }
  if (tiles != (int64_t)nbc * (nbc + 1) / 2 - 1) return m + 1;
  auto at = [&](int i, int j) { return pos[(size_t)i * nbc + j]; };
  // the latest task the chain's step s (and the assistant's step s) needs
  std::vector<int64_t> chain_need(nbc, -1);
  for (int s = 0; s < nb; s++) {
    int64_t need = s > 0 ? chain_need[s - 1] : -1;
    need = std::max(need, at(s, s + 1));
    if (s + 1 < nb) need = std::max(need, at(s + 1, s + 1));
    if (s >= 1) need = std::max(need, at(s - 1, s + 1));
    chain_need[s] = need;
  }
  for (int64_t t = 0; t < m; t++) {
    const int i = order[t] >> 16, nt = (order[t] & kPairBit) ? 2 : 1;
    for (int j = order[t] & 0x7fff, q = 0; q < nt; q++, j++) {
      const bool diag = i == j, nbr = j == i + 1;
      const int kend = ((diag && i < nb) || (nbr && i >= 1)) ? i - 1 : i;
      for (int k = 0; k < kend; k++)
        if (at(k, i) > t || at(k, j) > t || chain_need[k] > t) return t + 1;  // operands U_ki, U_kj (final after step k)
      if (!diag && !nbr && chain_need[i] > t) return t + 1;  // the solve waits for the chain's step i
    }
  }
  return 0;
}

namespace {

// device copy of flow_order(nbc) and its length, built once per (device, nbc, variant) and kept (a few KB)
int flow_order_dev(int nbc, const int32_t** out, int* count) {
  static std::mutex mu;
  static auto* cache = new std::map<std::pair<int, int>, std::pair<int32_t*, int>>;  // never freed
  int dev = 0;
  GBM_HIP_TRY(hipGetDevice(&dev));
  const int variant = flow_order_variant();
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache->find({dev, nbc * 8 + variant});
  if (it == cache->end()) {
    const std::vector<int32_t> o = flow_order(nbc, variant);
    int32_t* d = nullptr;
    GBM_HIP_TRY(hipMalloc((void**)&d, o.size() * sizeof(int32_t)));
    GBM_HIP_TRY(hipMemcpy(d, o.data(), o.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    it = cache->emplace(std::make_pair(dev, nbc * 8 + variant), std::make_pair(d, (int)o.size())).first;
  }
  *out = it->second.first;
  *count = it->second.second;
  return GBM_OK;
}

}  // namespace

// bytes of the flag block (queue word padded to 16 B + one int32 flag per tile), a multiple of 16
int64_t chol_flow_flag_bytes(int64_t gdim) {
  const int64_t nbc = gdim / FT;
  return round_up(16 + nbc * nbc * 4, 16);
}

// n up to this many padded rows use the dataflow factorisation (GBM_CHOL_FLOW_MAX, re-read at
// every solve; 0 = always the launch-per-panel path)
bool chol_flow_enabled(int64_t npad) {
  const char* e = ::gbm::knob("GBM_CHOL_FLOW_MAX");
  const int64_t lim = e ? (int64_t)atoll(e) : (int64_t)12288;  // n = 10 000: 10.1 vs 13.6 ms; n = 16 000: 37.2 vs 36.6
  return npad <= lim;
}

int launch_chol_flow(double* G, int64_t ldg, int64_t gdim, double* Ld, double* Dinv, void* flag_block, int32_t* info,
                     hipStream_t s) {
  const int64_t nbc = gdim / FT;
  const int64_t ntasks = nbc * (nbc + 1) / 2;
  if (nbc < 2 || (int64_t)FT * ldg * 8 > 0x7fffffff || nbc * nbc > 0x3fffffff || nbc > 0x7fff)
    return fail(GBM_E_ARG, "dataflow Cholesky: matrix too large for 32-bit buffer offsets");
  const int32_t* order = nullptr;
  int nwork = 0;  // dequeue-order entries (tiles, or pairs of tiles)
  GBM_TRY(flow_order_dev((int)nbc, &order, &nwork));
  GBM_HIP_TRY(hipMemsetAsync(flag_block, 0, (size_t)chol_flow_flag_bytes(gdim), s));
  // GBM_TEST_CHOL_FLOW_ABORT (tests): start as if a wait had already timed out (info = −1), so the
  // early exit of the chain and the workers runs; the solve then fails loudly, without a hang
  if (::gbm::knob("GBM_TEST_CHOL_FLOW_ABORT")) GBM_HIP_TRY(hipMemsetAsync(info, 0xFF, sizeof(int32_t), s));
  // one workgroup per CU; GBM_CHOL_FLOW_WGS (re-read per solve) caps the workers: with 1, one worker
  // runs every tile task in dequeue order beside the chain, which checks that no wait targets a later
  // task
  const char* ew = ::gbm::knob("GBM_CHOL_FLOW_WGS");
  const int64_t workers = ew && atoll(ew) > 0 ? atoll(ew) : flow_cus() - 2;
  // + the chain and the assistant
  const unsigned grid = (unsigned)(2 + (nwork < workers ? nwork : (workers < 1 ? 1 : workers)));
  int32_t* q = (int32_t*)flag_block;
  const char* ex = ::gbm::knob("GBM_CHOL_FLOW_XN");  // 0: wave 1 always fetches the next diagonal partial first (A/B)
  const int xn_defer = ex && atoi(ex) == 0 ? 0 : 1;
  if (::gbm::knob("GBM_CHOL_FLOW_TRACE")) {
    // timing tool only: one record of 16 int64 per task, read back by gbm_debug_chol_flow_trace
    const int64_t nrec = ntasks + nbc;  // the workers' tasks, then the chain's steps
    if (g_trace_cap < nrec) {
      if (g_trace) (void)hipFree(g_trace);
      g_trace = nullptr;
      GBM_HIP_TRY(hipMalloc((void**)&g_trace, (size_t)nrec * kTraceRec * 8));
      g_trace_cap = nrec;
    }
    GBM_HIP_TRY(hipMemsetAsync(g_trace, 0, (size_t)nrec * kTraceRec * 8, s));
    g_trace_n = nrec;
    // GBM_CHOL_FLOW_TRACE = a mask of the roles that record (1 chain, 2 assistant, 4 workers; 1 = all)
    const int tm = atoi(::gbm::knob("GBM_CHOL_FLOW_TRACE"));
    const int roles = tm > 1 ? (tm & 7) : 7;
    if (::gbm::knob("GBM_CHOL_FLOW_TRACE_PLAIN"))  // (debug) the untraced kernel with the trace buffer set up
      chol_flow_kernel<false><<<grid, 256, 0, s>>>(G, ldg, (int)nbc, Ld, Dinv, q, q + 4, info, order, nwork, xn_defer, nullptr, 0);
    else
    chol_flow_kernel<true><<<grid, 256, 0, s>>>(G, ldg, (int)nbc, Ld, Dinv, q, q + 4, info, order, nwork, xn_defer, g_trace, roles);
  } else {
    chol_flow_kernel<false><<<grid, 256, 0, s>>>(G, ldg, (int)nbc, Ld, Dinv, q, q + 4, info, order, nwork, xn_defer, nullptr, 0);
  }
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

}  // namespace gbm

// Timing tool (GBM_CHOL_FLOW_TRACE=1): copy the last traced launch's per-task records of 24 int64
// (i, j, XCC_ID * 1000 + workgroup, then 100 MHz ticks: start, k-loop end, tile in LDS, factor
// done / diagonal seen, stores issued, published).
extern "C" int64_t gbm_debug_chol_flow_trace(int64_t* host, int64_t cap) {
  using namespace gbm;
  if (!g_trace || !host) return 0;
  const int64_t n = g_trace_n < cap ? g_trace_n : cap;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(host, g_trace, (size_t)n * kTraceRec * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}

// Host check of the dataflow factorisation's dequeue order (no device work): 0 when valid for nbc tiles per
// side, else the first failing task position + 1; the order (nbc (nbc + 1)/2 − 1 entries of (i << 16) | j) is
// copied to order_out when it is not NULL and cap is large enough.
extern "C" int64_t gbm_debug_chol_flow_order(int nbc, int32_t* order_out, int64_t cap) {
  if (nbc < 2 || nbc > 0x7fff) return -1;
  const std::vector<int32_t> o = gbm::flow_order(nbc);
  if (order_out && cap >= (int64_t)o.size()) std::copy(o.begin(), o.end(), order_out);
  return gbm::flow_order_check(nbc, o.data(), (int64_t)o.size());
}

extern "C" int64_t gbm_debug_chol_flow_order_size(int nbc) {
  if (nbc < 2 || nbc > 0x7fff) return -1;
  return (int64_t)gbm::flow_order(nbc).size();
}

extern "C" int64_t gbm_debug_chol_flow_order_check(int nbc, const int32_t* order, int64_t m) {
  if (nbc < 2 || nbc > 0x7fff || !order) return -1;
  return gbm::flow_order_check(nbc, order, m);
}
