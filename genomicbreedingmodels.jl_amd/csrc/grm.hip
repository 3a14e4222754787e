// GRM build: G = Σ_j z_j z_jᵀ over the standardised locus rows of Zt — an fp64 SYRK on the
// CDNA4 matrix cores (v_mfma_f64_16x16x4_f64), the dominant cost of the path.
// Also the trailing-update kernels of the upper Cholesky (chol.hip), which share the tile core.
//
// Geometry:
//   * workgroup tile 128 x 128 of G (upper-triangular tiles only: nt(nt+1)/2 tiles),
//     256 threads = 4 waves in 2 x 2, each wave a 64 x 64 sub-tile = 4 x 4 MFMA 16x16 tiles
//     (16 f64x4 accumulators per lane);
//   * K (= loci) consumed in stages of 16 rows; each stage is 2 x 16 rows x 1 KB of Zt brought
//     straight into LDS by global_load_lds_dwordx4 (one wave-instruction = one 1-KB locus row
//     segment), double-buffered; LDS row pitch 1040 B (≡ 4 dwords mod 64 banks), so the
//     ds_read_b128 fragment reads are conflict-free;
//   * work units (loci range, tile): every tile is cut into the same guided loci ranges (plan());
//     persistent workgroups (one per resident slot) take units from per-XCD queues; partial
//     tiles go to workspace slabs summed in a fixed order (deterministic, no float atomics), or,
//     for large n, are accumulated in order straight into G (carry mode).
//
// Tuning knobs are read from the environment at every plan (grm_tuning()), so a test can force
// a mode per call: GBM_GRM_CARRY (0/1: slabs / in-order carry; unset: automatic),
// GBM_GRM_PERSIST=0 (hardware-dispatched workgroups), GBM_GRM_EDGE=0 (no ragged-edge kernel),
// GBM_GRM_EDGE_CONCURRENT=0 (edge kernel after the tiles), GBM_GRM_SPLIT=w0,w1,... (relative
// loci-range sizes instead of the planner's), GBM_GRM_FUSED=1 (the slab reduce inside the persistent tile
// kernel; same bits, opt-in: DESIGN.md §7, round 6).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <queue>
#include <tuple>
#include <vector>

#include "chol_device.h"

namespace gbm {

constexpr int BT = 128;            // tile edge
constexpr int BK = 16;             // loci per stage
constexpr int WPS = 2;             // waves per SIMD (= resident 256-thread workgroups per CU)
constexpr int LROW = BT + 2;       // LDS row pitch in doubles (1040 B ≡ 4 dwords mod 64 banks)
constexpr int STAGE = 2 * BK * LROW;  // doubles per stage (A rows then B rows)

__device__ __forceinline__ void tile_of(int64_t t, int64_t& ti, int64_t& tj) {
  // t -> upper-triangular tile (ti <= tj): enumerate the lower triangle row-major, then swap
  int64_t r = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) r++;
  while (r * (r + 1) / 2 > t) r--;
  tj = r;
  ti = t - r * (r + 1) / 2;
}

// kPersistFused: kPersist with the slab reduce inside (SliceBounds::fuse; its own instantiation, so the default
// persistent kernel keeps its registers)
enum SyrkMode { kSub = 0, kSplit = 1, kPersist = 2, kPersistFused = 3 };

// Column ownership of a distributed Cholesky trailing update (kSub): with nranks > 1 this rank
// updates only the 128-column tiles J (absolute, column J·128) with J mod nranks == rank, plus the
// bordered right-hand-side tile column rhs_tile, which every rank keeps current. The launch grid
// then covers only those columns: blockIdx.y = c picks the c-th own column J = j_first + c·nranks
// (c = ncols: the right-hand-side column, when rhs), blockIdx.x the tile row ti0 + blockIdx.x (a row
// range of the update: the look-ahead updates the next panel group's rows first).
struct TileOwner {
  int32_t rank = 0, nranks = 1;
  int64_t rhs_tile = -1;
  int64_t j_first = 0, ncols = 0;
  int32_t rhs = 0;
  int64_t ti0 = 0;
};

// acc[m][q] += (NEG ? −1 : 1) Σ_k U[k][i0 + ·] U[k][j0 + ·] over the stages [kstep0, kstep0 + nsteps)
// (BK loci each) of one BT x BT tile. Operands are staged by global_load_lds into the two LDS
// buffers (double-buffered); returns after a barrier, so the buffers are free again. `wave` is
// wave-uniform (SGPR): the staging branches are scalar.
template <bool NEG>
__device__ __forceinline__ void tile_pass(const double* __restrict__ U, int64_t ldu, int64_t K, int64_t i0,
                                          int64_t j0, bool diag, bool active, int64_t kstep0, int64_t nsteps,
                                          double* lds, d4 (&acc)[4][4], int wave, int lane) {
  const int wm = wave >> 1, wn = wave & 1;
  // each wave stages BK/4 locus rows r = wave*BK/4 + rr of A (and of B off-diagonal)
  auto stage_row = [&](int64_t kstep, int buf, int rr) {
    double* base = lds + buf * STAGE;
    const int r = wave * (BK / 4) + rr;
    const int64_t k = kstep * BK + r;
    double* la = base + r * LROW;
    double* lb = base + (BK + r) * LROW;
#ifdef GBM_SYRK_TIMING_NOLOAD
    // timing variant only (tools/build_grm_variants.sh): no operand traffic, the LDS keeps whatever it holds
    if (k < K) {
    } else {
#else
    if (k < K) {
      const double* src = U + k * ldu;
      __builtin_amdgcn_global_load_lds((const void*)(src + i0 + lane * 2), (void*)la, 16, 0, 0);
      if (!diag) __builtin_amdgcn_global_load_lds((const void*)(src + j0 + lane * 2), (void*)lb, 16, 0, 0);
    } else {
#endif
      *reinterpret_cast<double2*>(la + lane * 2) = make_double2(0.0, 0.0);
      if (!diag) *reinterpret_cast<double2*>(lb + lane * 2) = make_double2(0.0, 0.0);
    }
  };
  const int frag_row = lane >> 4;  // k within a 4-deep MFMA step
  const int frag_col = lane & 15;

  if (nsteps > 0) {
#pragma unroll
    for (int rr = 0; rr < BK / 4; rr++) stage_row(kstep0, 0, rr);
  }
  __syncthreads();
  for (int64_t st = 0; st < nsteps; st++) {
    const int buf = (int)(st & 1);
    // the next stage's rows go out first, all together (issuing them one per k-step between
    // the MFMA groups measured 3 % slower)
    if (st + 1 < nsteps) {
#pragma unroll
      for (int rr = 0; rr < BK / 4; rr++) stage_row(kstep0 + st + 1, buf ^ 1, rr);
    }
    const double* A = lds + buf * STAGE;
    const double* B = diag ? A : A + BK * LROW;
#pragma unroll
    for (int ks = 0; ks < BK / 4; ks++) {
      if (active) {
        const int kr = ks * 4 + frag_row;
        // interleaved wave tile: MFMA tile m holds quadrant rows 4ρ + m (ρ = MFMA row), tile q
        // holds quadrant columns 4γ + q, so a lane's four A (B) operands are adjacent: two
        // ds_read_b128 each (conflict-free at the 1040-B pitch)
        const double2 a01 = *reinterpret_cast<const double2*>(&A[kr * LROW + wm * 64 + 4 * frag_col]);
        const double2 a23 = *reinterpret_cast<const double2*>(&A[kr * LROW + wm * 64 + 4 * frag_col + 2]);
        const double2 b01 = *reinterpret_cast<const double2*>(&B[kr * LROW + wn * 64 + 4 * frag_col]);
        const double2 b23 = *reinterpret_cast<const double2*>(&B[kr * LROW + wn * 64 + 4 * frag_col + 2]);
        double af[4] = {a01.x, a01.y, a23.x, a23.y};
        const double bf[4] = {b01.x, b01.y, b23.x, b23.y};
        if constexpr (NEG) {
#pragma unroll
          for (int m = 0; m < 4; m++) af[m] = -af[m];
        }
        // the wave in its MFMA group wins issue arbitration over its SIMD partner's staging and
        // LDS instructions (GRM at C2 on one box: 18.87 -> 18.68 ms)
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
          for (int q = 0; q < 4; q++)
            acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[q], acc[m][q], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    __syncthreads();
  }
  __syncthreads();
}

// Loci split of the GRM: every tile is cut into the same nslices stage ranges
// [b[s], b[s+1]); workgroup (s, t) = blockIdx s * ntiles + t sums range s of tile t into slab
// slot (s, t). The ranges shrink from first to last (plan() below), so the hardware's in-order
// dispatch onto freed slots works like guided self-scheduling: large chunks first, small ones
// fill the tail.
constexpr int kMaxSlices = 32;
struct SliceBounds {
  int32_t n;
  int32_t b[kMaxSlices + 1];
  // carry = 1: the loci ranges of a tile are summed in order straight into G (range s waits for
  // range s − 1's flag, adds its partial, stores, flags s + 1); workspace = ntiles flags + 1.
  // carry = 0: one workspace slab per (range, tile), summed by grm_slab_reduce_kernel.
  int32_t carry;
  // ragged last tile column (grm_edge_pass): columns [e0, e0 + er) of G, er <= 64, in et 16-column
  // MFMA tiles, for all rows, by erb x es extra workgroups (256-row blocks x ekper-loci ranges)
  // appended to the grid; partials at slab + eslab_off, summed by grm_edge_reduce_kernel
  int32_t er, et, erb, es, ekper;
  int64_t e0, eslab_off;
  // carry mode with accumulation (G += this GRM): range 0 adds G's existing tile as well
  int32_t accum = 0;
  // fuse = 1 (persistent slabs mode, GBM_GRM_FUSED): the reduce runs inside the tile kernel — each unit stores
  // its slab, releases it (agent scope) and takes a ticket on its tile's counter; the unit that draws the last
  // ticket sums the tile's slabs into G in range order (the reduce kernel's order), so grm_slab_reduce_kernel
  // is not launched
  int32_t fuse = 0;
};

// Ragged last tile column of the GRM: when n = 128 (nt − 1) + r with small r, the last tile
// column would cost nt full 128x128 tiles (a workgroup whose waves idle still holds its slot
// for the whole tile time) for r useful columns. Instead the tiles cover [0, e0)^2 and extra
// workgroups compute G[i][e0 + c] = Σ_k U[k][i] U[k][e0 + c], c < r, for every row i: a
// 256-row block over a loci range per workgroup, operands straight from global memory into
// MFMA registers (A: 4 row tiles of 16 per wave, B: et column tiles), HBM-bound (one extra
// read of U). A separate launch after the tiles: as extra workgroups of the tile kernel it
// raised that kernel's VGPR allocation and slowed its tiles by ~2 %. Behind the persistent tile
// kernel it runs concurrently, on a helper stream (launch_grm_syrk).
template <int ET>
__device__ __forceinline__ void grm_edge_pass(const double* __restrict__ U, int64_t ldu, int64_t K,
                                              const SliceBounds& sb, int64_t e, double* __restrict__ part,
                                              int lane, int wave) {
  const int rb = (int)(e % sb.erb), ks = (int)(e / sb.erb);
  const int64_t k0 = (int64_t)ks * sb.ekper;
  const int64_t k1 = (k0 + sb.ekper < K) ? k0 + sb.ekper : K;
  const int64_t i0 = (int64_t)rb * 256 + wave * 64;
  const int fr = lane >> 4, fc = lane & 15;
  d4 acc[4][ET];
#pragma unroll
  for (int m = 0; m < 4; m++)
#pragma unroll
    for (int q = 0; q < ET; q++) acc[m][q] = (d4){0.0, 0.0, 0.0, 0.0};
  for (int64_t k = k0; k < k1; k += 16) {  // 4 MFMA k-steps per iteration, all loads first
    double a[4][4], b[4][ET];
#pragma unroll
    for (int st = 0; st < 4; st++) {
      const int64_t kk = k + st * 4 + fr;
      const bool kv = kk < k1;
      const double* row = U + kk * ldu;
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const int64_t i = i0 + m * 16 + fc;
        a[st][m] = (kv && i < ldu) ? row[i] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < ET; q++) b[st][q] = kv ? row[sb.e0 + q * 16 + fc] : 0.0;
    }
#pragma unroll
    for (int st = 0; st < 4; st++)
#pragma unroll
      for (int q = 0; q < ET; q++)
#pragma unroll
        for (int m = 0; m < 4; m++) acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[st][m], b[st][q], acc[m][q], 0, 0, 0);
  }
  const int64_t rows = (int64_t)sb.erb * 256;
  constexpr int w = 16 * ET;
#pragma unroll
  for (int m = 0; m < 4; m++)
#pragma unroll
    for (int q = 0; q < ET; q++)
#pragma unroll
      for (int r = 0; r < 4; r++)
        part[((int64_t)ks * rows + i0 + m * 16 + fr + 4 * r) * w + q * 16 + fc] = acc[m][q][r];
}

// ET = ⌈r/16⌉ column tiles: few enough registers (ET = 1: ≤ 128) that the edge workgroups fit
// beside the persistent tile kernel's two workgroups per CU and run concurrently with it
template <int ET>
__global__ void __launch_bounds__(256, ET == 1 ? 4 : 1) grm_edge_kernel(const double* __restrict__ U, int64_t ldu, int64_t K,
                                                       SliceBounds sb, double* __restrict__ part) {
  grm_edge_pass<ET>(U, ldu, K, sb, blockIdx.x, part, threadIdx.x & 63, threadIdx.x >> 6);
}

// G[i][e0 + c] = Σ_s part[s][i][c] in range order (deterministic), i < n, c < er; with `accum`,
// G[i][e0 + c] += that sum (the chunked host upload adds each chunk's GRM into G)
__global__ void __launch_bounds__(256) grm_edge_reduce_kernel(const double* __restrict__ part, int64_t n,
                                                              SliceBounds sb, double* __restrict__ G, int64_t ldg,
                                                              int accum) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n * sb.er) return;
  const int64_t i = idx / sb.er;
  const int c = (int)(idx - i * sb.er);
  const int64_t rows = (int64_t)sb.erb * 256;
  const int w = 16 * sb.et;
  double acc = 0.0;
  for (int s = 0; s < sb.es; s++) acc += part[((int64_t)s * rows + i) * w + c];
  double* g = G + i * ldg + sb.e0 + c;
  *g = accum ? *g + acc : acc;
}

// Two epilogues over one staging/MFMA core:
//   kSplit   slab[s][t] = Σ_{k in range s} U[k][i] U[k][j]   (the GRM, split over loci)
//   kSub     C[i][j]   -= Σ_k U[k][i] U[k][j]               (the upper-Cholesky trailing update, K = 64)
// U is k-major: row k holds columns c contiguous (U[k*ldu + c]); the tiles are the upper
// (ti <= tj) BT x BT tiles of the square [c0, c0 + lim)^2, in absolute column coordinates of U
// and C. Wave quadrants entirely outside `lim` skip their MFMAs and stores (padding / ragged
// last tile), as does the strictly-lower quadrant of a diagonal tile (upper storage); their
// operand columns may be read past `lim` (the caller guarantees those reads stay inside the
// allocation).
template <int MODE>
__global__ void __launch_bounds__(256, WPS)
syrk_kernel(const double* __restrict__ U, int64_t ldu, int64_t K, int64_t c0, int64_t lim,
            double* __restrict__ C, int64_t ldc, double* __restrict__ slab, int64_t ntiles, SliceBounds sb,
            double* __restrict__ Ld, double* __restrict__ Dinv, int32_t* __restrict__ info, int64_t fk0,
            TileOwner own) {
  // 2 stages (72 KB at BK = 16); kSub's first workgroup reuses it for the 64x64 factor image
  constexpr int LDS_DOUBLES = (2 * STAGE > CNB * PS + CNB + 16) ? 2 * STAGE : CNB * PS + CNB + 16;
  __shared__ __attribute__((aligned(16))) double lds[LDS_DOUBLES];

  const int64_t wg = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // f64 MFMA C/D map: MFMA column = lane & 15, MFMA row = (lane >> 4) + 4 * reg; with the
  // interleaved wave tile (tile_pass), acc[m][q][r] is quadrant element
  // (row 4 * frag_row + 16 * r + m, column 4 * frag_col + q)
  const int frag_row = lane >> 4, frag_col = lane & 15;
  const int64_t nst = (K + BK - 1) / BK;
  const int64_t rlim = c0 + lim;

  if constexpr (MODE == kSplit || MODE == kPersist || MODE == kPersistFused) {
    // one (loci range sl, tile t) unit: the tile's partial sum over the range, then the slab /
    // carry / direct epilogue
    auto run_unit = [&](int sl, int64_t t) {
    int64_t ti, tj;
    tile_of(t, ti, tj);
    const bool diag = (ti == tj);
    const int64_t i0 = c0 + ti * BT, j0 = c0 + tj * BT;
    const bool active = (i0 + wm * 64 < rlim) && (j0 + wn * 64 < rlim) && !(diag && wm == 1 && wn == 0);
    d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 4; b++) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
    const int64_t ks0 = sb.b[sl];
    const int64_t ks1 = sb.b[sl + 1] < nst ? sb.b[sl + 1] : nst;
    tile_pass<false>(U, ldu, K, i0, j0, diag, active, ks0, ks1 > ks0 ? ks1 - ks0 : 0, lds, acc, wave, lane);
    if (MODE == kSplit && sb.carry && sb.n > 1) {  // (not compiled into the persistent kernel)
      // in-order carry: G tile = ((P_0 + P_1) + P_2) + ..., the same order (and rounding) as the
      // slab reduce. Range sl's predecessor was dispatched 1+ rounds earlier (lower workgroup
      // id), so the wait is normally already satisfied and can never deadlock. The tile goes
      // through agent-scope (write-through) stores; the successor may run on another XCD.
      int32_t* tflags = reinterpret_cast<int32_t*>(slab);
      double* out = C + i0 * ldc + j0 + (wm * 64 + 4 * frag_row) * ldc + wn * 64 + 4 * frag_col;
      if (sl > 0 || sb.accum) {
        if (sl > 0) {
          if (threadIdx.x == 0) wait_flag(&tflags[t], sl, tflags + ntiles);
          __syncthreads();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        if (active) {
          double2 prev[4][4][2];
#pragma unroll
          for (int m = 0; m < 4; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
              const double* o = out + (16 * r + m) * ldc;
              prev[m][r][0] = *reinterpret_cast<const double2*>(o);
              prev[m][r][1] = *reinterpret_cast<const double2*>(o + 2);
            }
#pragma unroll
          for (int m = 0; m < 4; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
              acc[m][0][r] = prev[m][r][0].x + acc[m][0][r];
              acc[m][1][r] = prev[m][r][0].y + acc[m][1][r];
              acc[m][2][r] = prev[m][r][1].x + acc[m][2][r];
              acc[m][3][r] = prev[m][r][1].y + acc[m][3][r];
            }
        }
      }
      if (active) {
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            double* o = out + (16 * r + m) * ldc;
#pragma unroll
            for (int q = 0; q < 4; q++) st_agent(o + q, acc[m][q][r]);
          }
      }
      publish_flag(&tflags[t], sl + 1, threadIdx.x);
    } else if (MODE == kPersistFused && sb.n > 1) {
      // the fused reduce (SliceBounds::fuse), the guide's split-K hand-off in its plain-store form: the unit's
      // slab with plain stores, every wave drains them, barrier, ONE agent-scope release (L2 write-back) and
      // the relaxed agent-scope ticket; the unit that draws the tile's last ticket acquires (agent scope) and
      // reads every range's slab (its own too) with plain loads, adding them from 0.0 in range order exactly
      // as grm_slab_reduce_kernel does
      const int64_t per = (int64_t)BT * BT;
      const int64_t eoff = (wm * 64 + 4 * frag_row) * BT + wn * 64 + 4 * frag_col;
      if (active) {
        double* out = slab + ((int64_t)sl * ntiles + t) * per + eoff;
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            double* o = out + (16 * r + m) * BT;
            *reinterpret_cast<double2*>(o) = make_double2(acc[m][0][r], acc[m][1][r]);
            *reinterpret_cast<double2*>(o + 2) = make_double2(acc[m][2][r], acc[m][3][r]);
          }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* s_last = reinterpret_cast<int*>(lds);  // (the staging buffers are free: tile_pass ended in a barrier)
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const bool lt = __hip_atomic_fetch_add(&info[8 + t], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == sb.n - 1;
        if (lt) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *s_last = lt;
      }
      __syncthreads();
      const bool last = *s_last != 0;
      __syncthreads();  // every wave has read s_last before the next unit stages into lds
      if (last && active) {
        double* gout = C + (i0 + wm * 64 + 4 * frag_row) * ldc + j0 + wn * 64 + 4 * frag_col;
        const double* tbase = slab + t * per + eoff;
#pragma unroll 1
        for (int mr = 0; mr < 16; mr++) {
          const int m = mr & 3, r = mr >> 2;
          double2 v01 = make_double2(0.0, 0.0), v23 = make_double2(0.0, 0.0);
          for (int s2 = 0; s2 < sb.n; s2++) {
            const double* src = tbase + (int64_t)s2 * ntiles * per + (16 * r + m) * BT;
            const double2 x01 = *reinterpret_cast<const double2*>(src), x23 = *reinterpret_cast<const double2*>(src + 2);
            v01.x += x01.x;
            v01.y += x01.y;
            v23.x += x23.x;
            v23.y += x23.y;
          }
          double* g = gout + (16 * r + m) * ldc;
          if (sb.accum) {
            const double2 a01 = *reinterpret_cast<const double2*>(g), a23 = *reinterpret_cast<const double2*>(g + 2);
            v01 = make_double2(a01.x + v01.x, a01.y + v01.y);
            v23 = make_double2(a23.x + v23.x, a23.y + v23.y);
          }
          *reinterpret_cast<double2*>(g) = v01;
          *reinterpret_cast<double2*>(g + 2) = v23;
        }
      }
    } else if (active) {
      // a single slice stores straight into G (no workspace, the reduce is a no-op)
      const int64_t ld = sb.n == 1 ? ldc : BT;
      double* out = (sb.n == 1 ? C + i0 * ldc + j0 : slab + ((int64_t)sl * ntiles + t) * (BT * BT)) +
                    (wm * 64 + 4 * frag_row) * ld + wn * 64 + 4 * frag_col;
#pragma unroll
      for (int m = 0; m < 4; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          double* o = out + (16 * r + m) * ld;
          *reinterpret_cast<double2*>(o) = make_double2(acc[m][0][r], acc[m][1][r]);
          *reinterpret_cast<double2*>(o + 2) = make_double2(acc[m][2][r], acc[m][3][r]);
        }
    }
    };
    // XCD-aware order: XCD x owns the contiguous tile range [x T8/8, (x+1) T8/8) of every loci
    // range (T8 = round_up(ntiles, 8)), so neighbouring tiles share A/B strips in that XCD's L2
    // and later ranges revisit the same tiles
    const int64_t T8 = (ntiles + 7) & ~(int64_t)7;
    if constexpr (MODE == kPersist || MODE == kPersistFused) {
      // persistent workgroups (one per resident slot): each takes units from its own XCD's queue
      // (XCC_ID hardware register; units in range-major order over the XCD's tiles) through an
      // atomic counter, then steals from the other XCDs' queues once its own is empty. Dynamic
      // to the last unit, so the XCDs finish together (with hardware dispatch every XCD ran a
      // fixed 1/8 of the workgroups and they ended up to 1 ms apart).
      __shared__ int64_t s_unit;
      int32_t* ctr = info;  // 8 queue counters, zeroed before the launch
      const int xcc = (int)(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) & 7);
      const int64_t per = T8 >> 3;
      int q = xcc;
      for (int tries = 0; tries < 8;) {
        const int64_t qt0 = q * per;
        const int64_t qt1 = qt0 + per < ntiles ? qt0 + per : ntiles;
        const int64_t nq = qt1 > qt0 ? qt1 - qt0 : 0;
        if (threadIdx.x == 0) s_unit = atomicAdd(&ctr[q], 1);
        __syncthreads();
        const int64_t u = s_unit;
        __syncthreads();
        if (u >= nq * sb.n) {
          q = (q + 1) & 7;
          tries++;
          continue;
        }
        const int sl = (int)(u / nq);
        run_unit(sl, qt0 + (u - (int64_t)sl * nq));
      }
      return;
    } else {
      // hardware dispatch is round-robin over the 8 XCDs (workgroup id mod 8): each range is
      // launched as T8 workgroups and id u of a range maps to tile (u & 7) T8/8 + (u >> 3)
      const int sl = (int)(wg / T8);
      const int64_t u = wg - (int64_t)sl * T8;
      const int64_t t = (u & 7) * (T8 >> 3) + (u >> 3);
      if (t >= ntiles) return;
      run_unit(sl, t);
    }
    return;
  } else {
    int64_t ti, tj;
    if (own.nranks > 1) {  // the compact grid over this rank's tile columns
      const int64_t c = blockIdx.y;
      const int64_t J = c < own.ncols ? own.j_first + c * own.nranks : own.rhs_tile;
      tj = J - c0 / BT;
      ti = own.ti0 + blockIdx.x;
      if (ti > tj) return;  // (workgroup-uniform) below the diagonal
    } else {
      tile_of(wg, ti, tj);
    }
    const bool diag = (ti == tj);
    const int64_t i0 = c0 + ti * BT, j0 = c0 + tj * BT;
    const bool active = (i0 + wm * 64 < rlim) && (j0 + wn * 64 < rlim) && !(diag && wm == 1 && wn == 0);
    // the C tile goes straight into the accumulators (its loads overlap the operand staging)
    // and the A fragments are negated: the MFMA chain produces C − Σ_k U[k][i] U[k][j]
    d4 acc[4][4];
    // (rlim is a multiple of 4: a lane's 4 adjacent columns are in or out together)
    const int64_t col0 = j0 + wn * 64 + 4 * frag_col;
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int64_t row = i0 + wm * 64 + 4 * frag_row + 16 * r + m;
        double2 c01 = make_double2(0.0, 0.0), c23 = make_double2(0.0, 0.0);
        if (active && row < rlim && col0 < rlim) {
          c01 = *reinterpret_cast<const double2*>(C + row * ldc + col0);
          c23 = *reinterpret_cast<const double2*>(C + row * ldc + col0 + 2);
        }
        acc[m][0][r] = c01.x;
        acc[m][1][r] = c01.y;
        acc[m][2][r] = c23.x;
        acc[m][3][r] = c23.y;
      }
    tile_pass<true>(U, ldu, K, i0, j0, diag, active, 0, nst, lds, acc, wave, lane);
    // first workgroup (tile (0,0)), fk0 >= 0: factor the next diagonal block afterwards
    const bool factor_next = fk0 >= 0 && wg == 0;
    if (!active && !factor_next) return;
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int64_t row = i0 + wm * 64 + 4 * frag_row + 16 * r + m;
        if (active && row < rlim && col0 < rlim) {
          *reinterpret_cast<double2*>(C + row * ldc + col0) = make_double2(acc[m][0][r], acc[m][1][r]);
          *reinterpret_cast<double2*>(C + row * ldc + col0 + 2) = make_double2(acc[m][2][r], acc[m][3][r]);
        }
      }
    if (factor_next) {
      // the next panel's diagonal block [c0, c0+64)^2 is wave (0,0)'s 64x64 quadrant of this tile
      double* Us = lds;  // the staging buffers are free now (tile_pass ended in a barrier)
      double* rinv = lds + CNB * PS;
      if (wave == 0) {
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
          for (int q = 0; q < 4; q++)
#pragma unroll
            for (int r = 0; r < 4; r++) Us[(4 * frag_row + 16 * r + m) * PS + 4 * frag_col + q] = acc[m][q][r];
      }
      __syncthreads();
      const int bad = factor_diag_block(Us, rinv, threadIdx.x);
      if (threadIdx.x == 0 && bad >= 0) atomicCAS(info, 0, (int32_t)(fk0 + bad + 1));
      store_factor(Us, rinv, Ld + fk0 * CNB, Dinv + (fk0 / 16) * 256, threadIdx.x);
    }
  }
}

// G tile = Σ_s slab[s][tile] in slice order (deterministic, no float atomics); with `accum`,
// G tile += that sum.
// the slabs read with the nontemporal hint (each read once): C2 reduce 0.181 → 0.160 ms, same bits
// (profiles/r06_nt_reduce_transpose_ab.txt; GBM_GRM_RED_NT=0 builds the plain loads)
#ifndef GBM_GRM_RED_NT
#define GBM_GRM_RED_NT 1
#endif
__global__ void __launch_bounds__(256) grm_slab_reduce_kernel(const double* __restrict__ slab, int64_t ntiles,
                                                              int nslices, double* __restrict__ G, int64_t ldg,
                                                              int accum) {
  const int64_t t = blockIdx.x;
  int64_t ti, tj;
  tile_of(t, ti, tj);
  const int64_t per = (int64_t)BT * BT;
  for (int e = threadIdx.x * 2; e < BT * BT; e += 256 * 2) {
    double2 acc = make_double2(0.0, 0.0);
    for (int sl = 0; sl < nslices; sl++) {
#if GBM_GRM_RED_NT
      typedef double d2v __attribute__((ext_vector_type(2)));
      const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(slab + ((int64_t)sl * ntiles + t) * per + e));
#else
      const double2 v = *reinterpret_cast<const double2*>(slab + ((int64_t)sl * ntiles + t) * per + e);
#endif
      acc.x += v.x;
      acc.y += v.y;
    }
    const int row = e / BT, col = e % BT;
    double2* g = reinterpret_cast<double2*>(G + (ti * BT + row) * ldg + tj * BT + col);
    if (accum) {
      const double2 old = *g;
      acc.x = old.x + acc.x;
      acc.y = old.y + acc.y;
    }
    *g = acc;
  }
}

static int resident_wgs() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
  }
  return cus * WPS;  // WPS workgroups per CU (LDS 2 x 2 x BK x 1152 B each)
}

// Tuning of the GRM launch (GBM_* knobs, knobs.cpp), read at every plan (a few table lookups), so the
// modes can be forced per call (tests, through gbm_debug_set) without a process restart.
struct GrmTuning {
  int carry = -1;              // GBM_GRM_CARRY: 0 slabs, 1 in-order carry, -1 automatic
  bool edge = true;            // GBM_GRM_EDGE: ragged-edge kernel for a last tile column of <= 64
  bool persist = true;         // GBM_GRM_PERSIST: persistent workgroups with per-XCD queues
  bool edge_concurrent = true; // GBM_GRM_EDGE_CONCURRENT: edge kernel on the helper stream
  bool fuse = false;           // GBM_GRM_FUSED: the slab reduce inside the persistent tile kernel
  std::vector<double> split;   // GBM_GRM_SPLIT: relative loci-range sizes (tuning experiments)
};

static GrmTuning grm_tuning() {
  GrmTuning t;
  auto flag = [](const char* name, bool dflt) {
    const char* e = ::gbm::knob(name);
    return e ? atoi(e) != 0 : dflt;
  };
  if (const char* e = ::gbm::knob("GBM_GRM_CARRY")) t.carry = atoi(e) != 0 ? 1 : 0;
  t.edge = flag("GBM_GRM_EDGE", true);
  t.persist = flag("GBM_GRM_PERSIST", true);
  t.edge_concurrent = flag("GBM_GRM_EDGE_CONCURRENT", true);
  t.fuse = flag("GBM_GRM_FUSED", false);
  if (const char* ov = ::gbm::knob("GBM_GRM_SPLIT")) {
    for (const char* q = ov; *q;) {
      char* end = nullptr;
      const double x = strtod(q, &end);
      if (end == q) break;
      if (x > 0) t.split.push_back(x);
      q = (*end == ',') ? end + 1 : end;
    }
    if ((int)t.split.size() > kMaxSlices) t.split.clear();
  }
  return t;
}

// Plan of the GRM loci split. Candidate partitions of a tile's nst stages — uniform (1..8
// slices) and guided (one large first range, then geometrically shrinking ones) — are scored by
// simulating the dispatch of the ntiles x nslices units onto the resident slots (list
// scheduling with per-tile costs; slot speeds jittered by ~2 %, as measured with per-unit
// timelines), plus the slab-reduce cost; the fastest wins. Cached per (n, p, slots, mode).
struct GrmPlan {
  int64_t ntiles, nst, tile_elems;
  SliceBounds sb;
  int64_t main_doubles, edge_doubles;  // workspace: loci-slice partial tiles (or carry flags), edge partials
  bool persist, edge_concurrent;
};

static double simulate_split(const std::vector<int64_t>& sizes, const std::vector<double>& cost, int64_t R,
                             double tile_bytes, double stage_s, bool carry) {
  std::vector<double> speed(R);
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int64_t k = 0; k < R; k++) {  // deterministic jitter, sd ≈ 2 %
    h = h * 6364136223846793005ull + 1442695040888963407ull;
    speed[k] = 1.0 + 0.035 * (((double)(h >> 11) / 9007199254740992.0) * 2.0 - 1.0);
  }
  std::priority_queue<std::pair<double, int64_t>, std::vector<std::pair<double, int64_t>>, std::greater<>> slots;
  for (int64_t k = 0; k < R; k++) slots.push({0.0, k});
  double makespan = 0.0;
  for (size_t s = 0; s < sizes.size(); s++)
    for (double c : cost) {
      auto [f, k] = slots.top();
      slots.pop();
      // first-range units that start after the first round run ~10 % slower (measured: they
      // overlap other K ranges instead of streaming the same strips as their XCD's neighbours,
      // so fewer of their operand rows hit L2); fitted on 11 measured splits at C2
      f += (double)sizes[s] * c * ((s == 0 && f > 0.0) ? 1.10 : 1.0) / speed[k];
      if (carry && s > 0) f += 0.5;  // read-add-write of the running tile sum (~2 µs)
      if (f > makespan) makespan = f;
      slots.push({f, k});
    }
  // slab reduce: one tile partial read per (slice, tile) at ~4 TB/s, in stage-time units
  const double reduce_stages =
      carry ? 0.0 : (double)sizes.size() * (double)cost.size() * tile_bytes / 4e12 / stage_s;
  return makespan + reduce_stages;
}

static GrmPlan plan(int64_t n, int64_t p) {
  const GrmTuning tune = grm_tuning();
  GrmPlan g;
  const int64_t nt_all = npad_of(n) / BT;
  // ragged last tile column with r <= 64 useful columns: computed by the edge workgroups
  const int64_t r_last = n - (nt_all - 1) * BT;
  const bool edge = tune.edge && nt_all >= 8 && r_last <= 64;
  const int64_t nt = edge ? nt_all - 1 : nt_all;
  g.nst = (p + BK - 1) / BK;
  std::vector<double> cost;
  const int64_t R = resident_wgs();
  for (int64_t tj = 0; tj < nt; tj++)
    for (int64_t ti = 0; ti <= tj; ti++) cost.push_back(ti == tj ? 0.93 : 1.0);
  g.ntiles = nt * (nt + 1) / 2;
  g.tile_elems = (int64_t)BT * BT;
  auto finish = [&](GrmPlan& gp) {
    gp.main_doubles = gp.sb.n == 1 ? 0
                      : gp.sb.carry ? (gp.ntiles + 1 + 1) / 2 + 1  // int32 flags + error cell
                                    : (int64_t)gp.sb.n * gp.ntiles * gp.tile_elems;
    gp.sb.er = 0;
    gp.sb.et = gp.sb.erb = gp.sb.es = gp.sb.ekper = 0;
    gp.sb.e0 = gp.sb.eslab_off = 0;
    gp.edge_doubles = 0;
    if (edge) {
      gp.sb.e0 = nt * BT;
      gp.sb.er = (int32_t)r_last;
      gp.sb.et = (int32_t)((r_last + 15) / 16);
      gp.sb.erb = (int32_t)((n + 255) / 256);
      // ~2048 edge workgroups in all (loci ranges of >= 256, multiples of 16): bounded partials
      const int64_t es_want = std::max<int64_t>(1, std::min<int64_t>((2048 + gp.sb.erb - 1) / gp.sb.erb, (p + 255) / 256));
      gp.sb.ekper = (int32_t)(((p + es_want - 1) / es_want + 15) / 16 * 16);
      gp.sb.es = (int32_t)((p + gp.sb.ekper - 1) / gp.sb.ekper);
      gp.sb.eslab_off = gp.main_doubles;
      gp.edge_doubles = (int64_t)gp.sb.es * gp.sb.erb * 256 * 16 * gp.sb.et;
    }
    gp.persist = tune.persist && !gp.sb.carry;
    gp.sb.fuse = (gp.persist && gp.sb.n > 1 && tune.fuse) ? 1 : 0;
    // the ragged-column kernel and its reduce run on the helper stream, beside the persistent tiles
    gp.edge_concurrent = gp.sb.er > 0 && gp.persist && tune.edge_concurrent;
  };
  static std::mutex mu;
  static std::map<std::tuple<int64_t, int64_t, int64_t, int, std::vector<double>>, SliceBounds> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_tuple(nt, g.nst, R, tune.carry, tune.split);
  auto it = cache.find(key);
  if (it != cache.end()) {
    g.sb = it->second;
    finish(g);
    return g;
  }
  const int64_t minc = 16;  // stages per workgroup at least
  const bool big = g.ntiles > 2048;  // keep the one-off planning cost small for large n
  // stage time: ~3.9 us per 16-locus stage of a 128x128 tile at 2 workgroups per CU
  const double stage_s = 3.9e-6;
  double best = 1e300;
  auto choose = [&](bool carry) {
    std::vector<std::vector<int64_t>> cands;
    const int max_uniform = big ? 3 : (carry ? kMaxSlices : 8);
    for (int S = 1; S <= max_uniform; S++) {
      if (S > 1 && g.nst / S < minc) break;
      std::vector<int64_t> v;
      for (int i = 0; i < S; i++) v.push_back((g.nst * (i + 1)) / S - (g.nst * i) / S);
      cands.push_back(v);
    }
    for (double f = big ? 0.60 : 0.40; f < 0.90; f += big ? 0.10 : 0.05)
      for (double r : {0.3, 0.4, 0.5, 0.6, 0.7}) {
        if (big && r != 0.5) continue;
        std::vector<int64_t> v;
        int64_t first = (int64_t)(f * (double)g.nst);
        if (first < minc || g.nst - first < minc) continue;
        v.push_back(first);
        int64_t rem = g.nst - first;
        while (rem > 0) {
          int64_t c = (int64_t)std::ceil(r * (double)rem);
          if (c < minc) c = minc;
          if (rem - c < minc || (int)v.size() == (carry ? kMaxSlices : 12) - 1) c = rem;
          v.push_back(c);
          rem -= c;
        }
        cands.push_back(v);
      }
    if (!tune.split.empty()) {
      double tot = 0;
      for (double x : tune.split) tot += x;
      cands.clear();
      std::vector<int64_t> v;
      int64_t acc = 0;
      double cum = 0;
      for (size_t i = 0; i < tune.split.size(); i++) {
        cum += tune.split[i];
        const int64_t e = (i + 1 == tune.split.size()) ? g.nst : (int64_t)std::llround(cum / tot * (double)g.nst);
        if (e > acc) v.push_back(e - acc);
        acc = e > acc ? e : acc;
      }
      cands.push_back(v);
    }
    std::vector<int64_t> bv{g.nst};
    best = 1e300;
    for (const auto& v : cands) {
      const double m = simulate_split(v, cost, R, (double)g.tile_elems * 8.0, stage_s, carry);
      if (m < best * 0.999) {
        best = m;
        bv = v;
      }
    }
    return bv;
  };
  // slabs (+ reduce kernel) unless they would exceed 4 GiB (or GBM_GRM_CARRY forces a mode):
  // the in-order carry needs no workspace but its write-through epilogue costs ~1 % at C2
  int carry_mode = tune.carry;
  std::vector<int64_t> bestv = choose(carry_mode == 1);
  if (carry_mode < 0 && bestv.size() > 1 &&
      (double)bestv.size() * (double)g.ntiles * (double)g.tile_elems * 8.0 > 4.0 * 1073741824.0) {
    carry_mode = 1;
    bestv = choose(true);
  }
  g.sb.carry = (carry_mode == 1 && bestv.size() > 1) ? 1 : 0;
  g.sb.n = (int32_t)bestv.size();
  g.sb.b[0] = 0;
  for (int i = 0; i < g.sb.n; i++) g.sb.b[i + 1] = g.sb.b[i] + (int32_t)bestv[i];
  cache.emplace(key, g.sb);
  finish(g);
  return g;
}

// Small-tile variant of the Cholesky trailing update (64x64 upper tiles, K = 64, 4 waves of
// 32x32): more workgroups for the small trailing matrices of late panels. The C tile is loaded
// into the accumulators first and the A fragments are negated, so the MFMA chain itself
// produces C − Σ_k U[k][i] U[k][j] (no separate read-modify-write).
constexpr int P64 = 80;  // LDS pitch: the two 16-lane halves of a fragment read hit disjoint banks
// PIPE (the multi-chunk row updates): chunk c + 1's loads are in flight in registers while chunk c's MFMAs
// run (round 5: each chunk's loads used to wait behind the previous chunk's MFMAs — the distributed panel
// phase's row updates, 52 of 190 ms per rank at n = 50 000, R = 8); 32 more registers, still two
// workgroups per CU.
template <bool PIPE>
__global__ void __launch_bounds__(256, 2)
syrk64_sub_kernel(const double* __restrict__ U, int64_t ldu, int64_t c0, int64_t lim, double* __restrict__ C,
                  int64_t ldc, double* Ld, double* Dinv, int32_t* __restrict__ info,
                  int64_t fk0, int rowonly, int kchunks, ColKeep keep) {
  __shared__ __attribute__((aligned(16))) double As[64 * P64];
  __shared__ __attribute__((aligned(16))) double Bs[64 * P64];
  int64_t ti = 0, tj = blockIdx.x;  // rowonly: the first tile row only (the next panel's rows)
  if (!rowonly) tile_of(blockIdx.x, ti, tj);
  const bool diag = ti == tj;
  const int64_t i0 = c0 + ti * 64, j0 = c0 + tj * 64;
  // a distributed panel phase: only this rank's columns (and the group's area, the right-hand sides)
  if (rowonly && !col_kept(keep, j0)) return;  // (workgroup-uniform; block 0 is the group's area)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane >> 4, fc = lane & 15;
  const int64_t rlim = c0 + lim;
  const bool active = (i0 + wm * 32 < rlim) && (j0 + wn * 32 < rlim);
  d4 acc[2][2];
  if (active) {
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
      for (int q = 0; q < 2; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = i0 + wm * 32 + m * 16 + fr + 4 * r;
          const int64_t col = j0 + wn * 32 + q * 16 + fc;
          acc[m][q][r] = (row < rlim && col < rlim) ? C[row * ldc + col] : 0.0;
        }
  }
  // K = 64 kchunks: the chunks are staged one after the other (kchunks > 1 only for the row
  // updates that bring a later panel of a panel group up to date)
  const double* B = Bs;
  // thread t stages 16 bytes of rows (t >> 5) + 8 e, e < 8: one load instruction of a wave covers two whole
  // 512-byte rows (8 cache lines; 16 rows x 16 bytes per instruction left each line to 8 instructions — round
  // 5: 12 us per K = 64 chunk of the distributed row updates), and the LDS stores of a row are contiguous
  const int lrow = tid >> 5, lcol = 2 * (tid & 31);
  // all 16 loads in flight before the LDS stores (interleaving them with the diag-conditional stores
  // made the compiler wait for each load in turn)
  // (one 16-double vector each: as arrays carried across the chunk loop they went to scratch)
  typedef double d16 __attribute__((ext_vector_type(16)));
  d16 va, vb;
  auto load_chunk = [&](int c) {
    const double* sa = U + (c * 64 + lrow) * ldu + i0 + lcol;
    const double* sb = U + (c * 64 + lrow) * ldu + j0 + lcol;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const double2 x = *reinterpret_cast<const double2*>(sa + 8 * e * ldu);
      const double2 y = *reinterpret_cast<const double2*>(sb + 8 * e * ldu);
      va[2 * e] = x.x;
      va[2 * e + 1] = x.y;
      vb[2 * e] = y.x;
      vb[2 * e + 1] = y.y;
    }
  };
  load_chunk(0);
  for (int c = 0; c < kchunks; c++) {
    if (c > 0) __syncthreads();  // every wave is done with the previous chunk
#pragma unroll
    for (int e = 0; e < 8; e++) {  // (on diagonal tiles vb == va: storing it anyway keeps this branch-free)
      *reinterpret_cast<double2*>(&As[(lrow + 8 * e) * P64 + lcol]) = make_double2(va[2 * e], va[2 * e + 1]);
      *reinterpret_cast<double2*>(&Bs[(lrow + 8 * e) * P64 + lcol]) = make_double2(vb[2 * e], vb[2 * e + 1]);
    }
    __syncthreads();
    if (PIPE && c + 1 < kchunks) load_chunk(c + 1);  // in flight during this chunk's MFMAs
    if (active) {
#pragma unroll
      for (int ks = 0; ks < 16; ks++) {
        double af[2], bf[2];
#pragma unroll
        for (int m = 0; m < 2; m++) af[m] = -As[(ks * 4 + fr) * P64 + wm * 32 + m * 16 + fc];
#pragma unroll
        for (int q = 0; q < 2; q++) bf[q] = B[(ks * 4 + fr) * P64 + wn * 32 + q * 16 + fc];
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
          for (int q = 0; q < 2; q++)
            acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[q], acc[m][q], 0, 0, 0);
      }
    }
    if (!PIPE && c + 1 < kchunks) load_chunk(c + 1);
  }
  const bool factor_next = fk0 >= 0 && blockIdx.x == 0;
  if (!active && !factor_next) return;
#pragma unroll
  for (int m = 0; m < 2; m++)
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int64_t row = i0 + wm * 32 + m * 16 + fr + 4 * r;
        const int64_t col = j0 + wn * 32 + q * 16 + fc;
        if (active && row < rlim && col < rlim) C[row * ldc + col] = acc[m][q][r];
      }
  if (factor_next) {
    // this tile is the next panel's diagonal block: factor it straight from the accumulators
    __syncthreads();  // every wave is done reading As/Bs
    double* Us = As;  // pitch P64 == PS
    double* rinv = Bs;
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
      for (int q = 0; q < 2; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) Us[(wm * 32 + m * 16 + fr + 4 * r) * PS + wn * 32 + q * 16 + fc] = acc[m][q][r];
    __syncthreads();
    const int bad = factor_diag_block(Us, rinv, tid);
    if (tid == 0 && bad >= 0) atomicCAS(info, 0, (int32_t)(fk0 + bad + 1));
    store_factor(Us, rinv, Ld + fk0 * CNB, Dinv + (fk0 / 16) * 256, tid);
  }
}

// single-panel steps with 64x64-tile updates below this many trailing rows (GBM_UPD64_LIM,
// re-read at every solve so tests can force the grouped paths on small matrices)
static std::atomic<int64_t> g_small_lim{2048};
void chol_refresh_tuning() {
  const char* e = ::gbm::knob("GBM_UPD64_LIM");
  g_small_lim.store(e ? (int64_t)atoll(e) : (int64_t)2048, std::memory_order_relaxed);
}
int64_t chol_small_lim() { return g_small_lim.load(std::memory_order_relaxed); }

// Block row [k1, k1+64) only, k1 = k0 + 64 kch: C[k1 : k1+64, k1 : gdim] -= U[k0:k1, ·]ᵀ U[k0:k1, ·]
// (a later panel's rows of a panel group, brought up to date with the group's earlier panels so
// that the whole group shares one K = 64 g trailing update); the first workgroup factors the
// diagonal block at k1 afterwards.
int launch_chol_row_update(double* G, int64_t ldg, int64_t k0, int kch, int64_t gdim, double* Ld, double* Dinv,
                           int32_t* info, hipStream_t s, ColKeep keep) {
  const int64_t k1 = k0 + 64 * (int64_t)kch;
  const int64_t lim = gdim - k1;
  if (kch > 1)
    syrk64_sub_kernel<true><<<(unsigned)(lim / 64), 256, 0, s>>>(G + k0 * ldg, ldg, k1, lim, G, ldg, Ld, Dinv, info, k1,
                                                             1, kch, keep);
  else
    syrk64_sub_kernel<false><<<(unsigned)(lim / 64), 256, 0, s>>>(G + k0 * ldg, ldg, k1, lim, G, ldg, Ld, Dinv, info, k1,
                                                              1, kch, keep);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// Upper-Cholesky trailing update: C[k1:gdim, k1:gdim] (upper tiles) -= U[k0:k1, k1:]ᵀ U[k0:k1, k1:]
// with k1 = k0 + nb; the first workgroup then factors the diagonal block at next_k0 (if >= 0).
// 64x64 tiles (syrk64_sub_kernel) for single panels below chol_small_lim() trailing rows (more
// workgroups for the small trailing matrices of late panels), else the 128x128 tile kernel.
// Distributed (nranks > 1): this rank's tile columns in [col_lo, col_hi) and, when col_hi >= gdim,
// the right-hand sides (a launch grid over those columns only); the next diagonal block is factored
// after the ranks exchange its area (gbm_dev_chol_area_*).
int launch_chol_update(double* G, int64_t ldg, int64_t k0, int64_t nb, int64_t gdim, double* Ld, double* Dinv,
                       int32_t* info, int64_t next_k0, int rank, int nranks, hipStream_t s, int64_t col_lo,
                       int64_t col_hi, int64_t row_lo, int64_t row_hi) {
  const int64_t k1 = k0 + nb;
  const int64_t lim = gdim - k1;
  if (lim <= 0) return GBM_OK;
  TileOwner own;
  if (nranks > 1) {
    if ((k1 % BT) != 0 || nb == 64 || (col_lo % BT) != 0 || (row_lo % BT) != 0)
      return fail(GBM_E_ARG, "distributed Cholesky update: panel groups, column and row ranges on 128-column tiles");
    own.rank = rank;
    own.nranks = nranks;
    own.rhs_tile = (gdim - kRhsRows) / BT;
    const int64_t jlo = std::max(k1, col_lo) / BT;
    const int64_t jhi = col_hi >= gdim ? own.rhs_tile : std::min((col_hi + BT - 1) / BT, own.rhs_tile);  // regular only
    own.j_first = jlo + ((rank - jlo) % nranks + nranks) % nranks;
    own.ncols = own.j_first < jhi ? (jhi - own.j_first + nranks - 1) / nranks : 0;
    own.rhs = col_hi >= gdim ? 1 : 0;
    if (own.ncols + own.rhs == 0) return GBM_OK;
    // row tiles [ti0, ti1) of the update (rows [row_lo, row_hi) ∩ [k1, gdim))
    own.ti0 = (std::max(row_lo, k1) - k1) / BT;
    const int64_t ti1 = (std::min(row_hi, gdim) - k1 + BT - 1) / BT;
    if (ti1 <= own.ti0) return GBM_OK;
    const int64_t m = ti1 - own.ti0;
    syrk_kernel<kSub><<<dim3((unsigned)m, (unsigned)(own.ncols + own.rhs)), 256, 0, s>>>(
        G + k0 * ldg, ldg, nb, k1, lim, G, ldg, nullptr, 0, SliceBounds{}, Ld, Dinv, info, -1, own);
    GBM_LAUNCH_CHECK();
    return GBM_OK;
  }
  if (nb == 64 && lim <= chol_small_lim()) {
    const int64_t m = (lim + 63) / 64;
    syrk64_sub_kernel<false><<<(unsigned)(m * (m + 1) / 2), 256, 0, s>>>(G + k0 * ldg, ldg, k1, lim, G, ldg, Ld, Dinv, info,
                                                                  next_k0, 0, (int)(nb / 64), ColKeep{});
    GBM_LAUNCH_CHECK();
    return GBM_OK;
  }
  const int64_t m = (lim + BT - 1) / BT;
  const int64_t ntiles = m * (m + 1) / 2;
  syrk_kernel<kSub><<<(unsigned)ntiles, 256, 0, s>>>(G + k0 * ldg, ldg, nb, k1, lim, G, ldg, nullptr, ntiles, SliceBounds{}, Ld,
                                                     Dinv, info, next_k0, own);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// The helper stream of the forked edge kernel: one per device for the process (bounded, created
// on first use), with fork/join events made per call, so concurrent callers never share an event
// (two callers on one device only queue their edge kernels behind each other). No fork when the
// caller's stream belongs to another device than the current one.
struct AuxStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  ~AuxStream() {
    if (fork) (void)hipEventDestroy(fork);  // destruction is deferred until the event completes
    if (join) (void)hipEventDestroy(join);
  }
};
static int aux_stream(hipStream_t caller, AuxStream& a, bool* usable) {
  *usable = false;
  int dev = 0;
  GBM_HIP_TRY(hipGetDevice(&dev));
  if (caller) {
    int sdev = -1;
    if (hipStreamGetDevice(caller, &sdev) != hipSuccess) {
      (void)hipGetLastError();
      return GBM_OK;
    }
    if (sdev != dev) return GBM_OK;
  }
  static std::mutex mu;
  static std::map<int, hipStream_t> streams;
  {
    std::lock_guard<std::mutex> lock(mu);
    hipStream_t& hs = streams[dev];
    if (!hs) GBM_HIP_TRY(hipStreamCreateWithFlags(&hs, hipStreamNonBlocking));
    a.s = hs;
  }
  GBM_HIP_TRY(hipEventCreateWithFlags(&a.fork, hipEventDisableTiming));
  GBM_HIP_TRY(hipEventCreateWithFlags(&a.join, hipEventDisableTiming));
  *usable = true;
  return GBM_OK;
}

// workspace: [slabs or carry flags][edge partials][8 queue counters of the persistent launch, then (fused
// reduce) one ticket counter per tile]
static int64_t grm_counter_doubles(const GrmPlan& g) { return 4 + (g.sb.fuse ? (g.ntiles + 1) / 2 : 0); }
int64_t grm_workspace_bytes(int64_t n, int64_t p) {
  const GrmPlan g = plan(n, p);
  return (g.main_doubles + g.edge_doubles + grm_counter_doubles(g)) * (int64_t)sizeof(double);
}

static int check_grm_args(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg) {
  const int64_t npad = npad_of(n);
  if (!Zt || !G || p < 1 || n < 1 || ldz < npad || ldg < npad || (ldz & 1) || (ldg & 1))
    return fail(GBM_E_ARG, "gbm_dev_grm: bad arguments (need ldz, ldg >= npad(n), both even)");
  if (((uintptr_t)Zt & 15) != 0 || ((uintptr_t)G & 15) != 0)
    return fail(GBM_E_ARG, "gbm_dev_grm: Zt and G must be 16-byte aligned");
  return GBM_OK;
}

// stage 1: the MFMA SYRK (one partial tile per (slice, tile) into the workspace slabs, or the
// in-order carry into G)
int launch_grm_syrk(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg, void* ws,
                    int64_t ws_bytes, hipStream_t s, int accum = 0) {
  int rc = check_grm_args(Zt, ldz, p, n, G, ldg);
  if (rc != GBM_OK) return rc;
  const GrmPlan g = plan(n, p);
  SliceBounds sb = g.sb;
  sb.accum = accum;
  const int64_t need = (g.main_doubles + g.edge_doubles + grm_counter_doubles(g)) * (int64_t)sizeof(double);
  if (need > 0 && (!ws || ws_bytes < need))
    return fail(GBM_E_ARG, "gbm_dev_grm: workspace too small (" + std::to_string(ws_bytes) + " < " +
                               std::to_string(need) + ")");
  const unsigned grid = (unsigned)(g.sb.n * ((g.ntiles + 7) & ~(int64_t)7));
  if (g.sb.carry) GBM_HIP_TRY(hipMemsetAsync(ws, 0, (size_t)(g.ntiles + 1) * sizeof(int32_t), s));
  int32_t* ctr = reinterpret_cast<int32_t*>((double*)ws + g.main_doubles + g.edge_doubles);
  const int64_t lim = g.sb.er > 0 ? g.sb.e0 : n;  // with an edge, the tiles cover [0, e0)^2 exactly
  // the ragged-column kernel beside the persistent tiles: forked (before the tile launch) onto
  // the device's helper stream; its workgroups fit in the registers the two tile workgroups of a
  // CU leave free. Joined back before returning.
  AuxStream aux;
  AuxStream* ax = nullptr;
  if (g.edge_concurrent) {
    bool usable = false;
    rc = aux_stream(s, aux, &usable);
    if (rc != GBM_OK) return rc;
    if (usable) {
      ax = &aux;
      GBM_HIP_TRY(hipEventRecord(ax->fork, s));
      GBM_HIP_TRY(hipStreamWaitEvent(ax->s, ax->fork, 0));
    }
  }
  if (g.persist) {
    GBM_HIP_TRY(hipMemsetAsync(ctr, 0, (size_t)(8 + (g.sb.fuse ? g.ntiles : 0)) * sizeof(int32_t), s));
    const int64_t units = (int64_t)g.sb.n * g.ntiles;
    const unsigned pgrid = (unsigned)(units < resident_wgs() ? units : resident_wgs());
    if (g.sb.fuse)
      syrk_kernel<kPersistFused><<<pgrid, 256, 0, s>>>(Zt, ldz, p, 0, lim, G, ldg, (double*)ws, g.ntiles, sb, nullptr,
                                                       nullptr, ctr, -1, TileOwner{});
    else
      syrk_kernel<kPersist><<<pgrid, 256, 0, s>>>(Zt, ldz, p, 0, lim, G, ldg, (double*)ws, g.ntiles, sb, nullptr,
                                                  nullptr, ctr, -1, TileOwner{});
  } else {
    syrk_kernel<kSplit><<<grid, 256, 0, s>>>(Zt, ldz, p, 0, lim, G, ldg, (double*)ws, g.ntiles, sb, nullptr, nullptr,
                                             nullptr, -1, TileOwner{});
  }
  GBM_LAUNCH_CHECK();
  if (g.sb.er > 0) {
    const hipStream_t es = ax ? ax->s : s;
    const unsigned eg = (unsigned)((int64_t)g.sb.erb * g.sb.es);
    double* part = (double*)ws + g.sb.eslab_off;
    switch (g.sb.et) {
      case 1: grm_edge_kernel<1><<<eg, 256, 0, es>>>(Zt, ldz, p, g.sb, part); break;
      case 2: grm_edge_kernel<2><<<eg, 256, 0, es>>>(Zt, ldz, p, g.sb, part); break;
      case 3: grm_edge_kernel<3><<<eg, 256, 0, es>>>(Zt, ldz, p, g.sb, part); break;
      default: grm_edge_kernel<4><<<eg, 256, 0, es>>>(Zt, ldz, p, g.sb, part); break;
    }
    GBM_LAUNCH_CHECK();
    if (g.edge_concurrent) {
      // the edge columns of G are disjoint from the tiles: sum their partials here, on the helper
      // stream when there is one (launch_grm_reduce then skips them)
      grm_edge_reduce_kernel<<<(unsigned)((n * g.sb.er + 255) / 256), 256, 0, es>>>(part, n, g.sb, G, ldg, accum);
      GBM_LAUNCH_CHECK();
    }
    if (ax) {
      GBM_HIP_TRY(hipEventRecord(ax->join, ax->s));
      GBM_HIP_TRY(hipStreamWaitEvent(s, ax->join, 0));
    }
  }
  return GBM_OK;
}

// stage 2: sum the slice partials of each tile into G. In carry mode, read back the error cell
// of the inter-workgroup waits (tflags[ntiles]; set to −1 if a wait gave up) and fail loudly:
// a timed-out wait would otherwise leave a silently wrong G.
// With err_out (device int32) the carry mode's error cell is copied there instead (no host sync: a
// caller that queues several GRMs back to back checks them all at the end).
int launch_grm_reduce(int64_t n, int64_t p, double* G, int64_t ldg, const void* ws, hipStream_t s, int accum = 0,
                      int32_t* err_out = nullptr) {
  const GrmPlan g = plan(n, p);
  if (g.sb.n == 1 && g.sb.er == 0) return GBM_OK;
  if (!ws) return fail(GBM_E_ARG, "gbm_dev_grm_reduce: workspace required");
  if (g.sb.er > 0 && !g.edge_concurrent) {
    grm_edge_reduce_kernel<<<(unsigned)((n * g.sb.er + 255) / 256), 256, 0, s>>>((const double*)ws + g.sb.eslab_off, n,
                                                                                 g.sb, G, ldg, accum);
    GBM_LAUNCH_CHECK();
  }
  if (g.sb.n == 1 || g.sb.fuse) return GBM_OK;  // (fused: the tile kernel has summed the slabs)
  if (g.sb.carry && err_out) {
    GBM_HIP_TRY(hipMemcpyAsync(err_out, (const int32_t*)ws + g.ntiles, sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    return GBM_OK;
  }
  if (g.sb.carry) {
    int32_t err = 0;
    GBM_HIP_TRY(hipMemcpyAsync(&err, (const int32_t*)ws + g.ntiles, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    GBM_HIP_TRY(hipStreamSynchronize(s));
    if (err < 0)
      return fail(GBM_E_HIP, "GRM in-order carry accumulation: an inter-workgroup wait timed out (G is invalid)");
    return GBM_OK;
  }
  grm_slab_reduce_kernel<<<(unsigned)g.ntiles, 256, 0, s>>>((const double*)ws, g.ntiles, g.sb.n, G, ldg, accum);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

int launch_grm(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg, void* ws,
               int64_t ws_bytes, hipStream_t s, int accum, int32_t* err_out) {
  if (accum && !grm_can_accumulate(n, p)) return fail(GBM_E_ARG, "GRM: accumulation needs the slab split");
  int rc = launch_grm_syrk(Zt, ldz, p, n, G, ldg, ws, ws_bytes, s, accum);
  if (rc != GBM_OK) return rc;
  return launch_grm_reduce(n, p, G, ldg, ws, s, accum, err_out);
}

// G += the GRM of these loci is possible with several loci ranges: their slabs' reduce adds into G,
// or, in the in-order carry, range 0 adds G's tile. A single range stores straight into G.
bool grm_can_accumulate(int64_t n, int64_t p) {
  const GrmPlan g = plan(n, p);
  return g.sb.n > 1;
}

}  // namespace gbm

namespace gbm {
// Upper 128x128 tiles of G <-> a contiguous tile array (half the bytes of the npad x gdim rows):
// the form the multi-GPU all-reduce moves.
__global__ void __launch_bounds__(256) grm_pack_kernel(const double* __restrict__ G, int64_t ldg,
                                                       double* __restrict__ packed, int unpack) {
  const int64_t t = blockIdx.x;
  int64_t ti, tj;
  tile_of(t, ti, tj);
  double* pt = packed + t * (int64_t)(BT * BT);
  for (int e = threadIdx.x * 2; e < BT * BT; e += 512) {
    const int r = e / BT, c = e % BT;
    double* g = const_cast<double*>(G) + (ti * BT + r) * ldg + tj * BT + c;
    if (unpack)
      *reinterpret_cast<double2*>(g) = *reinterpret_cast<const double2*>(pt + e);
    else
      *reinterpret_cast<double2*>(pt + e) = *reinterpret_cast<const double2*>(g);
  }
}
}  // namespace gbm

extern "C" int64_t gbm_dev_grm_packed_size(int64_t n) {
  const int64_t nt = gbm::npad_of(n) / gbm::BT;
  return nt * (nt + 1) / 2 * gbm::BT * gbm::BT;
}

extern "C" int gbm_dev_grm_pack(const double* G, int64_t ldg, int64_t n, double* packed, void* stream) {
  if (!G || !packed || n < 1 || ldg < gbm::npad_of(n) || (ldg & 1)) return gbm::fail(GBM_E_ARG, "gbm_dev_grm_pack: bad arguments");
  const int64_t nt = gbm::npad_of(n) / gbm::BT;
  gbm::grm_pack_kernel<<<(unsigned)(nt * (nt + 1) / 2), 256, 0, (hipStream_t)stream>>>(G, ldg, packed, 0);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

extern "C" int gbm_dev_grm_unpack(const double* packed, int64_t n, double* G, int64_t ldg, void* stream) {
  if (!G || !packed || n < 1 || ldg < gbm::npad_of(n) || (ldg & 1)) return gbm::fail(GBM_E_ARG, "gbm_dev_grm_unpack: bad arguments");
  const int64_t nt = gbm::npad_of(n) / gbm::BT;
  gbm::grm_pack_kernel<<<(unsigned)(nt * (nt + 1) / 2), 256, 0, (hipStream_t)stream>>>(G, ldg, const_cast<double*>(packed), 1);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

extern "C" int64_t gbm_dev_grm_workspace(int64_t n, int64_t p) { return gbm::grm_workspace_bytes(n, p); }

extern "C" int gbm_dev_grm(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
                           void* workspace, int64_t ws_bytes, void* stream) {
  return gbm::launch_grm(Zt, ldz, p, n, G, ldg, workspace, ws_bytes, (hipStream_t)stream);
}

extern "C" int gbm_dev_grm_accumulate(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
                                      void* workspace, int64_t ws_bytes, void* stream) {
  if (!gbm::grm_can_accumulate(n, p))
    return gbm::fail(GBM_E_ARG, "gbm_dev_grm_accumulate: this (n, p) plans a single loci range (gbm_dev_grm_slices == 1); "
                                "use more loci per call");
  return gbm::launch_grm(Zt, ldz, p, n, G, ldg, workspace, ws_bytes, (hipStream_t)stream, 1);
}

extern "C" int gbm_dev_grm_syrk(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
                                void* workspace, int64_t ws_bytes, void* stream) {
  return gbm::launch_grm_syrk(Zt, ldz, p, n, G, ldg, workspace, ws_bytes, (hipStream_t)stream);
}

extern "C" int gbm_dev_grm_reduce(int64_t n, int64_t p, double* G, int64_t ldg, const void* workspace, void* stream) {
  if (!G || n < 1 || p < 1 || ldg < gbm::npad_of(n)) return gbm::fail(GBM_E_ARG, "gbm_dev_grm_reduce: bad arguments");
  return gbm::launch_grm_reduce(n, p, G, ldg, workspace, (hipStream_t)stream);
}

extern "C" int gbm_dev_grm_slices(int64_t n, int64_t p) {
  return gbm::plan(n, p).sb.n;
}

namespace gbm {
// a += b over n doubles (fixed order per element): the sum of two packed partial GRMs of SNP
// shards that live on the same device (capi.cpp), before the RCCL all-reduce across devices.
__global__ void __launch_bounds__(256) add_inplace_kernel(double* __restrict__ a, const double* __restrict__ b,
                                                          int64_t n) {
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2; i < n; i += (int64_t)gridDim.x * 512) {
    if (i + 1 < n) {
      double2 x = *reinterpret_cast<const double2*>(a + i);
      const double2 y = *reinterpret_cast<const double2*>(b + i);
      x.x += y.x;
      x.y += y.y;
      *reinterpret_cast<double2*>(a + i) = x;
    } else {
      a[i] += b[i];
    }
  }
}

int launch_add_inplace(double* a, const double* b, int64_t n, hipStream_t s) {
  if (n <= 0) return GBM_OK;
  const int64_t want = (n + 511) / 512;
  add_inplace_kernel<<<(unsigned)(want < 8192 ? want : 8192), 256, 0, s>>>(a, b, n);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// out[i, j] = inv_q * G[min(i,j), max(i,j)] for i, j < n (full symmetric export of the upper-stored GRM)
__global__ void __launch_bounds__(256) grm_export_kernel(const double* __restrict__ G, int64_t ldg, int64_t n,
                                                         double inv_q, double* __restrict__ out, int64_t ldo) {
  const int64_t i = blockIdx.x;
  for (int64_t j = threadIdx.x; j < n; j += 256)
    out[i * ldo + j] = inv_q * (j >= i ? G[i * ldg + j] : G[j * ldg + i]);
}

int launch_grm_export(const double* G, int64_t ldg, int64_t n, double inv_q, double* out, int64_t ldo, hipStream_t s) {
  grm_export_kernel<<<(unsigned)n, 256, 0, s>>>(G, ldg, n, inv_q, out, ldo);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}
}  // namespace gbm
