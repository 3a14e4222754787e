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
// Scheduling. Workgroups (one per CU) take tiles from one atomic counter in row-major order, except
// that each row's right neighbour (i, i + 1) comes before its diagonal tile (i, i). A tile waits
// only for tiles of earlier rows, for its row's diagonal tile (tiles right of the neighbour), or
// for the neighbour's partial (the diagonal tile): every one precedes it in that order and was
// therefore taken by a running workgroup, so the dependency chain always ends in a running
// workgroup, whatever the residency (one resident workgroup suffices): the launch cannot
// deadlock. Waits are bounded (~1 s, info = −1, as in chol_device.h).
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

#include "chol_device.h"

namespace gbm {

namespace {

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef unsigned int u2 __attribute__((ext_vector_type(2)));
constexpr int FT = 64;         // tile edge
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

// tile flags: kPartial = the accumulated (not yet solved) right neighbour of a diagonal tile,
// handed to the diagonal task; kFinal = the tile's U (or, on the diagonal, Ld + Dinv) is stored
constexpr int32_t kPartial = 1, kFinal = 2;
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
__device__ __forceinline__ bool wave_ready2(const int32_t* fa, const int32_t* fb, int lane) {
  int r = 0;
  if (lane == 0) r = (flag_set(fa) && flag_set(fb)) ? 1 : 0;
  return __builtin_amdgcn_readfirstlane(r) != 0;
}

// Upper Cholesky of the 64x64 block in X (LDS, pitch PS, upper part valid) by a 256-thread
// workgroup, together with the inverses of its four 16x16 diagonal blocks. Four 16-row leaves:
// wave 0 eliminates the leaf's rows over all remaining columns (lane l = column o + l) and, in
// lanes 0..15, carries identity columns through the same eliminations, so that column l of
// U_leaf⁻ᵀ (= row l of U_leaf⁻¹, the Dinv layout) comes out beside the factor and is stored
// straight to Dinv (sc1) and to Dl (LDS, same layout). Step c is split so that only its first two
// row updates are near the chain to the next pivot: rows c + 1, c + 2 are updated from v_readlane
// of U[c][c+1], U[c][c+2]; the rows beyond take U[c][·]
// from an LDS broadcast written in step c, read in step c + 1 and applied in step c + 2, so
// neither the LDS round trip nor those updates sit on the pivot chain.
// Between leaves all waves update the block's remaining upper 16x16 tiles by MFMA. Leaves U in X
// (zeros below the diagonal); bc = 48 doubles of LDS scratch. Returns the first failing column or -1.
__device__ __forceinline__ int factor_block_inv(double* X, double* bc, double* Dl, int tid,
                                                __amdgpu_buffer_rsrc_t rDi, uint32_t dinv_base,
                                                int64_t* tt = nullptr) {
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll 1
  for (int kb = 0; kb < 4; kb++) {
    const int o = kb * 16;
    if (wave == 0) {
      const int ncols = CNB - o;
      const int cc = o + (lane < ncols ? lane : 0);
      double x[16], y[16], b1[16], b2[16];
#pragma unroll
      for (int t = 0; t < 16; t++) {
        x[t] = X[(o + t) * PS + cc];
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
            y[c + d] = fma(-yc, u, y[c + d]);
          }
        __builtin_amdgcn_sched_barrier(0);
        // U[c − 1][·] (written last step) -> b1; this step's row -> LDS (three buffers: a row is
        // overwritten three steps after it was written, long after its reads completed)
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        if (c >= 1 && c + 2 < 16) {
#pragma unroll
          for (int t = c + 2; t < 16; t++) b1[t] = bc[((c - 1) % 3) * 16 + t];
        }
        if (c + 3 < 16 && lane < 16) bc[(c % 3) * 16 + lane] = lc;
        // step c − 2's updates of rows c + 1.. (rows c − 1 and c were its chain part)
        if (c >= 2) {
#pragma unroll
          for (int t = c + 1; t < 16; t++) {
            x[t] = fma(-l2, b2[t], x[t]);
            y[t] = fma(-m2, b2[t], y[t]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        l2 = l1;
        m2 = m1;
        l1 = lc;
        m1 = yc;
#pragma unroll
        for (int t = 0; t < 16; t++) b2[t] = b1[t];
      }
      if (tt) tt[kb] = (int64_t)__builtin_amdgcn_s_memrealtime();
      if (lane < ncols) {
#pragma unroll
        for (int t = 0; t < 16; t++) X[(o + t) * PS + cc] = (lane < 16 && t > lane) ? 0.0 : x[t];
      }
      if (lane < 16) {
        const uint32_t b = dinv_base + (uint32_t)((kb * 256 + lane * 16) * 8);
#pragma unroll
        for (int e = 0; e < 16; e += 2) {
          dbl2 v;
          v.x = y[e];
          v.y = y[e + 1];
          st2(rDi, b + e * 8, v);
          *reinterpret_cast<dbl2*>(&Dl[kb * 256 + lane * 16 + e]) = v;
        }
      }
    }
    __syncthreads();
    // update of the block's remaining upper 16x16 tiles (b <= a < m) by leaf kb's rows: the first
    // tile row (the next leaf's rows) by waves 1..m, then wave 0 goes on with the next leaf while
    // waves 1.. update the rest (done before the next leaf's closing barrier, i.e. before any
    // later leaf reads those rows)
    const int m = 3 - kb;  // remaining 16-blocks
    if (wave >= 1 && wave <= m) {
      const int c0 = o + 16 + (wave - 1) * 16;
      mfma_tile_sub_t(X, o + 16, c0, X, o + 16, X, c0, o, 4, lane);
    }
    __syncthreads();
    if (wave >= 1) {
      for (int t = wave - 1; t < m * (m - 1) / 2; t += 3) {
        int a = 1;
        while (a * (a + 1) / 2 <= t) a++;
        const int b = t - (a - 1) * a / 2 + 1;  // 1 <= b <= a: tile (row b, col a)
        const int r0 = o + 16 + b * 16, c0 = o + 16 + a * 16;
        mfma_tile_sub_t(X, r0, c0, X, r0, X, c0, o, 4, lane);
      }
    }
    if (tt && kb < 3) tt[4 + kb] = (int64_t)__builtin_amdgcn_s_memrealtime();
  }
  // (the lower parts of the diagonal 16x16 blocks hold leftovers of the MFMA updates; nothing
  // reads below the diagonal of a factored block)
  __syncthreads();
  const double dg = X[lane * PS + lane];
  const unsigned long long bm = __ballot(!(dg > 0.0) || !isfinite(dg));
  return bm ? (int)__builtin_ctzll(bm) : -1;
}

// task t (row-major over the upper tile triangle) -> tile (i, j)
__device__ __forceinline__ void task_tile(int t, int nbc, int& i, int& j) {
  auto start = [nbc](int r) { return r * nbc - r * (r - 1) / 2; };
  const double b = 2.0 * nbc + 1.0;
  int r = (int)((b - sqrt(b * b - 8.0 * (double)t)) * 0.5);
  if (r < 0) r = 0;
  while (r > 0 && start(r) > t) r--;
  while (r + 1 < nbc && start(r + 1) <= t) r++;
  i = r;
  j = r + (t - start(r));
  // within a row the right neighbour (i, i + 1) is dequeued before the diagonal tile (i, i), which
  // waits for the neighbour's partial: every wait then targets a task taken earlier
  if (i + 1 < nbc) {
    if (j == i) j = i + 1;
    else if (j == i + 1) j = i;
  }
}

// kTrace: per-task timestamps (s_memrealtime, 100 MHz) into trace[t * 24 ...] for the timeline tool
//
// Task kinds (tile (i, j)):
//   diagonal (i == j < nb): k-loop; U_ii = chol(A_ii) with the 16x16 inverses (Ld, Dinv); then the
//     right neighbour's U_i,i+1 = U_ii⁻ᵀ A_i,i+1 from the partial that the neighbour task handed
//     over (waves 1-3 fetch it while wave 0 factors), so that the next diagonal tile's last
//     update waits for one hand-off, not two; publishes (i, i) and (i, i+1) final.
//   right neighbour (j == i + 1): k-loop, then the accumulated tile is stored as a partial.
//   other (j > i + 1): k-loop; once (i, i) is final, U_ij = U_ii⁻ᵀ A_ij.
//   Schur (i == j == nb): k-loop; −WᵀW for the later kernels.
template <bool kTrace>
__global__ void __launch_bounds__(256, 1)
chol_flow_kernel(double* __restrict__ G, int64_t ld, int nbc, double* __restrict__ Ld, double* __restrict__ Dinv,
                 int32_t* __restrict__ queue, int32_t* __restrict__ flags, int32_t* __restrict__ info,
                 int64_t* __restrict__ trace) {
  // ≈ 90 KB: one workgroup per CU (the chain's serial steps then share no SIMD with other tiles)
  __shared__ __attribute__((aligned(16))) double X[FT * PS];
  __shared__ __attribute__((aligned(16))) double X2[FT * PS];
  __shared__ __attribute__((aligned(16))) double Dl[4 * 256];
  __shared__ double bcast[48];
  __shared__ int s_task;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int fr = lane >> 4, fc = lane & 15;
  const int nb = nbc - 1;  // diagonal tiles with a factor; tile (nb, nb) is the Schur block
  const int ntasks = nbc * (nbc + 1) / 2;
  const int64_t gbytes_rowblk = (int64_t)FT * ld * 8;
  const __amdgpu_buffer_rsrc_t rLd = rsrc(Ld, (int64_t)nb * FT * CNB * 8);
  const __amdgpu_buffer_rsrc_t rDi = rsrc(Dinv, (int64_t)nb * FT * 16 * 8);

  // U_ij in X (LDS) -> G upper (sc1: later tiles of this launch read it) ...
  auto store_upper = [&](const double* Xs, int64_t i0, int64_t j0) {
    const int row = tid >> 2, quarter = tid & 3;
    const __amdgpu_buffer_rsrc_t rG = rsrc(G + i0 * ld, gbytes_rowblk);
    const uint32_t base = (uint32_t)(((int64_t)row * ld + j0 + quarter * 16) * 8);
#pragma unroll
    for (int e = 0; e < 16; e += 2) st2(rG, base + e * 8, *reinterpret_cast<const dbl2*>(&Xs[row * PS + quarter * 16 + e]));
  };
  // ... and its transposed copy -> G lower (rows j0.., columns i0..; read only by the back
  // substitution / μ̂ kernels after this launch, so stored after the tile's flag)
  auto store_lower = [&](const double* Xs, int64_t i0, int64_t j0) {
    const int row = tid >> 2, quarter = tid & 3;
    double* dl = G + (j0 + row) * ld + i0 + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      dbl2 v;
      v.x = Xs[(quarter * 16 + e) * PS + row];
      v.y = Xs[(quarter * 16 + e + 1) * PS + row];
      *reinterpret_cast<dbl2*>(dl + e) = v;
    }
  };

  for (;;) {
    if (tid == 0) s_task = atomicAdd(queue, 1);
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    if (t >= ntasks) return;
    int i, j;
    task_tile(t, nbc, i, j);
    i = __builtin_amdgcn_readfirstlane(i);
    j = __builtin_amdgcn_readfirstlane(j);
    const bool diag = i == j;
    const bool nbr = j == i + 1;
    // the factorisation chain runs through the diagonal tiles and their right neighbours
    if (diag || nbr) __builtin_amdgcn_s_setprio(2);
    const int64_t i0 = (int64_t)i * FT, j0 = (int64_t)j * FT;
    int64_t tr[16] = {};
    if (kTrace) tr[0] = (int64_t)__builtin_amdgcn_s_memrealtime();

    // ---- accumulators = A_ij (interleaved wave tile: MFMA tile m holds rows 32wr + 2ρ + m,
    // tile q columns 32wc + 2γ + q, so a lane's two A (B) operands are one 16-byte load)
    d4 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int64_t row = i0 + 32 * wr + 2 * (fr + 4 * r) + m;
        const dbl2 v = *reinterpret_cast<const dbl2*>(G + row * ld + j0 + 32 * wc + 2 * fc);
        acc[m][0][r] = v.x;
        acc[m][1][r] = v.y;
      }

    // ---- A_ij −= Σ_k U_kiᵀ U_kj, 64-deep steps in two 32-deep halves (8 k-steps of 4); the next
    // half's loads are in flight while this one's MFMAs run. The lower quadrant of a diagonal (or
    // Schur) tile is never read: that wave skips the loop.
    if (i > 0 && !(diag && wr == 1 && wc == 0)) {
      const uint32_t offA = (uint32_t)(((int64_t)fr * ld + i0 + 32 * wr + 2 * fc) * 8);
      const uint32_t offB = (uint32_t)(((int64_t)fr * ld + j0 + 32 * wc + 2 * fc) * 8);
      const uint32_t kstep = (uint32_t)(4 * ld * 8);
      dbl2 a0[8], b0[8], a1[8], b1[8];
      auto issue = [&](dbl2(&A)[8], dbl2(&B)[8], int k, int h) {
        const __amdgpu_buffer_rsrc_t r = rsrc(G + (int64_t)k * FT * ld, gbytes_rowblk);
#pragma unroll
        for (int ks = 0; ks < 8; ks++) {
          const uint32_t so = (uint32_t)(h * 8 + ks) * kstep;
          A[ks] = ld2(r, offA, so);
          B[ks] = ld2(r, offB, so);
        }
      };
      auto mfma = [&](const dbl2(&A)[8], const dbl2(&B)[8]) {
#pragma unroll
        for (int ks = 0; ks < 8; ks++) {
          const double na0 = -A[ks].x, na1 = -A[ks].y;
          acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(na0, B[ks].x, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(na0, B[ks].y, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(na1, B[ks].x, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(na1, B[ks].y, acc[1][1], 0, 0, 0);
        }
      };
      auto fa = [&](int k) { return flags + (int64_t)k * nbc + i; };
      auto fb = [&](int k) { return flags + (int64_t)k * nbc + j; };
      wave_wait2(fa(0), fb(0), info, lane);
      issue(a0, b0, 0, 0);
      issue(a1, b1, 0, 1);
      for (int k = 0; k < i; k++) {
        mfma(a0, b0);
        const bool more = k + 1 < i;
        if (more) {
          wave_wait2(fa(k + 1), fb(k + 1), info, lane);
          issue(a0, b0, k + 1, 0);
        }
        mfma(a1, b1);
        if (more) issue(a1, b1, k + 1, 1);
      }
    }
    if (kTrace) tr[1] = (int64_t)__builtin_amdgcn_s_memrealtime();

    int32_t publish = kFinal;
    const double* low = nullptr;  // a solved tile whose lower copy is still to be stored
    int64_t lj0 = j0;
    if (nbr && i < nb) {
      // ---- right neighbour: hand the accumulated tile to the diagonal task (sc1, straight from
      // the accumulators into the tile's place in G; the diagonal task overwrites it with U)
      const __amdgpu_buffer_rsrc_t rG = rsrc(G + i0 * ld, gbytes_rowblk);
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int64_t row = 32 * wr + 2 * (fr + 4 * r) + m;
          dbl2 v;
          v.x = acc[m][0][r];
          v.y = acc[m][1][r];
          st2(rG, (uint32_t)((row * ld + j0 + 32 * wc + 2 * fc) * 8), v);
        }
      publish = kPartial;
    } else {
      // ---- accumulators -> X (natural layout)
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int row = 32 * wr + 2 * (fr + 4 * r) + m;
          dbl2 v;
          v.x = acc[m][0][r];
          v.y = acc[m][1][r];
          *reinterpret_cast<dbl2*>(&X[row * PS + 32 * wc + 2 * fc]) = v;
        }
      __syncthreads();
      if (kTrace) tr[2] = (int64_t)__builtin_amdgcn_s_memrealtime();

      if (diag && i < nb) {
        // ---- U_ii = chol(A_ii) -> Ld (row-major, zeros below), its 16x16 diagonal inverses ->
        // Dinv (and Dl)
        const int bad = factor_block_inv(X, bcast, Dl, tid, rDi, (uint32_t)((i0 / 16) * 256 * 8), kTrace ? tr + 6 : nullptr);
        if (tid == 0 && bad >= 0) atomicCAS(info, 0, (int32_t)(i0 + bad + 1));
        if (kTrace) tr[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
        // the neighbour's partial (its last update ran beside this factor; loads issued before the
        // Ld stores so that waiting for them does not wait for the stores)
        const int32_t* fn = flags + (int64_t)i * nbc + i + 1;
        wave_wait2(fn, fn, info, lane, kPartial);
        if (kTrace) tr[13] = (int64_t)__builtin_amdgcn_s_memrealtime();
        dbl2 pv[8];
        {
          const __amdgpu_buffer_rsrc_t rG = rsrc(G + i0 * ld, gbytes_rowblk);
#pragma unroll
          for (int q = 0; q < 8; q++) {
            const int e = tid + q * 256;
            pv[q] = ld2(rG, (uint32_t)(((int64_t)(e >> 5) * ld + j0 + FT + 2 * (e & 31)) * 8), 0);
          }
        }
        {
          // Ld: the six off-diagonal 16x16 blocks that the row's other solves read, write-through
          // now; the diagonal blocks (read only by later kernels) after the flags
          const int row = tid >> 2, quarter = tid & 3;
          const uint32_t base = (uint32_t)(((i0 + row) * CNB + quarter * 16) * 8);
          if (quarter > (row >> 4)) {
#pragma unroll
            for (int e = 0; e < 16; e += 2)
              st2(rLd, base + e * 8, *reinterpret_cast<const dbl2*>(&X[row * PS + quarter * 16 + e]));
          }
        }
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const int e = tid + q * 256;
          *reinterpret_cast<dbl2*>(&X2[(e >> 5) * PS + 2 * (e & 31)]) = pv[q];
        }
        __syncthreads();
        if (kTrace) tr[14] = (int64_t)__builtin_amdgcn_s_memrealtime();
        // ---- the right neighbour: U_i,i+1 = U_ii⁻ᵀ A_i,i+1 (all MFMA, operands in LDS); each
        // 16-row block of a wave's columns is stored (write-through) as soon as it is final, so
        // the hand-off's stores overlap the rest of the solve
        const __amdgpu_buffer_rsrc_t rN = rsrc(G + i0 * ld, gbytes_rowblk);
        panel_chunk_solve(
            X2, X, [&](int rb, int ks) { return Dl[rb * 256 + (ks * 4 + fr) * 16 + fc]; }, lane, wave,
            [&](int rb, const d4& a) {
#pragma unroll
              for (int r = 0; r < 4; r++)
                st1(rN, (uint32_t)(((int64_t)(rb * 16 + fr + 4 * r) * ld + j0 + FT + wave * 16 + fc) * 8), a[r]);
            });
        __syncthreads();
        if (kTrace) tr[15] = (int64_t)__builtin_amdgcn_s_memrealtime();
        low = X2;
        lj0 = j0 + FT;
      } else if (!diag) {
        // ---- U_ij = U_ii⁻ᵀ A_ij once U_ii is final. Operands of U_ii and its 16x16 inverses come
        // straight from the sc1-stored Ld / Dinv into registers; X (LDS) is solved in place:
        //   X_rb <- (D_rb⁻¹)ᵀ (X_rb − U[0:o, rb]ᵀ X[0:o]),  rb = 0..3, wave w on columns 16w..16w+15
        const int32_t* fd = flags + (int64_t)i * nbc + i;
        wave_wait2(fd, fd, info, lane);
        if (kTrace) tr[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
        double u[24], di[16];
        {
          int c = 0;
#pragma unroll
          for (int rb = 1; rb < 4; rb++)
#pragma unroll
            for (int ks = 0; ks < 4 * rb; ks++)
              u[c++] = ld1(rLd, (uint32_t)(((i0 + ks * 4 + fr) * CNB + rb * 16 + fc) * 8));
#pragma unroll
          for (int rb = 0; rb < 4; rb++)
#pragma unroll
            for (int ks = 0; ks < 4; ks++)
              di[rb * 4 + ks] = ld1(rDi, (uint32_t)(((i0 / 16) * 256 + rb * 256 + (ks * 4 + fr) * 16 + fc) * 8));
        }
        const int cw = wave * 16;
        int c = 0;
#pragma unroll
        for (int rb = 0; rb < 4; rb++) {
          const int o = rb * 16;
          if (rb > 0) {
            d4 s = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int ks = 0; ks < 4 * rb; ks++)
              s = __builtin_amdgcn_mfma_f64_16x16x4f64(u[c++], X[(ks * 4 + fr) * PS + cw + fc], s, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; r++) X[(o + fr + 4 * r) * PS + cw + fc] -= s[r];
          }
          d4 s = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ks = 0; ks < 4; ks++)
            s = __builtin_amdgcn_mfma_f64_16x16x4f64(di[rb * 4 + ks], X[(o + ks * 4 + fr) * PS + cw + fc], s, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; r++) X[(o + fr + 4 * r) * PS + cw + fc] = s[r];
        }
        __syncthreads();
        store_upper(X, i0, j0);
        low = X;
      } else {
        // ---- the Schur block −WᵀW (read by later kernels only)
        const int row = tid >> 2, quarter = tid & 3;
        double* d = G + (i0 + row) * ld + j0 + quarter * 16;
#pragma unroll
        for (int e = 0; e < 16; e += 2)
          *reinterpret_cast<dbl2*>(d + e) = *reinterpret_cast<const dbl2*>(&X[row * PS + quarter * 16 + e]);
      }
    }
    // ---- publish: every storing wave drains its write-through stores, then one flag store (a
    // diagonal task also publishes its right neighbour, whose U it stored)
    if (kTrace) tr[4] = (int64_t)__builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_store(flags + (int64_t)i * nbc + j, publish, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (diag && i < nb)
        __hip_atomic_store(flags + (int64_t)i * nbc + j + 1, kFinal, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (low) store_lower(low, i0, lj0);
    if (diag && i < nb) {
      const int row = tid >> 2, quarter = tid & 3;
      if (quarter == (row >> 4)) {
        double* d = Ld + (i0 + row) * CNB + quarter * 16;
#pragma unroll
        for (int e = 0; e < 16; e += 2) *reinterpret_cast<dbl2*>(d + e) = *reinterpret_cast<const dbl2*>(&X[row * PS + quarter * 16 + e]);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (kTrace && tid == 0) {
      tr[5] = (int64_t)__builtin_amdgcn_s_memrealtime();
      int64_t* o = trace + (int64_t)t * 24;
      o[0] = i;
      o[1] = j;
      o[2] = (int64_t)(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) & 7) /* XCC_ID */ * 1000 +
             (int64_t)blockIdx.x;
#pragma unroll
      for (int e = 0; e < 16; e++) o[3 + e] = tr[e];
    }
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

// bytes of the flag block (queue word padded to 16 B + one int32 flag per tile), a multiple of 16
int64_t chol_flow_flag_bytes(int64_t gdim) {
  const int64_t nbc = gdim / FT;
  return round_up(16 + nbc * nbc * 4, 16);
}

// n up to this many padded rows use the dataflow factorisation (GBM_CHOL_FLOW_MAX, re-read at
// every solve; 0 = always the launch-per-panel path)
bool chol_flow_enabled(int64_t npad) {
  const char* e = getenv("GBM_CHOL_FLOW_MAX");
  const int64_t lim = e ? (int64_t)atoll(e) : (int64_t)12288;  // n = 10 000: 10.1 vs 13.6 ms; n = 16 000: 37.2 vs 36.6
  return npad <= lim;
}

int launch_chol_flow(double* G, int64_t ldg, int64_t gdim, double* Ld, double* Dinv, void* flag_block, int32_t* info,
                     hipStream_t s) {
  const int64_t nbc = gdim / FT;
  const int64_t ntasks = nbc * (nbc + 1) / 2;
  if (nbc < 2 || (int64_t)FT * ldg * 8 > 0x7fffffff || nbc * nbc > 0x3fffffff)
    return fail(GBM_E_ARG, "dataflow Cholesky: matrix too large for 32-bit buffer offsets");
  GBM_HIP_TRY(hipMemsetAsync(flag_block, 0, (size_t)chol_flow_flag_bytes(gdim), s));
  // one workgroup per CU; GBM_CHOL_FLOW_WGS (re-read per solve) caps the grid: with 1 the whole
  // factorisation runs on one workgroup, which checks that no wait targets a later task
  const char* ew = getenv("GBM_CHOL_FLOW_WGS");
  const int64_t slots = ew && atoll(ew) > 0 ? atoll(ew) : flow_cus();
  const unsigned grid = (unsigned)(ntasks < slots ? ntasks : slots);
  int32_t* q = (int32_t*)flag_block;
  if (getenv("GBM_CHOL_FLOW_TRACE")) {
    // timing tool only: one record of 16 int64 per task, read back by gbm_debug_chol_flow_trace
    if (g_trace_cap < ntasks) {
      if (g_trace) (void)hipFree(g_trace);
      g_trace = nullptr;
      GBM_HIP_TRY(hipMalloc((void**)&g_trace, (size_t)ntasks * 192));
      g_trace_cap = ntasks;
    }
    g_trace_n = ntasks;
    chol_flow_kernel<true><<<grid, 256, 0, s>>>(G, ldg, (int)nbc, Ld, Dinv, q, q + 4, info, g_trace);
  } else {
    chol_flow_kernel<false><<<grid, 256, 0, s>>>(G, ldg, (int)nbc, Ld, Dinv, q, q + 4, info, nullptr);
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
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(host, g_trace, (size_t)n * 192, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}
