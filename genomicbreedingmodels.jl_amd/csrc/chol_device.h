// Device helpers shared by the Cholesky kernels (chol.hip) and the trailing-update kernels
// (grm.hip), which factor the next diagonal block in their first workgroup.
#pragma once
#include "gbm_internal.h"

namespace gbm {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int CNB = 64;        // Cholesky block (== kCholNB)
constexpr int PS = CNB + 16;   // LDS pitch of 64x64 images: fragment reads conflict-free

// Columns a rank computes in the panel phase of a distributed factorisation (chol.hip): its own
// 128-column tiles (J ≡ rank mod nranks), plus, on every rank, the columns left of keep_hi (the
// panel group's own diagonal area, which the group's later panels read) and the bordered
// right-hand sides from rhs0 on. nranks = 1: every column.
struct ColKeep {
  int32_t rank = 0, nranks = 1;
  int64_t keep_hi = 0, rhs0 = INT64_MAX;
};
__device__ __forceinline__ bool col_kept(const ColKeep& k, int64_t col) {
  return k.nranks == 1 || col < k.keep_hi || col >= k.rhs0 || (col / 128) % k.nranks == k.rank;
}

__device__ __forceinline__ double rsqrt_nr(double a) {  // v_rsq_f64 + one Newton step
  double y = __builtin_amdgcn_rsq(a);
  const double h = 0.5 * a * y;
  return y * fma(-h, y, 1.5);
}
__device__ __forceinline__ double rcp_nr(double a) {  // v_rcp_f64 + one Newton step
  double y = __builtin_amdgcn_rcp(a);
  const double e = fma(-a, y, 1.0);
  return fma(y, e, y);
}
__device__ __forceinline__ double readlane_d(double x, int lane) {
  union {
    double d;
    int i[2];
  } u;
  u.d = x;
  u.i[0] = __builtin_amdgcn_readlane(u.i[0], lane);
  u.i[1] = __builtin_amdgcn_readlane(u.i[1], lane);
  return u.d;
}

// Agent-scope (L2-bypassing) 64-bit accesses and a bounded flag wait, for data exchanged
// between workgroups of one launch (the 8 XCD L2s are not coherent with each other)
__device__ __forceinline__ double ld_agent(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}
// workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global
// loads and stores in flight (__syncthreads' workgroup fence would drain those too)
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// spin until *flag >= value; gives up (info = −1, every waiter then ends) after ~1 s — a wait
// that cannot end in a correct run must not hang the device
// The spin itself is relaxed (an acquire per iteration would invalidate this XCD's L2 every
// time, for every waiting wave); one acquire fence once the flag is seen.
// kAcquire = false: no fence at all — for a consumer that reads the payload only through sc1
// (L1-bypassing) buffer loads of write-through stores, as chol_flow.hip does; an agent acquire
// (the cache invalidate) costs ~1.7 µs per hand-off.
template <bool kAcquire = true>
__device__ __forceinline__ bool wait_flag(int32_t* flag, int32_t value, int32_t* info) {
  for (int64_t it = 0;; it++) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= value) {
      if constexpr (kAcquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      return true;
    }
    if ((it & 255) == 255) {
      if (__hip_atomic_load(info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 0) return false;
      if (it > (int64_t)1 << 22) {
        __hip_atomic_store(info, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Publish a flag after this workgroup's agent-scope (write-through) stores: wait for the
// stores to complete, barrier, then one relaxed agent-scope store. (A release store would first
// write back the XCD's whole L2 — every dirty tile of the launch — which costs several µs.)
__device__ __forceinline__ void publish_flag(int32_t* flag, int32_t value, int tid) {
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0): this wave's stores are done
  __syncthreads();
  if (tid == 0) __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// D(16x16 at (r0, c0) of dst) -= Σ_k S[kb + k][ra + row] T[kb + k][cb + col], k < 4*ksteps
// (all operands pitch PS)
__device__ __forceinline__ void mfma_tile_sub_t(double* dst, int r0, int c0, const double* S, int ra,
                                                const double* T, int cb, int kb, int ksteps, int lane) {
  d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
  const int fr = lane >> 4, fc = lane & 15;
  for (int ks = 0; ks < ksteps; ks++) {
    const double a = S[(kb + ks * 4 + fr) * PS + ra + fc];
    const double b = T[(kb + ks * 4 + fr) * PS + cb + fc];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) dst[(r0 + fr + 4 * r) * PS + c0 + fc] -= acc[r];
}

// rinv must hold CNB + 16 doubles (the last 16 are scratch).
// Upper Cholesky of the 64x64 block in Us (U-layout, pitch PS, upper part valid) by a
// 256-thread workgroup: four 16-row sub-panels, each a right-looking 16-step loop on wave 0
// (lane r owns column o + r; u_cs broadcast by v_readlane) followed by the MFMA update of the
// block's remaining upper 16x16 tiles on all waves. Leaves U in Us (zeros below the diagonal)
// and 1/U_ii in rinv. Returns, in every lane, the first failing column or -1.
__device__ __forceinline__ int factor_diag_block(double* Us, double* rinv, int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  for (int kb = 0; kb < 4; kb++) {
    const int o = kb * 16;
    if (wave == 0) {
      const int ncols = CNB - o;
      const int cc = o + (lane < ncols ? lane : 0);
      double x[16];
#pragma unroll
      for (int t = 0; t < 16; t++) x[t] = Us[(o + t) * PS + cc];
      // serial chain per step: readlane pivot → rsqrt → scale → row c of U through LDS (one
      // store, broadcast reads; LDS ops of one wave complete in order) → update. A
      // non-positive or non-finite pivot propagates NaN/≤0 onto the diagonal (checked below),
      // so the loop has no branches.
      double* bc = rinv + CNB;  // 16-double broadcast row
#pragma unroll
      for (int c = 0; c < 16; c++) {
        const double piv = readlane_d(x[c], c);
        const double lc = x[c] * rsqrt_nr(piv);  // lane c: piv/sqrt(piv) = U[c][c]
        if (lane < 16) bc[lane] = lc;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the row is in LDS before it is read
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int sidx = c + 1; sidx < 16; sidx++) x[sidx] = fma(-lc, bc[sidx], x[sidx]);
        x[c] = lc;
      }
      if (lane < ncols) {
#pragma unroll
        for (int t = 0; t < 16; t++) Us[(o + t) * PS + cc] = (lane < 16 && t > lane) ? 0.0 : x[t];
      }
      if (lane < 16) rinv[o + lane] = rcp_nr(x[lane & 15]);
    }
    __syncthreads();
    const int m = 3 - kb;  // remaining 16-blocks
    const int ntile = m * (m + 1) / 2;
    for (int t = wave; t < ntile; t += 4) {
      int a = 0;
      while ((a + 1) * (a + 2) / 2 <= t) a++;
      const int b = t - a * (a + 1) / 2;  // b <= a: tile (row b, col a)
      const int r0 = o + 16 + b * 16, c0 = o + 16 + a * 16;
      mfma_tile_sub_t(Us, r0, c0, Us, r0, Us, c0, o, 4, lane);
    }
    __syncthreads();
  }
  // the 16x16 lower parts of the trailing diagonal sub-blocks were touched by the MFMA updates
  for (int e = tid; e < CNB * CNB; e += 256) {
    const int r = e / CNB, c = e % CNB;
    if (c < r) Us[r * PS + c] = 0.0;
  }
  __syncthreads();
  // first failing column: U_cc = sqrt(pivot) is not a positive finite number
  const double dg = Us[lane * PS + lane];
  const bool bad = !(dg > 0.0) || !isfinite(dg);
  const unsigned long long m = __ballot(bad);
  return m ? (int)__builtin_ctzll(m) : -1;
}

// Write-through (sc1) buffer stores and sc1 (L1-bypassing) buffer loads: data handed between workgroups of one
// launch (chol_group_kernel; chol_flow.hip has its own copies). One resource per 64-row block of G keeps the
// byte offsets 32-bit.
typedef double wt_d2 __attribute__((ext_vector_type(2)));
typedef unsigned int wt_u4 __attribute__((ext_vector_type(4)));
typedef unsigned int wt_u2 __attribute__((ext_vector_type(2)));
constexpr int kWtSc1 = 16;  // buffer instruction aux bits: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ wt_d2 wt_ld2(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(wt_d2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, kWtSc1));
}
__device__ __forceinline__ double wt_ld1(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, 0, kWtSc1));
}
__device__ __forceinline__ void wt_st2(__amdgpu_buffer_rsrc_t r, uint32_t voff, wt_d2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(wt_u4, v), r, (int)voff, 0, kWtSc1);
}
__device__ __forceinline__ void wt_st1(__amdgpu_buffer_rsrc_t r, uint32_t voff, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(wt_u2, v), r, (int)voff, 0, kWtSc1);
}

// Store a factored block: Ld_blk (64x64 row-major, upper, zeros below) and the inverses of its
// four 16x16 diagonal sub-blocks Dinv_blk[w][i][j] = (D_w⁻¹)[i][j] (upper). Wave w computes D_w⁻¹
// column by column (lane j < 16), the dot products split over 2 partial sums.
// st_ld(e, v): Ld_blk[e..e+1] = v (e even); st_di(e, x): Dinv_blk[e] = x.
template <typename StLd, typename StDi>
__device__ __forceinline__ void store_factor_with(const double* Us, const double* rinv, int tid, StLd st_ld,
                                                  StDi st_di) {
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int k = 0; k < 8; k++) {  // the block is contiguous: a wave instruction stores 1 KB
    const int e = 2 * tid + 512 * k;
    st_ld(e, *reinterpret_cast<const wt_d2*>(&Us[(e >> 6) * PS + (e & 63)]));
  }
  const int o = wave * 16;
  const int j = lane & 15;
  double x[16];
#pragma unroll
  for (int i = 15; i >= 0; i--) {
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int k = i + 1; k < 16; k += 2) {
      p0 = fma(Us[(o + i) * PS + o + k], x[k], p0);
      if (k + 1 < 16) p1 = fma(Us[(o + i) * PS + o + k + 1], x[k + 1], p1);
    }
    x[i] = (i <= j) ? (((i == j) ? 1.0 : 0.0) - (p0 + p1)) * rinv[o + i] : 0.0;
  }
  if (lane < 16) {
#pragma unroll
    for (int i = 0; i < 16; i++) st_di(wave * 256 + i * 16 + j, x[i]);
  }
}
__device__ __forceinline__ void store_factor(const double* Us, const double* rinv, double* Ld_blk,
                                             double* Dinv_blk, int tid) {
  store_factor_with(
      Us, rinv, tid, [&](int e, wt_d2 v) { *reinterpret_cast<wt_d2*>(Ld_blk + e) = v; },
      [&](int e, double x) { Dinv_blk[e] = x; });
}

// Block forward substitution of one 64-column chunk X (LDS, pitch PS) of a panel row, given the
// factored diagonal block U_kk (LDS Us, pitch PS) and the inverses of its four 16x16 diagonal
// sub-blocks: load(rb, ks) returns this lane's MFMA A operand Dinv_rb[ks*4 + (lane>>4)][lane&15]
// (rb, ks compile-time after unrolling, so a register array can back it):
//   X_rb <- (D_rb⁻¹)ᵀ (X_rb − U[0:o, rb]ᵀ X[0:o])  for the 16-row blocks rb = 0..3.
// Wave w owns columns 16w..16w+15 of the chunk. All MFMA, no serial chain.
// emit(rb, acc): block row rb of the wave's 16 columns is final (acc[r] = X[16 rb + fr + 4 r][cw + fc]),
// e.g. to store it while the later block rows are solved
template <typename LoadDi, typename Emit>
__device__ __forceinline__ void panel_chunk_solve(double* X, const double* Us, LoadDi load, int lane, int wave,
                                                  Emit emit) {
  const int fr = lane >> 4, fc = lane & 15;
  const int cw = wave * 16;
#pragma unroll
  for (int rb = 0; rb < 4; rb++) {
    const int o = rb * 16;
    if (rb > 0) mfma_tile_sub_t(X, o, cw, Us, o, X, cw, 0, rb * 4, lane);  // X_rb -= U[0:o,rb]ᵀ X[0:o]
    // X_rb = (D_rb⁻¹)ᵀ X_rb : A[i][k] = Dinv[k][i], B[k][j] = X[o+k][cw+j]
    d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 4; ks++) {
      const double a = load(rb, ks);
      const double bv = X[(o + ks * 4 + fr) * PS + cw + fc];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) X[(o + fr + 4 * r) * PS + cw + fc] = acc[r];
    emit(rb, acc);
  }
}
template <typename LoadDi>
__device__ __forceinline__ void panel_chunk_solve(double* X, const double* Us, LoadDi load, int lane, int wave) {
  panel_chunk_solve(X, Us, load, lane, wave, [](int, const d4&) {});
}

}  // namespace gbm
