// GBLUP solve: upper Cholesky V = UᵀU of the bordered matrix (row-major, upper triangle stored)
//
//        [ V    R ]      V = G/q + λI  (npad x npad; padding rows/cols = identity)
//   M =  [ Rᵀ   0 ]      R = [1, y_1, ..., y_t, 0...]  (npad x 64, extra columns)
//
// Right-looking blocked factorisation over the first npad rows, panel height NB = 64:
//   panel k:  U_kk = chol(A_kk)ᵀ (64x64), U_k,J = U_kk⁻ᵀ A_k,J for every column block J > k —
//             including the R columns, which turns them into W = U⁻ᵀR = L⁻¹R (the forward
//             substitution is fused into the factorisation);
//   update k: A_IJ -= U_kIᵀ U_kJ (I <= J) — the same fp64-MFMA SYRK kernel as the GRM
//             (k-major operands: the panel rows), see grm.hip syrk_kernel<kSub>.
// The bottom-right block ends as −WᵀW, so 1ᵀV⁻¹1 and 1ᵀV⁻¹y come out of the factorisation
// (GLS intercept of reference src/gwas.jl:596-597 with X = 1). Then a = U⁻¹(W_y − μ̂ W_1) by
// a blocked back substitution, and GEBV = μ̂ + (y − μ̂) − λa (= μ̂ + G a).
// The reference inverts V with pinv/SVD (src/gwas.jl:472,595); for λ > 0 V is SPD and the
// Cholesky solution is the same up to rounding.
#include <cstdlib>
#include <string>

#include "chol_device.h"

namespace gbm {

constexpr int NB = kCholNB;  // 64
constexpr int MAXRHS = 63;

int launch_chol_update(double* G, int64_t ldg, int64_t k0, int64_t nb, int64_t gdim, double* Ld, double* Dinv,
                       int32_t* info, int64_t next_k0, int rank, int nranks, hipStream_t s, int64_t col_lo = 0,
                       int64_t col_hi = INT64_MAX, int64_t row_lo = 0, int64_t row_hi = INT64_MAX);
int launch_chol_row_update(double* G, int64_t ldg, int64_t k0, int kch, int64_t gdim, double* Ld, double* Dinv,
                           int32_t* info, hipStream_t s, ColKeep keep = ColKeep{});
int64_t chol_small_lim();
void chol_refresh_tuning();
int64_t chol_flow_flag_bytes(int64_t gdim);
bool chol_flow_enabled(int64_t npad);
int launch_chol_flow(double* G, int64_t ldg, int64_t gdim, double* Ld, double* Dinv, void* flag_block, int32_t* info,
                     hipStream_t s);

// ---- V = G/q + λI (upper part), padding = identity, bordered R columns -----------------------
// keep (a distributed factorisation, nranks > 1): only the columns the rank reads before an exchange
// overwrites them — its own 128-column tiles, the first panel group's area (< keep_hi) and the
// right-hand sides; the other columns keep G until the exchanges bring their owners' rows.
__global__ void __launch_bounds__(256) prepare_v_kernel(double* __restrict__ G, int64_t ld, int64_t n,
                                                        int64_t npad, int64_t gdim, double inv_q,
                                                        const int64_t* __restrict__ q_dev, double lambda,
                                                        const double* __restrict__ Y, int64_t ldy, int64_t nrhs,
                                                        int32_t* __restrict__ info, ColKeep keep) {
  const int64_t i = blockIdx.x;  // row
  if (i == 0 && threadIdx.x == 0) *info = 0;
  if (q_dev) inv_q = 1.0 / (double)(*q_dev);
  double* row = G + i * ld;
  const int64_t jbeg = (i / NB) * NB;  // from the start of the diagonal block
  for (int64_t j = jbeg + threadIdx.x; j < gdim; j += 256) {
    if (keep.nranks > 1 && !col_kept(keep, j)) continue;
    double v = 0.0;
    if (i < npad) {
      if (j < i) v = 0.0;
      else if (j < npad) v = (i < n && j < n) ? row[j] * inv_q + (i == j ? lambda : 0.0) : (i == j ? 1.0 : 0.0);
      else if (i < n) {
        const int64_t t = j - npad;
        v = t == 0 ? 1.0 : (t <= nrhs ? Y[(t - 1) * ldy + i] : 0.0);
      }
    }
    row[j] = v;
  }
}

// ---- a diagonal block on its own: the first one, and in a distributed factorisation the first of
// each panel group after the area exchange (otherwise the previous trailing update factors it) ---
__global__ void __launch_bounds__(256) factor_diag_kernel(const double* __restrict__ G, int64_t ld, int64_t k,
                                                          double* __restrict__ Ld, double* __restrict__ Dinv,
                                                          int32_t* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) double Us[CNB * PS];
  __shared__ double rinv[CNB + 16];
  const int tid = threadIdx.x;
  {
    const int row = tid >> 2, quarter = tid & 3;
    const double* sa = G + (k + row) * ld + k + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2)
      *reinterpret_cast<double2*>(&Us[row * PS + quarter * 16 + e]) = *reinterpret_cast<const double2*>(sa + e);
  }
  __syncthreads();
  const int bad = factor_diag_block(Us, rinv, tid);
  if (tid == 0 && bad >= 0) atomicCAS(info, 0, (int32_t)(k + bad + 1));
  store_factor(Us, rinv, Ld + k * CNB, Dinv + (k / 16) * 256, tid);
}

// ---- strips of a distributed factorisation: rows [r0, r0 + rows) x the 128-column tiles
// J in [r0/128, npad/128) that one rank owns (J ≡ owner mod nranks), packed [m][row][128] with
// m < cnt = ⌈(npad/128 − r0/128)/nranks⌉ (the rank's m-th tile J = J0 + ((owner − J0) mod nranks)
// + m·nranks; absent tiles past the end are zero-filled). unpack: every rank's pack of an
// all-gather, written back into G.
// Grid (⌈rows/4⌉, cnt, unpack ? nranks : 1): a workgroup moves four 1 KB tile rows of one rank's tile m
// (round 5: a flat grid-stride loop with 64-bit divisions per element moved the 50 MB pack of a 16-panel
// group at 0.34 TB/s).
__global__ void __launch_bounds__(256) chol_strip_kernel(double* __restrict__ G, int64_t ld, int64_t r0,
                                                         int64_t rows, int64_t J0, int64_t Jend, int64_t cnt,
                                                         int owner, int nranks, double* __restrict__ buf,
                                                         int unpack) {
  const int src = unpack ? (int)blockIdx.z : owner;
  const int64_t m = blockIdx.y;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int c2 = threadIdx.x & 63;
  if (row >= rows) return;
  const int64_t r = (m * rows + row) * 64 + c2;  // double2 index in the rank's pack
  double2* b2 = reinterpret_cast<double2*>(buf) + (unpack ? (int64_t)src * cnt * rows * 64 + r : r);
  const int j0 = (int)J0;
  const int64_t J = J0 + ((src - j0) % nranks + nranks) % nranks + m * nranks;
  if (J >= Jend) {
    if (!unpack) *b2 = make_double2(0.0, 0.0);
    return;
  }
  double2* g2 = reinterpret_cast<double2*>(G + (r0 + row) * ld + J * 128) + c2;
  if (unpack)
    *g2 = *b2;
  else
    *b2 = *g2;
}

// ---- panel k: U_k,J = U_kk⁻ᵀ A_k,J for the column chunks J > k ----------------------------------
// U_kk arrives factored (Ld) together with the inverses of its four 16x16 diagonal sub-blocks
// (Dinv), so the block forward substitution is all MFMA, no serial chain:
//   X_rb <- (D_rb⁻¹)ᵀ (X_rb − U[0:o, rb]ᵀ X[0:o])  for 16-row blocks rb = 0..3.
// Wave w owns columns 16w..16w+15 of the chunk, so the four waves never touch each other's data.
// The solved chunk is also written transposed into the (otherwise unused) lower triangle: L = Uᵀ
// row-major, so the back substitution and the μ̂ kernel read coalesced rows. Those entries are
// never overwritten later: every later trailing update covers only rows/cols >= its own origin.
// keep: in a distributed factorisation's panel phase, only the chunks of this rank's columns (the
// others arrive through the group's row exchange, chol_lower_copy_kernel adds their lower copy).
__global__ void __launch_bounds__(256) chol_panel_kernel(double* __restrict__ G, int64_t ld, int64_t k0,
                                                         const double* __restrict__ Ld,
                                                         const double* __restrict__ Dinv, ColKeep keep) {
  __shared__ __attribute__((aligned(16))) double Us[CNB * PS];
  __shared__ __attribute__((aligned(16))) double X[CNB * PS];
  __shared__ __attribute__((aligned(16))) double Di[4 * 256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t jx = k0 + ((int64_t)blockIdx.x + 1) * CNB;
  if (!col_kept(keep, jx)) return;  // (workgroup-uniform)
  // rows (tid >> 5) + 8 e, 16 bytes at column 2 (tid & 31): one wave instruction = two whole 512-byte rows
  const int lrow = tid >> 5, lcol = 2 * (tid & 31);
  {
    const double* sl = Ld + (k0 + lrow) * CNB + lcol;
    const double* sx = G + (k0 + lrow) * ld + jx + lcol;
    double2 vl[8], vx[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      vl[e] = *reinterpret_cast<const double2*>(sl + 8 * e * CNB);
      vx[e] = *reinterpret_cast<const double2*>(sx + 8 * e * ld);
    }
#pragma unroll
    for (int e = 0; e < 8; e++) {
      *reinterpret_cast<double2*>(&Us[(lrow + 8 * e) * PS + lcol]) = vl[e];
      *reinterpret_cast<double2*>(&X[(lrow + 8 * e) * PS + lcol]) = vx[e];
    }
    const double* sd = Dinv + (k0 / 16) * 256;
    *reinterpret_cast<double2*>(&Di[tid * 2]) = *reinterpret_cast<const double2*>(sd + tid * 2);
    *reinterpret_cast<double2*>(&Di[512 + tid * 2]) = *reinterpret_cast<const double2*>(sd + 512 + tid * 2);
  }
  __syncthreads();
  panel_chunk_solve(X, Us, [&](int rb, int ks) { return Di[rb * 256 + (ks * 4 + (lane >> 4)) * 16 + (lane & 15)]; },
                    lane, wave);
  __syncthreads();
  {
    double* dx = G + (k0 + lrow) * ld + jx + lcol;
#pragma unroll
    for (int e = 0; e < 8; e++)
      *reinterpret_cast<double2*>(dx + 8 * e * ld) = *reinterpret_cast<const double2*>(&X[(lrow + 8 * e) * PS + lcol]);
    const int row = tid >> 2, quarter = tid & 3;
    double* dl = G + (jx + row) * ld + k0 + quarter * 16;
#pragma unroll
    for (int e = 0; e < 16; e += 2)
      *reinterpret_cast<double2*>(dl + e) =
          make_double2(X[(quarter * 16 + e) * PS + row], X[(quarter * 16 + e + 1) * PS + row]);
  }
}

// ---- the transposed lower copy L = Uᵀ of a panel group's rows [r0, r0 + 64 g) for the column chunks
// another rank solved (received by the group's row exchange): one 64x64 block per workgroup, through
// LDS, so both the reads of U and the writes of L are coalesced rows. Chunks this rank kept (keep:
// its own, the group's area, the right-hand sides) were written by its chol_panel_kernel.
__global__ void __launch_bounds__(256) chol_lower_copy_kernel(double* __restrict__ G, int64_t ld, int64_t r0,
                                                              int64_t npad, ColKeep keep) {
  __shared__ double T[CNB][CNB + 1];
  const int64_t rb = blockIdx.y;                               // panel of the group
  const int64_t prow = r0 + rb * CNB;                          // its first row
  const int64_t jx = prow + ((int64_t)blockIdx.x + 1) * CNB;  // chunk right of its diagonal block
  if (jx >= npad || col_kept(keep, jx)) return;
  // rows (tid >> 5) + 8 e, 16 bytes at column 2 (tid & 31): each wave instruction reads / writes two whole rows
  const int tid = threadIdx.x, lrow = tid >> 5, lcol = 2 * (tid & 31);
  const double* su = G + (prow + lrow) * ld + jx + lcol;
  double2 v[8];
#pragma unroll
  for (int e = 0; e < 8; e++) v[e] = *reinterpret_cast<const double2*>(su + 8 * e * ld);
#pragma unroll
  for (int e = 0; e < 8; e++) {
    T[lrow + 8 * e][lcol] = v[e].x;
    T[lrow + 8 * e][lcol + 1] = v[e].y;
  }
  __syncthreads();
  double* dl = G + (jx + lrow) * ld + prow + lcol;
#pragma unroll
  for (int e = 0; e < 8; e++)
    *reinterpret_cast<double2*>(dl + 8 * e * ld) = make_double2(T[lcol][lrow + 8 * e], T[lcol + 1][lrow + 8 * e]);
}

// ---- a panel group's panel phase in ONE launch (round 5) -----------------------------------------
// The rows [k0, k0 + 64 g) of a panel group, for every column chunk right of the group's first
// diagonal block that the rank keeps, are the left-looking block forward substitution
//   A_jc −= Σ_{i<j} U_ijᵀ U_ic  (64-deep steps in i order),  then  U_jc = U_jj⁻ᵀ A_jc  (j < c)
//   or, on the area's diagonal (j = c), U_cc = chol(A_cc) → Ld, Dinv,
// the same arithmetic as the chain of g panel launches and g − 1 row-update launches it replaces
// (whose per-launch latency made the panel phase ~1.35 ms per 16-panel group at n = 50 000). One
// workgroup per column chunk walks its rows j = 0, 1, …; the area's chunks (c = 1 … g − 1: their
// tiles U_ij and U_jj are the other chunks' operands) publish a progress flag per row, the others
// wait for those flags only. Area chunk c keeps A_cc − Σ U_icᵀU_ic up to date after each of its
// rows, so its diagonal step is only the factor. Workgroups take their chunk from a ticket in
// dispatch order and wait only for smaller tickets: no deadlock whatever the residency. U tiles,
// Ld and Dinv handed between workgroups go through write-through stores and sc1 loads (no cache
// invalidate); flags as in chol_device.h (bounded waits, info = −1).
struct GroupCols {
  int32_t g = 0, nranks = 1;
  int64_t a0 = 0;       // first chunk right of the area
  int64_t n_own = 0;    // kept regular chunks right of the area
  int64_t J_first = 0;  // nranks > 1: the rank's first 128-column tile at or right of chunk a0
  int64_t rhs0 = 0, n_rhs = 0;  // the right-hand-side chunks
};

// Two workgroups per CU's worth of registers and at most 88 KB of LDS: a workgroup fits beside one of the
// trailing update's (72 KB), which the distributed solve runs concurrently (look-ahead).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) chol_group_kernel(double* __restrict__ G, int64_t ld, int64_t k0, GroupCols gc,
                                                            double* __restrict__ Ld, double* __restrict__ Dinv,
                                                            int32_t* __restrict__ prog, int32_t* __restrict__ info) {
  // staging of the update steps (As, Bs) | the solve (X, Us) | the diagonal step (rinv, Us): X aliases As, Us
  // aliases Bs, rinv lies in X's rows 1-2 (only used on the diagonal step); the three shared words sit in row 0's
  // padding columns (64-79 of every pitch-PS row are never touched). 80 KB: two workgroups per CU.
  __shared__ __attribute__((aligned(16))) double lds[2 * CNB * PS];
  int32_t* const sw = reinterpret_cast<int32_t*>(lds + CNB);
  int32_t& s_tk = sw[0];
  int32_t& s_seen = sw[1];
  int32_t& s_ok = sw[2];
  double* const As = lds;
  double* const Bs = lds + CNB * PS;
  double* const X = lds;
  double* const Us = lds + CNB * PS;
  double* const rinv = lds + PS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, fr = lane >> 4, fc = lane & 15;
  if (tid == 0) s_tk = atomicAdd(&prog[0], 1);
  __syncthreads();
  const int64_t b = s_tk;
  const int g = gc.g;
  const bool area = b < g - 1;
  const int c = area ? (int)b + 1 : g;  // area column, relative to the group
  int64_t chunk;
  if (area) {
    chunk = k0 / CNB + c;
  } else if (b - (g - 1) < gc.n_own) {
    const int64_t m = b - (g - 1);
    chunk = gc.nranks == 1 ? gc.a0 + m : 2 * (gc.J_first + (m >> 1) * gc.nranks) + (m & 1);
  } else {
    chunk = gc.rhs0 + (b - (g - 1) - gc.n_own);
  }
  const int64_t jx = chunk * CNB;
  const int jlast = area ? c : g - 1;
  // 16 bytes at column lcol of rows lrow + 8 e (e < 8): a wave instruction covers two whole 512-byte rows
  const int lrow = tid >> 5, lcol = 2 * (tid & 31);
  const int64_t slab = (int64_t)CNB * ld * 8;  // bytes of a 64-row block of G
  auto quad = [&](int m, int q, int r, int64_t& row, int64_t& col) {
    row = wm * 32 + m * 16 + fr + 4 * r;
    col = wn * 32 + q * 16 + fc;
  };
  d4 acc[2][2], accd[2][2];
  if (area) {  // A_cc, brought up to date row by row
    const double* src = G + (k0 + (int64_t)c * CNB) * ld + jx;
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
      for (int q = 0; q < 2; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          int64_t row, col;
          quad(m, q, r, row, col);
          accd[m][q][r] = src[row * ld + col];
        }
  }
  typedef double d16 __attribute__((ext_vector_type(16)));
  for (int j = 0; j <= jlast; j++) {
    const int64_t r0 = k0 + (int64_t)j * CNB;
    const __amdgpu_buffer_rsrc_t rrow = wt_rsrc(G + r0 * ld, slab);
    if (area && j == c) {
      // the diagonal block: store it updated (as the row updates did), factor it, publish Ld and Dinv
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            int64_t row, col;
            quad(m, q, r, row, col);
            G[(r0 + row) * ld + jx + col] = accd[m][q][r];
            Us[row * PS + col] = accd[m][q][r];
          }
      __syncthreads();
      const int bad = factor_diag_block(Us, rinv, tid);
      if (tid == 0 && bad >= 0) atomicCAS(info, 0, (int32_t)(r0 + bad + 1));
      const __amdgpu_buffer_rsrc_t rL = wt_rsrc(Ld + r0 * CNB, CNB * CNB * 8);
      const __amdgpu_buffer_rsrc_t rD = wt_rsrc(Dinv + (r0 / 16) * 256, 1024 * 8);
      store_factor_with(
          Us, rinv, tid, [&](int e, wt_d2 v) { wt_st2(rL, (uint32_t)(e * 8), v); },
          [&](int e, double x) { wt_st1(rD, (uint32_t)(e * 8), x); });
      publish_flag(&prog[c], j + 1, tid);
      break;
    }
    // acc = A_jc (written by earlier launches only)
    {
      const double* src = G + r0 * ld + jx;
#pragma unroll
      for (int m = 0; m < 2; m++)
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            int64_t row, col;
            quad(m, q, r, row, col);
            acc[m][q][r] = src[row * ld + col];
          }
    }
    // progress of area column j (row i final: prog[j] >= i + 1; its diagonal: >= j + 1). Column 0 is the
    // group's first diagonal block, factored before the launch. Workgroup-uniform.
    int seen = j == 0 ? 1 : 0;
    auto need = [&](int32_t v) -> bool {
      if (seen >= v) return true;
      __syncthreads();  // s_seen / s_ok are rewritten below
      if (tid == 0) {
        s_ok = wait_flag<false>(&prog[j], v, info) ? 1 : 0;
        s_seen = __hip_atomic_load(&prog[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      seen = s_seen;
      return s_ok != 0;
    };
    if (j > 0) {
      // acc −= Σ_{i<j} U_ijᵀ U_ic, staged through LDS; step i + 1's loads are in flight during step i's MFMAs
      d16 va, vb;
      auto load_step = [&](int i) {
        const __amdgpu_buffer_rsrc_t rk = wt_rsrc(G + (k0 + (int64_t)i * CNB) * ld, slab);
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const int64_t rowoff = (int64_t)(lrow + 8 * e) * ld;
          const wt_d2 x = wt_ld2(rk, (uint32_t)((rowoff + r0 + lcol) * 8));
          const wt_d2 y = wt_ld2(rk, (uint32_t)((rowoff + jx + lcol) * 8));
          va[2 * e] = x.x;
          va[2 * e + 1] = x.y;
          vb[2 * e] = y.x;
          vb[2 * e + 1] = y.y;
        }
      };
      if (!need(1)) return;
      load_step(0);
      for (int i = 0; i < j; i++) {
        if (i > 0) __syncthreads();  // every wave is done with step i − 1
#pragma unroll
        for (int e = 0; e < 8; e++) {
          *reinterpret_cast<wt_d2*>(&As[(lrow + 8 * e) * PS + lcol]) = (wt_d2){va[2 * e], va[2 * e + 1]};
          *reinterpret_cast<wt_d2*>(&Bs[(lrow + 8 * e) * PS + lcol]) = (wt_d2){vb[2 * e], vb[2 * e + 1]};
        }
        __syncthreads();
        if (i + 1 < j) {
          if (!need(i + 2)) return;
          load_step(i + 1);
        }
#pragma unroll
        for (int ks = 0; ks < 16; ks++) {
          double af[2], bf[2];
#pragma unroll
          for (int m = 0; m < 2; m++) af[m] = -As[(ks * 4 + fr) * PS + wm * 32 + m * 16 + fc];
#pragma unroll
          for (int q = 0; q < 2; q++) bf[q] = Bs[(ks * 4 + fr) * PS + wn * 32 + q * 16 + fc];
#pragma unroll
          for (int m = 0; m < 2; m++)
#pragma unroll
            for (int q = 0; q < 2; q++) acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[q], acc[m][q], 0, 0, 0);
        }
      }
      if (!need(j + 1)) return;  // U_jj factored
    }
    __syncthreads();  // As / Bs are free: X and Us alias them
    double di[16];
    // X = A_jc, Us = U_jj (Ld); di = this lane's MFMA operands of its 16x16 diagonal inverses (Dinv)
#pragma unroll
    for (int m = 0; m < 2; m++)
#pragma unroll
      for (int q = 0; q < 2; q++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          int64_t row, col;
          quad(m, q, r, row, col);
          X[row * PS + col] = acc[m][q][r];
        }
    {
      const __amdgpu_buffer_rsrc_t rL = wt_rsrc(Ld + r0 * CNB, CNB * CNB * 8);
      const __amdgpu_buffer_rsrc_t rD = wt_rsrc(Dinv + (r0 / 16) * 256, 1024 * 8);
      wt_d2 u[8];
#pragma unroll
      for (int k = 0; k < 8; k++) u[k] = wt_ld2(rL, (uint32_t)((2 * tid + 512 * k) * 8));
#pragma unroll
      for (int rb = 0; rb < 4; rb++)
#pragma unroll
        for (int ks = 0; ks < 4; ks++) di[rb * 4 + ks] = wt_ld1(rD, (uint32_t)((rb * 256 + (ks * 4 + fr) * 16 + fc) * 8));
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int e = 2 * tid + 512 * k;
        *reinterpret_cast<wt_d2*>(&Us[(e >> 6) * PS + (e & 63)]) = u[k];
      }
    }
    __syncthreads();
    panel_chunk_solve(X, Us, [&](int rb, int ks) { return di[rb * 4 + ks]; }, lane, wave);
    __syncthreads();
    // U_jc -> G (write-through: later steps of this and other workgroups read it), its transpose -> the lower copy
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int row = lrow + 8 * e;
      wt_st2(rrow, (uint32_t)(((int64_t)row * ld + jx + lcol) * 8), *reinterpret_cast<const wt_d2*>(&X[row * PS + lcol]));
    }
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int row = lrow + 8 * e;
      *reinterpret_cast<double2*>(G + (jx + row) * ld + r0 + lcol) = make_double2(X[lcol * PS + row], X[(lcol + 1) * PS + row]);
    }
    if (area) {
      // A_cc −= U_jcᵀ U_jc (from LDS), then row j of this column is published
#pragma unroll
      for (int ks = 0; ks < 16; ks++) {
        double af[2], bf[2];
#pragma unroll
        for (int m = 0; m < 2; m++) af[m] = -X[(ks * 4 + fr) * PS + wm * 32 + m * 16 + fc];
#pragma unroll
        for (int q = 0; q < 2; q++) bf[q] = X[(ks * 4 + fr) * PS + wn * 32 + q * 16 + fc];
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
          for (int q = 0; q < 2; q++) accd[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[q], accd[m][q], 0, 0, 0);
      }
      publish_flag(&prog[c], j + 1, tid);
    } else {
      __syncthreads();  // X is read before the next step's staging overwrites it
    }
  }
}

// ---- inverses of all diagonal blocks U_bb (one workgroup per block, all in parallel) --------
// lane = column j: X[i][j] = (δ_ij − Σ_{k>i} U[i][k] X[k][j]) / U[i][i], the dot product split
// over 4 partial sums so the dependent chain is a quarter of its length.
__global__ void __launch_bounds__(64) diag_inverse_kernel(const double* __restrict__ Ld, double* __restrict__ Linv) {
  __shared__ double Ub[NB][NB + 1];
  const int lane = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * NB;
  for (int r = 0; r < NB; r++) Ub[r][lane] = Ld[(b0 + r) * NB + lane];
  __syncthreads();
  double x[NB];
#pragma unroll
  for (int i = NB - 1; i >= 0; i--) {
    double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
    for (int k = i + 1; k < NB; k += 4) {
      p0 = fma(Ub[i][k], x[k], p0);
      if (k + 1 < NB) p1 = fma(Ub[i][k + 1], x[k + 1], p1);
      if (k + 2 < NB) p2 = fma(Ub[i][k + 2], x[k + 2], p2);
      if (k + 3 < NB) p3 = fma(Ub[i][k + 3], x[k + 3], p3);
    }
    x[i] = (i <= lane) ? (((lane == i) ? 1.0 : 0.0) - ((p0 + p1) + (p2 + p3))) * rcp_nr(Ub[i][i]) : 0.0;
  }
#pragma unroll
  for (int i = 0; i < NB; i++) Linv[(b0 + i) * NB + lane] = x[i];
}

// ---- μ̂ and the back-substitution right-hand sides w_t = W_{1+t} − μ̂_t W_0 ---------------------
// W_s is column npad + s of the factored rows (row npad + s of the lower copy); the Schur
// block holds −W_sᵀW_t.
// (also clears the per-block flags of back_solve_kernel, which runs next)
__global__ void __launch_bounds__(256) gls_mu_kernel(const double* __restrict__ G, int64_t ld, int64_t npad,
                                                     int64_t nrhs, double* __restrict__ W, int64_t lda,
                                                     double* __restrict__ mu, int32_t* __restrict__ flags) {
  const int64_t t = blockIdx.y;
  const double c11 = -G[npad * ld + npad];
  const double c1y = -G[npad * ld + npad + 1 + t];
  const double m = c1y / c11;
  if (blockIdx.x == 0 && threadIdx.x == 0) mu[t] = m;
  if (t == 0)
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < npad / NB; i += (int64_t)gridDim.x * 256) flags[i] = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < lda; i += (int64_t)gridDim.x * 256)
    W[t * lda + i] = i < npad ? G[(npad + 1 + t) * ld + i] - m * G[npad * ld + i] : 0.0;
}

// ---- REML ingredients of a finished solve (one workgroup) ------------------------------------
// terms[0] = logdet V = 2 Σ_i log U_ii (from the factored diagonal blocks in Ld; padding rows are
// identity and add log 1 = 0); terms[1] = 1ᵀV⁻¹1; terms[2 + 2t] = 1ᵀV⁻¹y_t; terms[3 + 2t] =
// y_tᵀV⁻¹y_t — the bordered Schur block ends as −WᵀW with W = U⁻ᵀ[1, y].
__global__ void __launch_bounds__(256) gblup_terms_kernel(const double* __restrict__ G, int64_t ld, int64_t npad,
                                                          int64_t nrhs, const double* __restrict__ Ld,
                                                          double* __restrict__ terms) {
  __shared__ double red[256];
  double sacc = 0.0;
  for (int64_t r = threadIdx.x; r < npad; r += 256) sacc += log(Ld[r * NB + (r % NB)]);
  red[threadIdx.x] = sacc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    terms[0] = 2.0 * red[0];
    terms[1] = -G[npad * ld + npad];
  }
  for (int64_t t = threadIdx.x; t < nrhs; t += 256) {
    terms[2 + 2 * t] = -G[npad * ld + npad + 1 + t];
    terms[3 + 2 * t] = -G[(npad + 1 + t) * ld + npad + 1 + t];
  }
}

constexpr int RC = 4;  // right-hand sides per chunk of the back substitution

// ---- sync-free blocked back substitution: one workgroup per PAIR of 64-blocks, flags between them ----
// U a = w with U's off-diagonal blocks read from the lower copy L = Uᵀ (coalesced along the rows
// i of a block) and the diagonal blocks through their inverses (Linv). Workgroup w owns the blocks
// bh = nb − 1 − 2w and bl = bh − 1: it folds in U_bh,c a_c and U_bl,c a_c for every c > bh as soon as
// block c publishes a_c (flag[c] = pass), then a_bh = U_bh,bh⁻¹ (w_bh − Σ_c U_bh,c a_c), publishes it, folds
// U_bl,bh a_bh from LDS (its L rows loaded before any wait) and solves a_bl. So the chain crosses
// workgroups once per two blocks (round 5: one workgroup per block made it one cross-workgroup hand-off,
// ≈ 1.3 µs, per 64 rows: 183 µs at C2); the per-row sums run in the same order as with one workgroup
// per block (c = nb − 1 .. b + 1, the same partials), so a is bit-identical. A workgroup only waits for
// lower-numbered workgroups, which the in-order dispatch has already placed, so the chain cannot
// deadlock whatever the residency. a travels through agent-scope (L2-bypassing) atomic stores and sc1
// loads: the 8 XCD L2s are not coherent with each other. A wait that does not end (it cannot in a
// correct run) gives up after ~1 s and reports info = −1 instead of hanging.
__global__ void __launch_bounds__(256) back_solve_kernel(const double* __restrict__ G, int64_t ld,
                                                         const double* __restrict__ Linv, int64_t nb,
                                                         const double* __restrict__ W, double* A,
                                                         int64_t lda, int64_t nrhs, int32_t* __restrict__ flags,
                                                         int32_t* __restrict__ info) {
  __shared__ double part[4][RC][NB];
  __shared__ double rl[RC][NB];
  __shared__ double ah[RC][NB];  // a_bh (the stored values), for the low block's last fold
  __shared__ int ok_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t bh = nb - 1 - 2 * (int64_t)blockIdx.x, bl = bh - 1;
  const bool lo = bl >= 0;
  const int64_t h0 = bh * NB, l0 = bl * NB;
  const int j0 = wave * 16;  // this wave's 16 of the 64 block columns
  const int64_t a_bytes = nrhs * lda * 8;
  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc(A, (short)0, (int)(a_bytes < 0x7fffffff ? a_bytes : 0x7fffffff), 0x00020000);
  double uh[16], ul[16], lb[16];  // (U_bh⁻¹)[lane][j0 + jj], (U_bl⁻¹)[lane][j0 + jj], L[h0 + j0 + jj][l0 + lane]
#pragma unroll
  for (int jj = 0; jj < 16; jj++) {
    uh[jj] = Linv[(h0 + lane) * NB + j0 + jj];
    ul[jj] = lo ? Linv[(l0 + lane) * NB + j0 + jj] : 0.0;
    lb[jj] = lo ? G[(h0 + j0 + jj) * ld + l0 + lane] : 0.0;
  }
  if (tid == 0) ok_s = 1;
  int32_t pass = 0;
  // a_b = U_bb⁻¹ (w_b − Σ acc) for the RHS chunk, through LDS; `out` also keeps the stored values
  // (w: wave 0's right-hand sides of the block, loaded before the chunk's waits so that no global load
  // latency sits on the chain; the barriers hand over LDS only)
  auto solve_block = [&](int64_t b0, const double (&ui)[16], const double (&acc)[RC], const double (&w)[RC], int tc,
                         int64_t t0, double (*out)[NB]) {
#pragma unroll
    for (int t = 0; t < RC; t++) part[wave][t][lane] = acc[t];
    lds_sync();
    if (wave == 0)
#pragma unroll
      for (int t = 0; t < RC; t++)
        if (t < tc) rl[t][lane] = w[t] - (((part[0][t][lane] + part[1][t][lane]) + part[2][t][lane]) + part[3][t][lane]);
    lds_sync();
    for (int t = 0; t < tc; t++) {
      double s = 0.0;
#pragma unroll
      for (int jj = 0; jj < 16; jj++) s = fma(ui[jj], rl[t][j0 + jj], s);
      part[wave][t][lane] = s;
    }
    lds_sync();
    if (wave == 0)
      for (int t = 0; t < tc; t++) {
        const double v = ((part[0][t][lane] + part[1][t][lane]) + part[2][t][lane]) + part[3][t][lane];
        st_agent(A + (t0 + t) * lda + b0 + lane, v);
        if (out) out[t][lane] = v;
      }
  };
  for (int64_t t0 = 0; t0 < nrhs; t0 += RC) {
    pass++;
    const int tc = (int)(nrhs - t0 < RC ? nrhs - t0 : RC);
    double acch[RC] = {0.0, 0.0, 0.0, 0.0}, accl[RC] = {0.0, 0.0, 0.0, 0.0};
    double wh[RC] = {0.0, 0.0, 0.0, 0.0}, wl[RC] = {0.0, 0.0, 0.0, 0.0};
    if (wave == 0)
#pragma unroll
      for (int t = 0; t < RC; t++)
        if (t < tc) {
          wh[t] = W[(t0 + t) * lda + h0 + lane];
          if (lo) wl[t] = W[(t0 + t) * lda + l0 + lane];
        }
    bool ok = true;
    for (int64_t c = nb - 1; c > bh && ok; c--) {
      double lh[16], ll[16];  // L[64c + j0 + jj][b0 + lane] = U[b0 + lane][64c + j0 + jj]
      const double* lp = G + (c * NB + j0) * ld + lane;
#pragma unroll
      for (int jj = 0; jj < 16; jj++) {
        lh[jj] = lp[(int64_t)jj * ld + h0];
        ll[jj] = lo ? lp[(int64_t)jj * ld + l0] : 0.0;
      }
      if (lane == 0) ok = wait_flag<false>(&flags[c], pass, info);
      ok = __builtin_amdgcn_readfirstlane((int)ok) != 0;
      // a_c was written through (agent-scope stores) before its flag was published; it is read
      // with sc1 buffer loads (all 16 in flight at once), so no agent acquire — an L1/L2
      // invalidate of ~1.7 µs that sat on the chain at every block — is needed. The wavefront
      // fence only keeps the compiler from hoisting the loads above the poll.
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int t = 0; t < tc; t++) {
        const uint32_t voff = (uint32_t)(((t0 + t) * lda + c * NB + j0) * 8);
        double av[16];
#pragma unroll
        for (int jj = 0; jj < 16; jj++)
          av[jj] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rA, (int)(voff + jj * 8), 0, 16));
        double sh = 0.0, sl = 0.0;
#pragma unroll
        for (int jj = 0; jj < 16; jj++) {
          sh = fma(lh[jj], av[jj], sh);
          sl = fma(ll[jj], av[jj], sl);
        }
        acch[t] += sh;
        accl[t] += sl;
      }
    }
    if (!ok) ok_s = 0;
    solve_block(h0, uh, acch, wh, tc, t0, lo ? ah : nullptr);
    // publish a_bh once its write-through stores are complete (a failed wait still publishes, so the
    // workgroups behind it end quickly); the barrier inside also makes ah visible to every wave
    publish_flag(&flags[bh], pass, tid);
    if (lo) {
      for (int t = 0; t < tc; t++) {
        double sl = 0.0;
#pragma unroll
        for (int jj = 0; jj < 16; jj++) sl = fma(lb[jj], ah[t][j0 + jj], sl);
        accl[t] += sl;
      }
      lds_sync();  // every wave has read ah and part before solve_block rewrites part
      solve_block(l0, ul, accl, wl, tc, t0, nullptr);
      publish_flag(&flags[bl], pass, tid);
    }
    if (!ok_s) return;
    lds_sync();  // ah / part / rl are rewritten by the next chunk
  }
}

// ---- GEBV = μ̂ + (y − μ̂) − λ a ------------------------------------------------------------
__global__ void __launch_bounds__(256) gebv_kernel(const double* __restrict__ Y, int64_t ldy, int64_t n,
                                                   const double* __restrict__ A, double* __restrict__ gebv,
                                                   int64_t lda, const double* __restrict__ mu, double lambda) {
  const int64_t t = blockIdx.y;
  const double m = mu[t];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < lda; i += (int64_t)gridDim.x * 256)
    gebv[t * lda + i] = i < n ? m + (Y[t * ldy + i] - m) - lambda * A[t * lda + i] : 0.0;
}

}  // namespace gbm

using namespace gbm;

extern "C" int64_t gbm_dev_npad(int64_t n) { return npad_of(n); }
extern "C" int64_t gbm_dev_gdim(int64_t n) { return gdim_of(n); }
// scratch: the factored 64x64 diagonal blocks (npad x 64), their inverses (npad x 64) and the
// inverses of their 16x16 diagonal sub-blocks (npad x 16)
// + one int32 flag per 64-block (back_solve_kernel), then (16-byte aligned) the dataflow
// factorisation's queue word and per-tile flags (chol_flow.hip)
static int64_t flow_block_offset(int64_t n) { return round_up(npad_of(n) * (2 * NB + 16) + npad_of(n) / NB / 2 + 1, 2); }
static int64_t solve_ws_doubles(int64_t n) { return flow_block_offset(n) + chol_flow_flag_bytes(gdim_of(n)) / 8; }
extern "C" int64_t gbm_dev_solve_workspace(int64_t n, int64_t nrhs) {
  (void)nrhs;
  return solve_ws_doubles(n) * (int64_t)sizeof(double);
}

namespace {

struct SolveWs {
  double *Ld, *Linv, *Dinv;
  int32_t* flags;
  void* flow;
};
SolveWs solve_ws(void* workspace, int64_t npad) {
  SolveWs w;
  w.Ld = (double*)workspace;
  w.Linv = w.Ld + npad * NB;
  w.Dinv = w.Linv + npad * NB;
  w.flags = reinterpret_cast<int32_t*>(w.Dinv + npad * 16);
  w.flow = (double*)workspace + flow_block_offset(npad);
  return w;
}

int check_solve_args(const double* G, int64_t ldg, int64_t n, const int32_t* info, const void* workspace,
                     int64_t ws_bytes, const char* who) {
  if (!G || !info || n < 1 || ldg < gdim_of(n) || (ldg & 1) || ((uintptr_t)G & 15))
    return fail(GBM_E_ARG, std::string(who) + ": bad arguments (G 16-byte aligned, even ldg >= gdim(n))");
  if (!workspace || ws_bytes < solve_ws_doubles(n) * (int64_t)sizeof(double) || ((uintptr_t)workspace & 15))
    return fail(GBM_E_ARG, std::string(who) + ": workspace too small (see gbm_dev_solve_workspace)");
  return GBM_OK;
}

// Remaining rows (64 kb .. gdim) at or below which the launch-per-panel path hands the rest of the
// factorisation to ONE dataflow launch on the trailing sub-matrix (chol_flow.hip: the remainder is itself a
// bordered matrix, the right-hand sides its last tile column). GBM_CHOL_TAIL_FLOW, re-read per call; by
// default 8192 when the whole matrix was too large for the dataflow launch (npad > 12 288), else 0 (off).
// Never the whole matrix (kb > 0).
static int64_t tail_flow_rows(int64_t npad) {
  const char* e = ::gbm::knob("GBM_CHOL_TAIL_FLOW");
  if (e) return (int64_t)atoll(e);
  return npad > 12288 ? 8192 : 0;
}
static bool tail_flow_at(int64_t kb, int64_t npad, int64_t gdim) {
  return kb > 0 && kb < npad / NB && gdim - kb * NB <= tail_flow_rows(npad);
}

// Panels per group of the factorisation step at 64-block kb: groups of g panels share one K = 64g
// trailing update (HBM/MALL-bound at K = 64, balanced at K = 128, MFMA-bound at K = 256). The
// thresholds are read at every call, so tests can force the grouped paths on small matrices.
// At the dataflow tail (tail_flow_at): every remaining panel, one group.
int group_size(int64_t kb, int64_t nb, int64_t gdim) {
  if (tail_flow_at(kb, nb * NB, gdim)) return (int)(nb - kb);
  auto lim = [](const char* name, int64_t dflt) {
    const char* e = ::gbm::knob(name);
    return e ? (int64_t)atoll(e) : dflt;
  };
  // 4-panel groups while the trailing matrix exceeds 8192 rows; 8-panel (K = 512) above 8192 and
  // 16-panel (K = 1024) above 16384: n = 50 000 solve 798 -> 746 -> 735 ms
  const int64_t g4 = lim("GBM_CHOL_G4_LIM", 8192), g8 = lim("GBM_CHOL_G8_LIM", 8192),
                g16 = lim("GBM_CHOL_G16_LIM", 16384);
  const int64_t k0 = kb * NB;
  if (g16 >= 0 && kb + 16 < nb && gdim - (k0 + 16 * NB) > g16) return 16;
  if (g8 >= 0 && kb + 8 < nb && gdim - (k0 + 8 * NB) > g8) return 8;
  if (g4 >= 0 && kb + 4 < nb && gdim - (k0 + 4 * NB) > g4) return 4;
  if (kb + 2 < nb && gdim - (k0 + 2 * NB) > chol_small_lim()) return 2;
  return 1;
}

int solve_prepare(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev, double lambda,
                  const double* Y, int64_t ldy, int64_t nrhs, int32_t* info, void* workspace, hipStream_t s,
                  bool factor_first = true, ColKeep keep = ColKeep{}) {
  const int64_t npad = npad_of(n), gdim = gdim_of(n);
  const SolveWs w = solve_ws(workspace, npad);
  chol_refresh_tuning();
  prepare_v_kernel<<<(unsigned)gdim, 256, 0, s>>>(G, ldg, n, npad, gdim, inv_q, q_dev, lambda, Y, ldy, nrhs, info,
                                                  keep);
  GBM_LAUNCH_CHECK();
  if (!factor_first) return GBM_OK;
  factor_diag_kernel<<<1, 256, 0, s>>>(G, ldg, 0, w.Ld, w.Dinv, info);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// GBM_CHOL_GROUP_KERNEL (re-read per group, default 1): a panel group's panel phase as one
// chol_group_kernel launch; 0: the chain of panel and row-update launches
static bool group_kernel_enabled() {
  const char* e = ::gbm::knob("GBM_CHOL_GROUP_KERNEL");
  return !e || atoi(e) != 0;
}

// The panel phase of the group at 64-block kb (its diagonal block already factored): the group's
// rows solved for every kept column chunk — one chol_group_kernel launch for g > 1 (default), or the
// chain of the first panel, then per later panel a row update (K = 64 j, factoring its diagonal
// block) and its panel. The trailing update (solve_group_update) follows.
// keep (distributed panel phase, nranks > 1): this rank's columns, the group's diagonal area and the
// right-hand sides only.
int solve_group_panels(double* G, int64_t ldg, int64_t n, int64_t kb, ColKeep keep, int32_t* info, void* workspace,
                       hipStream_t s, int64_t* g_out) {
  const int64_t npad = npad_of(n), gdim = gdim_of(n), nb = npad / NB;
  const SolveWs w = solve_ws(workspace, npad);
  const int64_t k0 = kb * NB;
  if (tail_flow_at(kb, npad, gdim))
    return fail(GBM_E_ARG, "gbm_dev_chol_group_panels: the dataflow tail (GBM_CHOL_TAIL_FLOW) runs as gbm_dev_chol_group");
  const int g = group_size(kb, nb, gdim);
  if (keep.nranks > 1) {
    if (g < 2 || (k0 % 128) != 0)
      return fail(GBM_E_ARG, "gbm_dev_chol_group_panels: a distributed step needs a panel group of >= 2 panels on a "
                             "128-row boundary (finish the tail with gbm_dev_chol_group, nranks = 1)");
    keep.keep_hi = k0 + g * NB;
    keep.rhs0 = npad;
  }
  if (g_out) *g_out = g;
  if (g > 1 && group_kernel_enabled()) {
    // the whole panel phase in one launch (chol_group_kernel)
    GroupCols gc;
    gc.g = g;
    gc.nranks = keep.nranks;
    gc.a0 = kb + g;
    gc.rhs0 = npad / NB;
    gc.n_rhs = (gdim - npad) / NB;
    if (keep.nranks == 1) {
      gc.n_own = npad / NB - gc.a0;
    } else {
      const int64_t R = keep.nranks, J0 = gc.a0 / 2;  // (a0 even: k0 on a 128-row boundary, g even)
      if ((gc.a0 & 1) != 0) return fail(GBM_E_ARG, "gbm_dev_chol_group_panels: odd panel group in a distributed step");
      gc.J_first = J0 + ((keep.rank - J0) % R + R) % R;
      for (int64_t J = gc.J_first; 2 * J < npad / NB; J += R) gc.n_own += (2 * J + 1 < npad / NB) ? 2 : 1;
    }
    if ((int64_t)(CNB + 1) * ldg * 8 > 0x7fffffff)
      return fail(GBM_E_ARG, "chol_group_kernel: ldg too large for 32-bit buffer offsets");
    int32_t* prog = reinterpret_cast<int32_t*>(w.flow);  // (the dataflow factorisation's flags: unused on this path)
    GBM_HIP_TRY(hipMemsetAsync(prog, 0, (size_t)g * sizeof(int32_t), s));
    const int64_t nwg = (g - 1) + gc.n_own + gc.n_rhs;
    chol_group_kernel<<<(unsigned)nwg, 256, 0, s>>>(G, ldg, k0, gc, w.Ld, w.Dinv, prog, info);
    GBM_LAUNCH_CHECK();
    return GBM_OK;
  }
  auto panel = [&](int64_t k) {
    const int64_t chunks = (gdim - k) / NB - 1;  // column chunks right of the diagonal block
    chol_panel_kernel<<<(unsigned)chunks, 256, 0, s>>>(G, ldg, k, w.Ld, w.Dinv, keep);
    return hipGetLastError() == hipSuccess;
  };
  if (!panel(k0)) return fail(GBM_E_HIP, "chol_panel_kernel launch failed");
  for (int j = 1; j < g; j++) {
    GBM_TRY(launch_chol_row_update(G, ldg, k0, j, gdim, w.Ld, w.Dinv, info, s, keep));
    if (!panel(k0 + j * NB)) return fail(GBM_E_HIP, "chol_panel_kernel launch failed");
  }
  return GBM_OK;
}

// The group's trailing update (its first workgroup factors the next diagonal block). nranks > 1:
// this rank's tile columns and the right-hand sides, once the group's rows are complete on every
// rank (row exchange + gbm_dev_chol_strip_unpack_rows); the next diagonal block is factored after
// the next group's area exchange (gbm_dev_chol_area_* + gbm_dev_chol_factor_diag).
int solve_group_update(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks, int32_t* info,
                       void* workspace, hipStream_t s, int64_t col_lo = 0, int64_t col_hi = INT64_MAX,
                       int64_t row_lo = 0, int64_t row_hi = INT64_MAX) {
  const int64_t npad = npad_of(n), gdim = gdim_of(n), nb = npad / NB;
  const SolveWs w = solve_ws(workspace, npad);
  const int64_t k0 = kb * NB;
  if (tail_flow_at(kb, npad, gdim))
    return fail(GBM_E_ARG, "gbm_dev_chol_group_update: the dataflow tail (GBM_CHOL_TAIL_FLOW) runs as gbm_dev_chol_group");
  const int g = group_size(kb, nb, gdim);
  const int64_t next = kb + g < nb ? k0 + g * NB : -1;
  if (g > 1)
    return launch_chol_update(G, ldg, k0, g * NB, gdim, w.Ld, w.Dinv, info, next, rank, nranks, s, col_lo, col_hi,
                              row_lo, row_hi);
  if (nranks > 1) return fail(GBM_E_ARG, "gbm_dev_chol_group_update: single-panel steps are not distributed");
  return launch_chol_update(G, ldg, k0, NB, gdim, w.Ld, w.Dinv, info, next, 0, 1, s);
}

// One whole panel group on one rank (the redundant factorisation and the distributed one's tail).
int solve_group(double* G, int64_t ldg, int64_t n, int64_t kb, int32_t* info, void* workspace, hipStream_t s,
                int64_t* g_out) {
  const int64_t npad = npad_of(n), gdim = gdim_of(n);
  if (tail_flow_at(kb, npad, gdim)) {
    // the rest in one dataflow launch on the trailing sub-matrix (its first diagonal block, already
    // factored by the last trailing update or factor_diag, is factored again from the same A)
    const SolveWs w = solve_ws(workspace, npad);
    const int64_t k0 = kb * NB;
    if (g_out) *g_out = npad / NB - kb;
    return launch_chol_flow(G + k0 * ldg + k0, ldg, gdim - k0, w.Ld + k0 * CNB, w.Dinv + (k0 / 16) * 256, w.flow,
                            info, s);
  }
  GBM_TRY(solve_group_panels(G, ldg, n, kb, ColKeep{}, info, workspace, s, g_out));
  return solve_group_update(G, ldg, n, kb, 0, 1, info, workspace, s);
}

// After the last panel: inverses of the diagonal blocks, μ̂ and the back-substitution right-hand
// sides from the bordered Schur block, the sync-free back substitution, GEBVs.
int solve_finish(double* G, int64_t ldg, int64_t n, const double* Y, int64_t ldy, int64_t nrhs, double lambda,
                 double* A_out, double* gebv, int64_t lda, double* mu, int32_t* info, void* workspace, hipStream_t s) {
  const int64_t npad = npad_of(n), nb = npad / NB;
  const SolveWs w = solve_ws(workspace, npad);
  diag_inverse_kernel<<<(unsigned)nb, 64, 0, s>>>(w.Ld, w.Linv);
  GBM_LAUNCH_CHECK();
  const unsigned gx = (unsigned)((lda + 255) / 256 < 1024 ? (lda + 255) / 256 : 1024);
  // the gebv buffer doubles as the w scratch: gebv_kernel (last) reads only Y and A
  gls_mu_kernel<<<dim3(gx, (unsigned)nrhs), 256, 0, s>>>(G, ldg, npad, nrhs, gebv, lda, mu, w.flags);
  GBM_LAUNCH_CHECK();
  back_solve_kernel<<<(unsigned)((nb + 1) / 2), 256, 0, s>>>(G, ldg, w.Linv, nb, gebv, A_out, lda, nrhs, w.flags, info);
  GBM_LAUNCH_CHECK();
  gebv_kernel<<<dim3(gx, (unsigned)nrhs), 256, 0, s>>>(Y, ldy, n, A_out, gebv, lda, mu, lambda);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// area: the square [r0, r0 + rows) x [r0, r0 + rows) only (a panel group's diagonal area)
void strip_geometry(int64_t n, int64_t kb, int64_t rows64, int nranks, int64_t& r0, int64_t& rows, int64_t& J0,
                    int64_t& Jend, int64_t& cnt, bool area = false) {
  r0 = kb * NB;
  rows = rows64 * NB;
  J0 = r0 / 128;
  Jend = area ? (r0 + rows + 127) / 128 : npad_of(n) / 128;
  cnt = Jend > J0 ? (Jend - J0 + nranks - 1) / nranks : 0;
}

}  // namespace

extern "C" int gbm_dev_gblup_solve(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev,
                                   double lambda, const double* Y, int64_t ldy, int64_t nrhs, double* A_out,
                                   double* gebv, int64_t lda, double* mu, int32_t* info, void* workspace,
                                   int64_t ws_bytes, void* stream) {
  const int64_t npad = npad_of(n);
  if (!Y || !A_out || !gebv || !mu || ldy < n || lda < npad || nrhs < 1 || nrhs > MAXRHS || !(lambda > 0.0) ||
      !(q_dev || inv_q > 0.0))
    return fail(GBM_E_ARG, "gbm_dev_gblup_solve: bad arguments (need ldg >= gdim(n), lda >= npad(n), "
                           "1 <= nrhs <= 63, lambda > 0, inv_q > 0)");
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_gblup_solve"));
  hipStream_t s = (hipStream_t)stream;
  if (chol_flow_enabled(npad)) {
    // one persistent dataflow launch factors the whole bordered matrix (chol_flow.hip)
    GBM_TRY(solve_prepare(G, ldg, n, inv_q, q_dev, lambda, Y, ldy, nrhs, info, workspace, s, false));
    const SolveWs w = solve_ws(workspace, npad);
    GBM_TRY(launch_chol_flow(G, ldg, gdim_of(n), w.Ld, w.Dinv, w.flow, info, s));
    return solve_finish(G, ldg, n, Y, ldy, nrhs, lambda, A_out, gebv, lda, mu, info, workspace, s);
  }
  GBM_TRY(solve_prepare(G, ldg, n, inv_q, q_dev, lambda, Y, ldy, nrhs, info, workspace, s));
  const int64_t nb = npad / NB;
  for (int64_t kb = 0; kb < nb;) {
    int64_t g = 1;
    GBM_TRY(solve_group(G, ldg, n, kb, info, workspace, s, &g));
    kb += g;
  }
  return solve_finish(G, ldg, n, Y, ldy, nrhs, lambda, A_out, gebv, lda, mu, info, workspace, s);
}

extern "C" int gbm_dev_chol_prepare(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev,
                                    double lambda, const double* Y, int64_t ldy, int64_t nrhs, int32_t* info,
                                    void* workspace, int64_t ws_bytes, void* stream) {
  if (!Y || ldy < n || nrhs < 1 || nrhs > MAXRHS || !(lambda > 0.0) || !(q_dev || inv_q > 0.0))
    return fail(GBM_E_ARG, "gbm_dev_chol_prepare: bad arguments");
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_prepare"));
  return solve_prepare(G, ldg, n, inv_q, q_dev, lambda, Y, ldy, nrhs, info, workspace, (hipStream_t)stream);
}

extern "C" int gbm_dev_chol_prepare_cols(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev,
                                         double lambda, const double* Y, int64_t ldy, int64_t nrhs, int rank,
                                         int nranks, int32_t* info, void* workspace, int64_t ws_bytes, void* stream) {
  if (!Y || ldy < n || nrhs < 1 || nrhs > MAXRHS || !(lambda > 0.0) || !(q_dev || inv_q > 0.0) || nranks < 1 ||
      rank < 0 || rank >= nranks)
    return fail(GBM_E_ARG, "gbm_dev_chol_prepare_cols: bad arguments");
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_prepare_cols"));
  ColKeep keep;
  keep.rank = rank;
  keep.nranks = nranks;
  if (nranks > 1) {
    chol_refresh_tuning();
    keep.keep_hi = (int64_t)group_size(0, npad_of(n) / NB, gdim_of(n)) * NB;  // the first group's area
    keep.rhs0 = npad_of(n);
  }
  return solve_prepare(G, ldg, n, inv_q, q_dev, lambda, Y, ldy, nrhs, info, workspace, (hipStream_t)stream, true, keep);
}

extern "C" int64_t gbm_dev_chol_group_size(int64_t n, int64_t kb) {
  const int64_t nb = npad_of(n) / NB;
  if (kb < 0 || kb >= nb) return 0;
  chol_refresh_tuning();
  return group_size(kb, nb, gdim_of(n));
}

extern "C" int gbm_dev_chol_group(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks, int32_t* info,
                                  void* workspace, int64_t ws_bytes, void* stream) {
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_group"));
  if (kb < 0 || kb >= npad_of(n) / NB || nranks != 1 || rank != 0)
    return fail(GBM_E_ARG, "gbm_dev_chol_group: one rank only (rank 0 of 1); a distributed step is "
                           "gbm_dev_chol_group_panels + row exchange + gbm_dev_chol_group_update");
  return solve_group(G, ldg, n, kb, info, workspace, (hipStream_t)stream, nullptr);
}

extern "C" int gbm_dev_chol_group_panels(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks,
                                         int32_t* info, void* workspace, int64_t ws_bytes, void* stream) {
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_group_panels"));
  if (kb < 0 || kb >= npad_of(n) / NB || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(GBM_E_ARG, "gbm_dev_chol_group_panels: bad step or rank");
  ColKeep keep;
  keep.rank = rank;
  keep.nranks = nranks;
  return solve_group_panels(G, ldg, n, kb, keep, info, workspace, (hipStream_t)stream, nullptr);
}

extern "C" int gbm_dev_chol_group_update(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks,
                                         int32_t* info, void* workspace, int64_t ws_bytes, void* stream) {
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_group_update"));
  if (kb < 0 || kb >= npad_of(n) / NB || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(GBM_E_ARG, "gbm_dev_chol_group_update: bad step or rank");
  return solve_group_update(G, ldg, n, kb, rank, nranks, info, workspace, (hipStream_t)stream);
}

extern "C" int gbm_dev_chol_group_update_cols(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks,
                                              int64_t col_lo, int64_t col_hi, int32_t* info, void* workspace,
                                              int64_t ws_bytes, void* stream) {
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_group_update_cols"));
  if (kb < 0 || kb >= npad_of(n) / NB || nranks < 2 || rank < 0 || rank >= nranks || col_lo < 0 || col_hi < col_lo)
    return fail(GBM_E_ARG, "gbm_dev_chol_group_update_cols: bad step, rank (nranks >= 2) or column range");
  return solve_group_update(G, ldg, n, kb, rank, nranks, info, workspace, (hipStream_t)stream, col_lo, col_hi);
}

extern "C" int gbm_dev_chol_group_update_tiles(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks,
                                               int64_t row_lo, int64_t row_hi, int64_t col_lo, int64_t col_hi,
                                               int32_t* info, void* workspace, int64_t ws_bytes, void* stream) {
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_group_update_tiles"));
  if (kb < 0 || kb >= npad_of(n) / NB || nranks < 2 || rank < 0 || rank >= nranks || col_lo < 0 || col_hi < col_lo ||
      row_lo < 0 || row_hi < row_lo)
    return fail(GBM_E_ARG, "gbm_dev_chol_group_update_tiles: bad step, rank (nranks >= 2), row or column range");
  return solve_group_update(G, ldg, n, kb, rank, nranks, info, workspace, (hipStream_t)stream, col_lo, col_hi, row_lo,
                            row_hi);
}

extern "C" int gbm_dev_chol_factor_diag(double* G, int64_t ldg, int64_t n, int64_t kb, int32_t* info, void* workspace,
                                        int64_t ws_bytes, void* stream) {
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_factor_diag"));
  if (kb < 0 || kb >= npad_of(n) / NB) return fail(GBM_E_ARG, "gbm_dev_chol_factor_diag: bad step");
  const SolveWs w = solve_ws(workspace, npad_of(n));
  factor_diag_kernel<<<1, 256, 0, (hipStream_t)stream>>>(G, ldg, kb * NB, w.Ld, w.Dinv, info);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

extern "C" int64_t gbm_dev_chol_strip_doubles(int64_t n, int64_t kb, int64_t rows64, int nranks) {
  if (nranks < 1 || kb < 0 || rows64 < 1) return 0;
  int64_t r0, rows, J0, Jend, cnt;
  strip_geometry(n, kb, rows64, nranks, r0, rows, J0, Jend, cnt);
  return cnt * rows * 128;
}

static int strip_launch(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank, int nranks,
                        double* buf, int unpack, hipStream_t s, bool area = false) {
  if (!G || !buf || n < 1 || ldg < gdim_of(n) || kb < 0 || rows64 < 1 || (kb * NB) % 128 != 0 || nranks < 1 ||
      rank < 0 || rank >= nranks || (kb + rows64) * NB > npad_of(n))
    return fail(GBM_E_ARG, "gbm_dev_chol_strip_pack/unpack: bad arguments (strip rows inside [0, npad), "
                           "starting on a 128-row boundary)");
  if (area && (rows64 & 1))
    return fail(GBM_E_ARG, "gbm_dev_chol_area_pack/unpack: the area must end on a 128-row boundary");
  int64_t r0, rows, J0, Jend, cnt;
  strip_geometry(n, kb, rows64, nranks, r0, rows, J0, Jend, cnt, area);
  if (cnt == 0) return GBM_OK;
  if (cnt > 65535 || nranks > 65535) return fail(GBM_E_ARG, "gbm_dev_chol_strip_*: too many tiles for the grid");
  const dim3 grid((unsigned)((rows + 3) / 4), (unsigned)cnt, (unsigned)(unpack ? nranks : 1));
  chol_strip_kernel<<<grid, 256, 0, s>>>(G, ldg, r0, rows, J0, Jend, cnt, rank, nranks, buf, unpack);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

extern "C" int gbm_dev_chol_strip_pack(const double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank,
                                       int nranks, double* buf, void* stream) {
  return strip_launch(const_cast<double*>(G), ldg, n, kb, rows64, rank, nranks, buf, 0, (hipStream_t)stream);
}

extern "C" int gbm_dev_chol_strip_unpack(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int nranks,
                                         const double* gathered, void* stream) {
  return strip_launch(G, ldg, n, kb, rows64, 0, nranks, const_cast<double*>(gathered), 1, (hipStream_t)stream);
}

extern "C" int64_t gbm_dev_chol_area_doubles(int64_t n, int64_t kb, int64_t rows64, int nranks) {
  if (nranks < 1 || kb < 0 || rows64 < 1) return 0;
  int64_t r0, rows, J0, Jend, cnt;
  strip_geometry(n, kb, rows64, nranks, r0, rows, J0, Jend, cnt, true);
  return cnt * rows * 128;
}

extern "C" int gbm_dev_chol_area_pack(const double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank,
                                      int nranks, double* buf, void* stream) {
  return strip_launch(const_cast<double*>(G), ldg, n, kb, rows64, rank, nranks, buf, 0, (hipStream_t)stream, true);
}

extern "C" int gbm_dev_chol_area_unpack(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int nranks,
                                        const double* gathered, void* stream) {
  return strip_launch(G, ldg, n, kb, rows64, 0, nranks, const_cast<double*>(gathered), 1, (hipStream_t)stream, true);
}

extern "C" int gbm_dev_chol_lower_copy(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank,
                                       int nranks, void* stream) {
  if (!G || n < 1 || ldg < gdim_of(n) || kb < 0 || rows64 < 1 || rank < 0 || rank >= nranks ||
      (kb + rows64) * NB > npad_of(n))
    return fail(GBM_E_ARG, "gbm_dev_chol_lower_copy: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  // the lower copy of the chunks other ranks solved (this rank's panel kernels wrote its own)
  const int64_t npad = npad_of(n), r0 = kb * NB;
  ColKeep keep;
  keep.rank = rank;
  keep.nranks = nranks;
  keep.keep_hi = r0 + rows64 * NB;
  keep.rhs0 = npad;
  const int64_t chunks = (npad - r0) / NB - 1;
  if (chunks > 0 && nranks > 1) {
    chol_lower_copy_kernel<<<dim3((unsigned)chunks, (unsigned)rows64), 256, 0, s>>>(G, ldg, r0, npad, keep);
    GBM_LAUNCH_CHECK();
  }
  return GBM_OK;
}

extern "C" int gbm_dev_chol_strip_unpack_rows(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank,
                                              int nranks, const double* gathered, void* stream) {
  if (rank < 0 || rank >= nranks) return fail(GBM_E_ARG, "gbm_dev_chol_strip_unpack_rows: bad rank");
  GBM_TRY(strip_launch(G, ldg, n, kb, rows64, 0, nranks, const_cast<double*>(gathered), 1, (hipStream_t)stream));
  return gbm_dev_chol_lower_copy(G, ldg, n, kb, rows64, rank, nranks, stream);
}

extern "C" int gbm_dev_chol_finish(double* G, int64_t ldg, int64_t n, const double* Y, int64_t ldy, int64_t nrhs,
                                   double lambda, double* A_out, double* gebv, int64_t lda, double* mu, int32_t* info,
                                   void* workspace, int64_t ws_bytes, void* stream) {
  if (!Y || !A_out || !gebv || !mu || ldy < n || lda < npad_of(n) || nrhs < 1 || nrhs > MAXRHS)
    return fail(GBM_E_ARG, "gbm_dev_chol_finish: bad arguments");
  GBM_TRY(check_solve_args(G, ldg, n, info, workspace, ws_bytes, "gbm_dev_chol_finish"));
  return solve_finish(G, ldg, n, Y, ldy, nrhs, lambda, A_out, gebv, lda, mu, info, workspace, (hipStream_t)stream);
}

extern "C" int gbm_dev_gblup_terms(const double* G, int64_t ldg, int64_t n, int64_t nrhs, const void* workspace,
                                   double* terms, void* stream) {
  if (!G || !workspace || !terms || n < 1 || nrhs < 1 || nrhs > MAXRHS || ldg < gdim_of(n))
    return fail(GBM_E_ARG, "gbm_dev_gblup_terms: bad arguments");
  gblup_terms_kernel<<<1, 256, 0, (hipStream_t)stream>>>(G, ldg, npad_of(n), nrhs, (const double*)workspace,
                                                         terms);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}
