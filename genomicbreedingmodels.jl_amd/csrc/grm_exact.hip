// Exact-integer GRM of dosage genotypes on the CDNA4 int8 matrix cores.
//
// The GRM of SURVEY.md §8a a3 (reference src/gwas.jl:112-126: Z = standardised X, G = Z Zᵀ/q) when
// X holds diploid dosages x = d/2, d ∈ {0, 1, 2}. With t_j = Σ_i d_ij and w_j = 1/var(d_·j) (ddof 1;
// the ploidy cancels: z_ij = (d_ij − t_j/n)·√w_j),
//
//   G_ik = Σ_j w_j (d_ij − t_j/n)(d_kj − t_j/n)
//        = 2^−F/n² · [ n² A_ik − n U_i − n U_k + C ],   A_ik = Σ_j W_j d_ij d_kj,
//                                                       U_i  = Σ_j W_j t_j d_ij,  C = Σ_j W_j t_j²,
//
// with W_j = w_j·2^F an integer: F is chosen so that every locus' fp64 weight w_j is an integer
// multiple of 2^−F (exact: its 53-bit significand lands on the integer grid) as long as the weights
// span ≤ 2^16 (xg_choose; beyond that the smallest are rounded to the grid, error ≤ 2^−(69−Δe) each).
// W_j is cut into S balanced base-128 digits W_j = Σ_s 128^s ω_sj, ω ∈ [−64, 63], so
// A_ik = Σ_s 128^s Σ_j d_ij (d_kj ω_sj) is S int8 GEMMs whose products d·ω ∈ [−128, 126] fit int8 and
// whose int32 sums are exact. The bracket is combined in 128-bit integers and rounded to fp64 once
// (plus the division by n²): the only approximation left is the fp64 rounding of w_j itself — the
// reference's own fp64 SYRK rounds every product and partial sum instead.
//
// Kernels (all stream-ordered, one host sync to size S):
//   xg_stats_kernel   per locus: t, Σd², mean, sd, keep, q (the standardisation's outputs), w_j, the
//                     exponent range of the kept weights, a flag for dosages outside {0, 1, 2} (block partials;
//                     xg_stats_reduce_kernel combines them)
//   xg_digits_kernel  per locus: the S digits (and doubled digits) in the GEMM's per-stage layout,
//                     V_j = W_j t_j (four 24-bit limbs), block partials of C
//   xg_transpose_u_kernel  locus-major dosages → individual-major Dt (the A operand) and St (B: each byte
//                     a v_perm selector picking 2ω, ω or 0 from the digit dwords), and partial U_i
//   xg_u_reduce_kernel   n·U_i and C in int128
//   xg_gemm_kernel<S> 128 x 64 output tiles of the upper triangle; 8 waves of 64 x 16, each holding S x 4
//                     v_mfma_i32_16x16x64_i8 accumulators; operands staged global → LDS by LDS-DMA into a
//                     4-deep ring (counted vmcnt, raw barriers); B scaled per slice in registers by one
//                     v_perm per dword (each scaled fragment feeds 4 MFMAs); the epilogue rebuilds the bracket in int128 and stores fp64 G.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "gbm_internal.h"

namespace gbm {

typedef __int128 i128;
typedef unsigned __int128 u128;
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int XG_BM = 128;       // tile rows (individuals i)
constexpr int XG_BN = 64;        // tile columns (individuals k)
constexpr int XG_BK = 128;       // loci per digit group (the GEMM stages 128 or 256 loci: XgStage)
constexpr int XG_KALIGN = 256;   // kp (padded loci) multiple: whole stages for either BK
constexpr int XG_SMIN = 8, XG_SMAX = 10;
constexpr int XG_UBLK = 256;      // threads per block of the U / digits kernels

struct XgInfo {  // device scratch written by the stats kernel, read by the host once
  unsigned long long wmax_bits;  // the largest kept weight (positive doubles order as their bits)
  int32_t emin, emax, bad, pad;
};
struct XgStatsPart {  // one stats block's partial (reduced by xg_stats_reduce_kernel: no same-address atomics
  unsigned long long kept, wmax_bits;  // from thousands of blocks, which serialise: measured 163 µs at C2)
  int32_t emin, emax, bad, pad;
};
constexpr int XG_SGRID = 4096;  // the most stats blocks

__device__ __forceinline__ double i128_to_double(i128 x) {
  const bool neg = x < 0;
  const u128 m = neg ? (u128)0 - (u128)x : (u128)x;
  const uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
  const double r = (double)hi * 18446744073709551616.0 + (double)lo;
  return neg ? -r : r;
}

// ---- per-locus statistics (one wave per locus row, grid-strided over waves) ----------------------------
// t = Σd and Σd² by v_dot4 over 4 dosages per lane per load when the rows are 4-byte aligned (ldd % 4 == 0),
// else byte loads. The exponent range and the largest weight are kept per wave, one atomic each at the end.
__global__ void __launch_bounds__(256) xg_stats_kernel(const int8_t* __restrict__ D, int64_t ldd, int64_t p, int64_t n,
                                                       double xs, double* __restrict__ mean, double* __restrict__ sd,
                                                       int32_t* __restrict__ keep, unsigned long long* __restrict__ q_dev,
                                                       double* __restrict__ w, int64_t* __restrict__ tcol,
                                                       XgStatsPart* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6, nw = ((int64_t)gridDim.x * 256) >> 6;
  const bool al4 = (ldd % 4) == 0 && ((uintptr_t)D % 4) == 0;
  unsigned long long kept = 0, wmaxb = 0;
  int emin = INT_MAX, emax = INT_MIN, bad = 0;
  for (int64_t j = wid; j < p; j += nw) {
    const int8_t* row = D + j * ldd;
    int t = 0, s2 = 0;
    int64_t tail = 0;
    if (al4) {
      const int64_t n4 = n / 4;
      const int* r4 = reinterpret_cast<const int*>(row);
#pragma unroll 8
      for (int64_t i = lane; i < n4; i += 64) {
        const int v = r4[i];
        t = __builtin_amdgcn_sdot4(v, 0x01010101, t, false);
        s2 = __builtin_amdgcn_sdot4(v, v, s2, false);
        // a byte outside {0, 1, 2}: any of bits 2-7 set, or both bits 0 and 1 (3)
        bad |= (v & 0xFCFCFCFC) | ((v & 0x02020202) & ((v & 0x01010101) << 1));
      }
      tail = 4 * n4;
    }
    for (int64_t i = tail + lane; i < n; i += 64) {
      const int d = row[i];
      t += d;
      s2 += d * d;
      bad |= (d < 0 || d > 2);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      t += __shfl_xor(t, off, 64);
      s2 += __shfl_xor(s2, off, 64);
    }
    // var(d) = (n Σd² − t²)/(n(n − 1)), exact integers up to the division
    const long long num = (long long)n * s2 - (long long)t * t;
    const bool kp = n > 1 && num > 0;
    const double dn = (double)n;
    const double wj = kp ? (dn * (dn - 1.0)) / (double)num : 0.0;
    if (lane == 0) {
      mean[j] = (double)t * xs / dn;
      sd[j] = kp ? sqrt((double)num / (dn * (dn - 1.0))) * xs : 0.0;
      keep[j] = kp ? 1 : 0;
      w[j] = wj;
      tcol[j] = t;
    }
    if (kp) {
      kept++;
      const int e = ilogb(wj);
      emin = e < emin ? e : emin;
      emax = e > emax ? e : emax;
      const unsigned long long bits = (unsigned long long)__double_as_longlong(wj);
      wmaxb = bits > wmaxb ? bits : wmaxb;
    }
  }
  // the block's four waves combine through LDS; one set of atomics per block
  __shared__ unsigned long long sk[4], sw[4];
  __shared__ int se0[4], se1[4], sb[4];
  bad = __any(bad != 0) ? 1 : 0;
  const int wv = threadIdx.x >> 6;
  if (lane == 0) {
    sk[wv] = kept;
    sw[wv] = wmaxb;
    se0[wv] = emin;
    se1[wv] = emax;
    sb[wv] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; k++) {
      kept += sk[k];
      wmaxb = sw[k] > wmaxb ? sw[k] : wmaxb;
      emin = se0[k] < emin ? se0[k] : emin;
      emax = se1[k] > emax ? se1[k] : emax;
      bad |= sb[k];
    }
    part[blockIdx.x] = XgStatsPart{kept, wmaxb, emin, emax, bad, 0};
  }
}

// one block: the stats blocks' partials → XgInfo (read by the host) and q (one atomic: q accumulates over calls)
__global__ void __launch_bounds__(256) xg_stats_reduce_kernel(const XgStatsPart* __restrict__ part, int nb,
                                                              unsigned long long* __restrict__ q_dev,
                                                              XgInfo* __restrict__ info) {
  __shared__ XgStatsPart red[256];
  XgStatsPart a{0, 0, INT_MAX, INT_MIN, 0, 0};
  for (int b = threadIdx.x; b < nb; b += 256) {
    const XgStatsPart x = part[b];
    a.kept += x.kept;
    a.wmax_bits = x.wmax_bits > a.wmax_bits ? x.wmax_bits : a.wmax_bits;
    a.emin = x.emin < a.emin ? x.emin : a.emin;
    a.emax = x.emax > a.emax ? x.emax : a.emax;
    a.bad |= x.bad;
  }
  red[threadIdx.x] = a;
  __syncthreads();
  for (int off = 128; off >= 1; off >>= 1) {
    if (threadIdx.x < off) {
      XgStatsPart& x = red[threadIdx.x];
      const XgStatsPart& y = red[threadIdx.x + off];
      x.kept += y.kept;
      x.wmax_bits = y.wmax_bits > x.wmax_bits ? y.wmax_bits : x.wmax_bits;
      x.emin = y.emin < x.emin ? y.emin : x.emin;
      x.emax = y.emax > x.emax ? y.emax : x.emax;
      x.bad |= y.bad;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const XgStatsPart& r = red[0];
    if (r.kept && !(r.bad & 1)) atomicAdd(q_dev, r.kept);  // a call that fails (bad dosage) leaves q untouched
    info->wmax_bits = r.wmax_bits;
    info->emin = r.emin;
    info->emax = r.emax;
    info->bad = r.bad;
    info->pad = 0;
  }
}

// ---- digits: W_j = w_j 2^F → S balanced base-128 digits in the GEMM's stage layout -----------------
// Stage layout (per 128-locus stage, S·256 bytes): [s][chunk c = 0..7][32 B: ω of loci 16c..16c+15,
// then 2ω of the same loci] (2ω from memory: computing it per dword costs two VALU ops per v_perm, and the
// kernel is VALU-issue-sensitive: measured slower).
__global__ void __launch_bounds__(XG_UBLK) xg_digits_kernel(const double* __restrict__ w, const int64_t* __restrict__ tcol,
                                                            int64_t p, int64_t kp, int S, int F,
                                                            int8_t* __restrict__ WW, uint4* __restrict__ VL,
                                                            i128* __restrict__ Cpart, XgInfo* __restrict__ info) {
  __shared__ i128 red[XG_UBLK];
  const int64_t j = (int64_t)blockIdx.x * XG_UBLK + threadIdx.x;
  i128 W = 0, c = 0;
  if (j < p && w[j] > 0.0) {
    int e;
    const double mant = frexp(w[j], &e);  // w = mant 2^e, mant ∈ [0.5, 1)
    const long long M = (long long)ldexp(mant, 53);
    const int sh = e - 53 + F;
    if (sh >= 0) {
      W = (i128)M << sh;
    } else {  // weights spanning > 2^16 (xg_choose): round the smallest to the grid
      const int r = -sh;
      W = r >= 63 ? (i128)0 : (i128)((M + (1LL << (r - 1))) >> r);
    }
    const i128 t = (i128)tcol[j];
    const i128 v = W * t;  // >= 0, < 2^89: four 24-bit limbs
    VL[j] = make_uint4((uint32_t)v & 0xFFFFFFu, (uint32_t)(v >> 24) & 0xFFFFFFu, (uint32_t)(v >> 48) & 0xFFFFFFu,
                       (uint32_t)(v >> 72) & 0xFFFFFFu);
    c = W * t * t;
  } else if (j < kp) {
    VL[j] = make_uint4(0, 0, 0, 0);
  }
  if (j < kp) {
    i128 x = W;
    const int64_t stage = j / XG_BK, c8 = (j / 16) % 8, pos = j % 16;
    for (int s = 0; s < S; s++) {
      int r = (int)(x & 127);
      if (r >= 64) r -= 128;
      x = (x - r) >> 7;
      const int64_t b = ((stage * S + s) * 8 + c8) * 32 + pos;
      WW[b] = (int8_t)r;
      WW[b + 16] = (int8_t)(2 * r);
    }
    if (x != 0) atomicOr(&info->bad, 2);  // W out of the digits' range (cannot happen with xg_choose's S)
  }
  red[threadIdx.x] = c;
  __syncthreads();
  for (int off = XG_UBLK / 2; off >= 1; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) Cpart[blockIdx.x] = red[0];
}

// ---- transpose + U: locus-major D (p rows of ldd bytes) → individual-major Dt, St ([npad][kp]) and the
// partial U_i = Σ_j V_j d_ij over this block's loci tiles --------------------------------------------------
// St byte at locus k (b = k mod 4, its byte in the dword): d = 2 → b (the 2ω dword, v_perm src1),
// d = 1 → 4 + b (the ω dword, src0), d = 0 → 12 (v_perm's constant zero).
// Block (x, y): individuals [256x, 256x + 256), the 64-locus tiles y, y + gridDim.y, ...: each tile read
// row by row (4 dosages per lane) into LDS, then one thread per individual assembles its 64 bytes of Dt and
// St and adds its V_j d_ij (V_j wave-uniform).
constexpr int XG_TP = 256 + 16;  // LDS row pitch of the 64-locus x 256-individual tile
// the dosage rows read with the nontemporal hint (read once here): C2 transpose 211 → 204 µs, same G digests
// (profiles/r06_nt_reduce_transpose_ab.txt; GBM_XG_TP_NT=0 builds the plain loads)
#ifndef GBM_XG_TP_NT
#define GBM_XG_TP_NT 1
#endif
__global__ void __launch_bounds__(256) xg_transpose_u_kernel(const int8_t* __restrict__ D, int64_t ldd, int64_t p,
                                                             int64_t n, int64_t kp, int64_t npad,
                                                             const uint4* __restrict__ VL, int8_t* __restrict__ Dt,
                                                             int8_t* __restrict__ St, i128* __restrict__ Upart) {
  __shared__ __attribute__((aligned(16))) int8_t tile[64 * XG_TP];
  const int64_t i0 = (int64_t)blockIdx.x * 256;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool al4 = (ldd % 4) == 0 && ((uintptr_t)D % 4) == 0;
  const int64_t i = i0 + threadIdx.x;
  // tiles strided over the blocks (a contiguous range per block measured slower: 0.60 vs 0.45 ms at C2)
  const int64_t nkt = kp / 64;
  i128 u = 0;
  uint32_t vr[16];
  auto load_rows = [&](int64_t kt) {  // this wave's 16 rows of tile kt, 4 dosages per lane, all in flight
#pragma unroll
    for (int rr = 0; rr < 16; rr++) {
      const int64_t k = kt * 64 + wv + 4 * rr;
      const int64_t ii = i0 + 4 * lane;
      uint32_t v = 0;
      if (k < p) {
        const int8_t* row = D + k * ldd;
        if (al4 && ii + 3 < n) {
#if GBM_XG_TP_NT
          v = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(row + ii));
#else
          v = *reinterpret_cast<const uint32_t*>(row + ii);
#endif
        } else {
#pragma unroll
          for (int b = 0; b < 4; b++)
            if (ii + b < n) v |= (uint32_t)(uint8_t)row[ii + b] << (8 * b);
        }
      }
      vr[rr] = v;
    }
  };
  if ((int64_t)blockIdx.y < nkt) load_rows(blockIdx.y);
  for (int64_t kt = blockIdx.y; kt < nkt; kt += gridDim.y) {
    const int64_t k0 = kt * 64;
    __syncthreads();  // the previous tile's reads are done
#pragma unroll
    for (int rr = 0; rr < 16; rr++) *reinterpret_cast<uint32_t*>(tile + (wv + 4 * rr) * XG_TP + 4 * lane) = vr[rr];
    if (kt + gridDim.y < nkt) load_rows(kt + gridDim.y);  // the next tile's rows in flight during this one
    __syncthreads();
    if (i < npad) {
      // U in four 24-bit limbs of V_j: one v_mad_u32_u24 per limb and dosage, 32-bit sums exact over the
      // tile's 64 loci (64·2·(2^24 − 1) < 2^31), carried into the int128 once per tile
      uint32_t dw[16], sw[16];
      uint32_t l0 = 0, l1 = 0, l2 = 0, l3 = 0;
#pragma unroll
      for (int q = 0; q < 16; q++) {
        uint32_t a = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int kk = q * 4 + b;
          const uint32_t d = (uint32_t)(uint8_t)tile[kk * XG_TP + threadIdx.x];
          a |= d << (8 * b);
          const uint4 vl = VL[k0 + kk];  // 0 beyond p
          l0 += __umul24(d, vl.x);
          l1 += __umul24(d, vl.y);
          l2 += __umul24(d, vl.z);
          l3 += __umul24(d, vl.w);
        }
        dw[q] = a;
        // the St selectors of the four bytes: 12 / 4 / 0 for d = 0 / 1 / 2 (a v_perm table lookup), plus the
        // byte's position b where d > 0
        const uint32_t h = __builtin_amdgcn_perm(0u, 0x0000040Cu, a);
        const uint32_t m = (a | (a >> 1)) & 0x01010101u;
        sw[q] = h + ((m * 0xFFu) & 0x03020100u);
      }
      u += (i128)l0 + ((i128)l1 << 24) + ((i128)l2 << 48) + ((i128)l3 << 72);
      const int64_t off = i * kp + k0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        *reinterpret_cast<uint4*>(Dt + off + 16 * q) = make_uint4(dw[4 * q], dw[4 * q + 1], dw[4 * q + 2], dw[4 * q + 3]);
        *reinterpret_cast<uint4*>(St + off + 16 * q) = make_uint4(sw[4 * q], sw[4 * q + 1], sw[4 * q + 2], sw[4 * q + 3]);
      }
    }
  }
  if (i < npad) Upart[blockIdx.y * npad + i] = u;
}

// ---- n·U_i and C from the partials ----------------------------------------------------------------------
// Block: 64 individuals, its four waves over the loci-tile partials r = wave, wave + 4, ... (the loads of a
// thread independent), combined through LDS; block 0 also sums the C partials with all its threads.
__global__ void __launch_bounds__(256) xg_u_reduce_kernel(const i128* __restrict__ Upart, int64_t nr, int64_t npad,
                                                          int64_t n, const i128* __restrict__ Cpart, int64_t ncp,
                                                          i128* __restrict__ NU, i128* __restrict__ C) {
  __shared__ i128 red[256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  i128 u = 0;
  if (i < npad)
#pragma unroll 4
    for (int64_t r = wv; r < nr; r += 4) u += Upart[r * npad + i];
  red[threadIdx.x] = u;
  __syncthreads();
  if (wv == 0 && i < npad) NU[i] = (red[lane] + red[64 + lane] + red[128 + lane] + red[192 + lane]) * (i128)n;
  if (blockIdx.x == 0) {
    __syncthreads();
    i128 c = 0;
    for (int64_t b = threadIdx.x; b < ncp; b += 256) c += Cpart[b];
    red[threadIdx.x] = c;
    __syncthreads();
    for (int off = 128; off >= 1; off >>= 1) {
      if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) *C = red[0];
  }
}

// ---- the int8 GEMM -----------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void wait_vm() {
  // s_waitcnt vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 encoding: vmcnt[3:0] | [15:14])
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// unit u → (row block I, column block J) over the upper-triangle units J >= 2I with columns below n
// (nI = ⌈n/128⌉ row blocks, nJ = ⌈n/64⌉ column blocks; every row block has at least one unit)
template <int RT>  // RT = row-block / column-block height ratio (2: 128 x 64 tiles, 1: 64 x 64)
__device__ __forceinline__ void xg_unit(int64_t u, int64_t nI, int64_t nJ, int64_t& I, int64_t& J) {
  int64_t base = 0, r = 0;
  while (r < nI && base + (nJ - RT * r) <= u) {
    base += nJ - RT * r;
    r++;
  }
  I = r;
  J = RT * r + (u - base);
}

// Blocked order (GBM_XG_ORDER=1; measured slower than the default row-major order): the units grouped in blocks of XG_OBI row blocks x XG_OBJ column
// blocks (32 = the CUs of an XCD), blocks row-major, units row-major inside a block; with the XCD remap an
// XCD's concurrently running units then share 4 A and 8 B operand strips (per stage 4·16 + 8·8 KB of distinct
// L2 lines instead of 16 + 32·8 KB in plain row-major order).
constexpr int XG_OBI = 4, XG_OBJ = 8;
template <int RT>
__device__ __forceinline__ void xg_unit_blocked(int64_t u, int64_t nI, int64_t nJ, int obi, int obj, int64_t& I,
                                                int64_t& J) {
  for (int64_t bi = 0; bi * obi < nI; bi++) {
    for (int64_t bj = 0; bj * obj < nJ; bj++) {
      const int64_t i1 = min(nI, (bi + 1) * obi), j0 = bj * obj, j1 = min(nJ, (bj + 1) * obj);
      for (int64_t ii = bi * obi; ii < i1; ii++) {
        const int64_t lo = max(RT * ii, j0), cnt = j1 > lo ? j1 - lo : 0;
        if (u < cnt) {
          I = ii;
          J = lo + u;
          return;
        }
        u -= cnt;
      }
    }
  }
  I = nI;  // not reached for u < nunits
  J = nJ;
}

// Stage geometry per BK (loci per LDS stage): operand rows of BK bytes, the stage's digits (BK/128 groups of
// S·256 bytes; up to 10 slices) in whole 1-KB DMA pieces, the ring depth that fits 160 KB of LDS.
template <int BK, int BM>
struct XgStage {
  static constexpr int kNW = BM / 16;                  // waves: 64 x 16 wave tiles over BM x 64
  static constexpr int kWW = BK == 128 ? 3072 : 5120;  // digit bytes in LDS (>= (BK/128)·XG_SMAX·256... at S <= 10)
  static constexpr int kBytes = BM * BK + XG_BN * BK + kWW;
  static constexpr int kNS = BK == 128 ? 4 : 3;        // ring depth: kNS − 1 stages in flight
  static constexpr int kA = BM * BK / 1024 / kNW;      // A pieces per wave
  static constexpr int kB = XG_BN * BK / 1024 / kNW;   // B pieces per wave
  static constexpr int kWWp = kWW / 1024;              // digit pieces (waves 0 .. kWWp − 1, one each)
  static constexpr int kRows = 1024 / BK;               // operand rows per piece
  __device__ static int swz(int r) { return BK == 128 ? (r & 7) : (r & 15); }  // conflict-free ds_read_b128
};

template <int N>
__device__ __forceinline__ void wait_vm_n(int pieces) {  // s_waitcnt vmcnt(N · pieces), pieces ∈ 3..7
  if (pieces == 3) wait_vm<3 * N>();
  else if (pieces == 4) wait_vm<4 * N>();
  else if (pieces == 5) wait_vm<5 * N>();
  else if (pieces == 6) wait_vm<6 * N>();
  else wait_vm<7 * N>();
}

template <int S, int BK, int BM>
__global__ void __launch_bounds__(BM * 4, BM == 128 ? 1 : 2)
xg_gemm_kernel(const int8_t* __restrict__ Dt, const int8_t* __restrict__ St, int64_t kp, const int8_t* __restrict__ WW,
               const i128* __restrict__ NU, const i128* __restrict__ Cp, int64_t n, int F, int64_t nI, int64_t nJ, int64_t nunits,
               double* __restrict__ G, int64_t ldg, int accum, int order, int64_t nfull, int ks_split,
               i32x4* __restrict__ part, int32_t* __restrict__ cnt) {
  using SG = XgStage<BK, BM>;
  constexpr int RT = BM / XG_BN;
  __shared__ __attribute__((aligned(16))) int8_t lds[SG::kNS * SG::kBytes];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // (BM/64) x 4 waves of 64 x 16

  // Blocks [0, nfull): whole units, XCD-aware bijective remap (the blocks the hardware deals to one XCD take
  // a contiguous unit range). Blocks [nfull, ...): the last nunits − nfull units (the partial last round of a
  // grid of one unit per CU) in ks_split loci ranges each, dispatched last and spread over every XCD; the
  // last range of a unit to finish (per wave: a counter per unit and wave) sums the others' int32 partials.
  const int64_t b = blockIdx.x;
  int64_t u, st0 = 0, st1 = kp / BK, slot = -1;
  int kpart = 0;
  if (b < nfull) {
    const int64_t xq = nfull / 8, xr = nfull % 8, x = b % 8;
    u = (x < xr ? x * (xq + 1) : xr * (xq + 1) + (x - xr) * xq) + b / 8;
  } else {
    const int64_t pc = b - nfull;
    slot = pc / ks_split;
    kpart = (int)(pc % ks_split);
    u = nfull + slot;
    const int64_t per = (st1 + ks_split - 1) / ks_split;
    st0 = kpart * per;
    st1 = st0 + per < st1 ? st0 + per : st1;
  }
  if (u >= nunits) return;
  int64_t I, J;
  if (order)
    xg_unit_blocked<RT>(u, nI, nJ, order >> 8, order & 255, I, J);
  else
    xg_unit<RT>(u, nI, nJ, I, J);
  const int64_t i0 = I * BM, j0 = J * XG_BN;
  const int64_t wr0 = i0 + wm * 64, wc0 = j0 + wn * 16;
  const bool active = !(wc0 + 15 < wr0) && wr0 < n && wc0 < n;

  // LDS-DMA pieces of one stage (1 KB = kRows operand rows): wave w takes A pieces w, w + 8, ..., B pieces
  // w, w + 8, ..., and waves 0 .. kWWp − 1 one digit piece each. Source chunk swizzled: LDS slot s of row r
  // holds chunk s ^ swz(r).
  const int prow = lane / (BK / 16), pslot = lane % (BK / 16);
  const bool wdig = wave < SG::kWWp;
  const int pieces = SG::kA + SG::kB + (wdig ? 1 : 0);
  auto issue = [&](int64_t st) {
    int8_t* base = lds + (int)(st % SG::kNS) * SG::kBytes;
#pragma unroll
    for (int a = 0; a < SG::kA; a++) {
      const int xx = wave + SG::kNW * a, r = xx * SG::kRows + prow;
      __builtin_amdgcn_global_load_lds((const void*)(Dt + (i0 + r) * kp + st * BK + ((pslot ^ SG::swz(r)) << 4)),
                                       (void*)(base + xx * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int a = 0; a < SG::kB; a++) {
      const int xx = wave + SG::kNW * a, r = xx * SG::kRows + prow;
      __builtin_amdgcn_global_load_lds((const void*)(St + (j0 + r) * kp + st * BK + ((pslot ^ SG::swz(r)) << 4)),
                                       (void*)(base + BM * BK + xx * 1024), 16, 0, 0);
    }
    if (wdig)
      __builtin_amdgcn_global_load_lds((const void*)(WW + st * (int64_t)((BK / 128) * S * 256) + wave * 1024 + lane * 16),
                                       (void*)(base + BM * BK + XG_BN * BK + wave * 1024), 16, 0, 0);
  };
  // stage st's pieces have landed (this wave's, by a counted wait; the others', by the barrier) and every
  // wave has finished reading the buffer the next issue overwrites (read one stage earlier)
  constexpr int PD = SG::kNS - 1;
  auto arrive = [&](int64_t st) {
    const int64_t ahead = (st1 - 1 - st) < (PD - 1) ? (st1 - 1 - st) : (PD - 1);
    if (ahead >= 2)
      wait_vm_n<2>(pieces);
    else if (ahead == 1)
      wait_vm_n<1>(pieces);
    else
      wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (st + PD < st1) issue(st + PD);
  };

  i32x4 acc[S][4];
#pragma unroll
  for (int s = 0; s < S; s++)
#pragma unroll
    for (int m = 0; m < 4; m++) acc[s][m] = (i32x4){0, 0, 0, 0};

  const int fr = lane & 15, g = lane >> 4;
  for (int64_t st = st0; st < st0 + PD && st < st1; st++) issue(st);
  if (!active) {  // a wave wholly below the diagonal or in the padding: stages and barriers only
    for (int64_t st = st0; st < st1; st++) arrive(st);
    return;
  }
  for (int64_t st = st0; st < st1; st++) {
    arrive(st);
    const int8_t* A = lds + (int)(st % SG::kNS) * SG::kBytes;
    const int8_t* B = A + BM * BK;
    const int8_t* Wd = B + XG_BN * BK;
    // the stage's NKS·S (k-step, slice) pairs in one unrolled sequence: digits two pairs ahead in a ring of
    // three register sets, the next k-step's fragments loaded during the current k-step (ring of two)
    constexpr int NKS = BK / 64;
    i32x4 af[2][4], bf[2], w1[3], w2[3];
    auto load_frags = [&](int ks) {
      const int c = ks * 4 + g;  // this lane group's 16-locus chunk
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const int r = wm * 64 + m * 16 + fr;
        af[ks & 1][m] = *reinterpret_cast<const i32x4*>(A + r * BK + ((c ^ SG::swz(r)) << 4));
      }
      const int rb = wn * 16 + fr;
      bf[ks & 1] = *reinterpret_cast<const i32x4*>(B + rb * BK + ((c ^ SG::swz(rb)) << 4));
    };
    auto load_digits = [&](int t) {
      const int ks = t / S;  // digit group ks/2 (128 loci), chunk (ks % 2)·4 + g inside it
      const int8_t* wp = Wd + (ks >> 1) * (S * 256) + (t % S) * 256 + ((ks & 1) * 4 + g) * 32;
      w1[t % 3] = *reinterpret_cast<const i32x4*>(wp);
      w2[t % 3] = *reinterpret_cast<const i32x4*>(wp + 16);
    };
    auto perm = [&](int t) {
      i32x4 r;
#pragma unroll
      for (int e = 0; e < 4; e++)
        r[e] = (int)__builtin_amdgcn_perm((uint32_t)w1[t % 3][e], (uint32_t)w2[t % 3][e], (uint32_t)bf[(t / S) & 1][e]);
      return r;
    };
    // software pipeline over the pairs t: the MFMAs of t issue beside the v_perms of t + 1 (digits loaded at
    // t − 2) and the digit loads of t + 3
    load_frags(0);
    load_digits(0);
    load_digits(1);
    load_digits(2);
    i32x4 bs = perm(0);
#pragma unroll
    for (int t = 0; t < NKS * S; t++) {
      const int ks = t / S, s = t % S;
      if (s == 1 && ks + 1 < NKS) load_frags(ks + 1);
      // each MFMA of t issued beside one v_perm of t + 1 (explicit pairs, no issue priority: 1.7 % faster
      // than the MFMAs grouped under s_setprio and the v_perms before them)
      i32x4 bn = bs;
      if (t + 3 < NKS * S) load_digits(t + 3);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 4; m++) {
        acc[s][m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[ks & 1][m], bs, acc[s][m], 0, 0, 0);
        if (t + 1 < NKS * S)
          bn[m] = (int)__builtin_amdgcn_perm((uint32_t)w1[(t + 1) % 3][m], (uint32_t)w2[(t + 1) % 3][m],
                                             (uint32_t)bf[((t + 1) / S) & 1][m]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int m = 0; m < 4; m++) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // one VALU (a v_perm of t + 1)
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);    // the digit loads of t + 3
      __builtin_amdgcn_sched_barrier(0);
      bs = bn;
    }
  }

  if (slot >= 0) {
    // split unit: publish this range's partials (write-back + agent release before the counter, the guide's
    // split-K hand-off per wave); the range that draws the last ticket acquires and adds the others'
    i32x4* mine = part + (((slot * ks_split + kpart) * 8 + wave) * S * 4) * 64 + lane;
#pragma unroll
    for (int s = 0; s < S; s++)
#pragma unroll
      for (int m = 0; m < 4; m++) mine[(s * 4 + m) * 64] = acc[s][m];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      last = __hip_atomic_fetch_add(&cnt[slot * 8 + wave], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ks_split - 1;
    }
    last = __builtin_amdgcn_readfirstlane(last);
    if (!last) return;
    if (lane == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    for (int kk = 0; kk < ks_split; kk++) {
      if (kk == kpart) continue;
      const i32x4* other = part + (((slot * ks_split + kk) * 8 + wave) * S * 4) * 64 + lane;
#pragma unroll
      for (int s = 0; s < S; s++)
#pragma unroll
        for (int m = 0; m < 4; m++) acc[s][m] += other[(s * 4 + m) * 64];
    }
  }

  // epilogue: T = n² Σ_s 128^s acc_s − NU_i − NU_k + C in int128 → G = T 2^−F / n²
  const i128 C = *Cp;
  const u128 n2 = (u128)n * (u128)n;
  const double dn2 = (double)n * (double)n;
  const int64_t col = wc0 + fr;
  const u128 nuk = (u128)NU[col];
#pragma unroll
  for (int m = 0; m < 4; m++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int64_t row = wr0 + m * 16 + g * 4 + r;
      // unsigned 128-bit arithmetic (wrap-around defined); the final T fits 127 bits (host range check)
      u128 a = 0;
#pragma unroll
      for (int s = S - 1; s >= 0; s--) a = a * 128u + (u128)(i128)acc[s][m][r];
      const i128 T = (i128)(n2 * a - (u128)NU[row] - nuk + (u128)C);
      const double v = (row < n && col < n) ? ldexp(i128_to_double(T) / dn2, -F) : 0.0;
      double* o = G + row * ldg + col;
      *o = accum ? *o + v : v;
    }
  }
}

// ---- host side ---------------------------------------------------------------------------------
constexpr int64_t kXgSplitPieces = 256;  // the most (unit, loci range) pieces of the split tail (one round of 256 CUs)
struct XgLayout {
  int64_t npad, kp, nst, nr, ncp;
  int64_t off_dt, off_st, off_ww, off_w, off_t, off_v, off_cp, off_up, off_nu, off_c, off_info, off_sp, off_part, off_cnt, total;
};

static XgLayout xg_layout(int64_t n, int64_t p) {
  XgLayout L{};
  L.npad = npad_of(n);
  L.kp = round_up(p < 1 ? 1 : p, XG_KALIGN);
  L.nst = L.kp / XG_BK;
  // loci-tile groups of the transpose + U kernel (GBM_XG_TNR: A/B knob, read at sizing and launch alike)
  // about 8192 blocks in all (more loci groups measured faster at C2: 64 → 312 µs, 512 → 215 µs), at
  // least 64 groups
  const int64_t xblocks = (L.npad + 255) / 256;  // the transpose grid's x
  int64_t tnr = std::max<int64_t>(64, (8192 + xblocks - 1) / xblocks);
  if (const char* te = ::gbm::knob("GBM_XG_TNR")) tnr = std::max<int64_t>(1, std::min<int64_t>(atoll(te), 1024));
  L.nr = std::min<int64_t>(L.kp / 64, tnr);
  L.ncp = (L.kp + XG_UBLK - 1) / XG_UBLK;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    const int64_t at = o;
    o = round_up(o + bytes, 256);
    return at;
  };
  L.off_dt = take(L.npad * L.kp);
  L.off_st = take(L.npad * L.kp);
  L.off_ww = take(L.nst * XG_SMAX * 256 + 4096);
  L.off_w = take(8 * L.kp);
  L.off_t = take(8 * L.kp);
  L.off_v = take(16 * L.kp);
  L.off_cp = take(16 * L.ncp);
  L.off_up = take(16 * L.nr * L.npad);
  L.off_nu = take(16 * L.npad);
  L.off_c = take(16);
  L.off_info = take(sizeof(XgInfo));
  L.off_sp = take((int64_t)XG_SGRID * sizeof(XgStatsPart));
  // split-unit partials: at most kXgSplitPieces (unit, range) pieces x 8 waves x XG_SMAX x 4 i32x4 per lane
  L.off_part = take((int64_t)kXgSplitPieces * 8 * XG_SMAX * 4 * 64 * 16);
  L.off_cnt = take((int64_t)kXgSplitPieces * 8 * 4);
  L.total = o;
  return L;
}

// S digits and the scale 2^F for the kept weights (exponents [emin, emax] by ilogb, largest wmax): F puts
// the smallest weight's significand on the integer grid (every weight exact), and S is the fewest
// balanced base-128 digits whose range (max 63·(128^S − 1)/127) holds W_max = wmax·2^F. With no such
// S ≤ XG_SMAX (weights spanning more than ~2^16), S = XG_SMAX and F shrinks: the smallest weights are
// rounded to the grid (relative error ≤ 2^−(69 − Δe) each). Returns 1 when exact.
// W = w·2^F as the digits kernel forms it (significand shifted, rounded half up below the grid)
static i128 xg_fixed(double w, int F) {
  if (!(w > 0.0)) return 0;
  int e;
  const double mant = std::frexp(w, &e);
  const long long M = (long long)std::ldexp(mant, 53);
  const int sh = e - 53 + F;
  if (sh >= 0) return (i128)M << sh;
  const int r = -sh;
  return r >= 63 ? (i128)0 : (i128)((M + (1LL << (r - 1))) >> r);
}

// the largest W that S balanced base-128 digits in [−64, 63] represent: 63·(128^S − 1)/127
static i128 xg_digit_max(int S) {
  i128 m = 0;
  for (int s = 0; s < S; s++) m = m * 128 + 63;
  return m;
}

static int xg_choose(int emin, int emax, double wmax, int& S, int& F) {
  (void)emax;
  F = 52 - emin;
  if (F + std::ilogb(wmax) < 7 * XG_SMAX) {  // W_max < 2^70: compare in exact integers
    const i128 W = xg_fixed(wmax, F);
    for (S = XG_SMIN; S <= XG_SMAX; S++)
      if (W <= xg_digit_max(S)) return 1;
  }
  S = XG_SMAX;
  F = 7 * S - 3 - std::ilogb(wmax);  // W_max < 2^(7S−2) < 63·(128^S − 1)/127
  return 0;
}

int64_t grm_exact_workspace_bytes(int64_t n, int64_t p) { return xg_layout(n, p).total; }

// The status launch_grm_exact leaves in its workspace, read after the stream has drained: bit 1 (a byte outside
// {0, 1, 2}; launch_grm_exact already failed with GBM_E_ARG) and bit 2 (a weight did not fit its S digits: the
// digit GEMMs summed a wrong W, so G is invalid — xg_choose's bound makes that impossible, this check makes a
// violation loud). Synchronises the stream.
int grm_exact_status(const void* ws, int64_t n, int64_t p, hipStream_t s) {
  if (!ws || n < 2 || p < 1) return fail(GBM_E_ARG, "gbm_dev_grm_exact_status: bad arguments");
  const XgLayout L = xg_layout(n, p);
  XgInfo h{};
  GBM_HIP_TRY(hipMemcpyAsync(&h, static_cast<const int8_t*>(ws) + L.off_info, sizeof(h), hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  if (h.bad & 2)
    return fail(GBM_E_HIP, "exact GRM: a locus weight did not fit its base-128 digits (XgInfo bit 2); G is invalid");
  if (h.bad & 1) return fail(GBM_E_ARG, "exact GRM: a dosage outside {0, 1, 2}");
  return GBM_OK;
}

int launch_grm_exact(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, double* G, int64_t ldg,
                     double* mean, double* sd, int32_t* keep, int64_t* q_dev, int accum, void* ws, int64_t ws_bytes,
                     int32_t* slices_out, hipStream_t s) {
  if (!D || !G || !mean || !sd || !keep || !q_dev || !ws || p < 1 || n < 2 || ldd < n || ldg < npad_of(n) || ploidy != 2)
    return fail(GBM_E_ARG, "gbm_dev_grm_exact_i8: bad arguments (diploid dosages {0,1,2}, p >= 1, n >= 2, ldg >= npad)");
  // int32 digit sums: |Σ_j d·ω| <= 252 p < 2^31 (p <= 2^23); the int128 bracket is checked below once W_max is known
  if (p > ((int64_t)1 << 23) || n > ((int64_t)1 << 19))
    return fail(GBM_E_ARG, "gbm_dev_grm_exact_i8: p <= 2^23 loci and n <= 2^19 individuals per call (integer ranges of the "
                           "exact sums); split the loci into shards (accum = 1) beyond that");
  const XgLayout L = xg_layout(n, p);
  if (ws_bytes < L.total) return fail(GBM_E_ARG, "gbm_dev_grm_exact_i8: workspace too small (gbm_dev_grm_exact_workspace)");
  int8_t* w8 = static_cast<int8_t*>(ws);
  int8_t* Dt = w8 + L.off_dt;
  int8_t* St = w8 + L.off_st;
  int8_t* WW = w8 + L.off_ww;
  double* w = reinterpret_cast<double*>(w8 + L.off_w);
  int64_t* tcol = reinterpret_cast<int64_t*>(w8 + L.off_t);
  uint4* VL = reinterpret_cast<uint4*>(w8 + L.off_v);
  i128* Cpart = reinterpret_cast<i128*>(w8 + L.off_cp);
  i128* Upart = reinterpret_cast<i128*>(w8 + L.off_up);
  i128* NU = reinterpret_cast<i128*>(w8 + L.off_nu);
  i128* C = reinterpret_cast<i128*>(w8 + L.off_c);
  XgInfo* info = reinterpret_cast<XgInfo*>(w8 + L.off_info);

  XgStatsPart* spart = reinterpret_cast<XgStatsPart*>(w8 + L.off_sp);
  const int sgrid = (int)std::min<int64_t>((p + 3) / 4, XG_SGRID);  // one wave per locus (grid-strided)
  xg_stats_kernel<<<sgrid, 256, 0, s>>>(D, ldd, p, n, 1.0 / ploidy, mean, sd, keep,
                                        reinterpret_cast<unsigned long long*>(q_dev), w, tcol, spart);
  GBM_LAUNCH_CHECK();
  xg_stats_reduce_kernel<<<1, 256, 0, s>>>(spart, sgrid, reinterpret_cast<unsigned long long*>(q_dev), info);
  GBM_LAUNCH_CHECK();
  XgInfo h{};
  GBM_HIP_TRY(hipMemcpyAsync(&h, info, sizeof(h), hipMemcpyDeviceToHost, s));
  GBM_HIP_TRY(hipStreamSynchronize(s));
  if (h.bad & 1) return fail(GBM_E_ARG, "gbm_dev_grm_exact_i8: a dosage outside {0, 1, 2}");
  int S = XG_SMIN, F = 0;
  if (h.emax >= h.emin) {  // else no kept locus: W = 0, G = 0
    double wmax;
    memcpy(&wmax, &h.wmax_bits, sizeof(wmax));
    xg_choose(h.emin, h.emax, wmax, S, F);
    // every term of the bracket T = n²A − nU_i − nU_k + C is at most 4 n² p W_max in magnitude (d, t/n <= 2),
    // so the int128 evaluation is exact when 16 n² p W_max < 2^127 (C3: 2^50.4 · W_max, W_max < 2^68: 2^122.4)
    const double lg = 4.0 + 2.0 * std::log2((double)n) + std::log2((double)p) + std::log2(std::ldexp(wmax, F));
    if (!(lg < 126.5))
      return fail(GBM_E_ARG, "gbm_dev_grm_exact_i8: n^2 p W_max exceeds the 128-bit bracket range; split the loci "
                             "into shards (accum = 1)");
  }
  // (tests) GBM_XG_TEST_S: force fewer digits than xg_choose's S, so the digits kernel flags W out of range
  // (XgInfo.bad bit 2) and grm_exact_status reports it instead of the caller using a wrong G
  if (const int64_t ts = knob_i64("GBM_XG_TEST_S", 0); ts >= 1 && ts < S) S = (int)std::max<int64_t>(XG_SMIN, ts);
  if (slices_out) *slices_out = S;
  xg_digits_kernel<<<(unsigned)L.ncp, XG_UBLK, 0, s>>>(w, tcol, p, L.kp, S, F, WW, VL, Cpart, info);
  GBM_LAUNCH_CHECK();
  xg_transpose_u_kernel<<<dim3((unsigned)((L.npad + 255) / 256), (unsigned)L.nr), 256, 0, s>>>(D, ldd, p, n, L.kp, L.npad,
                                                                                              VL, Dt, St, Upart);
  GBM_LAUNCH_CHECK();
  xg_u_reduce_kernel<<<(unsigned)((L.npad + 63) / 64), 256, 0, s>>>(Upart, L.nr, L.npad, n, Cpart,
                                                                                      L.ncp, NU, C);
  GBM_LAUNCH_CHECK();
  const char* be = ::gbm::knob("GBM_XG_BK");
  const int bk = (be && atoi(be) == 256) ? 256 : 128;
  const char* me = ::gbm::knob("GBM_XG_BM");  // 128: 128 x 64 tiles, one 8-wave workgroup per CU; 64 (default): 64 x 64, two
  const int bm = (bk == 128 && !(me && atoi(me) == 128)) ? 64 : 128;  // 64 x 64 measured fastest at C2
  const int64_t rt = bm / XG_BN;
  const int64_t nI = (n + bm - 1) / bm, nJ = (n + XG_BN - 1) / XG_BN;
  const int64_t nunits = nI * nJ - rt * nI * (nI - 1) / 2;
  // the partial last round of a grid with one unit per CU is split in loci ranges (GBM_XG_SPLIT=0: off)
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus < 1) cus = 256;
    if (bm == 64) cus *= 2;  // two workgroups per CU
    const char* ce = ::gbm::knob("GBM_XG_CUS");  // tests: pretend a chip of this many CUs (forces the split tail)
    if (ce && atoi(ce) > 0) cus = atoi(ce);
  }
  const char* se = ::gbm::knob("GBM_XG_SPLIT");
  int64_t nfull = nunits, ks = 1;
  if (!(se && *se && atoi(se) == 0)) {
    const int64_t tail = nunits % cus;
    if (nunits > cus && tail > 0) {
      ks = std::min<int64_t>(std::min<int64_t>(8, cus / tail), kXgSplitPieces / tail);
      if (ks >= 2) nfull = nunits - tail;
      else ks = 1;
    }
  }
  i32x4* part = reinterpret_cast<i32x4*>(w8 + L.off_part);
  int32_t* cnt = reinterpret_cast<int32_t*>(w8 + L.off_cnt);
  if (nfull < nunits) GBM_HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)(nunits - nfull) * 8 * 4, s));
  const unsigned grid = (unsigned)(nfull + (nunits - nfull) * ks);
  const char* oe = ::gbm::knob("GBM_XG_ORDER");
  // 0: row-major units (default); "AxB": blocks of A row blocks x B column blocks (row-major blocks)
  int order = 0;
  if (oe && *oe) {
    int a = 0, b = 0;
    if (sscanf(oe, "%dx%d", &a, &b) == 2 && a > 0 && b > 0 && a < 256 && b < 256) order = (a << 8) | b;
    else if (atoi(oe) == 1) order = (XG_OBI << 8) | XG_OBJ;
  }
#define XG_LAUNCH(SS, BKK, BMM) \
  xg_gemm_kernel<SS, BKK, BMM><<<grid, BMM * 4, 0, s>>>(Dt, St, L.kp, WW, NU, C, n, F, nI, nJ, nunits, G, ldg, accum, order, nfull, (int)ks, part, cnt)
  if (bk == 256) {
    if (S == 8) XG_LAUNCH(8, 256, 128); else if (S == 9) XG_LAUNCH(9, 256, 128); else XG_LAUNCH(10, 256, 128);
  } else if (bm == 64) {
    if (S == 8) XG_LAUNCH(8, 128, 64); else if (S == 9) XG_LAUNCH(9, 128, 64); else XG_LAUNCH(10, 128, 64);
  } else {
    if (S == 8) XG_LAUNCH(8, 128, 128); else if (S == 9) XG_LAUNCH(9, 128, 128); else XG_LAUNCH(10, 128, 128);
  }
#undef XG_LAUNCH
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// Training-set dosages of a resident fp64 genotype matrix whose values are dosages/2 (a session of int8
// or synthetic genotypes): D[j, i] = 2·Xt[j, idx[i]] as bytes (exact), the input of the exact GRM.
__global__ void __launch_bounds__(256) xg_gather_dosage_kernel(const double* __restrict__ Xt, int64_t ldx, int64_t p,
                                                               const int32_t* __restrict__ idx, int64_t nT,
                                                               int8_t* __restrict__ D) {
  const int64_t j = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nT; i += (int64_t)gridDim.x * 256)
    D[j * nT + i] = (int8_t)__double2int_rn(2.0 * Xt[j * ldx + idx[i]]);
}

int launch_gather_dosage(const double* Xt, int64_t ldx, int64_t p, const int32_t* idx, int64_t nT, int8_t* D,
                         hipStream_t s) {
  if (p < 1 || nT < 1) return GBM_OK;
  const unsigned gx = (unsigned)std::min<int64_t>((nT + 255) / 256, 64);
  for (int64_t j0 = 0; j0 < p; j0 += 65535) {
    const unsigned gy = (unsigned)std::min<int64_t>(65535, p - j0);
    xg_gather_dosage_kernel<<<dim3(gx, gy), 256, 0, s>>>(Xt + j0 * ldx, ldx, gy, idx, nT, D + j0 * nT);
    GBM_LAUNCH_CHECK();
  }
  return GBM_OK;
}

// ---- dosage detection (grm_mode exact / auto on fp64 input, include/gbm.h) -----------------------------
// p locus rows of n fp64 values (row j at X + j·ldx): D[j·ldd + i] = 2·x as a byte (if D != NULL), and
// *bad = 1 when any 2x is not exactly 0, 1 or 2 (NaN and ±Inf included). HBM-bound: 8 B read + 1 B written
// per cell; bad is only ever set to 1 (plain stores of one value, no atomics).
template <bool kWrite>
__global__ void __launch_bounds__(256) dosage_from_f64_kernel(const double* __restrict__ X, int64_t ldx, int64_t n,
                                                              int64_t p, int8_t* __restrict__ D, int64_t ldd,
                                                              int32_t* __restrict__ bad) {
  int off = 0;
  for (int64_t j = blockIdx.y; j < p; j += gridDim.y) {
    const double* row = X + j * ldx;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
      const double v = 2.0 * row[i];
      off |= !(v == 0.0 || v == 1.0 || v == 2.0);
      if (kWrite) D[j * ldd + i] = (int8_t)(v == 1.0 ? 1 : v == 2.0 ? 2 : 0);
    }
  }
  if (__any(off) && (threadIdx.x & 63) == 0) *bad = 1;
}

// the same check on dosage bytes: *bad = 1 when any byte is outside {0, 1, 2}
__global__ void __launch_bounds__(256) dosage_check_i8_kernel(const int8_t* __restrict__ D, int64_t ldd, int64_t n,
                                                              int64_t p, int32_t* __restrict__ bad) {
  int off = 0;
  for (int64_t j = blockIdx.y; j < p; j += gridDim.y) {
    const int8_t* row = D + j * ldd;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
      const int d = row[i];
      off |= (d < 0 || d > 2);
    }
  }
  if (__any(off) && (threadIdx.x & 63) == 0) *bad = 1;
}

static dim3 dosage_grid(int64_t n, int64_t p) {
  return dim3((unsigned)std::min<int64_t>((n + 255) / 256, 16), (unsigned)std::min<int64_t>(p, 8192));
}

int launch_dosage_from_f64(const double* X, int64_t ldx, int64_t n, int64_t p, int8_t* D, int64_t ldd, int32_t* bad,
                           hipStream_t s) {
  if (p < 1 || n < 1) return GBM_OK;
  if (D)
    dosage_from_f64_kernel<true><<<dosage_grid(n, p), 256, 0, s>>>(X, ldx, n, p, D, ldd, bad);
  else
    dosage_from_f64_kernel<false><<<dosage_grid(n, p), 256, 0, s>>>(X, ldx, n, p, nullptr, 0, bad);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

int launch_dosage_check_i8(const int8_t* D, int64_t ldd, int64_t n, int64_t p, int32_t* bad, hipStream_t s) {
  if (p < 1 || n < 1) return GBM_OK;
  dosage_check_i8_kernel<<<dosage_grid(n, p), 256, 0, s>>>(D, ldd, n, p, bad);
  GBM_LAUNCH_CHECK();
  return GBM_OK;
}

// host-side digit-count choice, exported for the CPU algebra tests (no device work)
int xg_choose_host(int emin, int emax, double wmax, int* S, int* F) {
  int s = 0, f = 0;
  const int exact = xg_choose(emin, emax, wmax, s, f);
  if (S) *S = s;
  if (F) *F = f;
  return exact;
}

}  // namespace gbm

extern "C" int gbm_debug_xg_choose(double wmin, double wmax, int* slices_out, int* shift_out) {
  if (!(wmin > 0.0) || !(wmax >= wmin)) return gbm::fail(GBM_E_ARG, "gbm_debug_xg_choose: need 0 < wmin <= wmax");
  return gbm::xg_choose_host(std::ilogb(wmin), std::ilogb(wmax), wmax, slices_out, shift_out);
}

extern "C" int64_t gbm_dev_grm_exact_workspace(int64_t n, int64_t p) { return gbm::grm_exact_workspace_bytes(n, p); }

extern "C" int gbm_dev_grm_exact_status(const void* workspace, int64_t n, int64_t p, void* stream) {
  return gbm::grm_exact_status(workspace, n, p, (hipStream_t)stream);
}

extern "C" int gbm_dev_grm_exact_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, double* G,
                                    int64_t ldg, double* mean, double* sd, int32_t* keep, int64_t* q_dev, int accum,
                                    void* workspace, int64_t ws_bytes, int32_t* slices_out, void* stream) {
  return gbm::launch_grm_exact(D, ldd, p, n, ploidy, G, ldg, mean, sd, keep, q_dev, accum, workspace, ws_bytes,
                               slices_out, (hipStream_t)stream);
}
