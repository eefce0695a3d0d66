// Blocked right-looking LDL^T (no pivoting) of a dense SPD matrix in lower 64x64 tiles,
// trailing updates on v_mfma_f64_16x16x4_f64, plus the forward / backward substitutions.
//
// Reference semantics: LinearSolverEigen::solve (ThirdParty/g2o/g2o/solvers/
// linear_solver_eigen.h:94-126) = Eigen SimplicialLDLT: A = L D L^T without pivoting, the
// solve fails only on an exact zero pivot.  Elimination order and the reduction order of
// every sum are fixed here (no atomics), so results are bitwise reproducible.
//
// One launch per panel step k (T launches) + one backward launch:
//   workgroup 0      : factor A_kk = L_kk D_k L_kk^T in LDS, Linv_kk = L_kk^-1,
//                      u_k = Linv_kk b_k, z_k = D_k^-1 u_k
//   workgroup (i, j) : k < j <= i < T.  Re-factors A_kk in LDS (cheaper than a grid-wide
//                      dependency), W_x = A_xk Linv_kk^T (MFMA), G_i = W_i D_k^-1 = L_ik,
//                      A_ij -= G_i W_j^T (MFMA).  Diagonal tiles also store L_ik and update
//                      the right-hand side b_i -= L_ik u_k.
// backward (one workgroup): x_k = Linv_kk^T z_k, z_j -= L_kj^T x_k for j < k.
#include "ldlt.hpp"
#include <atomic>
#include <map>
#include <mutex>
#include <set>
#include <utility>
#include <vector>
#include <algorithm>

namespace mcs {
namespace ldlt {

namespace {

// LDS row stride in doubles.  66 = 2 (mod 32): the MFMA operand reads (lane (r, k) of a
// 16 x 4 sub-block at r * LS + k) hit 32 distinct bank pairs per half-wave (conflict-free);
// the row-per-lane accesses of the panel elimination are 2-way.
constexpr int LS = TB + 2;
typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

// Tiles move global -> registers -> LDS in two phases so that all of a thread's loads (of
// every tile it needs) are in flight together: 8 x 16-byte loads per tile per thread.
__device__ __forceinline__ void fetch_tile(d2 (&v)[8], const double* __restrict__ g) {
  const d2* g2 = reinterpret_cast<const d2*>(g);
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = g2[threadIdx.x + 256 * i];
}
__device__ __forceinline__ void put_tile(double* s, const d2 (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int e = 2 * (threadIdx.x + 256 * i);
    *reinterpret_cast<d2*>(&s[(e >> 6) * LS + (e & 63)]) = v[i];
  }
}
// diagonal tile: only the lower triangle is defined (the strict upper part of the storage is
// never written by the producers and may hold stale bits), so it is stored as 0
__device__ __forceinline__ void put_tile_lower(double* s, const d2 (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int e = 2 * (threadIdx.x + 256 * i);
    const int r = e >> 6, c = e & 63;
    d2 w = v[i];
    if (c > r) w.x = 0.0;
    if (c + 1 > r) w.y = 0.0;
    *reinterpret_cast<d2*>(&s[r * LS + c]) = w;
  }
}
__device__ __forceinline__ void load_tile_lower(double* s, const double* __restrict__ g) {
  d2 v[8];
  fetch_tile(v, g);
  put_tile_lower(s, v);
}

#ifdef MCS_LDLT_PROBE
__device__ long long g_ldlt_stamps[16];
#define LDLT_STAMP(i) do { if (threadIdx.x == 0) g_ldlt_stamps[i] = __builtin_amdgcn_s_memtime(); } while (0)
// per (step, workgroup) phase clocks of k_panel: [k][wg][8]
__device__ long long g_panel_stamps[32 * 256 * 8];
#define PANEL_STAMP(i) do { if (threadIdx.x == 0 && k < 32 && blockIdx.x < 256) \
    g_panel_stamps[((size_t)k * 256 + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define LDLT_STAMP(i) do { } while (0)
#define PANEL_STAMP(i) do { } while (0)
#endif

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// X = L_BB^-1 of the unit-lower 16x16 diagonal block at (B, B), by one wave: lane column
// c = lane & 15 (four copies), column-oriented substitution (once x[k] is final it updates
// every later row: a 15-deep FMA chain instead of 120); the per-row accumulation order is
// still k ascending.  L entries are uniform LDS reads (broadcast).  Lanes 0..15 write X.
__device__ __forceinline__ void inv_diag16(const double* sA, double* sI, int B) {
  const int l = threadIdx.x & 63, c = l & 15;
  double x[16];
#pragma unroll
  for (int r = 0; r < 16; r++) x[r] = (r == c) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < 15; k++)
#pragma unroll
    for (int r = k + 1; r < 16; r++) x[r] = __builtin_fma(-sA[(B + r) * LS + B + k], x[k], x[r]);
  if (l < 16) {
#pragma unroll
    for (int r = 0; r < 16; r++) sI[(B + r) * LS + B + c] = x[r];
  }
}

// off-diagonal block X_ij = -X_ii (sum_{k=j}^{i-1} L_ik X_kj) of L^-1 (one wave, MFMA); the
// inner sum stays in accumulator layout, which is the B-operand layout of the outer product
__device__ __forceinline__ void offdiag_block(const double* sA, double* sI, int i, int j) {
  const int l = threadIdx.x & 63, r16 = l & 15, k4 = l >> 4;
  d4 s = {0.0, 0.0, 0.0, 0.0};
  for (int k = j; k < i; k++) {
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += 4) {
      const double av = sA[(16 * i + r16) * LS + 16 * k + k0 + k4];   // L_ik[m][kk]
      const double bv = sI[(16 * k + k0 + k4) * LS + 16 * j + r16];   // X_kj[kk][n]
      s = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, s, 0, 0, 0);
    }
  }
  d4 xo = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const double av = sI[(16 * i + r16) * LS + 16 * i + 4 * r + k4];  // X_ii[m][4r + kk]
    xo = __builtin_amdgcn_mfma_f64_16x16x4f64(av, s[r], xo, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) sI[(16 * i + k4 + 4 * r) * LS + 16 * j + r16] = -xo[r];
}

// Panel elimination of columns P..P+15 by wave p (lane l = row l, a[] = row l of the panel),
// the textbook right-looking step per column J = P + j:
//   d = a_J[j] (readlane), r = 1/d (v_rcp_f64 + two Newton steps), l = a[j] r,
//   a[m] -= l a_{P+m}[j]  (m > j)
// Measured on gfx950 (tools/bench/lat_probe2.hip, one wave): a dependent f64 FMA 7 cycles and
// an independent one 7 (f64 VALU issues at half the f32 rate), v_rcp_f64 18, readlane -> use
// 27 per link but ~10 issue cycles per v_readlane_b32, LDS write -> uniform read -> use 77.
// So the pivot and the next column's entry travel by readlane (they are on the
// column-to-column chain), the other entries of the column by one LDS write and uniform
// reads (off the chain: they feed the bulk updates), and every store is deferred past the
// loop, so the 16 columns are one basic block with no exec-mask branches.  The arithmetic is
// the same as a column-at-a-time elimination (same operations in the same order).
// Outputs: L (strict lower) and D (diagonal) of the panel's columns in sA, C^T of the rows
// below the panel in sA's strict upper triangle (row J, column l >= P + 16).  sx: 128
// doubles of wave-private LDS scratch.
__device__ __forceinline__ void panel_bulk(double (&a)[16], const double (&cm)[16], double lj, int m0, int m1) {
#pragma unroll
  for (int m = m0; m < m1; m++)
    if (m < 16) a[m] = __builtin_fma(-lj, cm[m], a[m]);
}

__device__ __forceinline__ void panel_elim(double* sA, double* sx, int P, double (&a)[16], int* fail) {
  const int l = threadIdx.x & 63;
  double lv[16], cm[16], cn[16];
  double dsel = 0.0;
  // software pipelined: iteration j finishes column j, publishes column j+1 to LDS and issues
  // the reads of its entries at once (they are consumed an iteration later), and computes the
  // reciprocal of the next pivot in between its own bulk updates; sched_barriers pin that
  // interleaving (the compiler otherwise issues bulk updates ahead of the chain and stalls the
  // in-order wave on them)
  sx[l] = a[0];
#pragma unroll
  for (int m = 2; m < 16; m++) cn[m] = sx[P + m];
  double dn = readlane_d(a[0], P), c1 = readlane_d(a[0], P + 1);
  double r = __builtin_amdgcn_rcp(dn);
  r = __builtin_fma(r, __builtin_fma(-dn, r, 1.0), r);
#ifndef MCS_LDLT_NEWTON1
  r = __builtin_fma(r, __builtin_fma(-dn, r, 1.0), r);
#endif
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const int J = P + j;
#pragma unroll
    for (int m = j + 2; m < 16; m++) cm[m] = cn[m];
    const double cj = a[j];
    const double lj = cj * r;
    lv[j] = lj;
    if (j == 15) {
      if (l == J) dsel = cj;
      break;
    }
    a[j + 1] = __builtin_fma(-lj, c1, a[j + 1]);
    double c1n = 0.0;
    if (j + 1 <= 13) {
      double* bn = sx + ((j + 1) & 1) * 64;
      bn[l] = a[j + 1];
#ifdef MCS_LDLT_PIVOT_RL
      dn = readlane_d(a[j + 1], J + 1);
      c1n = readlane_d(a[j + 1], J + 2);
#else
      dn = bn[J + 1];
      c1n = bn[J + 2];
#endif
#pragma unroll
      for (int m = j + 3; m < 16; m++) cn[m] = bn[P + m];
    } else {
      dn = readlane_d(a[j + 1], J + 1);
      if (j + 1 <= 14) c1n = readlane_d(a[j + 1], J + 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    panel_bulk(a, cm, lj, j + 2, j + 5);
    if (l == J) dsel = cj;
    __builtin_amdgcn_sched_barrier(0);
    double rn = __builtin_amdgcn_rcp(dn);
    __builtin_amdgcn_sched_barrier(0);
    panel_bulk(a, cm, lj, j + 5, j + 7);
    __builtin_amdgcn_sched_barrier(0);
    double e = __builtin_fma(-dn, rn, 1.0);
    __builtin_amdgcn_sched_barrier(0);
    panel_bulk(a, cm, lj, j + 7, j + 8);
    __builtin_amdgcn_sched_barrier(0);
    rn = __builtin_fma(rn, e, rn);
    __builtin_amdgcn_sched_barrier(0);
    panel_bulk(a, cm, lj, j + 8, j + 9);
#ifndef MCS_LDLT_NEWTON1
    __builtin_amdgcn_sched_barrier(0);
    e = __builtin_fma(-dn, rn, 1.0);
    __builtin_amdgcn_sched_barrier(0);
    panel_bulk(a, cm, lj, j + 9, j + 10);
    __builtin_amdgcn_sched_barrier(0);
    rn = __builtin_fma(rn, e, rn);
    __builtin_amdgcn_sched_barrier(0);
    panel_bulk(a, cm, lj, j + 10, 16);
#else
    panel_bulk(a, cm, lj, j + 9, 16);
#endif
    r = rn;
    c1 = c1n;
  }
  // L on and above the diagonal too (scratch of the strict upper triangle; the diagonal is
  // overwritten by D next, in-order LDS within the wave)
#pragma unroll
  for (int k = 0; k < 16; k++) sA[l * LS + P + k] = lv[k];
  const bool diag = (l >= P && l < P + 16);
  if (diag) sA[l * LS + l] = dsel;
  if (l >= P + 16) {
#pragma unroll
    for (int k = 0; k < 16; k++) sA[(P + k) * LS + l] = a[k];
  }
  if (__any(diag && dsel == 0.0) && l == 0) *fail = 1;
}

// Partial sum of an off-diagonal block of L^-1: s += L_ik X_kj (one wave, MFMA), the k-th term
// of S_ij = sum_{k=j}^{i-1} L_ik X_kj in offdiag_block's order (callers add k ascending).
__device__ __forceinline__ void xsum_add(const double* sA, const double* sI, d4& s, int i, int k, int j) {
  const int l = threadIdx.x & 63, r16 = l & 15, k4 = l >> 4;
#pragma unroll
  for (int k0 = 0; k0 < 16; k0 += 4) {
    const double av = sA[(16 * i + r16) * LS + 16 * k + k0 + k4];   // L_ik[m][kk]
    const double bv = sI[(16 * k + k0 + k4) * LS + 16 * j + r16];   // X_kj[kk][n]
    s = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, s, 0, 0, 0);
  }
}
// X_ij = -X_ii S_ij (one wave, MFMA), S in accumulator (= B-operand) layout, as offdiag_block
__device__ __forceinline__ void xfinish(double* sI, const d4& s, int i, int j) {
  const int l = threadIdx.x & 63, r16 = l & 15, k4 = l >> 4;
  d4 xo = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const double av = sI[(16 * i + r16) * LS + 16 * i + 4 * r + k4];  // X_ii[m][4r + kk]
    xo = __builtin_amdgcn_mfma_f64_16x16x4f64(av, s[r], xo, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) sI[(16 * i + k4 + 4 * r) * LS + 16 * j + r16] = -xo[r];
}
// Trailing update of the 16x16 block (bi, bj) by panel p: A_{bi,bj} -= C_{bi,p} L_{bj,p}^T
// (C^T from sA's upper triangle), one wave, four MFMAs.
__device__ __forceinline__ void upd_block(double* sA, int p, int bi, int bj) {
  const int l = threadIdx.x & 63, r16 = l & 15, k4 = l >> 4, P = 16 * p;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < 16; k0 += 4) {
    const double av = sA[(P + k0 + k4) * LS + 16 * bi + r16];   // C[16 bi + m][P + k]
    const double bv = sA[(16 * bj + r16) * LS + P + k0 + k4];   // L[16 bj + n][P + k]
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) sA[(16 * bi + k4 + 4 * r) * LS + 16 * bj + r16] -= acc[r];
}

// LDL^T of the 64x64 tile in sA (lower triangle read) and L^-1, blocked by 16-column panels,
// with every block operation that is off the column-to-column chain moved beside the next
// panel's elimination (which occupies one wave; the other three were idle):
//   panel p        : wave p eliminates columns 16p..16p+15 (panel_elim);
//   urgent update  : the block column p+1 of the trailing matrix (the next panel's input), one
//                    16x16 block per wave (upd_block), between two barriers;
//   beside panel p : the deferred trailing blocks of panel p-1 (not needed before panel p+1),
//                    X_{p-1,p-1} = inverse of the previous diagonal block (inv_diag16) and the
//                    partial sums S_ij = sum_k L_ik X_kj of the off-diagonal L^-1 blocks whose
//                    inputs are final;
//   tail           : X_33, then X_3j = -X_33 S_3j.
// Every block is updated by its panels in panel order and every S_ij accumulates k ascending
// in one wave's registers, so the arithmetic is the same as a panel-at-a-time factorisation
// followed by offdiag_block (same operations in the same order per element).  7 barriers.
// On return sA holds L (strict lower) and D (diagonal), sI holds L^-1 (0 above the diagonal).
__device__ __forceinline__ void factor_tile(double* sA, double* sI, int* fail) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  double* sx = sI + 62 * LS;   // panel scratch (block row 3 of sI is written last)
  d4 s0 = {0.0, 0.0, 0.0, 0.0}, s1 = {0.0, 0.0, 0.0, 0.0};
  // ---- panel 0; the other waves clear the strict upper blocks of L^-1
  if (w == 0) {
    double a[16];
#pragma unroll
    for (int c = 0; c < 16; c++) a[c] = sA[l * LS + c];
    panel_elim(sA, sx, 0, a, fail);
  } else {
    for (int e = t - 64; e < TB * TB; e += 192) {
      const int rr = e >> 6, cc = e & 63;
      if ((cc >> 4) > (rr >> 4)) sI[rr * LS + cc] = 0.0;
    }
  }
  __syncthreads();
  LDLT_STAMP(0);
  if (w >= 1) upd_block(sA, 0, w, 1);               // urgent: block column 1
  __syncthreads();
  // ---- panel 1 | X00 | panel-0 blocks (2,2), (3,2), (3,3)
  if (w == 1) {
    double a[16];
#pragma unroll
    for (int c = 0; c < 16; c++) a[c] = sA[l * LS + 16 + c];
    panel_elim(sA, sx, 16, a, fail);
  } else if (w == 0) {
    inv_diag16(sA, sI, 0);
  } else if (w == 2) {
    upd_block(sA, 0, 2, 2);
    upd_block(sA, 0, 3, 2);
  } else {
    upd_block(sA, 0, 3, 3);
  }
  __syncthreads();
  LDLT_STAMP(1);
  if (w >= 2) upd_block(sA, 1, w, 2);               // urgent: block column 2
  __syncthreads();
  // ---- panel 2 | X11 | S20, S30 (k = 0) | panel-1 block (3,3)
  if (w == 2) {
    double a[16];
#pragma unroll
    for (int c = 0; c < 16; c++) a[c] = sA[l * LS + 32 + c];
    panel_elim(sA, sx, 32, a, fail);
  } else if (w == 1) {
    inv_diag16(sA, sI, 16);
  } else if (w == 0) {
    xsum_add(sA, sI, s0, 2, 0, 0);                  // S20
    xsum_add(sA, sI, s1, 3, 0, 0);                  // S30
  } else {
    upd_block(sA, 1, 3, 3);
  }
  __syncthreads();
  LDLT_STAMP(2);
  if (w == 3) upd_block(sA, 2, 3, 3);               // urgent: block column 3
  __syncthreads();
  // ---- panel 3 | X22 | X10, S21, S31 (k = 1)
  if (w == 3) {
    double a[16];
#pragma unroll
    for (int c = 0; c < 16; c++) a[c] = sA[l * LS + 48 + c];
    panel_elim(sA, sx, 48, a, fail);
  } else if (w == 2) {
    inv_diag16(sA, sI, 32);
  } else if (w == 1) {
    d4 s10 = {0.0, 0.0, 0.0, 0.0};
    xsum_add(sA, sI, s10, 1, 0, 0);
    xfinish(sI, s10, 1, 0);                         // X10
    xsum_add(sA, sI, s0, 2, 1, 1);                  // S21
    xsum_add(sA, sI, s1, 3, 1, 1);                  // S31 (k = 1)
  }
  __syncthreads();
  LDLT_STAMP(3);
  // ---- X33 | S20, S30 (k = 1), X20, S30 (k = 2) | X21, then S31 (k = 2) | S32
  if (w == 3) {
    inv_diag16(sA, sI, 48);
  } else if (w == 0) {
    xsum_add(sA, sI, s0, 2, 1, 0);                  // S20 (k = 1)
    xsum_add(sA, sI, s1, 3, 1, 0);                  // S30 (k = 1)
    xfinish(sI, s0, 2, 0);
    __builtin_amdgcn_wave_barrier();
    xsum_add(sA, sI, s1, 3, 2, 0);
  } else if (w == 1) {
    xfinish(sI, s0, 2, 1);
    __builtin_amdgcn_wave_barrier();
    xsum_add(sA, sI, s1, 3, 2, 1);
  } else {
    xsum_add(sA, sI, s1, 3, 2, 2);                  // S32
  }
  __syncthreads();
  LDLT_STAMP(4);
  if (w < 3) xfinish(sI, s1, 3, w);                 // X30, X31, X32
  __syncthreads();
  LDLT_STAMP(8);
}

#ifdef MCS_LDLT_FACTOR_V0
// LDL^T of the 64x64 tile in sA (lower triangle read) and L^-1, blocked by 16-column panels.
//   panel p (wave p, lane = row): columns 16p..16p+15 are eliminated in registers; the value of
//     column j at another row comes from v_readlane (one wave: no barrier, no LDS).  The wave
//     writes L (strict lower) and D (diagonal) of its columns into sA, and the unscaled columns
//     C = L D of the rows below the panel, transposed, into the strict upper triangle (scratch:
//     only the lower triangle and the diagonal of sA are results).
//   trailing update: A[bi][bj] -= C_bi L_bj^T for the 16x16 blocks p < bj <= bi, on
//     v_mfma_f64_16x16x4_f64, blocks spread over the 4 waves.
//   L^-1: diagonal 16x16 blocks by forward substitution with lane = column (no cross-lane
//     traffic; the L entries are LDS broadcasts), then block rows i = 1..3:
//     X_ij = -X_ii (sum_{k=j}^{i-1} L_ik X_kj) on MFMA; the inner sum stays in accumulator
//     layout, which is already the B-operand layout of the outer product.
// The column-at-a-time version this replaces needed one barrier and a 64-row exchange per
// column (~138k cycles per tile); here 8 barriers remain.
// On return sA holds L (strict lower) and D (diagonal), sI holds L^-1 (0 above the diagonal).
__device__ __forceinline__ void factor_tile_v0(double* sA, double* sI, int* fail) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int r16 = l & 15, k4 = l >> 4;
  for (int p = 0; p < 4; p++) {
    const int P = 16 * p;
    if (w == p) {
      double a[16];
#pragma unroll
      for (int c = 0; c < 16; c++) a[c] = sA[l * LS + P + c];
#ifndef MCS_LDLT_FACTOR_STD
      panel_elim(sA, sI + 62 * LS, P, a, fail);
#else
      // column broadcast through LDS (sI is scratch until the L^-1 phase): the wave writes its
      // unscaled column once and reads the pivot and the panel rows back with uniform
      // addresses (in-order LDS within one wave, no barrier); the pivot's reciprocal is one
      // v_rcp_f64 + two Newton steps instead of a per-lane IEEE division
      double* sc = sI + 63 * LS;   // row 63 of sI: written last (block row 3)
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int J = P + j;
        const double cj = a[j];
        sc[l] = cj;
        __builtin_amdgcn_wave_barrier();
        double cm[16];
#pragma unroll
        for (int m = j; m < 16; m++) cm[m] = sc[P + m];
        __builtin_amdgcn_wave_barrier();
        const double dj = cm[j];
        double r = __builtin_amdgcn_rcp(dj);
        r = __builtin_fma(r, __builtin_fma(-dj, r, 1.0), r);
        r = __builtin_fma(r, __builtin_fma(-dj, r, 1.0), r);
        const double lj = cj * r;
#pragma unroll
        for (int m = j + 1; m < 16; m++) a[m] = __builtin_fma(-lj, cm[m], a[m]);
        if (dj == 0.0 && l == 0) *fail = 1;
        if (l >= J) sA[l * LS + J] = (l > J) ? lj : cj;
        if (l >= P + 16) sA[J * LS + l] = cj;
      }
#endif
    } else if (w == p - 1) {
      // the previous panel's diagonal block is final: invert it while this panel runs
      inv_diag16(sA, sI, 16 * (p - 1));
    }
    __syncthreads();
    LDLT_STAMP(2 * p);
    const int nb = 3 - p;
    for (int b = w; b < nb * (nb + 1) / 2; b += 4) {
      int q = 0, s = b;
      while (s > q) { s -= q + 1; q++; }
      const int bi = p + 1 + q, bj = p + 1 + s;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k0 = 0; k0 < 16; k0 += 4) {
        const double av = sA[(P + k0 + k4) * LS + 16 * bi + r16];   // C[16 bi + m][P + k]
        const double bv = sA[(16 * bj + r16) * LS + P + k0 + k4];   // L[16 bj + n][P + k]
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; r++) sA[(16 * bi + k4 + 4 * r) * LS + 16 * bj + r16] -= acc[r];
    }
    __syncthreads();
    LDLT_STAMP(2 * p + 1);
  }
  // L^-1: diagonal blocks 0..2 were inverted during the next panel; block 3 now (wave 3),
  // while wave 0 forms the off-diagonal block X_10 (it needs X_00, X_11 only) and the other
  // waves clear the upper blocks
  if (w == 3) inv_diag16(sA, sI, 48);
  else if (w == 0) offdiag_block(sA, sI, 1, 0);
  for (int e = t; e < TB * TB; e += 256) {
    const int rr = e >> 6, cc = e & 63;
    if ((cc >> 4) > (rr >> 4)) sI[rr * LS + cc] = 0.0;
  }
  __syncthreads();
  LDLT_STAMP(8);
  // remaining off-diagonal blocks, one block row at a time (row i needs the rows above it)
  for (int i = 2; i < 4; i++) {
    if (w < i) offdiag_block(sA, sI, i, w);
    __syncthreads();
  }
}

#endif

// acc = X Y^T (64x64x64), wave w owns output columns [16w, 16w+16), acc[q] rows [16q, 16q+16)
// v_mfma_f64_16x16x4_f64: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15];
// result reg r of lane l is D[(l>>4) + 4r][l&15].
__device__ __forceinline__ void gemm_xyt(const double* X, const double* Y, d4 (&acc)[4]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = l & 15, k4 = l >> 4;
#pragma unroll
  for (int q = 0; q < 4; q++) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < TB; k0 += 4) {
    const double bv = Y[(16 * w + r16) * LS + k0 + k4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const double av = X[(16 * q + r16) * LS + k0 + k4];
      acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q], 0, 0, 0);
    }
  }
}

// acc = X Linv^T with Linv unit lower (zero above the diagonal): output block (q, c) only
// needs k < 16 (c + 1).  Wave w computes row block q = w for the four column blocks
// (acc[c]); with the k loop fully unrolled the triangular bounds are static: 40 MFMAs per
// wave instead of 64, every wave the same.
__device__ __forceinline__ void gemm_xlt(const double* X, const double* Li, d4 (&acc)[4]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = l & 15, k4 = l >> 4;
#pragma unroll
  for (int c = 0; c < 4; c++) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < TB; k0 += 4) {
    const double av = X[(16 * w + r16) * LS + k0 + k4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      if (k0 < 16 * (c + 1)) {
        const double bv = Li[(16 * c + r16) * LS + k0 + k4];
        acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[c], 0, 0, 0);
      }
    }
  }
}

// out[r] = sum_m M[r][m] v[m] for 64 rows (M in LDS, stride LS); 4 lanes per row, fixed
// xor-tree order.  All 256 threads call; lanes with (t & 3) == 0 get the result.
__device__ __forceinline__ double gemv_row(const double* M, const double* v) {
  const int t = threadIdx.x, r = t >> 2, q = t & 3;
  double s = 0.0;
#pragma unroll
  for (int m = q; m < TB; m += 4) s += M[r * LS + m] * v[m];
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  return s;
}

__global__ __launch_bounds__(256) void k_panel(double* __restrict__ A, double* __restrict__ b,
                                               double* __restrict__ L, double* __restrict__ Linv,
                                               double* __restrict__ z, int k, int T, int* flag,
                                               const int* skip) {
  if (skip && *skip) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* sK = sm;               // A_kk -> L_kk (strict lower) + D (diagonal)
  double* sI = sK + TB * LS;     // Linv_kk
  double* sX = sI + TB * LS;     // A_ik -> G_i = L_ik
  double* sY = sX + TB * LS;     // A_jk -> W_j
  double* sv = sY + TB * LS;     // b_k
  double* su = sv + TB;          // u_k = Linv b_k
  // LDS ints live in the dynamic region too: a static __shared__ variable would shift the
  // dynamic base off 16 B and every 16-B LDS access would be replayed (Guideline 17)
  int& fail = *reinterpret_cast<int*>(su + TB);
  const int t = threadIdx.x;
  const int wg = blockIdx.x;
  int i = -1, j = -1;
  if (wg > 0) {
    const int q = wg - 1;
    int ii = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
    while ((ii + 1) * (ii + 2) / 2 <= q) ii++;
    while (ii * (ii + 1) / 2 > q) ii--;
    i = k + 1 + ii;
    j = k + 1 + (q - ii * (ii + 1) / 2);
  }
  const bool rhs = (wg == 0) || (i == j);
  PANEL_STAMP(0);
  if (t == 0) fail = 0;
  const int l = t & 63, w = t >> 6, r16 = l & 15, k4 = l >> 4;
  // every global read of the workgroup in flight together: A_kk, A_ik, A_jk, b_k and the
  // A_ij entries this thread updates at the end (accumulator layout, kept in registers)
  d2 vK[8], vX[8], vY[8];
  double aij[4][4];
  fetch_tile(vK, A + toff(k, k, T));
  if (wg > 0) {
    fetch_tile(vX, A + toff(i, k, T));
    if (j != i) fetch_tile(vY, A + toff(j, k, T));
    const double* Aij = A + toff(i, j, T);
    const int col = 16 * w + r16;
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) aij[q][r] = Aij[(16 * q + k4 + 4 * r) * TB + col];
  }
  if (rhs && t < TB) sv[t] = b[k * TB + t];
  put_tile_lower(sK, vK);
  if (wg > 0) {
    put_tile(sX, vX);
    if (j != i) put_tile(sY, vY);
  }
  __syncthreads();
  PANEL_STAMP(1);
  factor_tile(sK, sI, &fail);
  PANEL_STAMP(2);
  if (rhs) {
    const double u = gemv_row(sI, sv);
    if ((t & 3) == 0) su[t >> 2] = u;
    __syncthreads();
  }
  if (wg == 0) {
    double* gI = Linv + (size_t)k * TB * TB;
    for (int e = t; e < TB * TB; e += 256) gI[e] = sI[(e >> 6) * LS + (e & 63)];
    if (t < TB) z[k * TB + t] = su[t] / sK[t * LS + t];
    if (t == 0 && fail) atomicOr(flag, kFlagZeroPivot);
    return;
  }
  d4 wi[4], wj[4];
  gemm_xlt(sX, sI, wi);
  if (j != i) gemm_xlt(sY, sI, wj);
  __syncthreads();
  PANEL_STAMP(3);
  {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int col = 16 * c + r16;
      const double invd = 1.0 / sK[col * LS + col];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * w + k4 + 4 * r;
        sX[row * LS + col] = wi[c][r] * invd;
        sY[row * LS + col] = (j != i) ? wj[c][r] : wi[c][r];
      }
    }
  }
  __syncthreads();
  d4 p[4];
  gemm_xyt(sX, sY, p);
  PANEL_STAMP(4);
  {
    double* Aij = A + toff(i, j, T);
    const int col = 16 * w + r16;
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * q + k4 + 4 * r;
        Aij[row * TB + col] = aij[q][r] - p[q][r];
      }
  }
  if (i == j) {
    double* Lik = L + toff(i, k, T);
    for (int e = t; e < TB * TB; e += 256) Lik[e] = sX[(e >> 6) * LS + (e & 63)];
    const double s = gemv_row(sX, su);
    if ((t & 3) == 0) b[i * TB + (t >> 2)] -= s;
  }
  PANEL_STAMP(5);
}

// L^T x = z, one workgroup of 1024 threads, left-looking:
//   x_k = Linv_kk^T (z_k - sum_{i>k} L_ik^T x_i)
// thread (c = t & 63, g = t >> 6) sums rows r = g (mod 16) of every tile below the diagonal
// (all loads independent, coalesced over c); the 16 partials are combined in a fixed order.
constexpr int kBwdNT = 1024;
__global__ __launch_bounds__(kBwdNT) void k_backward(const double* __restrict__ L,
                                                     const double* __restrict__ Linv,
                                                     const double* __restrict__ z,
                                                     double* __restrict__ x, int T,
                                                     const int* skip) {
  if (skip && *skip) return;
  extern __shared__ __attribute__((aligned(16))) double sx[];   // 64 T: solved blocks of x
  __shared__ double part[16][TB];
  __shared__ double rk[TB];
  const int t = threadIdx.x, c = t & 63, g = t >> 6;
  for (int k = T - 1; k >= 0; k--) {
    double s0 = 0.0, s1 = 0.0;
    for (int ib = k + 1; ib < T; ib++) {
      const double* Lik = L + toff(ib, k, T);
      const double* xi = sx + ib * TB;
      s0 += Lik[g * TB + c] * xi[g];
      s1 += Lik[(g + 16) * TB + c] * xi[g + 16];
      s0 += Lik[(g + 32) * TB + c] * xi[g + 32];
      s1 += Lik[(g + 48) * TB + c] * xi[g + 48];
    }
    part[g][c] = s0 + s1;
    __syncthreads();
    if (t < TB) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < 16; q++) acc += part[q][t];
      rk[t] = z[k * TB + t] - acc;
    }
    __syncthreads();
    // x_k[c] = sum_m Linv[m][c] r[m], rows m = g (mod 16)
    const double* I = Linv + (size_t)k * TB * TB;
    double u = I[g * TB + c] * rk[g] + I[(g + 16) * TB + c] * rk[g + 16];
    u += I[(g + 32) * TB + c] * rk[g + 32] + I[(g + 48) * TB + c] * rk[g + 48];
    part[g][c] = u;
    __syncthreads();
    if (t < TB) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < 16; q++) acc += part[q][t];
      sx[k * TB + t] = acc;
      x[k * TB + t] = acc;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Pipelined factorisation: ONE launch for the whole LDL^T (instead of one k_panel launch per
// step, each of whose workgroups re-factors A_kk).  Same arithmetic as the k_panel steps, so
// the results are bitwise those of the launch-per-step path:
//   * workgroup "diag" (the holder of ticket 0) walks k = 0 .. T-1: applies the last product
//     (k, k, k-1) to A_kk and b_k, factors A_kk ONCE (L_kk, D_k, Linv_kk, u_k = Linv b_k,
//     z_k = u_k / D_k), publishes Linv_kk / D_k / u_k, then forms the next panel tile
//     L_{k+1,k} = A_{k+1,k} Linv^T D^-1 and W_{k+1,k} = A_{k+1,k} Linv^T itself (look-ahead:
//     the diagonal chain never waits for another workgroup's hand-off of its own outputs);
//   * every other workgroup takes tasks from a queue in step-major order:
//       TRSM (i, k), i >= k + 2:  L_ik, W_ik from A_ik (after products 0..k-1) and Linv_kk;
//       UPDATE (i, j, k):         A_ij -= L_ik W_jk^T (and b_i -= L_ik u_k when i == j), in k
//                                 order per tile (a per-tile product counter), except
//                                 (k+1, k+1, k), which the diag workgroup applies itself.
// Deadlock freedom does not depend on residency or dispatch order: tickets are taken from one
// device-scope counter; the diag workgroup at step k waits only on tasks of steps <= k - 1, and
// every task waits only on earlier tickets or on diag steps <= its own step.  Every wait is
// bounded (PipeArgs::wait_ticks): a timeout sets the error word and the solve's failure flag, and
// every workgroup then drains out.
// Hand-offs (MI355X_MICROARCH.md, visibility; cdna_hip_programming.md Guideline 16, R1):
// payload stored write-through (sc1: 16-B buffer stores from LDS, 8-B stores from registers),
// every storing wave drains vmcnt, a workgroup barrier, ONE lane stores the flag / counter
// (relaxed, agent scope); the consumer's lane 0 polls relaxed with s_sleep, then ONE agent-scope
// acquire + vmcnt drain before the workgroup barrier, then plain loads -- the MCS_PIPE_ACQUIRE
// build; by default the consumers read with sc1 loads instead (kSc1Consume below).  Flag words
// are zeroed by a memset on the stream before every launch.
namespace {

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef unsigned u4v __attribute__((ext_vector_type(4)));
// a wait gives up after PipeArgs::wait_ticks ticks of the 100 MHz real-time counter
constexpr long long kWaitTicksDefault = 25000000;   // 0.25 s

__device__ __forceinline__ unsigned pl_load(const unsigned* p) {
  return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pl_store(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// 64x64 tile from LDS (stride LS) to global (row-major), write-through, 16 B per store
__device__ __forceinline__ void store_tile_sc1(double* g, const double* s) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, TB * TB * 8, 0x00020000);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int e = 2 * (threadIdx.x + 256 * i);
    const d2 v = *reinterpret_cast<const d2*>(&s[(e >> 6) * LS + (e & 63)]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), rs, e * 8, 0, 16);
  }
}

// Consumer side of the hand-offs.  Every byte k_pipe hands off is stored sc1 (write-through,
// 16-B tiles / 8-B words) by a workgroup whose every storing wave drained vmcnt before ONE lane's
// sc1 flag store, the waiting lane polls that flag with sc1 loads and the other waves join it at
// a barrier, one workgroup per CU (LDS), hipMalloc memory: MI355X_MICROARCH.md's hand-off table,
// first row.  So the consumer reads the handed-off bytes with sc1 loads (16-B buffer loads for
// tiles, 8-B global loads for words) and skips the agent acquire after each wait (an L2
// invalidate on the diagonal chain twice per step).  Config E (n = 1194, 19 tile steps): solve
// 0.395 -> 0.390 ms per trial, parity tests green on both forms (round 5,
// profiles/r05_c_gba_host_ab.txt).
// MCS_PIPE_ACQUIRE builds the acquire form.
#ifdef MCS_PIPE_ACQUIRE
constexpr bool kSc1Consume = false;
#else
constexpr bool kSc1Consume = true;
#endif
__device__ __forceinline__ double ld_h(const double* p) {
  if (!kSc1Consume) return *p;
  return __longlong_as_double((long long)__hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void fetch_tile_h(d2 (&v)[8], const double* g) {
  if (!kSc1Consume) { fetch_tile(v, g); return; }
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(g), 0, TB * TB * 8, 0x00020000);
#pragma unroll
  for (int i = 0; i < 8; i++)
    v[i] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * (threadIdx.x + 256 * i), 0, 16));
}
__device__ __forceinline__ void load_acc_h(double (&a)[4][4], const double* Aij) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, r16 = l & 15, k4 = l >> 4;
  const int col = 16 * w + r16;
#pragma unroll
  for (int q = 0; q < 4; q++)
#pragma unroll
    for (int r = 0; r < 4; r++) a[q][r] = ld_h(&Aij[(16 * q + k4 + 4 * r) * TB + col]);
}

// Lane 0 waits until *w_i >= v_i for every non-null word (bounded in time), then acquires; all threads get the
// outcome (false: timed out here or elsewhere).
__device__ __forceinline__ bool wg_wait(const unsigned* w0, unsigned v0, const unsigned* w1, unsigned v1,
                                     const unsigned* w2, unsigned v2, unsigned* err, int* sh_ok,
                                     long long ticks) {
  if (threadIdx.x == 0) {
    int ok = 1;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      if ((!w0 || pl_load(w0) >= v0) && (!w1 || pl_load(w1) >= v1) && (!w2 || pl_load(w2) >= v2)) break;
      if (pl_load(err) != 0u) { ok = 0; break; }
      if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) { pl_store(err, 1u); ok = 0; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (ok && !kSc1Consume) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *sh_ok = ok;
  }
  __syncthreads();
  // wave-uniform by construction; readfirstlane makes that visible to the compiler, so every
  // branch on it is a scalar branch (no exec-mask structurisation around the barriers)
  const bool ok = __builtin_amdgcn_readfirstlane(*sh_ok) != 0;
  __syncthreads();
  return ok;
}

// every storing wave drains its write-through stores, then ONE lane raises the word
__device__ __forceinline__ void wg_publish(unsigned* word, unsigned v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) pl_store(word, v);
}

struct PipeArgs {
  double* A;            // tiles (destroyed)
  double* b;            // 64 T (destroyed)
  double* L;            // off-diagonal L tiles (out)
  double* W;            // off-diagonal W = L D tiles (scratch)
  double* Linv;         // T x 64 x 64 (out)
  double* du;           // T x 128: D_k, u_k
  double* z;            // 64 T (out)
  unsigned* sync;       // [0] ticket, [1] error, [4..] product counters, panel flags, diag flags
  const int4* tasks;    // (type 0 TRSM / 1 UPDATE, i, j, k)
  int ntasks, T, ntile;
  int D;                // tile bandwidth (tiles with I - J >= D are zero and never touched)
  int* flag;
  const int* skip;
  long long wait_ticks;
};

__device__ __forceinline__ int tix(int I, int J, int T) { return (int)band_tiles(I - J, T) + J; }
// the first step whose product reaches tile row i (L_ik = 0 for k < i - (D - 1)); the product
// counters count from there, so a tile's counter holds (products applied) = (next k) - kbase
__device__ __forceinline__ int kbase(int i, int D) { return max(0, i - (D - 1)); }

#ifdef MCS_LDLT_PROBE
// probe builds only: diag step stamps [k][8] and task stamps [ticket][4] (s_memrealtime, 100 MHz)
__device__ long long g_diag_stamps[128 * 8];
__device__ long long g_task_stamps[65536 * 4];
#define DSTAMP(k, i) do { if (threadIdx.x == 0 && (k) < 128) g_diag_stamps[(k) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TSTAMP(tk, i) do { if (threadIdx.x == 0 && (tk) < 65536) g_task_stamps[(tk) * 4 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define DSTAMP(k, i) do { } while (0)
#define TSTAMP(tk, i) do { } while (0)
#endif

#ifdef MCS_PIPE_TRACE
// debug builds only (tools/bench/pipe_debug.hip): events {wg, code, a, b} into host memory
__device__ unsigned* g_pipe_trace;
__device__ unsigned g_pipe_trace_n;
__device__ __forceinline__ void ptrace(unsigned code, unsigned a, unsigned b) {
  if (threadIdx.x == 0 && g_pipe_trace) {
    const unsigned i = atomicAdd(&g_pipe_trace_n, 1u);
    if (i < 65536) {
      unsigned* e = g_pipe_trace + 4 * (size_t)i;
      __hip_atomic_store(e + 1, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(e + 2, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(e + 3, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(e + 0, blockIdx.x + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
#define PTRACE(c, a, b) ptrace((c), (unsigned)(a), (unsigned)(b))
#else
#define PTRACE(c, a, b) do { } while (0)
#endif

// W = X Linv^T (registers, wave-row layout), then sX <- W D^-1 (= L), sY <- W, as k_panel does
__device__ __forceinline__ void trsm_to_lds(double* sX, double* sY, const double* sI, const double* dvec) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, r16 = l & 15, k4 = l >> 4;
  d4 wi[4];
  gemm_xlt(sX, sI, wi);
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const int col = 16 * c + r16;
    const double invd = 1.0 / dvec[col];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = 16 * w + k4 + 4 * r;
      sX[row * LS + col] = wi[c][r] * invd;
      sY[row * LS + col] = wi[c][r];
    }
  }
  __syncthreads();
}

// the 10 lower and 6 strict-upper 16x16 blocks of a diagonal tile
__constant__ int kLowBi[10] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3};
__constant__ int kLowBj[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
__constant__ int kUpBi[6] = {0, 0, 0, 1, 1, 2};
__constant__ int kUpBj[6] = {1, 2, 3, 2, 3, 3};
// one lane's four accumulator-layout values of block (bi, bj) into the LDS tile, the strict
// upper part of a diagonal block as 0
__device__ __forceinline__ void a3_store(double* sK, const double (&v)[4], int bi, int bj) {
  const int l = threadIdx.x & 63, r16 = l & 15, k4 = l >> 4;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int row = 16 * bi + k4 + 4 * r, col = 16 * bj + r16;
    sK[row * LS + col] = (col > row) ? 0.0 : v[r];
  }
}

__device__ void diag_role(const PipeArgs& g, double* sm, int* sh_ok, int* fail) {
  double* sK = sm;
  double* sI = sK + TB * LS;
  double* sX = sI + TB * LS;
  double* sY = sX + TB * LS;
  double* sv = sY + TB * LS;
  double* su = sv + TB;
  const int T = g.T, t = threadIdx.x, l = t & 63, w = t >> 6, r16 = l & 15, k4 = l >> 4;
  unsigned* err = g.sync + 1;
  unsigned* cnt = g.sync + 4;
  unsigned* pan = cnt + g.ntile;
  unsigned* dg = pan + g.ntile;
  for (int k = 0; k < T; k++) {
    PTRACE(10, k, 0);
    DSTAMP(k, 0);
    // A_kk after products 0 .. k-2 (UPDATE tasks), then product k-1 from the tiles this
    // workgroup formed at step k-1 (still in sX / sY, u_{k-1} in su)
    if (k >= 2 && !wg_wait(cnt + tix(k, k, T), (unsigned)max(0, k - 1 - kbase(k, g.D)), nullptr, 0, nullptr, 0, err,
                           sh_ok, g.wait_ticks))
      break;
    DSTAMP(k, 1);
    // A_kk -= L_{k,k-1} W_{k,k-1}^T on the 10 lower 16x16 blocks only (the upper ones are
    // not read by the factorisation), 3 / 3 / 2 / 2 blocks per wave; each block is the same
    // MFMA chain (k ascending) as the full gemm_xyt, so the bits are the full product's
    double bv = ld_h(&g.b[k * TB + (t >> 2)]);
    {
      const double* Akk = g.A + toff(k, k, T);
      const int nb = w < 2 ? 3 : 2, b0 = w < 2 ? 3 * w : 6 + 2 * (w - 2);
      double a[3][4];
#pragma unroll
      for (int q = 0; q < 3; q++) {
        if (q < nb) {
          const int bi = kLowBi[b0 + q], bj = kLowBj[b0 + q];
#pragma unroll
          for (int r = 0; r < 4; r++) a[q][r] = ld_h(&Akk[(16 * bi + k4 + 4 * r) * TB + 16 * bj + r16]);
        }
      }
      if (k >= 1) bv -= gemv_row(sX, su);
#pragma unroll
      for (int q = 0; q < 3; q++) {
        if (q < nb) {
          const int bi = kLowBi[b0 + q], bj = kLowBj[b0 + q];
          if (k >= 1) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k0 = 0; k0 < TB; k0 += 4)
              acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sX[(16 * bi + r16) * LS + k0 + k4],
                                                          sY[(16 * bj + r16) * LS + k0 + k4], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; r++) a[q][r] = a[q][r] - acc[r];
          }
          a3_store(sK, a[q], bi, bj);
        }
      }
      // the strict upper blocks are zero (the factorisation reads the lower triangle only, but
      // put_tile_lower's convention keeps the upper part defined)
      const int nz = w < 2 ? 2 : 1, z0 = w < 2 ? 2 * w : 4 + (w - 2);
      for (int q = 0; q < nz; q++) {
        const int bi = kUpBi[z0 + q], bj = kUpBj[z0 + q];
#pragma unroll
        for (int r = 0; r < 4; r++) sK[(16 * bi + k4 + 4 * r) * LS + 16 * bj + r16] = 0.0;
      }
    }
    __syncthreads();
    if ((t & 3) == 0) sv[t >> 2] = bv;
    if (t == 0) *fail = 0;
    __syncthreads();
    DSTAMP(k, 2);
    factor_tile(sK, sI, fail);
    {
      const double u = gemv_row(sI, sv);
      if ((t & 3) == 0) su[t >> 2] = u;
    }
    __syncthreads();
    store_tile_sc1(g.Linv + (size_t)k * TB * TB, sI);
    if (t < TB) {
      const double dk = sK[t * LS + t];
      st_sc1(g.du + (size_t)k * 128 + t, dk);
      st_sc1(g.du + (size_t)k * 128 + TB + t, su[t]);
      g.z[k * TB + t] = su[t] / dk;
    }
    if (t == 0 && *fail) atomicOr(g.flag, kFlagZeroPivot);
    DSTAMP(k, 3);
    wg_publish(dg + k, 1u);
    PTRACE(11, k, 0);
    DSTAMP(k, 4);
    if (k + 1 < T) {
      // the next panel tile: A_{k+1,k} after products 0 .. k-1
      if (!wg_wait(cnt + tix(k + 1, k, T), (unsigned)(k - kbase(k + 1, g.D)), nullptr, 0, nullptr, 0, err, sh_ok,
                   g.wait_ticks))
        break;
      DSTAMP(k, 5);
      {
        d2 v[8];
        fetch_tile_h(v, g.A + toff(k + 1, k, T));
        put_tile(sX, v);
      }
      if (t < TB) sv[t] = sK[t * LS + t];
      __syncthreads();
      trsm_to_lds(sX, sY, sI, sv);
      store_tile_sc1(g.L + toff(k + 1, k, T), sX);
      store_tile_sc1(g.W + toff(k + 1, k, T), sY);
      wg_publish(pan + tix(k + 1, k, T), 1u);
      PTRACE(12, k, 0);
      DSTAMP(k, 6);
    }
  }
  if (t == 0 && pl_load(err) != 0u) atomicOr(g.flag, kFlagTimeout);
}

__device__ bool trsm_task(const PipeArgs& g, int i, int k, double* sm, int* sh_ok, int tk) {
  double* sI = sm + TB * LS;
  double* sX = sI + TB * LS;
  double* sY = sX + TB * LS;
  double* sv = sY + TB * LS;
  const int T = g.T, t = threadIdx.x;
  unsigned* err = g.sync + 1;
  unsigned* cnt = g.sync + 4;
  unsigned* pan = cnt + g.ntile;
  unsigned* dg = pan + g.ntile;
  if (!wg_wait(dg + k, 1u, cnt + tix(i, k, T), (unsigned)(k - kbase(i, g.D)), nullptr, 0, err, sh_ok, g.wait_ticks))
    return false;
  TSTAMP(tk, 1);
  {
    d2 vx[8], vi[8];
    fetch_tile_h(vx, g.A + toff(i, k, T));
    fetch_tile_h(vi, g.Linv + (size_t)k * TB * TB);
    if (t < TB) sv[t] = ld_h(&g.du[(size_t)k * 128 + t]);
    put_tile(sX, vx);
    put_tile(sI, vi);
  }
  __syncthreads();
  TSTAMP(tk, 2);
  trsm_to_lds(sX, sY, sI, sv);
  store_tile_sc1(g.L + toff(i, k, T), sX);
  store_tile_sc1(g.W + toff(i, k, T), sY);
  wg_publish(pan + tix(i, k, T), 1u);
  return true;
}

__device__ bool update_task(const PipeArgs& g, int i, int j, int k, double* sm, int* sh_ok, int tk) {
  double* sX = sm + 2 * TB * LS;
  double* sY = sX + TB * LS;
  double* su = sY + TB * LS + TB;
  const int T = g.T, t = threadIdx.x, l = t & 63, w = t >> 6, r16 = l & 15, k4 = l >> 4;
  unsigned* err = g.sync + 1;
  unsigned* cnt = g.sync + 4;
  unsigned* pan = cnt + g.ntile;
  const int kb = kbase(i, g.D);
  if (!wg_wait(pan + tix(i, k, T), 1u, pan + tix(j, k, T), 1u, cnt + tix(i, j, T), (unsigned)(k - kb), err, sh_ok,
               g.wait_ticks))
    return false;
  TSTAMP(tk, 1);
  double a[4][4];
  double bv = 0.0;
  {
    d2 vx[8], vy[8];
    fetch_tile_h(vx, g.L + toff(i, k, T));
    fetch_tile_h(vy, g.W + toff(j, k, T));
    load_acc_h(a, g.A + toff(i, j, T));
    if (i == j) {
      bv = ld_h(&g.b[i * TB + (t >> 2)]);
      if (t < TB) su[t] = ld_h(&g.du[(size_t)k * 128 + TB + t]);
    }
    put_tile(sX, vx);
    put_tile(sY, vy);
  }
  __syncthreads();
  TSTAMP(tk, 2);
  d4 p[4];
  gemm_xyt(sX, sY, p);
  {
    double* Aij = g.A + toff(i, j, T);
    const int col = 16 * w + r16;
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) st_sc1(&Aij[(16 * q + k4 + 4 * r) * TB + col], a[q][r] - p[q][r]);
  }
  if (i == j) {
    const double s = gemv_row(sX, su);
    if ((t & 3) == 0) st_sc1(&g.b[i * TB + (t >> 2)], bv - s);
  }
  wg_publish(cnt + tix(i, j, T), (unsigned)(k + 1 - kb));
  __syncthreads();   // LDS tiles are rewritten by the next task
  return true;
}

__global__ __launch_bounds__(256) void k_pipe(PipeArgs g) {
  if (g.skip && *g.skip) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  int* ish = reinterpret_cast<int*>(sm + 4 * TB * LS + 2 * TB);   // dynamic region (Guideline 17)
  int& sh_tk = ish[0];
  int& sh_ok = ish[1];
  int& fail = ish[2];
  for (;;) {
    if (threadIdx.x == 0) sh_tk = (int)atomicAdd(g.sync, 1u);
    __syncthreads();
    const int tk = __builtin_amdgcn_readfirstlane(sh_tk);
    __syncthreads();
    PTRACE(1, tk, 0);
    if (tk == 0) {
      diag_role(g, sm, &sh_ok, &fail);
      break;
    }
    if (tk > g.ntasks) break;
    const int4 tq = g.tasks[tk - 1];
    const int ty = __builtin_amdgcn_readfirstlane(tq.x), ti = __builtin_amdgcn_readfirstlane(tq.y);
    const int tj = __builtin_amdgcn_readfirstlane(tq.z), tkk = __builtin_amdgcn_readfirstlane(tq.w);
    PTRACE(2, ty, (ti << 16) | (tj << 8) | tkk);
    TSTAMP(tk, 0);
    const bool ok = ty == 0 ? trsm_task(g, ti, tkk, sm, &sh_ok, tk) : update_task(g, ti, tj, tkk, sm, &sh_ok, tk);
    TSTAMP(tk, 3);
    PTRACE(3, ok, 0);
    if (!ok) {
      if (threadIdx.x == 0) atomicOr(g.flag, kFlagTimeout);
      break;
    }
  }
}

// Backward substitution L^T x = z across workgroups (one launch): the workgroup holding
// ticket t owns block column k = T - 1 - t and forms
//   r_k = z_k - sum_{k < i < k + D} L_ik^T x_i,   x_k = Linv_kk^T r_k   (D: the tile band),
// accumulating L_ik^T x_i as each x_i is published (i descending, the next tile prefetched
// into registers while it waits), so only the x_{k+1} term and the Linv product follow the
// hand-off of x_{k+1}.  Tickets make it deadlock-free without co-residency (a column waits only
// on columns with earlier tickets).  x_k is published write-through (8-B sc1 stores, every
// storing wave drained, then one flag), read with sc1 loads (MICROARCH visibility table, row 1).
// Thread (c = t & 63, q = t >> 6) sums rows q + 4m of each tile; x_k = Linv^T r_k uses
// k_solve1's partial layout and order (16 row groups), so a one-tile system gives the bits of
// the fused one-tile solve.  sync: [0] ticket, [1] error, [4 .. 4+T) column flags.
__global__ __launch_bounds__(256) void k_bwd(const double* __restrict__ L, const double* __restrict__ Linv,
                                             const double* __restrict__ z, double* x, unsigned* sync,
                                             int T, int D, int* flag, const int* skip, long long ticks) {
  if (skip && *skip) return;
  extern __shared__ __attribute__((aligned(16))) double bsm[];
  double* part = bsm;              // [16][64]
  double* rk = part + 16 * TB;     // [64]
  int* ish = reinterpret_cast<int*>(rk + TB);
  const int t = threadIdx.x, c = t & 63, q = t >> 6;
  unsigned* err = sync + 1;
  unsigned* xf = sync + 4;
  if (t == 0) ish[0] = (int)atomicAdd(sync, 1u);
  __syncthreads();
  const int tk = __builtin_amdgcn_readfirstlane(ish[0]);
  if (tk >= T) return;
  const int k = T - 1 - tk;
  // Linv_kk in registers: rows g + 16 h (h = 0..3) of the row groups g = q + 4 m (m = 0..3)
  double iv[4][4];
  {
    const double* I = Linv + (size_t)k * TB * TB;
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
      for (int h = 0; h < 4; h++) iv[m][h] = I[(q + 4 * m + 16 * h) * TB + c];
  }
  double acc = 0.0;
  double lt[16];
  const int ilast = min(T - 1, k + D - 1);   // L_ik = 0 beyond the band
  if (k + 1 <= ilast) {
    const double* Lt = L + toff(ilast, k, T);
#pragma unroll
    for (int m = 0; m < 16; m++) lt[m] = Lt[(q + 4 * m) * TB + c];
  }
  bool ok = true;
  for (int i = ilast; i > k; i--) {
    // wait for x_i
    if (t == 0) {
      int good = 1;
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      while (pl_load(xf + i) == 0u) {
        if (pl_load(err) != 0u) { good = 0; break; }
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) { pl_store(err, 1u); good = 0; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (good) {   // acquire x_i before the barrier, as wg_wait does
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      ish[1] = good;
    }
    __syncthreads();
    ok = __builtin_amdgcn_readfirstlane(ish[1]) != 0;
    __syncthreads();
    if (!ok) break;
    double xv[16];
#pragma unroll
    for (int m = 0; m < 16; m++)
      xv[m] = __longlong_as_double((long long)__hip_atomic_load((const gu64*)(x + (size_t)i * TB + q + 4 * m),
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    double cur[16];
#pragma unroll
    for (int m = 0; m < 16; m++) cur[m] = lt[m];
    if (i - 1 > k) {   // prefetch the next tile while this one is summed
      const double* Lt = L + toff(i - 1, k, T);
#pragma unroll
      for (int m = 0; m < 16; m++) lt[m] = Lt[(q + 4 * m) * TB + c];
    }
#pragma unroll
    for (int m = 0; m < 16; m++) acc = __builtin_fma(cur[m], xv[m], acc);
  }
  if (ok) {
    part[q * TB + c] = acc;
    __syncthreads();
    if (t < TB) rk[t] = z[(size_t)k * TB + t] - (((part[t] + part[TB + t]) + part[2 * TB + t]) + part[3 * TB + t]);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const int g = q + 4 * m;
      double u = iv[m][0] * rk[g] + iv[m][1] * rk[g + 16];
      u += iv[m][2] * rk[g + 32] + iv[m][3] * rk[g + 48];
      part[g * TB + c] = u;
    }
    __syncthreads();
    if (t < TB) {
      double a = 0.0;
#pragma unroll
      for (int g = 0; g < 16; g++) a += part[g * TB + t];
      st_sc1(x + (size_t)k * TB + t, a);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) pl_store(xf + k, 1u);
  } else if (t == 0) {
    atomicOr(flag, kFlagTimeout);
  }
}

}  // namespace

__global__ void k_pad(double* __restrict__ A, double* __restrict__ b, int n, int T, double dv,
                      const int* skip) {
  if (skip && *skip) return;
  const int Np = T * TB;
  const int r = n + blockIdx.x;   // one workgroup per padding row
  if (r >= Np) return;
  for (int c = threadIdx.x; c <= r; c += blockDim.x) A[sidx(r, c, T)] = (c == r) ? dv : 0.0;
  // the strict-upper part of the last diagonal tile in the padding columns of rows < n is
  // never read by the factorisation (lower triangle only)
  if (threadIdx.x == 0) b[r] = 0.0;
}

// The whole solve of a one-tile system (n <= 64: LocalBA-sized), one launch instead of
// k_pad + k_panel + k_backward, with the same arithmetic: the padding rows are set as k_pad
// writes them (diag_value on the diagonal, zero right-hand side), the tile is factored and
// u = Linv b, z = u / D formed as k_panel's workgroup 0 does, and x = Linv^T z as
// k_backward's one step (whose empty off-diagonal sum is +0: r = z exactly), in the same
// partial layout and summation order.
__global__ __launch_bounds__(256) void k_solve1(const double* __restrict__ A, const double* __restrict__ b,
                                                double* __restrict__ x, int n, double dv, int* flag,
                                                const int* skip) {
  if (skip && *skip) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* sK = sm;               // A -> L (strict lower) + D (diagonal)
  double* sI = sK + TB * LS;     // Linv
  double* sv = sI + TB * LS;     // b, then z
  double* su = sv + TB;          // u
  double* part = su + TB;        // [16][TB]
  int& fail = *reinterpret_cast<int*>(part + 16 * TB);
  const int t = threadIdx.x;
  if (t == 0) fail = 0;
  d2 vK[8];
  fetch_tile(vK, A);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int e = 2 * (t + 256 * i), r = e >> 6, c = e & 63;
    if (r >= n) {
      vK[i].x = (c == r) ? dv : 0.0;
      vK[i].y = (c + 1 == r) ? dv : 0.0;
    }
  }
  if (t < TB) sv[t] = t < n ? b[t] : 0.0;
  put_tile_lower(sK, vK);
  __syncthreads();
  factor_tile(sK, sI, &fail);
  const double u = gemv_row(sI, sv);
  if ((t & 3) == 0) su[t >> 2] = u;
  __syncthreads();
  if (t < TB) sv[t] = su[t] / sK[t * LS + t];
  if (t == 0 && fail) atomicOr(flag, kFlagZeroPivot);
  __syncthreads();
  const int c = t & 63;
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const int g = (t >> 6) + 4 * m;
    double v = sI[g * LS + c] * sv[g] + sI[(g + 16) * LS + c] * sv[g + 16];
    v += sI[(g + 32) * LS + c] * sv[g + 32] + sI[(g + 48) * LS + c] * sv[g + 48];
    part[g * TB + c] = v;
  }
  __syncthreads();
  if (t < TB) {
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) acc += part[q * TB + t];
    x[t] = acc;
  }
}

}  // namespace

constexpr size_t kSolve1Lds = (2 * (size_t)TB * LS + 18 * TB) * sizeof(double) + 16;

// hipFuncSetAttribute applies to the current device: set each kernel's dynamic-LDS limit once
// per (kernel, device), under a lock (a process may drive several GPUs from several threads)
hipError_t set_lds_limit(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(mu);
  if (done.count({fn, dev})) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert({fn, dev});
  return e;
}

hipError_t solve_one_tile(const double* A, const double* b, double* x, int n, double diag_value, int* flag,
                          hipStream_t st, const int* skip) {
  hipError_t e = set_lds_limit((const void*)k_solve1, (int)kSolve1Lds);
  if (e != hipSuccess) return e;
  if (n < 1 || n > TB) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_solve1, dim3(1), dim3(256), kSolve1Lds, st, A, b, x, n, diag_value, flag, skip);
  return hipGetLastError();
}

constexpr size_t kPanelLds = (4 * (size_t)TB * LS + 2 * TB) * sizeof(double) + 16;

// Task table of the pipelined factorisation, step-major: for each k the TRSM tasks (i, k),
// i = k+2 .. T-1, then the UPDATE tasks (i, j, k) by column j = k+1 .. T-1 and row i = j .. T-1,
// except (k+1, k+1, k) (the diag workgroup's).  Every task waits only on earlier tickets or on
// diag steps <= k, which in turn wait only on tasks of steps <= k - 1.
// Banded (D < T): only tasks inside the band, i - k < D (so j - k < D too): L_ik = 0 beyond it
// and A_ij receives no product from outside it; the same order otherwise.
static size_t pipe_task_count(int T, int D) {
  size_t n = 0;
  for (int k = 0; k + 1 < T; k++) {
    const int m = std::min(T - 1, k + D - 1) - k;   // rows k+1 .. k+m in the band
    n += (size_t)std::max(0, m - 1) + (size_t)m * (m + 1) / 2 - 1;
  }
  return n;
}

static std::vector<int4> pipe_tasks(int T, int D) {
  std::vector<int4> v;
  v.reserve(pipe_task_count(T, D));
  for (int k = 0; k + 1 < T; k++) {
    const int ie = std::min(T - 1, k + D - 1);
    for (int i = k + 2; i <= ie; i++) v.push_back(make_int4(0, i, k, k));
    for (int j = k + 1; j <= ie; j++)
      for (int i = j; i <= ie; i++)
        if (!(i == k + 1 && j == k + 1)) v.push_back(make_int4(1, i, j, k));
  }
  return v;
}

bool pipe_supported(int T, int D) {
  D = pipe_band(T, D);
  if (T < 2) return false;
  if (D >= T) return T <= kPipeMaxT;
  return T <= kPipeMaxTBand && pipe_task_count(T, D) <= kPipeMaxTasks;
}

static size_t bwd_sync_words(int T) { return (4 + (size_t)T + 3) & ~(size_t)3; }

size_t pipe_sync_words(int T, int D) {
  // factorisation words, then the backward's (ticket, error, column flags); multiple of 16 B
  const size_t ntile = band_tiles(pipe_band(T, D), T);
  return ((4 + 2 * ntile + (size_t)T + 3) & ~(size_t)3) + bwd_sync_words(T);
}

constexpr size_t kBwdLds = (17 * (size_t)TB) * sizeof(double) + 16;

const std::vector<int4>& pipe_tasks_host(int T, int D) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, std::vector<int4>> cache;   // node-based: entries never move
  D = pipe_band(T, D);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find({T, D});
  if (it == cache.end()) it = cache.emplace(std::make_pair(T, D), pipe_tasks(T, D)).first;
  return it->second;   // never reallocated afterwards: safe as an async-copy source
}

hipError_t pipe_prepare(Work& w, int T, hipStream_t st, int D) {
  if (T < 1 || !(T == 1 || pipe_supported(T, D))) return hipErrorInvalidValue;
  D = pipe_band(T, D);
  const std::vector<int4>& tasks = pipe_tasks_host(T, D);
  hipError_t e = hipMalloc(&w.W, tile_doubles(T) * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&w.du, (size_t)T * 128 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&w.sync, pipe_sync_words(T, D) * sizeof(unsigned));
  if (e == hipSuccess && !tasks.empty()) e = hipMalloc(&w.tasks, tasks.size() * sizeof(int4));
  if (e == hipSuccess && !tasks.empty())
    e = hipMemcpyAsync(w.tasks, tasks.data(), tasks.size() * sizeof(int4), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  w.ntasks = (int)tasks.size();
  w.pipe_T = T;
  w.band = D;
  return e;
}

void pipe_release(Work& w) {
  for (void* p : {(void*)w.W, (void*)w.du, (void*)w.sync, (void*)w.tasks})
    if (p) (void)hipFree(p);
  w.W = nullptr; w.du = nullptr; w.sync = nullptr; w.tasks = nullptr; w.ntasks = 0; w.pipe_T = 0; w.band = 0;
}

static int device_cus() {
  static std::mutex mu;
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  std::lock_guard<std::mutex> g(mu);
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

static std::atomic<long long> g_wait_ticks{kWaitTicksDefault};
void set_wait_ticks(long long ticks) { g_wait_ticks.store(ticks > 0 ? ticks : kWaitTicksDefault); }
long long wait_ticks() { return g_wait_ticks.load(); }

hipError_t solve(double* A, double* b, double* x, int T, const Work& w, int* flag, hipStream_t st,
                 const int* skip) {
  hipError_t e = set_lds_limit((const void*)k_panel, (int)kPanelLds);
  if (e == hipSuccess) e = set_lds_limit((const void*)k_backward, 96 * 1024);
  if (e == hipSuccess) e = set_lds_limit((const void*)k_pipe, (int)kPanelLds);
  if (e != hipSuccess) return e;
  if (w.sync && w.pipe_T == T) {
    const int D = pipe_band(T, w.band);
    if (w.per_step && D < T) return hipErrorInvalidValue;   // k_panel walks every tile
    e = hipMemsetAsync(w.sync, 0, pipe_sync_words(T, D) * sizeof(unsigned), st);
    if (e != hipSuccess) return e;
    const long long ticks = wait_ticks();
    PipeArgs g{A, b, w.L, w.W, w.Linv, w.du, w.z, w.sync, w.tasks, w.ntasks, T, (int)band_tiles(D, T), D, flag, skip,
               ticks};
    if (w.per_step) {
      for (int k = 0; k < T; k++) {
        const int m = T - 1 - k;
        const unsigned grid = 1u + (unsigned)(m * (m + 1) / 2);
        hipLaunchKernelGGL(k_panel, dim3(grid), dim3(256), kPanelLds, st, A, b, w.L, w.Linv, w.z, k, T, flag, skip);
      }
    } else {
      const int grid = std::max(1, std::min(device_cus(), w.ntasks + 1));
      hipLaunchKernelGGL(k_pipe, dim3(grid), dim3(256), kPanelLds, st, g);
    }
    hipLaunchKernelGGL(k_bwd, dim3(T), dim3(256), kBwdLds, st, (const double*)w.L, (const double*)w.Linv,
                       (const double*)w.z, x, w.sync + pipe_sync_words(T, D) - bwd_sync_words(T), T, D, flag, skip,
                       ticks);
    return hipGetLastError();
  }
  // one k_panel launch per step + the one-workgroup backward (its x lives in LDS: <= 192 tiles)
  if ((size_t)T * TB * sizeof(double) > 96 * 1024) return hipErrorInvalidValue;
  for (int k = 0; k < T; k++) {
    const int m = T - 1 - k;
    const unsigned grid = 1u + (unsigned)(m * (m + 1) / 2);
    hipLaunchKernelGGL(k_panel, dim3(grid), dim3(256), kPanelLds, st, A, b, w.L, w.Linv, w.z, k, T, flag, skip);
  }
  hipLaunchKernelGGL(k_backward, dim3(1), dim3(kBwdNT), (size_t)T * TB * sizeof(double), st,
                     (const double*)w.L, (const double*)w.Linv, (const double*)w.z, x, T, skip);
  return hipGetLastError();
}

hipError_t pad(double* A, double* b, int n, int T, double diag_value, hipStream_t st, const int* skip) {
  const int np = T * TB - n;
  if (np <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pad, dim3(np), dim3(256), 0, st, A, b, n, T, diag_value, skip);
  return hipGetLastError();
}

}  // namespace ldlt
}  // namespace mcs
