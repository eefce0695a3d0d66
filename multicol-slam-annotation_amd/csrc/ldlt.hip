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
#include <mutex>
#include <set>
#include <utility>

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
__device__ __forceinline__ void factor_tile(double* sA, double* sI, int* fail) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int r16 = l & 15, k4 = l >> 4;
  for (int p = 0; p < 4; p++) {
    const int P = 16 * p;
    if (w == p) {
      double a[16];
#pragma unroll
      for (int c = 0; c < 16; c++) a[c] = sA[l * LS + P + c];
#ifdef MCS_LDLT_FACTOR_V1
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int J = P + j;
        const double cj = a[j];
        const double dj = readlane_d(cj, J);
        const double lj = cj / dj;
#pragma unroll
        for (int m = j + 1; m < 16; m++) a[m] = __builtin_fma(-lj, readlane_d(cj, P + m), a[m]);
        if (dj == 0.0 && l == 0) *fail = 1;
        if (l >= J) sA[l * LS + J] = (l > J) ? lj : cj;
        if (l >= P + 16) sA[J * LS + l] = cj;
      }
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
  extern __shared__ double sm[];
  double* sK = sm;               // A_kk -> L_kk (strict lower) + D (diagonal)
  double* sI = sK + TB * LS;     // Linv_kk
  double* sX = sI + TB * LS;     // A_ik -> G_i = L_ik
  double* sY = sX + TB * LS;     // A_jk -> W_j
  double* sv = sY + TB * LS;     // b_k
  double* su = sv + TB;          // u_k = Linv b_k
  __shared__ int fail;
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
    if (t == 0 && fail) *flag = 1;
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
  extern __shared__ double sx[];   // 64 T: solved blocks of x
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
  extern __shared__ double sm[];
  double* sK = sm;               // A -> L (strict lower) + D (diagonal)
  double* sI = sK + TB * LS;     // Linv
  double* sv = sI + TB * LS;     // b, then z
  double* su = sv + TB;          // u
  double* part = su + TB;        // [16][TB]
  __shared__ int fail;
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
  if (t == 0 && fail) *flag = 1;
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

constexpr size_t kSolve1Lds = (2 * (size_t)TB * LS + 18 * TB) * sizeof(double);

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

constexpr size_t kPanelLds = (4 * (size_t)TB * LS + 2 * TB) * sizeof(double);

hipError_t solve(double* A, double* b, double* x, int T, const Work& w, int* flag, hipStream_t st,
                 const int* skip) {
  hipError_t e = set_lds_limit((const void*)k_panel, (int)kPanelLds);
  if (e == hipSuccess) e = set_lds_limit((const void*)k_backward, 96 * 1024);
  if (e != hipSuccess) return e;
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
