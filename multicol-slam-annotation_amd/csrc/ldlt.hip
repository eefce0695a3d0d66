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

namespace mcs {
namespace ldlt {

namespace {

constexpr int LS = TB + 1;   // LDS row stride in doubles (breaks the power-of-two stride)
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void load_tile(double* s, const double* __restrict__ g) {
  for (int e = threadIdx.x; e < TB * TB; e += 256) s[(e >> 6) * LS + (e & 63)] = g[e];
}

// diagonal tile: only the lower triangle is defined (the strict upper part of the storage is
// never written by the producers and may hold stale bits), so it is loaded as 0
__device__ __forceinline__ void load_tile_lower(double* s, const double* __restrict__ g) {
  for (int e = threadIdx.x; e < TB * TB; e += 256) {
    const int r = e >> 6, c = e & 63;
    s[r * LS + c] = (c <= r) ? g[e] : 0.0;
  }
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// LDL^T of the 64x64 tile in sA (lower triangle read) and L^-1, register resident:
// lane = row i, wave g owns the columns m = g + 4q.  A runtime loop runs over groups of 4
// columns (j = 4 jj + gj, gj unrolled): the trailing-matrix registers a[] are shifted by one
// after every group, so the column the owning wave gj works on is always a[0] and the code
// stays small (a fully unrolled sweep is ~55 KB and runs instruction-fetch bound).
// e[q] holds row i of E = L^-1 (column g + 4q), built by applying every elimination row
// operation to the identity.
// Per column j, before the barrier: the owning wave forms l_i = A[i][j] / d_j, publishes l_i
// and c_i = A[i][j] and writes L / D of column j into sA; lane j of every wave publishes its
// (final) row j of E is read from lane j of the same wave.  After the barrier every wave
// updates its registers:
// A[i][m] -= l_i c_m (m > j), E[i][m] -= l_i E[j][m] (m <= j).  Updates are branch-free
// (masked operands are 0 and l_i = 0 for rows i <= j, so the FMA leaves the value exact).
// Exchange buffers are double-buffered by column parity: one barrier per column.
// On return sA holds L (strict lower) and D (diagonal), sI holds L^-1 (0 above the diagonal).
__device__ __forceinline__ void factor_tile(double* sA, double* sI, double* scol, int* fail) {
  const int t = threadIdx.x, i = t & 63, g = t >> 6;
  double a[16], e[16];
#pragma unroll
  for (int q = 0; q < 16; q++) {
    a[q] = sA[i * LS + g + 4 * q];
    e[q] = (i == g + 4 * q) ? 1.0 : 0.0;
  }
  // scol layout (doubles): colL [2][64] | colC [2][4][16]
  double* colL = scol;
  double* colC = scol + 128;
  __syncthreads();   // sA is rewritten column by column below
  for (int jj = 0; jj < TB / 4; jj++) {
#pragma unroll
    for (int gj = 0; gj < 4; gj++) {
      const int j = 4 * jj + gj, bf = gj & 1;
      // every wave forms the candidate (only the owner's is published): no branch around
      // register updates
      const double dj = readlane_d(a[0], j);
      const double c = a[0];
      const double l = c / dj;
      if (g == gj) {
        if (dj == 0.0 && i == 0) *fail = 1;
        colL[bf * 64 + i] = l;
        const int slot = (i >> 2) - jj;   // register slot of row i's column after the shifts
        if (slot >= 0) colC[bf * 64 + (i & 3) * 16 + slot] = c;
        sA[i * LS + j] = (i > j) ? l : c;
      }
      __syncthreads();
      // unconditional loads, masks applied as multipliers (all operands finite), so the
      // compiler emits no branches between the LDS reads
      const double lv = colL[bf * 64 + i];
      const double li = (i > j) ? lv : 0.0;   // select, not a multiply: rows <= j may hold inf
      // c of column g + 4 (q + jj); slots past the tile hold stale values, which only reach
      // registers that stand for columns past the tile (never read back)
      const double2* cg = reinterpret_cast<const double2*>(colC + bf * 64 + g * 16);
      double cv[16];
#pragma unroll
      for (int q2 = 0; q2 < 8; q2++) {
        const double2 v = cg[q2];
        cv[2 * q2] = v.x;
        cv[2 * q2 + 1] = v.y;
      }
      // a[q] is column g + 4 (q + jj) > j  <=>  g + 4 q > gj: only q = 0 can be <= j
      cv[0] = (g > gj) ? cv[0] : 0.0;
#pragma unroll
      for (int q = 0; q < 16; q++) a[q] = __builtin_fma(-li, cv[q], a[q]);
      // E row j of this wave's columns lives in lane j of the same wave: readlane, no LDS
      // (a single-lane LDS publish of the row measured ~2000 cycles per column)
      // E[j][m] == 0 for m > j: skip those readlanes (wave-uniform branch; each readlane
      // pair costs ~25 cycles)
#pragma unroll
      for (int q = 0; q < 16; q++) {
        if (g + 4 * q <= j) {
          const double ej = readlane_d(e[q], j);
          e[q] = __builtin_fma(-li, ej, e[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 15; q++) a[q] = a[q + 1];
    a[15] = 0.0;
  }
#pragma unroll
  for (int q = 0; q < 16; q++) sI[i * LS + g + 4 * q] = e[q];
  __syncthreads();
}

// acc = X Y^T (64x64x64), wave w owns output columns [16w, 16w+16), acc[q] rows [16q, 16q+16)
// v_mfma_f64_16x16x4_f64: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15];
// result reg r of lane l is D[(l>>4) + 4r][l&15].
__device__ __forceinline__ void gemm_xyt(const double* X, const double* Y, d4 (&acc)[4]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r16 = l & 15, k4 = l >> 4;
#pragma unroll
  for (int q = 0; q < 4; q++) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k0 = 0; k0 < TB; k0 += 4) {
    const double bv = Y[(16 * w + r16) * LS + k0 + k4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const double av = X[(16 * q + r16) * LS + k0 + k4];
      acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q], 0, 0, 0);
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
                                               double* __restrict__ z, int k, int* flag) {
  extern __shared__ double sm[];
  double* sK = sm;               // A_kk -> L_kk (strict lower) + D (diagonal)
  double* sI = sK + TB * LS;     // Linv_kk
  double* sX = sI + TB * LS;     // A_ik -> G_i = L_ik
  double* sY = sX + TB * LS;     // A_jk -> W_j
  double* sv = sY + TB * LS;     // b_k
  double* su = sv + TB;          // u_k = Linv b_k
  double* scol = su + TB;        // factor_tile column exchange (512 doubles)
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
  if (t == 0) fail = 0;
  load_tile_lower(sK, A + toff(k, k));
  if (wg > 0) {
    load_tile(sX, A + toff(i, k));
    if (j != i) load_tile(sY, A + toff(j, k));
  }
  if (rhs && t < TB) sv[t] = b[k * TB + t];
  __syncthreads();
  factor_tile(sK, sI, scol, &fail);
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
  const int l = t & 63, w = t >> 6, r16 = l & 15, k4 = l >> 4;
  d4 wi[4], wj[4];
  gemm_xyt(sX, sI, wi);
  if (j != i) gemm_xyt(sY, sI, wj);
  __syncthreads();
  {
    const int col = 16 * w + r16;
    const double invd = 1.0 / sK[col * LS + col];
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * q + k4 + 4 * r;
        sX[row * LS + col] = wi[q][r] * invd;
        sY[row * LS + col] = (j != i) ? wj[q][r] : wi[q][r];
      }
  }
  __syncthreads();
  d4 p[4];
  gemm_xyt(sX, sY, p);
  {
    double* Aij = A + toff(i, j);
    const int col = 16 * w + r16;
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * q + k4 + 4 * r;
        Aij[row * TB + col] -= p[q][r];
      }
  }
  if (i == j) {
    double* Lik = L + toff(i, k);
    for (int e = t; e < TB * TB; e += 256) Lik[e] = sX[(e >> 6) * LS + (e & 63)];
    const double s = gemv_row(sX, su);
    if ((t & 3) == 0) b[i * TB + (t >> 2)] -= s;
  }
}

// L^T x = z, one workgroup of 1024 threads, left-looking:
//   x_k = Linv_kk^T (z_k - sum_{i>k} L_ik^T x_i)
// thread (c = t & 63, g = t >> 6) sums rows r = g (mod 16) of every tile below the diagonal
// (all loads independent, coalesced over c); the 16 partials are combined in a fixed order.
constexpr int kBwdNT = 1024;
__global__ __launch_bounds__(kBwdNT) void k_backward(const double* __restrict__ L,
                                                     const double* __restrict__ Linv,
                                                     const double* __restrict__ z,
                                                     double* __restrict__ x, int T) {
  extern __shared__ double sx[];   // 64 T: solved blocks of x
  __shared__ double part[16][TB];
  __shared__ double rk[TB];
  const int t = threadIdx.x, c = t & 63, g = t >> 6;
  for (int k = T - 1; k >= 0; k--) {
    double s0 = 0.0, s1 = 0.0;
    for (int ib = k + 1; ib < T; ib++) {
      const double* Lik = L + toff(ib, k);
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

__global__ void k_pad(double* __restrict__ A, double* __restrict__ b, int n, int T, double dv) {
  const int Np = T * TB;
  const int r = n + blockIdx.x;   // one workgroup per padding row
  if (r >= Np) return;
  for (int c = threadIdx.x; c <= r; c += blockDim.x) A[sidx(r, c)] = (c == r) ? dv : 0.0;
  // the strict-upper part of the last diagonal tile in the padding columns of rows < n is
  // never read by the factorisation (lower triangle only)
  if (threadIdx.x == 0) b[r] = 0.0;
}

}  // namespace

constexpr size_t kPanelLds = (4 * (size_t)TB * LS + 2 * TB + 512) * sizeof(double);

hipError_t solve(double* A, double* b, double* x, int T, const Work& w, int* flag, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_panel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)kPanelLds);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void*)k_backward, hipFuncAttributeMaxDynamicSharedMemorySize,
                            96 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  if ((size_t)T * TB * sizeof(double) > 96 * 1024) return hipErrorInvalidValue;
  for (int k = 0; k < T; k++) {
    const int m = T - 1 - k;
    const unsigned grid = 1u + (unsigned)(m * (m + 1) / 2);
    hipLaunchKernelGGL(k_panel, dim3(grid), dim3(256), kPanelLds, st, A, b, w.L, w.Linv, w.z, k, flag);
  }
  hipLaunchKernelGGL(k_backward, dim3(1), dim3(kBwdNT), (size_t)T * TB * sizeof(double), st,
                     (const double*)w.L, (const double*)w.Linv, (const double*)w.z, x, T);
  return hipGetLastError();
}

hipError_t pad(double* A, double* b, int n, int T, double diag_value, hipStream_t st) {
  const int np = T * TB - n;
  if (np <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pad, dim3(np), dim3(256), 0, st, A, b, n, T, diag_value);
  return hipGetLastError();
}

}  // namespace ldlt
}  // namespace mcs
