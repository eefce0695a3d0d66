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

// In-LDS LDL^T of a 64x64 tile (lower triangle read).  On return the strict lower triangle
// holds L, the diagonal holds D.  One barrier per column: column j is scaled by 1/d_j during
// step j+1 (nothing reads it after step j's update).
__device__ void factor_tile(double* sA, int* fail) {
  const int t = threadIdx.x, i = t & 63, g = t >> 6;
  double inv_prev = 0.0;
  for (int j = 0; j < TB; j++) {
    const double dj = sA[j * LS + j];
    if (dj == 0.0 && t == 0) *fail = 1;
    const double inv = 1.0 / dj;
    if (j > 0 && g == 0 && i > j - 1) sA[i * LS + j - 1] *= inv_prev;
    if (i > j) {
      const double aij = sA[i * LS + j] * inv;
      for (int m = j + 1 + g; m <= i; m += 4) sA[i * LS + m] -= aij * sA[m * LS + j];
    }
    inv_prev = inv;
    __syncthreads();
  }
}

// Linv = L^-1 (unit lower) into sI: lane c of wave 0 computes column c row by row,
// Linv[r][c] = [r == c] - sum_{m<r} L[r][m] Linv[m][c]; L reads are broadcasts, the column
// reads / writes are lane-consecutive (conflict-free).  Entries above the diagonal come out 0.
__device__ void invert_unit_lower(const double* sA, double* sI) {
  const int t = threadIdx.x;
  if (t < TB) {
    const int c = t;
    for (int r = 0; r < TB; r++) {
      const double* Lr = sA + r * LS;
      double s0 = (r == c) ? 1.0 : 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
      int m = 0;
      for (; m + 3 < r; m += 4) {
        s0 -= Lr[m] * sI[m * LS + c];
        s1 -= Lr[m + 1] * sI[(m + 1) * LS + c];
        s2 -= Lr[m + 2] * sI[(m + 2) * LS + c];
        s3 -= Lr[m + 3] * sI[(m + 3) * LS + c];
      }
      for (; m < r; m++) s0 -= Lr[m] * sI[m * LS + c];
      sI[r * LS + c] = (s0 + s1) + (s2 + s3);
    }
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
  load_tile(sK, A + toff(k, k));
  if (wg > 0) {
    load_tile(sX, A + toff(i, k));
    if (j != i) load_tile(sY, A + toff(j, k));
  }
  if (rhs && t < TB) sv[t] = b[k * TB + t];
  __syncthreads();
  factor_tile(sK, &fail);
  invert_unit_lower(sK, sI);
  __syncthreads();
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

// L^T x = z, one workgroup; z is staged in LDS and updated right-looking.
__global__ __launch_bounds__(256) void k_backward(const double* __restrict__ L,
                                                  const double* __restrict__ Linv,
                                                  const double* __restrict__ z,
                                                  double* __restrict__ x, int T) {
  extern __shared__ double sz[];   // 64 T
  __shared__ double part[4][TB];
  __shared__ double xk[TB];
  const int t = threadIdx.x, c = t & 63, g = t >> 6;
  const int Np = T * TB;
  for (int e = t; e < Np; e += 256) sz[e] = z[e];
  __syncthreads();
  for (int k = T - 1; k >= 0; k--) {
    // x_k = Linv_kk^T z_k : x[c] = sum_m Linv[m][c] z[m]
    const double* I = Linv + (size_t)k * TB * TB;
    double s = 0.0;
    for (int m = g; m < TB; m += 4) s += I[m * TB + c] * sz[k * TB + m];
    part[g][c] = s;
    __syncthreads();
    if (t < TB) {
      const double v = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
      xk[t] = v;
      x[k * TB + t] = v;
    }
    __syncthreads();
    // z_j[c] -= sum_r L_kj[r][c] x_k[r], j < k
    for (int o = t; o < k * TB; o += 256) {
      const int jb = o >> 6, cc = o & 63;
      const double* Lkj = L + toff(k, jb);
      double a0 = 0.0, a1 = 0.0;
      for (int r = 0; r < TB; r += 2) {
        a0 += Lkj[r * TB + cc] * xk[r];
        a1 += Lkj[(r + 1) * TB + cc] * xk[r + 1];
      }
      sz[jb * TB + cc] -= a0 + a1;
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

constexpr size_t kPanelLds = (4 * (size_t)TB * LS + 2 * TB) * sizeof(double);

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
  hipLaunchKernelGGL(k_backward, dim3(1), dim3(256), (size_t)T * TB * sizeof(double), st,
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
