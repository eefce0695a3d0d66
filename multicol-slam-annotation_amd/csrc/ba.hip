// MultiCol bundle adjustment on gfx950: per-edge residual/Jacobian, Huber-weighted
// normal equations, Schur complement onto the MultiKeyFrame poses, LDL^T of the reduced
// camera system, point back-substitution and the Levenberg-Marquardt control of g2o.
//
// Reference (billamiable/MultiCol-SLAM-Annotation):
//   EdgeProjectXYZ2MCS::computeError / linearizeOplus   src/g2o_MultiCol_vertices_edges.cpp:32-129
//   WorldToImg                                          src/cam_model_omni.cpp:147-163
//   cayley2rot / cayley2hom / invMat                    include/misc.h:134-226, src/cConverter.cpp:31-44
//   BaseMultiEdge::constructQuadraticForm + Huber       ThirdParty/g2o/g2o/core/base_multi_edge.hpp:36-48,171-222
//   BlockSolver<6,3>::buildSystem / solve (Schur)       ThirdParty/g2o/g2o/core/block_solver.hpp:354-604
//   OptimizationAlgorithmLevenberg::solve               ThirdParty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-189
//   SparseOptimizer::optimize / TerminateAction         sparse_optimizer.cpp:354-435, sparse_optimizer_terminate_action.cpp:21-72
//   cOptimizer::LocalBundleAdjustment rounds            src/cOptimizer.cpp:771-903
//
// Every reduction runs in a fixed order (no float atomics): results are bitwise
// reproducible run to run.  The LM accept/reject decision needs two scalars per trial
// (robust chi2, model decrease), read back by the host driver.
#include "common.hpp"
#include "../../include/mcs_ba.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <new>
#include <vector>

namespace mcs {
namespace ba {

// ---------------------------------------------------------------------------
// device math (same operation order as oracle/ba_oracle.cpp)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cay2rot(const double* c, double* R) {
  const double c1 = c[0], c2 = c[1], c3 = c[2];
  const double c1s = c1 * c1, c2s = c2 * c2, c3s = c3 * c3;
  const double scale = 1 + c1s + c2s + c3s;
  const double inv = 1 / scale;
  R[0] = inv * (1 + c1s - c2s - c3s); R[1] = inv * (2 * (c1 * c2 - c3)); R[2] = inv * (2 * (c1 * c3 + c2));
  R[3] = inv * (2 * (c1 * c2 + c3)); R[4] = inv * (1 - c1s + c2s - c3s); R[5] = inv * (2 * (c2 * c3 - c1));
  R[6] = inv * (2 * (c1 * c3 - c2)); R[7] = inv * (2 * (c2 * c3 + c1)); R[8] = inv * (1 - c1s - c2s + c3s);
}

__device__ __forceinline__ double horner12(const double* a, double x) {
  double r = 0.0;
#pragma unroll
  for (int i = 11; i >= 0; i--) r = r * x + a[i];
  return r;
}

// err = meas - WorldToImg((M_t M_c)^-1 X): the reference's 4x4 path (computeError)
__device__ void edge_error(const double* pose, const double* X, const double* mc,
                           const double* cam, const double* meas, double* err) {
  double Rt[9], Rc[9];
  cay2rot(pose, Rt);
  cay2rot(mc, Rc);
  // Mct = [Rt|tt][Rc|tc] (4x4 product, k = 0..3, last row 0 0 0 1)
  double R[9], t[3];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) {
      double s = 0;
      s += Rt[3 * i] * Rc[j];
      s += Rt[3 * i + 1] * Rc[3 + j];
      s += Rt[3 * i + 2] * Rc[6 + j];
      s += pose[3 + i] * 0.0;
      R[3 * i + j] = s;
    }
    double s = 0;
    s += Rt[3 * i] * mc[3];
    s += Rt[3 * i + 1] * mc[4];
    s += Rt[3 * i + 2] * mc[5];
    s += pose[3 + i] * 1.0;
    t[i] = s;
  }
  // invMat: R' = R^T, t' = (-R') t ; X_c = R' X + t'
  double ti[3];
  for (int i = 0; i < 3; i++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (-R[3 * k + i]) * t[k];
    ti[i] = s;
  }
  double Xc[3];
  for (int i = 0; i < 3; i++) {
    double s = 0;
    s += R[i] * X[0];
    s += R[3 + i] * X[1];
    s += R[6 + i] * X[2];
    s += ti[i] * 1.0;
    Xc[i] = s;
  }
  const double x = Xc[0], y = Xc[1], z = Xc[2];
  double norm = sqrt(x * x + y * y);
  if (norm == 0.0) norm = 1e-14;
  const double theta = atan(-z / norm);
  const double rho = horner12(cam + 5, theta);
  const double uu = x / norm * rho, vv = y / norm * rho;
  const double u = uu * cam[0] + vv * cam[1] + cam[3];
  const double v = uu * cam[2] + vv + cam[4];
  err[0] = meas[0] - u;
  err[1] = meas[1] - v;
}

__device__ void dcay(const double* c, int k, const double* R, double* D) {
  const double s = 1 + c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double v = (i == j) ? -2 * c[k] : 0.0;
      v += 2 * (((i == k) ? c[j] : 0.0) + ((j == k) ? c[i] : 0.0));
      // [e_k]x
      double ex = 0;
      if (k == 0) ex = (i == 1 && j == 2) ? -1 : ((i == 2 && j == 1) ? 1 : 0);
      if (k == 1) ex = (i == 0 && j == 2) ? 1 : ((i == 2 && j == 0) ? -1 : 0);
      if (k == 2) ex = (i == 0 && j == 1) ? -1 : ((i == 1 && j == 0) ? 1 : 0);
      v += 2 * ex;
      D[3 * i + j] = v / s - R[3 * i + j] * 2 * c[k] / s;
    }
}

// analytic Jacobians of err: jp [2][6], jl [2][3]
__device__ void edge_jac(const double* pose, const double* X, const double* mc, const double* cam,
                         double* jp, double* jl) {
  double Rt[9], Rc[9], R[9];
  cay2rot(pose, Rt);
  cay2rot(mc, Rc);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += Rt[3 * i + k] * Rc[3 * k + j];
      R[3 * i + j] = s;
    }
  double t[3];
  for (int i = 0; i < 3; i++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += Rt[3 * i + k] * mc[3 + k];
    t[i] = s + pose[3 + i];
  }
  double Xc[3];
  for (int i = 0; i < 3; i++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += R[3 * k + i] * (X[k] - t[k]);
    Xc[i] = s;
  }
  const double x = Xc[0], y = Xc[1], z = Xc[2];
  double rho = sqrt(x * x + y * y);
  if (rho == 0.0) rho = 1e-14;
  const double theta = atan(-z / rho);
  const double* a = cam + 5;
  const double r = horner12(a, theta);
  double dr = 0;
  for (int k = 11; k >= 1; k--) dr = dr * theta + k * a[k];
  const double den = rho * rho + z * z;
  const double dth_dx = z / den * x / rho, dth_dy = z / den * y / rho, dth_dz = -rho / den;
  const double g = r / rho;
  const double dg_dx = dr * dth_dx / rho - r * x / (rho * rho * rho);
  const double dg_dy = dr * dth_dy / rho - r * y / (rho * rho * rho);
  const double dg_dz = dr * dth_dz / rho;
  const double dm[2][3] = {{g + x * dg_dx, x * dg_dy, x * dg_dz}, {y * dg_dx, g + y * dg_dy, y * dg_dz}};
  const double c = cam[0], d = cam[1], e = cam[2];
  double Jm[2][3];
  for (int j = 0; j < 3; j++) {
    Jm[0][j] = c * dm[0][j] + d * dm[1][j];
    Jm[1][j] = e * dm[0][j] + dm[1][j];
  }
  double JX[2][3];
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += Jm[i][k] * R[3 * j + k];
      JX[i][j] = s;
    }
  const double q[3] = {X[0] - pose[3], X[1] - pose[4], X[2] - pose[5]};
  for (int k = 0; k < 3; k++) {
    double D[9];
    dcay(pose, k, Rt, D);
    double w[3], dx[3];
    for (int i = 0; i < 3; i++) {
      double s = 0;
      for (int m = 0; m < 3; m++) s += D[3 * m + i] * q[m];
      w[i] = s;
    }
    for (int i = 0; i < 3; i++) {
      double s = 0;
      for (int m = 0; m < 3; m++) s += Rc[3 * m + i] * w[m];
      dx[i] = s;
    }
    for (int i = 0; i < 2; i++) {
      double s = 0;
      for (int m = 0; m < 3; m++) s += Jm[i][m] * dx[m];
      jp[6 * i + k] = -s;
    }
  }
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 3; j++) {
      jp[6 * i + 3 + j] = JX[i][j];
      jl[3 * i + j] = -JX[i][j];
    }
}

__device__ __forceinline__ void huber(double e, double delta, double dsqr, double* rho0, double* rho1) {
  if (e <= dsqr) { *rho0 = e; *rho1 = 1.; }
  else { const double sq = sqrt(e); *rho0 = 2 * sq * delta - dsqr; *rho1 = delta / sq; }
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
struct Dev {
  // problem
  const double* mc; const double* cam;
  const int32_t* e_pose; const int32_t* e_point; const int32_t* e_cam;
  const double* e_meas; const double* e_info;
  double delta, dsqr;
  // state
  double* poses; double* points; const double* poses_bk; const double* points_bk;
  // active structure
  const int32_t* aedge; int nae;
  const int32_t* pose_h; const int32_t* point_h;      // hessian index per vertex (-1 inactive)
  const int32_t* hpose_vtx; const int32_t* hpt_vtx;   // vertex id per hessian index
  int np, nl;
  const int32_t* pt_ptr; const int32_t* pt_edges;     // CSR active points -> active edges
  const int32_t* ps_ptr; const int32_t* ps_edges;     // CSR active poses  -> active edges
  const int32_t* blk_i; const int32_t* blk_j;         // lower pose blocks (i >= j)
  const int32_t* pr_ptr; const int32_t* pr_e1; const int32_t* pr_e2;  // edge pairs per block
  // per-edge buffers (indexed by edge id)
  double* err; double* w; double* jp; double* jl; double* hpl; double* y; double* chi; double* rchi;
  // system
  double* Hpp; double* bp; double* Hll; double* bl; double* Dinv; double* db;
  double* S; double* bs; double* x;   // S: n x n row-major (lower triangle used)
  double* red;                         // reduction scratch
  int* flag;
};

// per active edge: error (+ robust chi2) and optionally Jacobians / weight
__global__ __launch_bounds__(256) void k_edges(Dev d, int linearize) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= d.nae) return;
  const int e = d.aedge[k];
  const int pi = d.e_pose[e], li = d.e_point[e], ci = d.e_cam[e];
  const double* pose = d.poses + 6 * pi;
  const double* X = d.points + 3 * li;
  double er[2];
  edge_error(pose, X, d.mc + 6 * ci, d.cam + 17 * ci, d.e_meas + 2 * e, er);
  const double c2 = d.e_info[e] * (er[0] * er[0] + er[1] * er[1]);
  double r0, r1;
  huber(c2, d.delta, d.dsqr, &r0, &r1);
  d.err[2 * e] = er[0]; d.err[2 * e + 1] = er[1];
  d.chi[e] = c2;
  d.rchi[k] = r0;
  if (linearize) {
    double jp[12], jl[6];
    edge_jac(pose, X, d.mc + 6 * ci, d.cam + 17 * ci, jp, jl);
    for (int i = 0; i < 12; i++) d.jp[12 * e + i] = jp[i];
    for (int i = 0; i < 6; i++) d.jl[6 * e + i] = jl[i];
    d.w[e] = r1 * d.e_info[e];
  }
}

// deterministic single-workgroup sum / max of n doubles -> out[0]
template <bool MAX>
__global__ __launch_bounds__(1024) void k_reduce(const double* __restrict__ v, int n, double* out) {
  __shared__ double s[1024];
  double acc = MAX ? 0.0 : 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) acc = MAX ? fmax(acc, fabs(v[i])) : acc + v[i];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) s[threadIdx.x] = MAX ? fmax(s[threadIdx.x], s[threadIdx.x + o]) : s[threadIdx.x] + s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = s[0];
}

// per active point: Hll (3x3), b_l over its edges in edge order; diag -> red (for lambda init)
__global__ __launch_bounds__(256) void k_points_build(Dev d) {
  const int l = blockIdx.x * 256 + threadIdx.x;
  if (l >= d.nl) return;
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
  for (int q = d.pt_ptr[l]; q < d.pt_ptr[l + 1]; q++) {
    const int e = d.pt_edges[q];
    const double* jl = d.jl + 6 * e;
    const double w = d.w[e];
    const double we0 = -w * d.err[2 * e], we1 = -w * d.err[2 * e + 1];
    for (int a = 0; a < 3; a++) {
      for (int bb = 0; bb < 3; bb++) H[3 * a + bb] += w * (jl[a] * jl[bb] + jl[3 + a] * jl[3 + bb]);
      b[a] += jl[a] * we0 + jl[3 + a] * we1;
    }
  }
  for (int i = 0; i < 9; i++) d.Hll[9 * l + i] = H[i];
  for (int i = 0; i < 3; i++) d.bl[3 * l + i] = b[i];
  d.red[l] = fmax(fmax(fabs(H[0]), fabs(H[4])), fabs(H[8]));
}

// Deterministic block sum of NV per-thread partials: fixed xor-butterfly inside each wave,
// then the 4 wave sums in wave order.  On return sm[v * 4] holds sum v (after the barrier).
template <int NV>
__device__ __forceinline__ void block_sum_vec(double (&acc)[NV], double* sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int v = 0; v < NV; v++) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc[v] += __shfl_xor(acc[v], o);
  }
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < NV; v++) sm[v * 4 + w] = acc[v];
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const int v = threadIdx.x;
    sm[v * 4] = ((sm[v * 4] + sm[v * 4 + 1]) + sm[v * 4 + 2]) + sm[v * 4 + 3];
  }
  __syncthreads();
}

constexpr int kRedNT = 256;
constexpr int kUpper6[21][2] = {{0, 0}, {0, 1}, {0, 2}, {0, 3}, {0, 4}, {0, 5}, {1, 1},
                                {1, 2}, {1, 3}, {1, 4}, {1, 5}, {2, 2}, {2, 3}, {2, 4},
                                {2, 5}, {3, 3}, {3, 4}, {3, 5}, {4, 4}, {4, 5}, {5, 5}};

// per active pose: Hpp (6x6, upper 21 mirrored), b_p; edges of the pose split over 256
// threads (fixed stride), block tree sum
__global__ __launch_bounds__(kRedNT) void k_poses_build(Dev d) {
  __shared__ double sm[27 * 4];
  const int i = blockIdx.x, t = threadIdx.x;
  double acc[27];
#pragma unroll
  for (int v = 0; v < 27; v++) acc[v] = 0.0;
  for (int q = d.ps_ptr[i] + t; q < d.ps_ptr[i + 1]; q += kRedNT) {
    const int e = d.ps_edges[q];
    const double* jp = d.jp + 12 * e;
    double j0[6], j1[6];
#pragma unroll
    for (int a = 0; a < 6; a++) { j0[a] = jp[a]; j1[a] = jp[6 + a]; }
    const double w = d.w[e];
    const double we0 = -w * d.err[2 * e], we1 = -w * d.err[2 * e + 1];
#pragma unroll
    for (int v = 0; v < 21; v++) {
      const int a = kUpper6[v][0], bb = kUpper6[v][1];
      acc[v] += w * (j0[a] * j0[bb] + j1[a] * j1[bb]);
    }
#pragma unroll
    for (int a = 0; a < 6; a++) acc[21 + a] += j0[a] * we0 + j1[a] * we1;
  }
  block_sum_vec<27>(acc, sm);
  if (t < 21) {
    const int a = kUpper6[t][0], bb = kUpper6[t][1];
    const double h = sm[t * 4];
    d.Hpp[36 * i + 6 * a + bb] = h;
    d.Hpp[36 * i + 6 * bb + a] = h;
    if (a == bb) d.red[d.nl + 6 * i + a] = fabs(h);
  } else if (t < 27) {
    d.bp[6 * i + t - 21] = sm[t * 4];
  }
}

// per active point: D = Hll + lambda I -> Dinv (cofactors), db = Dinv b_l;
// per edge with a non-fixed pose: Hpl_e = w Jp^T Jl, Y_e = Hpl_e Dinv
__global__ __launch_bounds__(256) void k_point_trial(Dev d, double lam) {
  const int l = blockIdx.x * 256 + threadIdx.x;
  if (l >= d.nl) return;
  double D[9];
  for (int k = 0; k < 9; k++) D[k] = d.Hll[9 * l + k];
  D[0] += lam; D[4] += lam; D[8] += lam;
  const double c00 = D[4] * D[8] - D[5] * D[7], c01 = D[5] * D[6] - D[3] * D[8], c02 = D[3] * D[7] - D[4] * D[6];
  const double det = D[0] * c00 + D[1] * c01 + D[2] * c02;
  const double id = 1.0 / det;
  double Di[9];
  Di[0] = c00 * id; Di[3] = c01 * id; Di[6] = c02 * id;
  Di[1] = (D[2] * D[7] - D[1] * D[8]) * id;
  Di[4] = (D[0] * D[8] - D[2] * D[6]) * id;
  Di[7] = (D[1] * D[6] - D[0] * D[7]) * id;
  Di[2] = (D[1] * D[5] - D[2] * D[4]) * id;
  Di[5] = (D[2] * D[3] - D[0] * D[5]) * id;
  Di[8] = (D[0] * D[4] - D[1] * D[3]) * id;
  for (int k = 0; k < 9; k++) d.Dinv[9 * l + k] = Di[k];
  const double* b = d.bl + 3 * l;
  for (int a = 0; a < 3; a++) d.db[3 * l + a] = Di[3 * a] * b[0] + Di[3 * a + 1] * b[1] + Di[3 * a + 2] * b[2];
  for (int q = d.pt_ptr[l]; q < d.pt_ptr[l + 1]; q++) {
    const int e = d.pt_edges[q];
    if (d.pose_h[d.e_pose[e]] < 0) continue;
    const double* jp = d.jp + 12 * e;
    const double* jl = d.jl + 6 * e;
    const double w = d.w[e];
    double B[18];
    for (int a = 0; a < 6; a++)
      for (int bb = 0; bb < 3; bb++) B[3 * a + bb] = w * (jp[a] * jl[bb] + jp[6 + a] * jl[3 + bb]);
    for (int k = 0; k < 18; k++) d.hpl[18 * e + k] = B[k];
    for (int a = 0; a < 6; a++)
      for (int bb = 0; bb < 3; bb++)
        d.y[18 * e + 3 * a + bb] = B[3 * a] * Di[bb] + B[3 * a + 1] * Di[3 + bb] + B[3 * a + 2] * Di[6 + bb];
  }
}

// reduced camera system, lower blocks (i >= j): S_ij = [i==j](Hpp_i + lambda I)
//   - sum over (e1 in pose i, e2 in pose j, same point) Y_e1 Hpl_e2^T;
// diagonal blocks also form bschur_i = b_i - sum_e Hpl_e db(point(e)).
// The pair list of a block is split over 256 threads (fixed stride) + block tree sum.
__global__ __launch_bounds__(kRedNT) void k_schur(Dev d, double lam) {
  __shared__ double sm[42 * 4];
  const int blk = blockIdx.x, t = threadIdx.x;
  const int bi = d.blk_i[blk], bj = d.blk_j[blk];
  const int n = 6 * d.np;
  double acc[42];
#pragma unroll
  for (int v = 0; v < 42; v++) acc[v] = 0.0;
  for (int q = d.pr_ptr[blk] + t; q < d.pr_ptr[blk + 1]; q += kRedNT) {
    const double* Y = d.y + 18 * d.pr_e1[q];
    const double* B = d.hpl + 18 * d.pr_e2[q];
    double y[18], bb[18];
#pragma unroll
    for (int k = 0; k < 18; k++) { y[k] = Y[k]; bb[k] = B[k]; }
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
      for (int c = 0; c < 6; c++)
        acc[6 * a + c] += y[3 * a] * bb[3 * c] + y[3 * a + 1] * bb[3 * c + 1] + y[3 * a + 2] * bb[3 * c + 2];
  }
  if (bi == bj) {
    for (int q = d.ps_ptr[bi] + t; q < d.ps_ptr[bi + 1]; q += kRedNT) {
      const int e = d.ps_edges[q];
      const double* B = d.hpl + 18 * e;
      const double* g = d.db + 3 * d.point_h[d.e_point[e]];
      const double g0 = g[0], g1 = g[1], g2 = g[2];
#pragma unroll
      for (int a = 0; a < 6; a++) acc[36 + a] += B[3 * a] * g0 + B[3 * a + 1] * g1 + B[3 * a + 2] * g2;
    }
  }
  block_sum_vec<42>(acc, sm);
  if (t < 36) {
    const int a = t / 6, c = t % 6;
    double s0 = 0.0;
    if (bi == bj) { s0 = d.Hpp[36 * bi + 6 * a + c]; if (a == c) s0 += lam; }
    d.S[(6 * bi + a) * n + 6 * bj + c] = s0 - sm[t * 4];
  } else if (t < 42 && bi == bj) {
    const int a = t - 36;
    d.bs[6 * bi + a] = d.bp[6 * bi + a] - sm[t * 4];
  }
}

// LDL^T of the reduced camera system held in LDS (n <= kLdsN), right-looking, no pivoting
// (Eigen SimplicialLDLT only fails on an exact zero pivot), then the two triangular solves
// column by column.  One workgroup; zero pivot -> flag = 1.
constexpr int kLdsN = 88;   // n*n + n doubles <= 62.6 KB of LDS
__global__ __launch_bounds__(256) void k_ldlt_lds(Dev d) {
  extern __shared__ double A[];   // n*n lower (row-major), then x[n]
  __shared__ int fail;
  const int n = 6 * d.np, t = threadIdx.x;
  double* x = A + n * n;
  for (int idx = t; idx < n * n; idx += 256) {
    const int i = idx / n, j = idx - i * n;
    A[idx] = (j <= i) ? d.S[idx] : 0.0;
  }
  for (int i = t; i < n; i += 256) x[i] = d.bs[i];
  if (t == 0) fail = 0;
  __syncthreads();
  for (int j = 0; j < n; j++) {
    const double dj = A[j * n + j];
    if (dj == 0.0) { if (t == 0) fail = 1; break; }   // uniform: every thread reads the same dj
    for (int i = j + 1 + t; i < n; i += 256) A[i * n + j] /= dj;
    __syncthreads();
    // trailing update A[i][m] -= (L_ij L_mj) d_j for j < m <= i
    const int r = n - 1 - j;
    for (int idx = t; idx < r * r; idx += 256) {
      const int ii = idx / r, mm = idx - ii * r;
      if (mm > ii) continue;
      const int i = j + 1 + ii, m = j + 1 + mm;
      A[i * n + m] -= (A[i * n + j] * A[m * n + j]) * dj;
    }
    __syncthreads();
  }
  __syncthreads();
  if (fail) { if (t == 0) *d.flag = 1; return; }
  // forward: L y = b (unit lower), column-oriented
  for (int k = 0; k < n; k++) {
    const double xk = x[k];
    for (int i = k + 1 + t; i < n; i += 256) x[i] -= A[i * n + k] * xk;
    __syncthreads();
  }
  for (int i = t; i < n; i += 256) x[i] /= A[i * n + i];
  __syncthreads();
  // backward: L^T x = y
  for (int k = n - 1; k >= 0; k--) {
    const double xk = x[k];
    for (int i = t; i < k; i += 256) x[i] -= A[k * n + i] * xk;
    __syncthreads();
  }
  for (int i = t; i < n; i += 256) d.x[i] = x[i];
  if (t == 0) *d.flag = 0;
}

// LDL^T (no pivoting, lower, left-looking) + solve, one workgroup; zero pivot -> flag=1
__global__ __launch_bounds__(256) void k_ldlt(Dev d) {
  const int n = 6 * d.np, t = threadIdx.x;
  double* S = d.S;  // overwritten with L (strictly lower) and D (diagonal)
  __shared__ int fail;
  if (t == 0) fail = 0;
  __syncthreads();
  for (int j = 0; j < n; j++) {
    // d_j = S_jj - sum_k L_jk^2 D_k  (single thread, fixed order)
    if (t == 0) {
      double dj = S[j * n + j];
      for (int k = 0; k < j; k++) dj -= S[j * n + k] * S[j * n + k] * S[k * n + k];
      if (dj == 0.0) fail = 1;
      S[j * n + j] = dj;
    }
    __syncthreads();
    if (fail) break;
    const double dj = S[j * n + j];
    for (int i = j + 1 + t; i < n; i += 256) {
      double s = S[i * n + j];
      for (int k = 0; k < j; k++) s -= S[i * n + k] * S[j * n + k] * S[k * n + k];
      S[i * n + j] = s / dj;
    }
    __syncthreads();
  }
  if (t == 0) {
    *d.flag = fail;
    if (!fail) {
      double* x = d.x;
      for (int i = 0; i < n; i++) {
        double s = d.bs[i];
        for (int k = 0; k < i; k++) s -= S[i * n + k] * x[k];
        x[i] = s;
      }
      for (int i = 0; i < n; i++) x[i] /= S[i * n + i];
      for (int i = n - 1; i >= 0; i--) {
        double s = x[i];
        for (int k = i + 1; k < n; k++) s -= S[k * n + i] * x[k];
        x[i] = s;
      }
    }
  }
}

// x_l = Dinv (b_l - sum_e Hpl_e^T x_p); point = backup + x_l; per-point model decrease term
__global__ __launch_bounds__(256) void k_update(Dev d, double lam) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int n = 6 * d.np;
  if (k < d.nl) {
    double c[3] = {d.bl[3 * k], d.bl[3 * k + 1], d.bl[3 * k + 2]};
    for (int q = d.pt_ptr[k]; q < d.pt_ptr[k + 1]; q++) {
      const int e = d.pt_edges[q];
      const int i1 = d.pose_h[d.e_pose[e]];
      if (i1 < 0) continue;
      const double* B = d.hpl + 18 * e;
      for (int b = 0; b < 3; b++)
        for (int a = 0; a < 6; a++) c[b] -= B[3 * a + b] * d.x[6 * i1 + a];
    }
    const double* Di = d.Dinv + 9 * k;
    double s = 0;
    const int v = d.hpt_vtx[k];
    for (int a = 0; a < 3; a++) {
      const double xa = Di[3 * a] * c[0] + Di[3 * a + 1] * c[1] + Di[3 * a + 2] * c[2];
      d.x[n + 3 * k + a] = xa;
      d.points[3 * v + a] = d.points_bk[3 * v + a] + xa;
      s += xa * (lam * xa + d.bl[3 * k + a]);
    }
    d.red[k] = s;
  } else if (k < d.nl + d.np) {
    const int i = k - d.nl;
    const int v = d.hpose_vtx[i];
    double s = 0;
    for (int a = 0; a < 6; a++) {
      const double xa = d.x[6 * i + a];
      d.poses[6 * v + a] = d.poses_bk[6 * v + a] + xa;
      s += xa * (lam * xa + d.bp[6 * i + a]);
    }
    d.red[k] = s;
  }
}

}  // namespace ba
}  // namespace mcs

using namespace mcs;
using namespace mcs::ba;

struct mcs_ba_ctx {
  int device = 0;
  hipStream_t st = nullptr;
  // Device buffers are cached across calls: the driver requests them in the same order
  // every call, so request k reuses slot k when it is large enough (grow-only).
  std::vector<void*> bufs;
  std::vector<size_t> caps;
  size_t next = 0;
  double* pinned = nullptr;   // host-pinned readback scalars
  int32_t* pinned_i = nullptr;
  void* alloc(size_t bytes) {
    bytes += 64;
    if (next < bufs.size() && caps[next] >= bytes) return bufs[next++];
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    if (next < bufs.size()) {
      (void)hipFree(bufs[next]);
      bufs[next] = p; caps[next] = bytes;
    } else {
      bufs.push_back(p); caps.push_back(bytes);
    }
    next++;
    return p;
  }
  void free_all() { next = 0; }   // recycle (buffers stay allocated)
  void release() {
    for (void* p : bufs) (void)hipFree(p);
    bufs.clear(); caps.clear(); next = 0;
  }
};

namespace {

struct HostStruct {
  std::vector<int32_t> aedge, pose_h, point_h, hpose_vtx, hpt_vtx, pt_ptr, pt_edges, ps_ptr,
      ps_edges, blk_i, blk_j, pr_ptr, pr_e1, pr_e2;
  int np = 0, nl = 0;
};

void build_structure(const mcs_ba_problem& p, const uint8_t* level, HostStruct& s) {
  s.aedge.clear();
  for (int e = 0; e < p.n_edges; e++)
    if (!level || level[e] == 0) s.aedge.push_back(e);
  std::vector<int> ph(p.n_poses, 0), lh(p.n_points, 0);
  for (int e : s.aedge) { ph[p.edge_pose[e]] = 1; lh[p.edge_point[e]] = 1; }
  s.pose_h.assign(p.n_poses, -1);
  s.point_h.assign(p.n_points, -1);
  s.hpose_vtx.clear(); s.hpt_vtx.clear();
  s.np = s.nl = 0;
  for (int i = 0; i < p.n_poses; i++)
    if (ph[i] && !p.pose_fixed[i]) { s.pose_h[i] = s.np++; s.hpose_vtx.push_back(i); }
  for (int i = 0; i < p.n_points; i++)
    if (lh[i]) { s.point_h[i] = s.nl++; s.hpt_vtx.push_back(i); }
  std::vector<std::vector<int>> pe(s.nl), se(s.np);
  for (int e : s.aedge) {
    pe[s.point_h[p.edge_point[e]]].push_back(e);
    const int h = s.pose_h[p.edge_pose[e]];
    if (h >= 0) se[h].push_back(e);
  }
  s.pt_ptr.assign(1, 0); s.pt_edges.clear();
  for (int l = 0; l < s.nl; l++) {
    for (int e : pe[l]) s.pt_edges.push_back(e);
    s.pt_ptr.push_back((int)s.pt_edges.size());
  }
  s.ps_ptr.assign(1, 0); s.ps_edges.clear();
  for (int i = 0; i < s.np; i++) {
    for (int e : se[i]) s.ps_edges.push_back(e);
    s.ps_ptr.push_back((int)s.ps_edges.size());
  }
  // lower pose blocks (i >= j) and their edge pairs, in (point, e1, e2) order
  std::vector<std::vector<int>> pairs((size_t)s.np * s.np);
  for (int l = 0; l < s.nl; l++)
    for (int e1 : pe[l]) {
      const int i1 = s.pose_h[p.edge_pose[e1]];
      if (i1 < 0) continue;
      for (int e2 : pe[l]) {
        const int i2 = s.pose_h[p.edge_pose[e2]];
        if (i2 < 0 || i2 > i1) continue;
        auto& v = pairs[(size_t)i1 * s.np + i2];
        v.push_back(e1);
        v.push_back(e2);
      }
    }
  s.blk_i.clear(); s.blk_j.clear(); s.pr_ptr.assign(1, 0); s.pr_e1.clear(); s.pr_e2.clear();
  for (int i = 0; i < s.np; i++)
    for (int j = 0; j <= i; j++) {
      s.blk_i.push_back(i);
      s.blk_j.push_back(j);
      auto& v = pairs[(size_t)i * s.np + j];
      for (size_t q = 0; q < v.size(); q += 2) { s.pr_e1.push_back(v[q]); s.pr_e2.push_back(v[q + 1]); }
      s.pr_ptr.push_back((int)s.pr_e1.size());
    }
}

template <typename T>
T* up(mcs_ba_ctx* c, const std::vector<T>& v, hipError_t& e) {
  T* d = (T*)c->alloc(std::max<size_t>(1, v.size()) * sizeof(T));
  if (!d) { e = hipErrorOutOfMemory; return nullptr; }
  if (!v.empty() && e == hipSuccess) e = hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->st);
  return d;
}

template <typename T>
T* up_raw(mcs_ba_ctx* c, const T* src, size_t n, hipError_t& e) {
  T* d = (T*)c->alloc(std::max<size_t>(1, n) * sizeof(T));
  if (!d) { e = hipErrorOutOfMemory; return nullptr; }
  if (n && src && e == hipSuccess) e = hipMemcpyAsync(d, src, n * sizeof(T), hipMemcpyHostToDevice, c->st);
  return d;
}

unsigned gb(int n) { return (unsigned)std::max(1, (n + 255) / 256); }

}  // namespace

extern "C" {

void mcs_ba_default_options(mcs_ba_options* o) {
  if (!o) return;
  o->max_iterations = 10; o->gain_threshold = 1e-6; o->terminate_max_iter = 15;
  o->max_trials = 10; o->tau = 1e-5;
}

int mcs_ba_create(int32_t device, mcs_ba_ctx** out) {
  if (!out) return MCS_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  if (device < 0 || device >= ndev) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(device));
  mcs_ba_ctx* c = new (std::nothrow) mcs_ba_ctx();
  if (!c) return MCS_ERR_ARG;
  c->device = device;
  MCS_HIP_CHECK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
  MCS_HIP_CHECK(hipHostMalloc((void**)&c->pinned, 64, hipHostMallocDefault));
  MCS_HIP_CHECK(hipHostMalloc((void**)&c->pinned_i, 64, hipHostMallocDefault));
  *out = c;
  return MCS_OK;
}

void mcs_ba_destroy(mcs_ba_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->st);
  c->release();
  if (c->pinned) (void)hipHostFree(c->pinned);
  if (c->pinned_i) (void)hipHostFree(c->pinned_i);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
}

int mcs_ba_optimize(mcs_ba_ctx* c, const mcs_ba_problem* p, const mcs_ba_options* o,
                    double* poses, double* points, const uint8_t* edge_level, double* edge_chi2,
                    volatile int32_t* stop_flag, mcs_ba_report* rep) {
  if (!c || !p || !o || !poses || !points) return MCS_ERR_ARG;
  if (p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0 || p->n_cams < 1) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(c->device));
  volatile int32_t aux = 0;
  volatile int32_t* stop = stop_flag ? stop_flag : &aux;
  HostStruct s;
  build_structure(*p, edge_level, s);
  if (rep) {
    rep->n_active_edges = (int)s.aedge.size();
    rep->n_active_poses = s.np;
    rep->n_active_points = s.nl;
    rep->iterations = 0;
  }
  const int n = 6 * s.np;
  if (n > 6 * 256) {
    set_error("more than 256 active poses: the dense LDL^T path is sized for LocalBA");
    return MCS_ERR_UNSUPPORTED;
  }
  c->free_all();
  hipError_t he = hipSuccess;
  Dev d;
  const int NE = p->n_edges;
  d.mc = up_raw(c, p->mc, 6 * (size_t)p->n_cams, he);
  d.cam = up_raw(c, p->cam, 17 * (size_t)p->n_cams, he);
  d.e_pose = up_raw(c, p->edge_pose, NE, he);
  d.e_point = up_raw(c, p->edge_point, NE, he);
  d.e_cam = up_raw(c, p->edge_cam, NE, he);
  d.e_meas = up_raw(c, p->edge_meas, 2 * (size_t)NE, he);
  d.e_info = up_raw(c, p->edge_info, NE, he);
  d.delta = p->huber_delta;
  d.dsqr = p->huber_delta * p->huber_delta;
  double* d_poses = up_raw(c, (const double*)poses, 6 * (size_t)p->n_poses, he);
  double* d_points = up_raw(c, (const double*)points, 3 * (size_t)p->n_points, he);
  double* d_poses_bk = up_raw(c, (const double*)poses, 6 * (size_t)p->n_poses, he);
  double* d_points_bk = up_raw(c, (const double*)points, 3 * (size_t)p->n_points, he);
  d.poses = d_poses; d.points = d_points; d.poses_bk = d_poses_bk; d.points_bk = d_points_bk;
  d.aedge = up(c, s.aedge, he); d.nae = (int)s.aedge.size();
  d.pose_h = up(c, s.pose_h, he); d.point_h = up(c, s.point_h, he);
  d.hpose_vtx = up(c, s.hpose_vtx, he); d.hpt_vtx = up(c, s.hpt_vtx, he);
  d.np = s.np; d.nl = s.nl;
  d.pt_ptr = up(c, s.pt_ptr, he); d.pt_edges = up(c, s.pt_edges, he);
  d.ps_ptr = up(c, s.ps_ptr, he); d.ps_edges = up(c, s.ps_edges, he);
  d.blk_i = up(c, s.blk_i, he); d.blk_j = up(c, s.blk_j, he);
  d.pr_ptr = up(c, s.pr_ptr, he); d.pr_e1 = up(c, s.pr_e1, he); d.pr_e2 = up(c, s.pr_e2, he);
  auto dz = [&](size_t cnt) { double* q = (double*)c->alloc(std::max<size_t>(1, cnt) * 8); if (!q) he = hipErrorOutOfMemory; return q; };
  d.err = dz(2 * (size_t)NE); d.w = dz(NE); d.jp = dz(12 * (size_t)NE); d.jl = dz(6 * (size_t)NE);
  d.hpl = dz(18 * (size_t)NE); d.y = dz(18 * (size_t)NE); d.chi = dz(NE); d.rchi = dz(NE);
  d.Hpp = dz(36 * (size_t)s.np); d.bp = dz(6 * (size_t)s.np);
  d.Hll = dz(9 * (size_t)s.nl); d.bl = dz(3 * (size_t)s.nl);
  d.Dinv = dz(9 * (size_t)s.nl); d.db = dz(3 * (size_t)s.nl);
  d.S = dz((size_t)n * n); d.bs = dz(n); d.x = dz(n + 3 * (size_t)s.nl);
  d.red = dz((size_t)NE + 6 * (size_t)s.np + s.nl + 16);
  double* d_scalar = dz(4);
  d.flag = (int*)c->alloc(16);
  if (he != hipSuccess || !d.flag) { set_hip_error(he, "BA upload", __FILE__, __LINE__); return MCS_ERR_HIP; }
  hipStream_t st = c->st;
  const int nvar = s.np + s.nl;

  auto chi_now = [&](double* out) -> int {   // robust chi2 of the current estimate
    hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, d, 0);
    hipLaunchKernelGGL(k_reduce<false>, dim3(1), dim3(1024), 0, st, (const double*)d.rchi, d.nae, d_scalar);
    MCS_HIP_CHECK(hipMemcpyAsync(c->pinned + 3, d_scalar, 8, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipStreamSynchronize(st));
    *out = c->pinned[3];
    return MCS_OK;
  };
  auto copy_state = [&](double* dp, double* dl, const double* sp, const double* sl) -> int {
    MCS_HIP_CHECK(hipMemcpyAsync(dp, sp, 48 * (size_t)p->n_poses, hipMemcpyDeviceToDevice, st));
    MCS_HIP_CHECK(hipMemcpyAsync(dl, sl, 24 * (size_t)p->n_points, hipMemcpyDeviceToDevice, st));
    return MCS_OK;
  };
  int rc;
  double chi0 = 0;
  if (nvar == 0 || d.nae == 0) {
    if (rep) rep->chi2_initial = rep->chi2_final = 0;
  } else {
    if ((rc = chi_now(&chi0))) return rc;
    if (rep) rep->chi2_initial = chi0;
    double lambda = 0, lastChi = 0;
    int ni = 2, nBad = 0, it = 0;
    bool ok = true;
    double currentChi = chi0;
    for (int i = 0; i < o->max_iterations && !(*stop) && ok; i++) {
      // ---- OptimizationAlgorithmLevenberg::solve(i)
      // The robust chi2 of the linearisation point equals the chi2 the previous iteration
      // ended with (same kernel, same state: accepted trial or restored backup), so only
      // the first iteration reads anything back (the max diagonal for lambda's init).
      hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, d, 1);
      hipLaunchKernelGGL(k_points_build, dim3(gb(s.nl)), dim3(256), 0, st, d);
      if (s.np) hipLaunchKernelGGL(k_poses_build, dim3(s.np), dim3(kRedNT), 0, st, d);
      if (i == 0) {
        hipLaunchKernelGGL(k_reduce<true>, dim3(1), dim3(1024), 0, st, (const double*)d.red, s.nl + 6 * s.np, d_scalar + 1);
        MCS_HIP_CHECK(hipMemcpyAsync(c->pinned + 1, d_scalar + 1, 8, hipMemcpyDeviceToHost, st));
        MCS_HIP_CHECK(hipStreamSynchronize(st));
        lambda = o->tau * c->pinned[1]; ni = 2; nBad = 0;
      }
      const double iniChi = currentChi;
      double rho = 0;
      int qmax = 0;
      do {
        if ((rc = copy_state(d_poses_bk, d_points_bk, d_poses, d_points))) return rc;  // push
        hipLaunchKernelGGL(k_point_trial, dim3(gb(s.nl)), dim3(256), 0, st, d, lambda);
        if (s.np) {
          hipLaunchKernelGGL(k_schur, dim3((unsigned)s.blk_i.size()), dim3(kRedNT), 0, st, d, lambda);
          if (n <= kLdsN)
            hipLaunchKernelGGL(k_ldlt_lds, dim3(1), dim3(256), ((size_t)n * n + n) * 8, st, d);
          else
            hipLaunchKernelGGL(k_ldlt, dim3(1), dim3(256), 0, st, d);
        } else {
          MCS_HIP_CHECK(hipMemsetAsync(d.flag, 0, 4, st));
        }
        hipLaunchKernelGGL(k_update, dim3(gb(nvar)), dim3(256), 0, st, d, lambda);
        hipLaunchKernelGGL(k_reduce<false>, dim3(1), dim3(1024), 0, st, (const double*)d.red, nvar, d_scalar + 2);
        hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, d, 0);
        hipLaunchKernelGGL(k_reduce<false>, dim3(1), dim3(1024), 0, st, (const double*)d.rchi, d.nae, d_scalar);
        MCS_HIP_CHECK(hipMemcpyAsync(c->pinned, d_scalar, 24, hipMemcpyDeviceToHost, st));
        MCS_HIP_CHECK(hipMemcpyAsync(c->pinned_i, d.flag, 4, hipMemcpyDeviceToHost, st));
        MCS_HIP_CHECK(hipStreamSynchronize(st));
        const double tr[3] = {c->pinned[0], c->pinned[1], c->pinned[2]};
        const int fl = c->pinned_i[0];
        double tempChi = tr[0];
        if (fl) tempChi = std::numeric_limits<double>::max();
        rho = currentChi - tempChi;
        double scale = tr[2];
        scale += 1e-3;
        rho /= scale;
        if (rho > 0 && std::isfinite(tempChi)) {
          double alpha = 1. - std::pow((2 * rho - 1), 3);
          alpha = std::min(alpha, 2. / 3.);
          lambda *= std::max(1. / 3., alpha);
          ni = 2;
          currentChi = tempChi;
        } else {
          lambda *= ni;
          ni *= 2;
          if ((rc = copy_state(d_poses, d_points, d_poses_bk, d_points_bk))) return rc;  // pop
        }
        qmax++;
      } while (rho < 0 && qmax < o->max_trials && !(*stop));
      int result = 0;
      if (qmax == o->max_trials || rho == 0) result = 1;
      else {
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) result = 1;
      }
      ok = (result == 0);
      ++it;
      // ---- SparseOptimizerTerminateAction (post-iteration): activeRobustChi2 of the
      // current state == currentChi (see above)
      const double cur = currentChi;
      if (rep && rep->trace_chi2 && i < rep->trace_cap) rep->trace_chi2[i] = cur;
      if (i == 0) lastChi = cur;
      else {
        bool stopOpt = false;
        if (i < o->terminate_max_iter) {
          const double gain = (lastChi - cur) / cur;
          lastChi = cur;
          if (gain >= 0 && gain < o->gain_threshold) stopOpt = true;
        } else {
          stopOpt = true;
        }
        if (stopOpt) *stop = 1;
      }
      if (rep) rep->lambda_final = lambda;
    }
    if (rep) rep->iterations = it;
    const double fin = currentChi;
    if (rep) rep->chi2_final = fin;
  }
  if (rep) rep->stop_flag = *stop;
  MCS_HIP_CHECK(hipMemcpyAsync(poses, d_poses, 48 * (size_t)p->n_poses, hipMemcpyDeviceToHost, st));
  MCS_HIP_CHECK(hipMemcpyAsync(points, d_points, 24 * (size_t)p->n_points, hipMemcpyDeviceToHost, st));
  if (edge_chi2) {
    // chi2 of every edge (active or not) at the final estimate
    std::vector<int32_t> all(NE);
    for (int e = 0; e < NE; e++) all[e] = e;
    int32_t* d_all = up(c, all, he);
    if (he != hipSuccess) { set_hip_error(he, "BA chi2", __FILE__, __LINE__); return MCS_ERR_HIP; }
    Dev d2 = d;
    d2.aedge = d_all;
    d2.nae = NE;
    d2.rchi = dz(NE);
    hipLaunchKernelGGL(k_edges, dim3(gb(NE)), dim3(256), 0, st, d2, 0);
    MCS_HIP_CHECK(hipMemcpyAsync(edge_chi2, d.chi, 8 * (size_t)NE, hipMemcpyDeviceToHost, st));
  }
  MCS_HIP_CHECK(hipStreamSynchronize(st));
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_local_ba(mcs_ba_ctx* c, const mcs_ba_problem* p, double* poses, double* points,
                 uint8_t* edge_inlier, int32_t* write_back, volatile int32_t* stop_flag,
                 mcs_ba_report* r1, mcs_ba_report* r2) {
  if (!c || !p || !poses || !points || !edge_inlier || !write_back) return MCS_ERR_ARG;
  mcs_ba_options o;
  mcs_ba_default_options(&o);
  const double huberK2 = p->huber_delta * p->huber_delta;
  std::vector<uint8_t> level(p->n_edges, 0);
  std::vector<double> chi(p->n_edges);
  *write_back = 0;
  for (int e = 0; e < p->n_edges; e++) edge_inlier[e] = 1;
  if (stop_flag && *stop_flag) return MCS_OK;               // :771-773
  o.max_iterations = 10;
  int rc = mcs_ba_optimize(c, p, &o, poses, points, level.data(), chi.data(), stop_flag, r1);
  if (rc) return rc;
  if (stop_flag && *stop_flag) return MCS_OK;               // bDoMore = false (:790-794)
  for (int e = 0; e < p->n_edges; e++)                      // :798-817
    if (chi[e] > huberK2) { level[e] = 1; edge_inlier[e] = 0; }
  o.max_iterations = 15;                                    // :819-820
  rc = mcs_ba_optimize(c, p, &o, poses, points, level.data(), chi.data(), stop_flag, r2);
  if (rc) return rc;
  for (int e = 0; e < p->n_edges; e++)                      // :830-849
    if (edge_inlier[e] && chi[e] > huberK2) edge_inlier[e] = 0;
  *write_back = 1;
  return MCS_OK;
}

int mcs_ba_linearize(mcs_ba_ctx* c, const mcs_ba_problem* p, double* err, double* jac_pose,
                     double* jac_point) {
  if (!c || !p || !err || !jac_pose || !jac_point) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(c->device));
  c->free_all();
  hipError_t he = hipSuccess;
  Dev d;
  std::memset(&d, 0, sizeof(d));
  const int NE = p->n_edges;
  d.mc = up_raw(c, p->mc, 6 * (size_t)p->n_cams, he);
  d.cam = up_raw(c, p->cam, 17 * (size_t)p->n_cams, he);
  d.e_pose = up_raw(c, p->edge_pose, NE, he);
  d.e_point = up_raw(c, p->edge_point, NE, he);
  d.e_cam = up_raw(c, p->edge_cam, NE, he);
  d.e_meas = up_raw(c, p->edge_meas, 2 * (size_t)NE, he);
  d.e_info = up_raw(c, p->edge_info, NE, he);
  d.delta = p->huber_delta; d.dsqr = p->huber_delta * p->huber_delta;
  d.poses = up_raw(c, p->poses, 6 * (size_t)p->n_poses, he);
  d.points = up_raw(c, p->points, 3 * (size_t)p->n_points, he);
  std::vector<int32_t> all(NE);
  for (int e = 0; e < NE; e++) all[e] = e;
  d.aedge = up(c, all, he); d.nae = NE;
  auto dz = [&](size_t cnt) { double* q = (double*)c->alloc(std::max<size_t>(1, cnt) * 8); if (!q) he = hipErrorOutOfMemory; return q; };
  d.err = dz(2 * (size_t)NE); d.w = dz(NE); d.jp = dz(12 * (size_t)NE); d.jl = dz(6 * (size_t)NE);
  d.chi = dz(NE); d.rchi = dz(NE);
  if (he != hipSuccess) { set_hip_error(he, "BA linearize upload", __FILE__, __LINE__); return MCS_ERR_HIP; }
  hipLaunchKernelGGL(k_edges, dim3(gb(NE)), dim3(256), 0, c->st, d, 1);
  MCS_HIP_CHECK(hipMemcpyAsync(err, d.err, 16 * (size_t)NE, hipMemcpyDeviceToHost, c->st));
  MCS_HIP_CHECK(hipMemcpyAsync(jac_pose, d.jp, 96 * (size_t)NE, hipMemcpyDeviceToHost, c->st));
  MCS_HIP_CHECK(hipMemcpyAsync(jac_point, d.jl, 48 * (size_t)NE, hipMemcpyDeviceToHost, c->st));
  MCS_HIP_CHECK(hipStreamSynchronize(c->st));
  return MCS_OK;
}

}  // extern "C"
