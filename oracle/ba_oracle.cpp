// ============================================================================
// ORACLE -- TEST INFRASTRUCTURE ONLY (checker / CPU baseline; never in the product).
//
// CPU restatement of the MultiCol bundle adjustment on the hot path:
//   * EdgeProjectXYZ2MCS::computeError      src/g2o_MultiCol_vertices_edges.cpp:32-63
//     via cayley2hom/cayley2rot (include/misc.h:134-226), cConverter::invMat
//     (src/cConverter.cpp:31-44), cCamModelGeneral_::WorldToImg (src/cam_model_omni.cpp:147-163)
//   * edge Jacobian: chain rule of the same projection -- replaces the
//     900-temporary symbolic mcsJacs1 (:134-1145); checked against central differences
//   * g2o LM: OptimizationAlgorithmLevenberg::solve (optimization_algorithm_levenberg.cpp:61-189),
//     BlockSolver<6,3> Schur complement (block_solver.hpp:354-486, 502-604), quadratic form
//     with Huber (base_multi_edge.hpp:36-48,171-222; robust_kernel_impl.cpp:78-91),
//     SparseOptimizer::optimize / initializeOptimization / buildIndexMapping
//     (sparse_optimizer.cpp:166-267, 354-435), SparseOptimizerTerminateAction (:21-72)
//   * the reduced camera system is solved by LDLT without pivoting: Eigen's SimplicialLDLT
//     (linear_solver_eigen.h:94-126) also only fails on an exact zero pivot
//   * cOptimizer::LocalBundleAdjustment rounds + culling (src/cOptimizer.cpp:771-903),
//     BundleAdjustment (:73-261) and PoseOptimization (:264-486)
//
// PARITY STATUS: unpinned against the reference binary.  The MultiCol edge needs OpenCV
// (absent); the vendored g2o core needs the cmake-generated ThirdParty/g2o/config.h
// (core/openmp_mutex.h:30 includes "../../config.h"), so it is unbuildable here without a
// stand-in header.  The restatement is checked by the properties in tests/test_ba.py.
// ============================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <list>
#include <map>
#include <vector>

#include "../include/mcs_ba.h"

namespace {

// computeScale test hook (tests/test_ba_scale_order.py): per LM trial {currentChi - tempChi,
// computeScale in g2o's index order, the product's split order (points' sum + poses' sum),
// sum of |terms|, number of terms, lambda}
bool g_scale_trace_on = false;
std::vector<double> g_scale_trace;


void cay2rot(const double* c, double* R) {  // misc.h:134-162
  const double c1 = c[0], c2 = c[1], c3 = c[2];
  const double c1s = c1 * c1, c2s = c2 * c2, c3s = c3 * c3;
  const double scale = 1 + c1s + c2s + c3s;
  double M[9] = {1 + c1s - c2s - c3s, 2 * (c1 * c2 - c3), 2 * (c1 * c3 + c2),
                 2 * (c1 * c2 + c3), 1 - c1s + c2s - c3s, 2 * (c2 * c3 - c1),
                 2 * (c1 * c3 - c2), 2 * (c2 * c3 + c1), 1 - c1s - c2s + c3s};
  const double inv = 1 / scale;
  for (int i = 0; i < 9; i++) R[i] = inv * M[i];
}

void cay2hom(const double* p, double* T) {  // 4x4 row-major
  double R[9];
  cay2rot(p, R);
  const double t[3] = {p[3], p[4], p[5]};
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) T[4 * i + j] = R[3 * i + j];
    T[4 * i + 3] = t[i];
  }
  T[12] = T[13] = T[14] = 0; T[15] = 1;
}

void mat44(const double* A, const double* B, double* C) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      double s = 0;
      for (int k = 0; k < 4; k++) s += A[4 * i + k] * B[4 * k + j];
      C[4 * i + j] = s;
    }
}

void inv_mat(const double* M, double* O) {  // cConverter::invMat
  double R[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R[3 * i + j] = M[4 * j + i];  // transpose
  const double t[3] = {M[3], M[7], M[11]};
  for (int i = 0; i < 3; i++) {
    double s = 0;
    for (int k = 0; k < 3; k++) s += (-R[3 * i + k]) * t[k];
    for (int j = 0; j < 3; j++) O[4 * i + j] = R[3 * i + j];
    O[4 * i + 3] = s;
  }
  O[12] = O[13] = O[14] = 0; O[15] = 1;
}

inline double horner(const double* c, int s, double x) {
  double r = 0.0;
  for (int i = s - 1; i >= 0; i--) r = r * x + c[i];
  return r;
}

void world_to_img(const double* cam, double x, double y, double z, double& u, double& v) {
  double norm = std::sqrt(x * x + y * y);
  if (norm == 0.0) norm = 1e-14;
  const double theta = std::atan(-z / norm);
  const double rho = horner(cam + 5, 12, theta);
  const double uu = x / norm * rho, vv = y / norm * rho;
  u = uu * cam[0] + vv * cam[1] + cam[3];
  v = uu * cam[2] + vv + cam[4];
}

// EdgeProjectXYZ2MCS::computeError
void edge_error(const double* pose, const double* X, const double* mc, const double* cam,
                const double* meas, double* err) {
  double Tt[16], Tc[16], Tct[16], Ti[16];
  cay2hom(pose, Tt);
  cay2hom(mc, Tc);
  mat44(Tt, Tc, Tct);
  inv_mat(Tct, Ti);
  const double v4[4] = {X[0], X[1], X[2], 1.0};
  double r[4];
  for (int i = 0; i < 4; i++) {
    double s = 0;
    for (int k = 0; k < 4; k++) s += Ti[4 * i + k] * v4[k];
    r[i] = s;
  }
  double u, v;
  world_to_img(cam, r[0], r[1], r[2], u, v);
  err[0] = meas[0] - u;
  err[1] = meas[1] - v;
}

// d R(c)/d c_k (Cayley), 3x3 row-major
void dcay(const double* c, int k, double* D) {
  double R[9];
  cay2rot(c, R);
  const double s = 1 + c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
  double dN[9];
  // N = (1 - c'c) I + 2 c c' + 2 [c]x
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double v = (i == j) ? -2 * c[k] : 0.0;
      v += 2 * (((i == k) ? c[j] : 0.0) + ((j == k) ? c[i] : 0.0));
      dN[3 * i + j] = v;
    }
  // [e_k]x
  const double ex[3][9] = {{0, 0, 0, 0, 0, -1, 0, 1, 0}, {0, 0, 1, 0, 0, 0, -1, 0, 0},
                           {0, -1, 0, 1, 0, 0, 0, 0, 0}};
  for (int i = 0; i < 9; i++) dN[i] += 2 * ex[k][i];
  for (int i = 0; i < 9; i++) D[i] = dN[i] / s - R[i] * 2 * c[k] / s;
}

// analytic Jacobians of err = meas - proj: jp [2][6], jl [2][3]
void edge_jac(const double* pose, const double* X, const double* mc, const double* cam,
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
  double rho = std::sqrt(x * x + y * y);
  if (rho == 0.0) rho = 1e-14;
  const double theta = std::atan(-z / rho);
  const double* a = cam + 5;
  const double r = horner(a, 12, theta);
  double dr = 0;
  for (int k = 11; k >= 1; k--) dr = dr * theta + k * a[k];
  const double den = rho * rho + z * z;
  const double dth_dx = z / den * x / rho, dth_dy = z / den * y / rho, dth_dz = -rho / den;
  const double g = r / rho;
  const double dg_dx = dr * dth_dx / rho - r * x / (rho * rho * rho);
  const double dg_dy = dr * dth_dy / rho - r * y / (rho * rho * rho);
  const double dg_dz = dr * dth_dz / rho;
  const double dm[2][3] = {{g + x * dg_dx, x * dg_dy, x * dg_dz},
                           {y * dg_dx, g + y * dg_dy, y * dg_dz}};
  const double c = cam[0], d = cam[1], e = cam[2];
  double Jm[2][3];
  for (int j = 0; j < 3; j++) {
    Jm[0][j] = c * dm[0][j] + d * dm[1][j];
    Jm[1][j] = e * dm[0][j] + dm[1][j];
  }
  // d Xc / d X = R^T  -> J_X = Jm R^T
  double JX[2][3];
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += Jm[i][k] * R[3 * j + k];
      JX[i][j] = s;
    }
  // rotation columns: d Xc / d c_k = Rc^T dRt_k^T (X - t_t)
  const double q[3] = {X[0] - pose[3], X[1] - pose[4], X[2] - pose[5]};
  for (int k = 0; k < 3; k++) {
    double D[9];
    dcay(pose, k, D);
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
      jp[6 * i + 3 + j] = JX[i][j];   // d proj / d t_t = -J_X  -> edge jac = +J_X
      jl[3 * i + j] = -JX[i][j];
    }
}

// RobustKernelHuber::dsqr is a float member (ThirdParty/g2o/g2o/core/robust_kernel_impl.h:84),
// setDelta stores delta*delta into it (robust_kernel_impl.cpp:65-69)
static inline double huber_dsqr(double delta) { return (double)(float)(delta * delta); }

struct Huber {
  double delta, dsqr;
  void robustify(double e, double* rho) const {
    if (e <= dsqr) { rho[0] = e; rho[1] = 1.; rho[2] = 0.; }
    else {
      const double sq = std::sqrt(e);
      rho[0] = 2 * sq * delta - dsqr;
      rho[1] = delta / sq;
      rho[2] = -0.5 * rho[1] / e;
    }
  }
};

// ---------------------------------------------------------------------------
// One SparseOptimizer configured like LocalBundleAdjustment.
// ---------------------------------------------------------------------------
struct Graph {
  const mcs_ba_problem* P;
  std::vector<double> poses, points;   // current estimate
  std::vector<uint8_t> level;          // per edge, 0 active
  bool points_fixed = false;           // BundleAdjustment(poseOnly): setFixed(poseOnly) (:178)
  const double* pose_cnt = nullptr;    // optional: active-edge count per pose over ALL shards
  Huber hk;
  // active structure
  std::vector<int> aedges;             // active edges in id order
  std::vector<int> pose_h, point_h;    // hessian index (-1 inactive)
  int np = 0, nl = 0;
  std::vector<double> err;             // [n_edges][2]
  // system
  std::vector<double> Hpp, Hll, bp, bl;   // Hpp: np 6x6 blocks (diagonal only), Hll: nl 3x3
  std::vector<double> Hpl;                // per active edge 6x3 block (summed per (pose,point) implicitly)
  std::vector<double> x;                  // [6np + 3nl]
  std::vector<double> stack_poses, stack_points;
  double lambda = 0; int ni = 2, nBad = 0;

  void compute_errors() {
    for (int e : aedges) {
      const mcs_ba_problem& p = *P;
      edge_error(&poses[6 * p.edge_pose[e]], &points[3 * p.edge_point[e]], p.mc + 6 * p.edge_cam[e],
                 p.cam + 17 * p.edge_cam[e], p.edge_meas + 2 * e, &err[2 * e]);
    }
  }
  double chi2_edge(int e) const {
    return P->edge_info[e] * (err[2 * e] * err[2 * e] + err[2 * e + 1] * err[2 * e + 1]);
  }
  double robust_chi2() const {
    double chi = 0, rho[3];
    for (int e : aedges) { hk.robustify(chi2_edge(e), rho); chi += rho[0]; }
    return chi;
  }

  void initialize() {  // initializeOptimization(0) + buildIndexMapping
    const mcs_ba_problem& p = *P;
    aedges.clear();
    // initializeOptimization (sparse_optimizer.cpp:206-267): level-0 edges that are not
    // allVerticesFixed (Mc / IO are always fixed, so: pose fixed and point fixed)
    for (int e = 0; e < p.n_edges; e++)
      if (level[e] == 0 && !(p.pose_fixed[p.edge_pose[e]] && points_fixed)) aedges.push_back(e);
    std::vector<int> pose_has(p.n_poses, 0), pt_has(p.n_points, 0);
    for (int e : aedges) { pose_has[p.edge_pose[e]] = 1; pt_has[p.edge_point[e]] = !points_fixed; }
    if (pose_cnt)
      for (int i = 0; i < p.n_poses; i++) pose_has[i] = pose_cnt[i] > 0;
    pose_h.assign(p.n_poses, -1);
    point_h.assign(p.n_points, -1);
    np = nl = 0;
    for (int i = 0; i < p.n_poses; i++)
      if (pose_has[i] && !p.pose_fixed[i]) pose_h[i] = np++;
    for (int i = 0; i < p.n_points; i++)
      if (pt_has[i]) point_h[i] = nl++;
  }

  void build_system() {  // BlockSolver::buildSystem
    const mcs_ba_problem& p = *P;
    Hpp.assign(36 * np, 0); bp.assign(6 * np, 0);
    Hll.assign(9 * nl, 0); bl.assign(3 * nl, 0);
    Hpl.assign(18 * p.n_edges, 0);
    for (int e : aedges) {
      const int pi = pose_h[p.edge_pose[e]], li = point_h[p.edge_point[e]];
      if (pi < 0 && li < 0) continue;   // every vertex fixed: no contribution
      double jp[12], jl[6];
      edge_jac(&poses[6 * p.edge_pose[e]], &points[3 * p.edge_point[e]], p.mc + 6 * p.edge_cam[e],
               p.cam + 17 * p.edge_cam[e], jp, jl);
      double rho[3];
      hk.robustify(chi2_edge(e), rho);
      const double w = rho[1] * p.edge_info[e];            // robustInformation
      const double we[2] = {-w * err[2 * e], -w * err[2 * e + 1]};  // omega_r = -Omega e rho'
      if (pi >= 0) {
        for (int a = 0; a < 6; a++) {
          for (int b = 0; b < 6; b++) Hpp[36 * pi + 6 * a + b] += w * (jp[a] * jp[b] + jp[6 + a] * jp[6 + b]);
          bp[6 * pi + a] += jp[a] * we[0] + jp[6 + a] * we[1];
        }
      }
      if (li >= 0)
        for (int a = 0; a < 3; a++) {
          for (int b = 0; b < 3; b++) Hll[9 * li + 3 * a + b] += w * (jl[a] * jl[b] + jl[3 + a] * jl[3 + b]);
          bl[3 * li + a] += jl[a] * we[0] + jl[3 + a] * we[1];
        }
      if (pi >= 0 && li >= 0)
        for (int a = 0; a < 6; a++)
          for (int b = 0; b < 3; b++) Hpl[18 * e + 3 * a + b] = w * (jp[a] * jl[b] + jp[6 + a] * jl[3 + b]);
    }
  }

  double lambda_init(double tau) const {
    double m = 0;
    for (int i = 0; i < np; i++)
      for (int j = 0; j < 6; j++) m = std::max(m, std::fabs(Hpp[36 * i + 7 * j]));
    for (int i = 0; i < nl; i++)
      for (int j = 0; j < 3; j++) m = std::max(m, std::fabs(Hll[9 * i + 4 * j]));
    return tau * m;
  }

  // BlockSolver::solve with lambda on the diagonal; returns false on an exact zero pivot
  bool solve(double lam) {
    std::vector<double> S, bs;
    schur(lam, lam, S, bs);
    return factor_solve(S, bs);
  }

  // reduced camera system S = Hpp + lam_diag I - sum Hpl Hll(lam)^-1 Hpl^T, bs; also Dinv_
  std::vector<double> Dinv_;
  std::vector<std::vector<int>> pe_;
  void schur(double lam, double lam_diag, std::vector<double>& S, std::vector<double>& bs) {
    const mcs_ba_problem& p = *P;
    const int n = 6 * np;
    S.assign((size_t)n * n, 0.0);
    bs.assign(n, 0.0);
    for (int i = 0; i < np; i++)
      for (int a = 0; a < 6; a++) {
        for (int b = 0; b < 6; b++) S[(6 * i + a) * n + 6 * i + b] = Hpp[36 * i + 6 * a + b];
        S[(6 * i + a) * n + 6 * i + a] += lam_diag;
        bs[6 * i + a] = bp[6 * i + a];
      }
    std::vector<double>& Dinv = Dinv_;
    Dinv.assign(9 * nl, 0.0);
    // edges grouped per point in edge order
    std::vector<std::vector<int>>& pe = pe_;
    pe.assign(nl, {});
    for (int e : aedges)
      if (point_h[p.edge_point[e]] >= 0) pe[point_h[p.edge_point[e]]].push_back(e);
    for (int l = 0; l < nl; l++) {
      double D[9];
      for (int k = 0; k < 9; k++) D[k] = Hll[9 * l + k];
      D[0] += lam; D[4] += lam; D[8] += lam;
      // Dinv = D.inverse(): Eigen 3.2.10 fixed 3x3 (ThirdParty/Eigen/Eigen/src/LU/Inverse.h:117-159),
      // det summed c0 + (c1 + c2) (Redux.h:77-106, no packet access for 3-vectors)
      auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return D[3 * i1 + j1] * D[3 * i2 + j2] - D[3 * i1 + j2] * D[3 * i2 + j1];
      };
      const double k0 = cof(0, 0), k1 = cof(1, 0), k2 = cof(2, 0);
      const double det = k0 * D[0] + (k1 * D[3] + k2 * D[6]);
      const double id = 1.0 / det;
      double* Di = &Dinv[9 * l];
      Di[0] = k0 * id; Di[1] = k1 * id; Di[2] = k2 * id;
      Di[3] = cof(0, 1) * id; Di[4] = cof(1, 1) * id; Di[5] = cof(2, 1) * id;
      Di[6] = cof(0, 2) * id; Di[7] = cof(1, 2) * id; Di[8] = cof(2, 2) * id;
      double db[3];
      for (int a = 0; a < 3; a++) db[a] = Di[3 * a] * bl[3 * l] + Di[3 * a + 1] * bl[3 * l + 1] + Di[3 * a + 2] * bl[3 * l + 2];
      for (int e1 : pe[l]) {
        const int i1 = pose_h[p.edge_pose[e1]];
        if (i1 < 0) continue;
        const double* B1 = &Hpl[18 * e1];
        double BD[18];
        for (int a = 0; a < 6; a++)
          for (int b = 0; b < 3; b++)
            BD[3 * a + b] = B1[3 * a] * Di[b] + B1[3 * a + 1] * Di[3 + b] + B1[3 * a + 2] * Di[6 + b];
        for (int a = 0; a < 6; a++) bs[6 * i1 + a] -= B1[3 * a] * db[0] + B1[3 * a + 1] * db[1] + B1[3 * a + 2] * db[2];
        for (int e2 : pe[l]) {
          const int i2 = pose_h[p.edge_pose[e2]];
          if (i2 < 0) continue;
          const double* B2 = &Hpl[18 * e2];
          for (int a = 0; a < 6; a++)
            for (int b = 0; b < 6; b++)
              S[(6 * i1 + a) * n + 6 * i2 + b] -=
                  BD[3 * a] * B2[3 * b] + BD[3 * a + 1] * B2[3 * b + 1] + BD[3 * a + 2] * B2[3 * b + 2];
        }
      }
    }
  }

  bool factor_solve(const std::vector<double>& S, const std::vector<double>& bs) {
    const mcs_ba_problem& p = *P;
    const int n = 6 * np;
    const std::vector<double>& Dinv = Dinv_;
    const std::vector<std::vector<int>>& pe = pe_;
    // LDL^T without pivoting (lower), solve
    std::vector<double> L((size_t)n * n, 0.0), Dg(n, 0.0);
    for (int j = 0; j < n; j++) {
      double d = S[j * n + j];
      for (int k = 0; k < j; k++) d -= L[j * n + k] * L[j * n + k] * Dg[k];
      if (d == 0.0) return false;
      Dg[j] = d;
      L[j * n + j] = 1.0;
      for (int i = j + 1; i < n; i++) {
        double s = S[i * n + j];
        for (int k = 0; k < j; k++) s -= L[i * n + k] * L[j * n + k] * Dg[k];
        L[i * n + j] = s / d;
      }
    }
    x.assign(6 * np + 3 * nl, 0.0);
    std::vector<double> yv(n);
    for (int i = 0; i < n; i++) {
      double s = bs[i];
      for (int k = 0; k < i; k++) s -= L[i * n + k] * yv[k];
      yv[i] = s;
    }
    for (int i = 0; i < n; i++) yv[i] /= Dg[i];
    for (int i = n - 1; i >= 0; i--) {
      double s = yv[i];
      for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
      x[i] = s;
    }
    // back-substitute the points: x_l = Dinv (b_l - Hpl^T x_p)
    for (int l = 0; l < nl; l++) {
      double c[3] = {bl[3 * l], bl[3 * l + 1], bl[3 * l + 2]};
      for (int e : pe[l]) {
        const int i1 = pose_h[p.edge_pose[e]];
        if (i1 < 0) continue;
        const double* B = &Hpl[18 * e];
        for (int b = 0; b < 3; b++)
          for (int a = 0; a < 6; a++) c[b] -= B[3 * a + b] * x[6 * i1 + a];
      }
      const double* Di = &Dinv[9 * l];
      for (int a = 0; a < 3; a++) x[n + 3 * l + a] = Di[3 * a] * c[0] + Di[3 * a + 1] * c[1] + Di[3 * a + 2] * c[2];
    }
    return true;
  }

  void update() {  // SparseOptimizer::update: oplus (additive) on non-fixed active vertices
    const mcs_ba_problem& p = *P;
    for (int i = 0; i < p.n_poses; i++)
      if (pose_h[i] >= 0)
        for (int a = 0; a < 6; a++) poses[6 * i + a] += x[6 * pose_h[i] + a];
    for (int i = 0; i < p.n_points; i++)
      if (point_h[i] >= 0)
        for (int a = 0; a < 3; a++) points[3 * i + a] += x[6 * np + 3 * point_h[i] + a];
  }

  // computeScale's terms summed with |.|: the bound on any other summation order (test hook)
  void scale_terms(double lam, double* sum_abs, double* split, int* n) const {
    double a = 0, sp = 0, sl = 0;
    int k = 0;
    for (int i = 0; i < 6 * np; i++, k++) {
      const double t = x[i] * (lam * x[i] + bp[i]);
      a += std::fabs(t); sp += t;
    }
    for (int j = 0; j < 3 * nl; j++, k++) {
      const double t = x[6 * np + j] * (lam * x[6 * np + j] + bl[j]);
      a += std::fabs(t); sl += t;
    }
    *sum_abs = a; *split = sl + sp; *n = k;
  }

  double compute_scale(double lam) const {
    double s = 0;
    for (int i = 0; i < np; i++)
      for (int a = 0; a < 6; a++) s += x[6 * i + a] * (lam * x[6 * i + a] + bp[6 * i + a]);
    for (int l = 0; l < nl; l++)
      for (int a = 0; a < 3; a++) s += x[6 * np + 3 * l + a] * (lam * x[6 * np + 3 * l + a] + bl[3 * l + a]);
    return s;
  }

  // OptimizationAlgorithmLevenberg::solve: 0 OK, 1 Terminate
  int lm_solve(int iteration, const mcs_ba_options& o, volatile int32_t* stop) {
    compute_errors();
    double currentChi = robust_chi2();
    const double iniChi = currentChi;
    build_system();
    if (iteration == 0) { lambda = lambda_init(o.tau); ni = 2; nBad = 0; }
    double rho = 0;
    int qmax = 0;
    do {
      stack_poses = poses; stack_points = points;           // push
      const bool ok2 = solve(lambda);
      update();
      compute_errors();
      double tempChi = robust_chi2();
      if (!ok2) tempChi = std::numeric_limits<double>::max();
      rho = currentChi - tempChi;
      double scale = compute_scale(lambda);
      if (g_scale_trace_on) {
        double sa, split; int nt;
        scale_terms(lambda, &sa, &split, &nt);
        const double rec[6] = {rho, scale, split, sa, (double)nt, lambda};
        g_scale_trace.insert(g_scale_trace.end(), rec, rec + 6);
      }
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tempChi)) {
        double alpha = 1. - std::pow((2 * rho - 1), 3);
        alpha = std::min(alpha, 2. / 3.);
        const double sf = std::max(1. / 3., alpha);
        lambda *= sf;
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        poses = stack_poses; points = stack_points;           // pop
      }
      qmax++;
    } while (rho < 0 && qmax < o.max_trials && !(stop && *stop));
    if (qmax == o.max_trials || rho == 0) return 1;
    if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
    else nBad = 0;
    if (nBad >= 3) return 1;
    return 0;
  }
};

int optimize(Graph& g, const mcs_ba_options& o, volatile int32_t* stop_in, mcs_ba_report* rep) {
  int32_t aux = 0;
  volatile int32_t* stop = stop_in ? stop_in : &aux;
  g.initialize();
  g.err.assign(2 * g.P->n_edges, 0.0);
  if (rep) {
    rep->n_active_edges = (int32_t)g.aedges.size();
    rep->n_active_poses = g.np;
    rep->n_active_points = g.nl;
  }
  if (g.np + g.nl == 0) return 0;
  g.compute_errors();
  if (rep) rep->chi2_initial = g.robust_chi2();
  // terminate action (iteration < 0 never reached by optimize(): the flag is not reset)
  double lastChi = 0;
  int it = 0;
  bool ok = true;
  for (int i = 0; i < o.max_iterations && !(*stop) && ok; i++) {
    const int r = g.lm_solve(i, o, stop);
    ok = (r == 0);
    ++it;
    // SparseOptimizerTerminateAction (post-iteration)
    g.compute_errors();
    const double cur = g.robust_chi2();
    if (rep && rep->trace_chi2 && i < rep->trace_cap) rep->trace_chi2[i] = cur;
    if (i == 0) lastChi = cur;
    else {
      bool stopOpt = false;
      if (i < o.terminate_max_iter) {
        const double gain = (lastChi - cur) / cur;
        lastChi = cur;
        if (gain >= 0 && gain < o.gain_threshold) stopOpt = true;
      } else {
        stopOpt = true;
      }
      if (stopOpt) *stop = 1;
    }
  }
  g.compute_errors();
  if (rep) {
    rep->iterations = it;
    rep->stop_flag = *stop;
    rep->chi2_final = g.robust_chi2();
    rep->lambda_final = g.lambda;
  }
  return it;
}

}  // namespace

extern "C" {

void oracle_scale_trace(int32_t enable) {
  g_scale_trace_on = enable != 0;
  g_scale_trace.clear();
}
int32_t oracle_scale_trace_read(double* out, int32_t cap) {
  const int32_t n = (int32_t)(g_scale_trace.size() / 6);
  for (int32_t i = 0; i < n && i < cap; i++)
    for (int k = 0; k < 6; k++) out[6 * i + k] = g_scale_trace[6 * i + k];
  return n;
}

// ComputeE (src/misc.cpp:72-86) for every camera pair as SearchForTriangulationRaw's Es table
// (src/cORBmatcher.cpp:985-998): E[i][j] = ComputeE(invMat(M_t1 M_c[i]), M_t2 M_c[j]).
int oracle_compute_e_rig(const double* mt1, const double* mt2, const double* mc, int ncams,
                         double* E) {
  auto matmul = [](const double* a, const double* b, double* c, int m, int l, int n) {
    for (int i = 0; i < m; i++)
      for (int j = 0; j < n; j++) {
        double s = 0;
        for (int k = 0; k < l; k++) s += a[i * l + k] * b[k * n + j];
        c[i * n + j] = s;
      }
  };
  double T1[16], T2[16], Mc[16], M1[16], M2[16], I1[16];
  cay2hom(mt1, T1);
  cay2hom(mt2, T2);
  for (int i = 0; i < ncams; i++)
    for (int j = 0; j < ncams; j++) {
      cay2hom(mc + 6 * i, Mc);
      mat44(T1, Mc, M1);
      inv_mat(M1, I1);
      cay2hom(mc + 6 * j, Mc);
      mat44(T2, Mc, M2);
      double R1w[9], R2w[9], R2wt[9], nR1w[9], R12[9], A[9], t12[3], t1w[3], t2w[3];
      for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) {
          R1w[3 * r + c] = I1[4 * r + c];
          R2w[3 * r + c] = M2[4 * r + c];
        }
        t1w[r] = I1[4 * r + 3];
        t2w[r] = M2[4 * r + 3];
      }
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
          R2wt[3 * r + c] = R2w[3 * c + r];
          nR1w[3 * r + c] = -R1w[3 * r + c];
        }
      matmul(R1w, R2wt, R12, 3, 3, 3);
      matmul(nR1w, R2wt, A, 3, 3, 3);
      matmul(A, t2w, t12, 3, 3, 1);
      for (int r = 0; r < 3; r++) t12[r] += t1w[r];
      double ss = 0;
      for (int r = 0; r < 3; r++) ss += t12[r] * t12[r];
      const double ia = 1. / std::sqrt(ss);
      for (int r = 0; r < 3; r++) t12[r] *= ia;
      const double S[9] = {0.0, -t12[2], t12[1], t12[2], 0.0, -t12[0], -t12[1], t12[0], 0.0};
      matmul(S, R12, E + 9 * ((size_t)i * ncams + j), 3, 3, 3);
    }
  return 0;
}

int oracle_ba_edge(const double* pose, const double* X, const double* mc, const double* cam,
                   const double* meas, double* err, double* jp, double* jl) {
  edge_error(pose, X, mc, cam, meas, err);
  if (jp && jl) edge_jac(pose, X, mc, cam, jp, jl);
  return 0;
}

int oracle_ba_optimize_ex(const mcs_ba_problem* p, const mcs_ba_options* o, double* poses,
                          double* points, const uint8_t* edge_level, double* edge_chi2,
                          int32_t* stop_flag, mcs_ba_report* rep, int32_t points_fixed);
int oracle_ba_optimize(const mcs_ba_problem* p, const mcs_ba_options* o, double* poses,
                       double* points, const uint8_t* edge_level, double* edge_chi2,
                       int32_t* stop_flag, mcs_ba_report* rep) {
  return oracle_ba_optimize_ex(p, o, poses, points, edge_level, edge_chi2, stop_flag, rep, 0);
}

// the same with every point vertex fixed (BundleAdjustment(poseOnly) :178, PoseOptimization :382)
int oracle_ba_optimize_ex(const mcs_ba_problem* p, const mcs_ba_options* o, double* poses,
                          double* points, const uint8_t* edge_level, double* edge_chi2,
                          int32_t* stop_flag, mcs_ba_report* rep, int32_t points_fixed) {
  Graph g;
  g.P = p;
  g.points_fixed = points_fixed != 0;
  g.poses.assign(poses, poses + 6 * p->n_poses);
  g.points.assign(points, points + 3 * p->n_points);
  g.level.assign(p->n_edges, 0);
  if (edge_level) g.level.assign(edge_level, edge_level + p->n_edges);
  g.hk.delta = p->huber_delta;
  g.hk.dsqr = huber_dsqr(p->huber_delta);
  optimize(g, *o, stop_flag, rep);
  std::memcpy(poses, g.poses.data(), sizeof(double) * 6 * p->n_poses);
  std::memcpy(points, g.points.data(), sizeof(double) * 3 * p->n_points);
  if (edge_chi2) {
    // chi2 of every edge at the final estimate (culling reads e->chi2(), which holds the
    // last computed error; the terminate action recomputes errors after each iteration)
    std::vector<double> err(2);
    for (int e = 0; e < p->n_edges; e++) {
      edge_error(&g.poses[6 * p->edge_pose[e]], &g.points[3 * p->edge_point[e]], p->mc + 6 * p->edge_cam[e],
                 p->cam + 17 * p->edge_cam[e], p->edge_meas + 2 * e, err.data());
      edge_chi2[e] = p->edge_info[e] * (err[0] * err[0] + err[1] * err[1]);
    }
  }
  return 0;
}

// cOptimizer::BundleAdjustment (src/cOptimizer.cpp:73-261) after graph construction:
// optimize(15) with the terminate action; poseOnly fixes every point (:178)
int oracle_global_ba(const mcs_ba_problem* p, int32_t pose_only, double* poses, double* points,
                     int32_t* stop_flag, mcs_ba_report* rep) {
  mcs_ba_options o;
  o.max_iterations = 15; o.gain_threshold = 1e-6; o.terminate_max_iter = 15; o.max_trials = 10;
  o.tau = 1e-5;
  Graph g;
  g.P = p;
  g.poses.assign(poses, poses + 6 * p->n_poses);
  g.points.assign(points, points + 3 * p->n_points);
  g.level.assign(p->n_edges, 0);
  g.points_fixed = pose_only != 0;
  g.hk.delta = p->huber_delta;
  g.hk.dsqr = huber_dsqr(p->huber_delta);
  optimize(g, o, stop_flag, rep);
  std::memcpy(poses, g.poses.data(), sizeof(double) * 6 * p->n_poses);
  std::memcpy(points, g.points.data(), sizeof(double) * 3 * p->n_points);
  return 0;
}

// One rank's share of the reduced camera system at the given estimate:
// S_r = Hpp_r + lam_diag I - sum_{own points} Hpl Hll(lam)^-1 Hpl^T (n x n row-major, full)
// and bs_r; pose_cnt = active-edge count per pose over all shards (nullable = this problem).
// Summing S_r / bs_r over the shards (lam_diag = lam on one rank, 0 elsewhere) gives the
// unsharded system.  Returns n = 6 * (active poses).
int oracle_ba_partial_schur(const mcs_ba_problem* p, const double* pose_cnt, double lam,
                            double lam_diag, double* S_out, int32_t s_cap, double* bs_out) {
  Graph g;
  g.P = p;
  g.poses.assign(p->poses, p->poses + 6 * p->n_poses);
  g.points.assign(p->points, p->points + 3 * p->n_points);
  g.level.assign(p->n_edges, 0);
  g.pose_cnt = pose_cnt;
  g.hk.delta = p->huber_delta;
  g.hk.dsqr = huber_dsqr(p->huber_delta);
  g.initialize();
  g.err.assign(2 * p->n_edges, 0.0);
  g.compute_errors();
  g.build_system();
  std::vector<double> S, bs;
  g.schur(lam, lam_diag, S, bs);
  const int n = 6 * g.np;
  if (n > s_cap) return -1;
  std::memcpy(S_out, S.data(), sizeof(double) * (size_t)n * n);
  std::memcpy(bs_out, bs.data(), sizeof(double) * n);
  return n;
}

// cOptimizer::LocalBundleAdjustment (src/cOptimizer.cpp:771-903) after graph construction,
// with cMapPoint's bookkeeping: EraseObservation (src/cMapPoint.cpp:120-152) turns a point
// bad below 2 observations (extra_obs = observations from bad keyframes, which have no
// edge), the culling loops skip bad points (:805-806, :836-837), the write-back needs a good
// point with TotalNrObservations() > 1 (:166-178, :885-887) and >= 2 vertex edges (:895).
int oracle_local_ba_ex(const mcs_ba_problem* p, const int32_t* extra_obs, double* poses,
                       double* points, uint8_t* edge_inlier, uint8_t* point_write,
                       int32_t* write_back, int32_t* stop_flag, mcs_ba_report* r1,
                       mcs_ba_report* r2) {
  mcs_ba_options o;
  o.max_iterations = 10; o.gain_threshold = 1e-6; o.terminate_max_iter = 15; o.max_trials = 10;
  o.tau = 1e-5;
  const double huberK2 = p->huber_delta * p->huber_delta;
  std::vector<uint8_t> level(p->n_edges, 0);
  std::vector<double> chi(p->n_edges);
  // per map point: its observation lists as the reference keeps them
  struct MP { int good_obs; int bad_kf_obs; bool bad; int vertex_edges; };
  std::vector<MP> mp(p->n_points);
  for (int i = 0; i < p->n_points; i++) mp[i] = MP{0, extra_obs ? extra_obs[i] : 0, false, 0};
  for (int e = 0; e < p->n_edges; e++) { mp[p->edge_point[e]].good_obs++; mp[p->edge_point[e]].vertex_edges++; }
  auto erase_observation = [&](int i) {          // cMapPoint::EraseObservation
    MP& m = mp[i];
    m.good_obs--;
    const int nrObs = m.good_obs + m.bad_kf_obs;
    if (nrObs < 2) m.bad = true;                   // SetBadFlag (observations cleared)
  };
  // pbStopFlag == NULL: g2o installs the terminate action's auxiliary flag as the force-stop
  // flag the first time the action stops (sparse_optimizer_terminate_action.cpp:64-72) and
  // nothing resets it, so it is shared by both rounds
  int32_t aux = 0;
  int32_t* sf = stop_flag ? stop_flag : &aux;
  mcs_ba_report t1{}, t2{};
  if (!r1) r1 = &t1;
  if (!r2) r2 = &t2;
  *write_back = 0;
  if (point_write) std::memset(point_write, 0, (size_t)p->n_points);
  std::vector<char> vpEdges(p->n_edges, 1);      // NULL once an observation is erased
  for (int e = 0; e < p->n_edges; e++) edge_inlier[e] = 1;
  if (stop_flag && *stop_flag) return 0;
  oracle_ba_optimize(p, &o, poses, points, level.data(), chi.data(), sf, r1);
  // optimize() == -1 == OptimizationAlgorithm::Fail: empty active graph (:784-788)
  if (r1->n_active_poses + r1->n_active_points == 0) return 0;
  if (stop_flag && *stop_flag) return 0;   // bDoMore = false: no culling, no write-back
  for (int e = 0; e < p->n_edges; e++) {          // :798-817
    if (mp[p->edge_point[e]].bad) continue;
    if (chi[e] > huberK2) {
      erase_observation(p->edge_point[e]);
      level[e] = 1;
      vpEdges[e] = 0;
      edge_inlier[e] = 0;
    }
  }
  o.max_iterations = 15;
  oracle_ba_optimize(p, &o, poses, points, level.data(), chi.data(), sf, r2);
  if (r2->n_active_poses + r2->n_active_points == 0) return 0;   // :822-826
  for (int e = 0; e < p->n_edges; e++) {          // :830-849
    if (!vpEdges[e]) continue;
    if (mp[p->edge_point[e]].bad) continue;
    if (chi[e] > huberK2) {
      erase_observation(p->edge_point[e]);
      vpEdges[e] = 0;
      edge_inlier[e] = 0;
    }
  }
  *write_back = 1;
  if (point_write)                                 // :874-902
    for (int i = 0; i < p->n_points; i++)
      point_write[i] = !mp[i].bad && mp[i].good_obs > 1 && mp[i].vertex_edges >= 2;
  return 0;
}

int oracle_local_ba(const mcs_ba_problem* p, double* poses, double* points, uint8_t* edge_inlier,
                    int32_t* write_back, int32_t* stop_flag, mcs_ba_report* r1, mcs_ba_report* r2) {
  return oracle_local_ba_ex(p, nullptr, poses, points, edge_inlier, nullptr, write_back, stop_flag,
                            r1, r2);
}

// Local keyframe / point / fixed keyframe selection and edge list of LocalBundleAdjustment
// (src/cOptimizer.cpp:503-769), restated with the reference's containers and marks
// (std::list, mnBALocalForKF / mnBAFixedForKF) over index arrays.  Same outputs as
// mcs_local_ba_select (include/mcs_ba.h).  Returns 0, 1 (<= 1 local keyframe) or -2.
int oracle_local_ba_select(const mcs_lba_map* m, int32_t cur, const int32_t* covis, int32_t n_covis,
                           mcs_lba_graph* g) {
  const long long pKF_id = m->kf_id[cur] + 1000000007LL;   // a mark value no keyframe holds yet
  std::vector<long long> mnBALocalForKF(m->n_kf, -1), mnBAFixedForKF(m->n_kf, -1);
  std::vector<long long> mpLocal(m->n_points, -1);
  std::list<int> lLocalKeyFrames;
  lLocalKeyFrames.push_back(cur);
  mnBALocalForKF[cur] = pKF_id;
  for (int i = 0; i < n_covis; i++) {
    const int k = covis[i];
    mnBALocalForKF[k] = pKF_id;
    if (!m->kf_bad[k]) lLocalKeyFrames.push_back(k);
  }
  g->n_local = g->n_fixed = g->n_points = g->n_edges = 0;
  for (int k : lLocalKeyFrames) g->local_kf[g->n_local++] = k;
  if (lLocalKeyFrames.size() <= 1) return 1;
  std::list<int> lLocalMapPoints;
  for (int k : lLocalKeyFrames)
    for (int q = m->kf_mp_off[k]; q < m->kf_mp_off[k + 1]; q++) {
      const int pMP = m->kf_mp[q];
      if (pMP >= 0)
        if (!m->pt_bad[pMP])
          if (mpLocal[pMP] != pKF_id) { lLocalMapPoints.push_back(pMP); mpLocal[pMP] = pKF_id; }
    }
  std::list<int> lFixedCameras;
  for (int pMP : lLocalMapPoints)
    for (int o = m->pt_obs_off[pMP]; o < m->pt_obs_off[pMP + 1]; o++) {
      const int k = m->obs_kf[o];
      if (mnBALocalForKF[k] != pKF_id && mnBAFixedForKF[k] != pKF_id) {
        mnBAFixedForKF[k] = pKF_id;
        if (!m->kf_bad[k]) lFixedCameras.push_back(k);
      }
    }
  std::map<int, int> vertex;   // keyframe -> pose slot (g2o vertex of id mnId)
  bool oneFixed = false;
  int slot = 0;
  for (int k : lLocalKeyFrames) {
    oneFixed = m->kf_id[k] == 0;
    g->pose_fixed[slot] = oneFixed;
    vertex[k] = slot++;
  }
  if (!oneFixed && lFixedCameras.size() == 0) g->pose_fixed[vertex[*lLocalKeyFrames.begin()]] = 1;
  for (int k : lFixedCameras) {
    g->fixed_kf[g->n_fixed++] = k;
    g->pose_fixed[slot] = 1;
    vertex[k] = slot++;
  }
  int ne = 0, ip = 0;
  for (int pMP : lLocalMapPoints) {
    if (m->pt_bad[pMP]) continue;
    g->points[g->n_points] = pMP;
    int extra = 0;
    for (int o = m->pt_obs_off[pMP]; o < m->pt_obs_off[pMP + 1]; o++) {
      const int k = m->obs_kf[o];
      if (m->kf_bad[k]) { extra++; continue; }
      if (ne < g->edge_cap) { g->edge_obs[ne] = o; g->edge_pose[ne] = vertex[k]; g->edge_point[ne] = ip; }
      ne++;
    }
    g->point_extra_obs[g->n_points++] = extra;
    ip++;
  }
  g->n_edges = ne;
  return ne > g->edge_cap ? -2 : 0;
}

// cOptimizer::PoseOptimization (src/cOptimizer.cpp:264-486) after graph construction: one pose
// vertex (p->n_poses == 1, optimised), every map point fixed (:382), Huber delta =
// p->huber_delta (1.345 * huberMultiplier, :344), information invSigma2(octave) (:405-406).
// optimize(10); chi2 > delta^2 -> outlier, edge level 1; optimize(10); classify the remaining
// edges (:432-474).  No force-stop flag is set, so the terminate action's auxiliary flag
// carries over from round 1 to round 2.  Returns nInitialCorrespondences - nBad;
// *bad_ratio = nBad / nInitialCorrespondences (the reference's `inliers` output).
int oracle_pose_optimization(const mcs_ba_problem* p, double* pose, uint8_t* outlier,
                             double* bad_ratio, mcs_ba_report* r1, mcs_ba_report* r2) {
  mcs_ba_options o;
  o.max_iterations = 10; o.gain_threshold = 1e-6; o.terminate_max_iter = 15; o.max_trials = 10;
  o.tau = 1e-5;
  const double th2 = p->huber_delta * p->huber_delta;
  const int N = p->n_edges;
  std::vector<uint8_t> level(N, 0);
  const uint8_t not_fixed = 0;
  mcs_ba_problem q = *p;
  q.pose_fixed = &not_fixed;
  int32_t aux = 0;
  auto round = [&](mcs_ba_report* rep) {
    Graph g;
    g.P = &q;
    g.poses.assign(pose, pose + 6);
    g.points.assign(p->points, p->points + 3 * p->n_points);
    g.level = level;
    g.points_fixed = true;
    g.hk.delta = p->huber_delta;
    g.hk.dsqr = huber_dsqr(p->huber_delta);
    optimize(g, o, &aux, rep);
    std::memcpy(pose, g.poses.data(), sizeof(double) * 6);
    std::vector<double> chi(N);
    double err[2];
    for (int e = 0; e < N; e++) {
      edge_error(pose, &g.points[3 * p->edge_point[e]], p->mc + 6 * p->edge_cam[e],
                 p->cam + 17 * p->edge_cam[e], p->edge_meas + 2 * e, err);
      chi[e] = p->edge_info[e] * (err[0] * err[0] + err[1] * err[1]);
    }
    return chi;
  };
  int nBad = 0;
  std::vector<double> chi = round(r1);
  for (int e = 0; e < N; e++) {
    if (chi[e] > th2) { outlier[e] = 1; level[e] = 1; nBad++; }
    else outlier[e] = 0;
  }
  chi = round(r2);
  for (int e = 0; e < N; e++) {
    if (level[e]) continue;
    if (chi[e] > th2) { outlier[e] = 1; nBad++; }
    else outlier[e] = 0;
  }
  if (bad_ratio) *bad_ratio = N > 0 ? (double)nBad / N : 0.0;
  return N - nBad;
}

// cMultiFrame::isInFrustum (src/cMultiFrame.cpp:218-270) for every (point, camera): the
// reference's 4x4 path (WorldToCamHom_fast, src/cam_system_omni.cpp:92-112), mirror-mask test
// (src/cam_model_omni.cpp:165-180), distance invariance 0.8 / 1.2 (src/cMapPoint.cpp:498-508),
// viewCos, lower_bound scale level.  Arrays as mcs_is_in_frustum_device (host memory).
int oracle_is_in_frustum(const double* pose, const double* mc, const double* camv, int32_t C,
                         const uint8_t* masks, int32_t mw, int32_t mh, const double* pts,
                         const double* nrm, const double* dist, int32_t n, const double* scale,
                         int32_t L, uint8_t* in_view, double* proj, int32_t* level,
                         double* view_cos) {
  for (int p = 0; p < n; p++)
    for (int c = 0; c < C; c++) {
      const long q = (long)p * C + c;
      in_view[q] = 0;
      double Mt[16], Mc[16], M[16], Mi[16];
      cay2hom(pose, Mt);
      cay2hom(mc + 6 * c, Mc);
      mat44(Mt, Mc, M);
      inv_mat(M, Mi);
      const double* P = pts + 3 * p;
      const double pt4[4] = {P[0], P[1], P[2], 1.0};
      double r[4];
      for (int i = 0; i < 4; i++) {
        double s = 0;
        for (int k = 0; k < 4; k++) s += Mi[4 * i + k] * pt4[k];
        r[i] = s;
      }
      double u = 0.0, v = 0.0;
      world_to_img(camv + 17 * c, r[0], r[1], r[2], u, v);
      const int ur = (int)std::lrint(u), vr = (int)std::lrint(v);   // cvRound
      if (ur >= mw || ur <= 0 || vr >= mh || vr <= 0) continue;
      if (!(masks[(long)c * mw * mh + (long)vr * mw + ur] > 0)) continue;
      const double maxDistance = 1.2 * dist[2 * p + 1];
      const double minDistance = 0.8 * dist[2 * p];
      const double PO[3] = {P[0] - M[3], P[1] - M[7], P[2] - M[11]};
      double ss = 0;
      for (int k = 0; k < 3; k++) ss += PO[k] * PO[k];
      const double d = std::sqrt(ss);                                  // cv::norm
      if (d < minDistance || d > maxDistance) continue;
      const double* Pn = nrm + 3 * p;
      double dot = 0;
      for (int k = 0; k < 3; k++) dot += PO[k] * Pn[k];
      const double viewCos = dot / d;
      const double ratio = d / minDistance;
      int lv = (int)(std::lower_bound(scale, scale + L, ratio) - scale);
      if (lv >= L) lv = L - 1;
      in_view[q] = 1;
      proj[2 * q] = u;
      proj[2 * q + 1] = v;
      level[q] = lv;
      view_cos[q] = viewCos;
    }
  return 0;
}

}  // extern "C"
