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
#include "ldlt.hpp"
#include "ba_structure.hpp"
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <new>
#include <thread>
#include <vector>
#include <string.h>
#include <rocprim/rocprim.hpp>

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

// RobustKernelHuber keeps delta^2 in a FLOAT member (ThirdParty/g2o/g2o/core/robust_kernel_impl.h:84,
// `float dsqr;`, set by setDelta as dsqr = delta*delta, robust_kernel_impl.cpp:65-69), so the
// inlier test and rho(e) = 2 sqrt(e) delta - dsqr use delta^2 rounded to float.  (The culling
// thresholds of cOptimizer, thHuber2 = thHuber*thHuber, stay double: src/cOptimizer.cpp:436.)
static inline double huber_dsqr(double delta) { return (double)(float)(delta * delta); }

__device__ __forceinline__ void huber(double e, double delta, double dsqr, double* rho0, double* rho1) {
  if (e <= dsqr) { *rho0 = e; *rho1 = 1.; }
  else { const double sq = sqrt(e); *rho0 = 2 * sq * delta - dsqr; *rho1 = delta / sq; }
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// Device-side Levenberg-Marquardt control (Optimizer::run_device): the accept / reject
// decision, the lambda schedule, Raul's nBad stop and the terminate action of g2o run in
// k_edges_end after every trial, so the host enqueues trial after trial without reading anything
// back.  Kernels of a step that is no longer needed (done) return at once; the linearisation
// of a step runs only when the previous trial ended an iteration (lin).
constexpr int kLmTraceCap = 64;
struct LmCtl {
  double lambda, currentChi, iniChi, lastChi, tau, gain_threshold;
  double chi0, lambda_final;
  int ni, qmax, nBad, it, iter;
  int done, lin, restore, stop_out, ext_stop;
  int dev_err;       // a solve's hand-off wait timed out (ldlt::kFlagTimeout): the run is aborted
  int spec_lin;      // k_edges_end linearises every trial into the other Jacobian buffer
  int jbuf;          // the linearisation buffer of the current iteration (0 / 1)
  int max_iterations, max_trials, terminate_max_iter;
  unsigned arrive;   // k_edges_end's arrival counter (0 between launches)
  double trace[kLmTraceCap];
};
// host-coherent progress word of run_device (written by k_edges_end after every step)
struct LmSig { uint64_t seq; int32_t done, iter; int32_t ext_stop, pad_; };

struct Dev {
  LmCtl* ctl;   // device-driven LM (null: host-driven, lambda by value below)
  // device-driven trial sums: per-workgroup partials of the robust chi2 (k_edges), of the
  // points' and the poses' model decrease (k_update); null = the per-element arrays only
  double* part_chi; double* part_pt; double* part_ps;
  // problem
  const double* mc; const double* cam;
  const int32_t* e_pose; const int32_t* e_point; const int32_t* e_cam;
  const double* e_meas; const double* e_info;
  double delta, dsqr;
  // state
  double* poses; double* points; const double* poses_bk; const double* points_bk;
  // active structure
  const int32_t* aedge; int nae;
  const uint8_t* elevel;   // per edge: 1 = level 1 (LocalBA round 2 keeps round 1's list), null = none
  const int32_t* pose_h; const int32_t* point_h;      // hessian index per vertex (-1 inactive)
  const int32_t* hpose_vtx; const int32_t* hpt_vtx;   // vertex id per hessian index
  int np, nl;
  const int32_t* pt_ptr; const int32_t* pt_edges;     // CSR active points -> active edges
  const int32_t* pt_h;                                // pose Hessian index per pt_edges entry
  const int32_t* ps_ptr; const int32_t* ps_edges;     // CSR active poses  -> active edges
  const int32_t* blk_i; const int32_t* blk_j;         // lower pose blocks (i >= j)
  const int32_t* it_blk; const int32_t* it_chunk; const int32_t* it_slot;  // k_schur items
  const int32_t* blk_nch; const int32_t* blk_slot0;  // chunks / first partial slot per block
  double* schur_part;                                 // [slots][42]
  uint32_t* blk_arrive;                               // per block: chunks arrived (fused fin; null: k_schur_fin)
  double lam, lam0;                                   // lambda; lambda on rank 0, 0 elsewhere
  const int32_t* pr_ptr; const uint2* pr;             // edge pairs (e1, e2) per block
  const int32_t* nitem;                               // k_schur items (device-built count)
  int npe;                                            // entries of pt_edges
  // per-edge buffers (indexed by edge id)
  double* err; double* w; double* jp; double* jl; double* hpl; double* y; double* chi; double* rchi;
  // the second linearisation buffer of a device-driven run (null: one buffer): k_edges_end
  // linearises each trial there, and an accepted trial makes it the iteration's (ctl->jbuf)
  double* alt_err; double* alt_w; double* alt_jp; double* alt_jl; double* alt_hpl;
  // system
  double* Hpp; double* bp; double* Hll; double* bl; double* Dinv; double* db;
  double* S; double* bs; double* xp;   // S: lower 64x64 tiles (ldlt.hpp), bs / xp: 64 T
  int T;                               // tiles per side of S
  double* hdiag; double* bpf;          // [6 np] Hpp diagonal and b_p (all-reduced when sharded)
  double* red;                         // reduction scratch
  // trial bookkeeping folded into k_point_trial (each was a 4-5 us copy / fill launch)
  double* push_poses; double* push_points;  // backups (== poses_bk / points_bk)
  int n_pose_dbl, n_point_dbl;              // 6 n_poses, 3 n_points
  int* flag;                                // solve failure flag
};

// deterministic sum over a 256-thread workgroup: xor butterfly per wave, then the 4 wave sums
// in wave order (every thread calls; the result is valid in every thread)
__device__ __forceinline__ double block_sum256(double v) {
  __shared__ double sm[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();   // sm may still be read by a previous call
  if (lane == 0) sm[w] = v;
  __syncthreads();
  return ((sm[0] + sm[1]) + sm[2]) + sm[3];
}

__device__ __forceinline__ double lam_of(const Dev& d) { return d.ctl ? d.ctl->lambda : d.lam; }
// the linearisation buffer a kernel of a device-driven step reads (spec: the one a trial
// linearises into); host-driven runs have one buffer
__device__ __forceinline__ Dev lin_buf(const Dev& d, bool spec) {
  Dev r = d;
  if (d.ctl && d.alt_err && ((d.ctl->jbuf ^ (spec ? 1 : 0)) & 1)) {
    r.err = d.alt_err; r.w = d.alt_w; r.jp = d.alt_jp; r.jl = d.alt_jl; r.hpl = d.alt_hpl;
  }
  return r;
}
__device__ __forceinline__ double lam0_of(const Dev& d) { return d.ctl ? d.ctl->lambda : d.lam0; }
// a kernel of a device-driven step that is not needed (the loop has ended)
__device__ __forceinline__ bool lm_done(const Dev& d) { return d.ctl && d.ctl->done; }

constexpr int kRedNT = 256;   // reduction workgroup (k_edges_end's LM tail, k_update partials)
#ifndef MCS_BUILD_NT
#define MCS_BUILD_NT 256
#endif
// k_build / k_build_trial workgroup (1024 measured slower: 18.3 vs 12.9 us at config C)
constexpr int kBuildNT = MCS_BUILD_NT;

// per active edge: error (+ robust chi2) and optionally Jacobians / weight / Hpl = w Jp^T Jl
// (device-driven linearisation: only when the previous trial ended an iteration)
__global__ __launch_bounds__(256) void k_edges(Dev d0, int linearize) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (lm_done(d0) || (linearize && d0.ctl && !d0.ctl->lin)) return;
  const Dev d = lin_buf(d0, false);
  if (!linearize && d.part_chi) {   // trial chi2 of a device-driven step: + workgroup partial
    double r0 = 0.0;
    const int e = k < d.nae ? (d.aedge ? d.aedge[k] : k) : 0;
    if (k < d.nae && d.elevel && d.elevel[e]) {
      d.rchi[k] = 0.0;   // level 1: outside the graph
    } else if (k < d.nae) {
      const int pi = d.e_pose[e], li = d.e_point[e], ci = d.e_cam[e];
      double er[2];
      edge_error(d.poses + 6 * pi, d.points + 3 * li, d.mc + 6 * ci, d.cam + 17 * ci, d.e_meas + 2 * e, er);
      const double c2 = d.e_info[e] * (er[0] * er[0] + er[1] * er[1]);
      double r1;
      huber(c2, d.delta, d.dsqr, &r0, &r1);
      d.err[2 * e] = er[0]; d.err[2 * e + 1] = er[1];
      d.chi[e] = c2;
      d.rchi[k] = r0;
    }
    const double sum = block_sum256(r0);
    if (threadIdx.x == 0) d.part_chi[blockIdx.x] = sum;
    return;
  }
  if (k >= d.nae) return;
  const int e = d.aedge ? d.aedge[k] : k;   // null: every edge
  if (d.elevel && d.elevel[e]) { d.rchi[k] = 0.0; return; }   // level 1: terms stay zero
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
    const double w = r1 * d.e_info[e];
    d.w[e] = w;
    if (d.hpl && d.pose_h[pi] >= 0 && d.point_h[li] >= 0) {
      for (int a = 0; a < 6; a++)
        for (int bb = 0; bb < 3; bb++)
          d.hpl[18 * e + 3 * a + bb] = w * (jp[a] * jl[bb] + jp[6 + a] * jl[3 + bb]);
    }
  }
}

// deterministic sum / max|.| of n doubles -> out[0], two stages with fixed orders:
// k_reduce_part: workgroup g owns the contiguous chunk [g*chunk, (g+1)*chunk), each thread
// 8 strided accumulators (loads in flight, short add chains), a fixed tree over the block;
// k_reduce: one workgroup over the partials.  Small inputs skip the first stage.
constexpr int kRedPartMax = 256;
template <bool MAX>
__global__ __launch_bounds__(256) void k_reduce_part(const double* __restrict__ v, int n, int chunk,
                                                     double* __restrict__ part) {
  __shared__ double s[256];
  const int g = blockIdx.x, t = threadIdx.x;
  const int b0 = g * chunk, b1 = min(n, b0 + chunk);
  double acc[8];
#pragma unroll
  for (int u = 0; u < 8; u++) acc[u] = 0.0;
  for (int i = b0 + t; i < b1; i += 8 * 256) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int q = i + u * 256;
      if (q < b1) acc[u] = MAX ? fmax(acc[u], fabs(v[q])) : acc[u] + v[q];
    }
  }
  double a = acc[0];
#pragma unroll
  for (int u = 1; u < 8; u++) a = MAX ? fmax(a, acc[u]) : a + acc[u];
  s[t] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) s[t] = MAX ? fmax(s[t], s[t + o]) : s[t] + s[t + o];
    __syncthreads();
  }
  if (t == 0) part[g] = s[0];
}

template <bool MAX>
__global__ __launch_bounds__(1024) void k_reduce(const double* __restrict__ v, int n, double* out) {
  __shared__ double s[1024];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) acc = MAX ? fmax(acc, fabs(v[i])) : acc + v[i];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) s[threadIdx.x] = MAX ? fmax(s[threadIdx.x], s[threadIdx.x + o]) : s[threadIdx.x] + s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = s[0];
}

// The closing sums of an LM trial (robust chi2, point and pose step norms), one workgroup
// each, in exactly k_reduce<false>'s order (1024-strided partials, then the LDS tree); every
// sum goes straight to host-coherent memory with its own released sequence number (the solve
// flag with the first), so the host sees the trial's outcome without a readback copy or a
// stream synchronisation.
struct Sum3 { const double* v[3]; int n[3]; };
struct TrialSig { double v[3]; int32_t flag, pad; uint64_t seq[3]; };
__global__ __launch_bounds__(1024) void k_reduce3(Sum3 q, const int* flag, TrialSig* sig, uint64_t seq) {
  __shared__ double s[1024];
  const int t = threadIdx.x, b = blockIdx.x;
  const double* v = q.v[b];
  const int n = q.n[b];
  double acc = 0.0;
  for (int i = t; i < n; i += 1024) acc = acc + v[i];
  s[t] = acc;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (t < o) s[t] = s[t] + s[t + o];
    __syncthreads();
  }
  if (t == 0) {
    sig->v[b] = s[0];
    if (b == 0) sig->flag = *flag;
    __hip_atomic_store(&sig->seq[b], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- device-driven Levenberg-Marquardt control (one thread) ------------------------------
// x^3 rounded once (double-double product), the value std::pow(x, 3) returns: host and device
// (and every rank) take the identical lambda step
__host__ __device__ inline double cube_rn(double x) {
  const double p = x * x;
  const double pe = __builtin_fma(x, x, -p);       // x^2 = p + pe exactly
  const double h = p * x;
  // overflow: pow(x, 3) returns +-inf (the error terms would turn it into NaN, and the LM's
  // alpha = 1 - pow(2 rho - 1, 3) must become -inf so that lambda *= 1/3; g2o_solver.npz
  // scenario 27 has such a step)
  if (!__builtin_isfinite(h)) return h;
  const double he = __builtin_fma(p, x, -h);       // p x = h + he exactly
  return h + (he + pe * x);
}

// The end of a device-driven step, run by the last-arriving workgroup of k_edges_end: the
// trial's three sums from the workgroup partials (each summed exactly as k_reduce3's 1024-thread
// workgroups do: 1024 strided slots, then the LDS tree -- emulated here by kRedNT threads, so
// the bits are the same), the LM control (lm_control) and the pop of a rejected trial.
__device__ void lm_control(LmCtl* c, const double* sc, int flag, LmSig* sig);
struct LmEnd { double* sc; const int* flag; LmSig* sig; uint64_t seq; LmCtl* host_ctl; };
#ifndef MCS_LM_AHEAD
#define MCS_LM_AHEAD 2      // LM steps the host keeps enqueued ahead of the device
#endif
#ifndef MCS_EXP_PUB_DONE
#define MCS_EXP_PUB_DONE 0  // experiment builds: publish progress only once the run is done
#endif
__device__ __forceinline__ void lm_publish(const LmCtl* c, const LmEnd& le) {
  if (MCS_EXP_PUB_DONE && !c->done) return;
  // relaxed: a stale `done` only costs the host one more (no-op) step
  __hip_atomic_store(&le.sig->done, c->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&le.sig->iter, c->iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&le.sig->seq, le.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// (blockDim >= 256: threads past 256 only take part in the barriers)
__device__ void lm_end_body(const Dev& d, const Sum3& q, const LmEnd& le) {
  static_assert(kRedNT == 256, "the tree below folds 1024 slots onto 256 threads");
  __shared__ double s[3][256];
  __shared__ int rej;
  LmCtl* c = d.ctl;
  const int t = threadIdx.x;
  const bool act = t < 256;
  // slot ts = t + 256 u (u = 0..3) sums v[ts], v[ts + 1024], ... in order; the tree levels 512
  // and 256 (s[ts] += s[ts + o]) pair slots of one thread, so they run in registers; 128 and 64
  // cross waves (LDS); 32 .. 1 stay in wave 0 (shuffles).  Same additions in the same order.
  double a[3];
  if (act) {
#pragma unroll
    for (int b = 0; b < 3; b++) {
      const double* v = q.v[b];
      double x[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        double acc = 0.0;
        // sc1 loads: k_edges_end's partials arrive write-through, without an acquire
        for (int i = t + 256 * u; i < q.n[b]; i += 1024)
          acc = acc + __longlong_as_double((long long)__hip_atomic_load(
                          (const __attribute__((address_space(1))) unsigned long long*)(v + i), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT));
        x[u] = acc;
      }
      x[0] = x[0] + x[2];   // o = 512
      x[1] = x[1] + x[3];
      a[b] = x[0] + x[1];   // o = 256
      s[b][t] = a[b];
    }
  }
  __syncthreads();
  if (t < 128)
    for (int b = 0; b < 3; b++) a[b] = s[b][t] + s[b][t + 128];   // o = 128
  __syncthreads();
  if (t < 128)
    for (int b = 0; b < 3; b++) s[b][t] = a[b];
  __syncthreads();
  if (t < 64) {
    for (int b = 0; b < 3; b++) {
      double w = s[b][t] + s[b][t + 64];                           // o = 64
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) w = w + __shfl_down(w, o, 64);
      if (t == 0) le.sc[b] = w;
    }
  }
  if (t == 0) {
    lm_control(c, le.sc, *le.flag, le.sig);
    rej = c->restore;
  }
  __syncthreads();
  if (rej && act) {   // pop: every pose and point back to the backups of the trial's push
    for (int i = t; i < d.n_pose_dbl; i += kRedNT) d.poses[i] = d.push_poses[i];
    for (int i = t; i < d.n_point_dbl; i += kRedNT) d.points[i] = d.push_points[i];
  }
  // the run's last step: the control block straight into host memory (the report), read by
  // the host once the stream has drained -- no readback copy
  if (le.host_ctl && c->done && act) {
    constexpr int nw = (int)(sizeof(LmCtl) / 4);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(c);
    uint32_t* dst = reinterpret_cast<uint32_t*>(le.host_ctl);
    for (int i = t; i < nw; i += kRedNT) dst[i] = src[i];
  }
  if (t == 0) lm_publish(c, le);
}

// The trial's evaluation (k_edges without linearisation: error, robust chi2, workgroup partial)
// and the end of the step in one launch: each workgroup releases its partial and counts itself
// in; the last one (device-scope counter, agent-scope acquire) closes the step.  A step past
// the end still publishes its sequence number (workgroup 0), as the host waits for each.
// A workgroup holds 256 edges and 512 threads: waves 0-3 evaluate the error / robust chi2 / weight
// of edge k (slot t), waves 4-7 its Jacobians (speculative linearisation), the two independent
// halves of one edge's dependent chain side by side; Hpl = w Jp^T Jl follows once the weight
// has crossed over in LDS.  Every value is the single-thread form's, bit for bit.
constexpr int kEdgeEndNT = 512;
__global__ __launch_bounds__(kEdgeEndNT) void k_edges_end(Dev d0, Sum3 q, LmEnd le) {
  __shared__ int last;
  __shared__ double wsh[256];
  __shared__ double sm[4];
  LmCtl* c = d0.ctl;
  if (c->done) {
    if (blockIdx.x == 0 && threadIdx.x == 0) lm_publish(c, le);
    return;
  }
  // with speculative linearisation the trial's error, Jacobians, weight and Hpl go to the
  // other buffer: if lm_control accepts the trial they are the next iteration's linearisation
  // (k_edges at the accepted state, the same arithmetic), and no linearising launch is needed
  const bool spec = c->spec_lin != 0;
  const Dev d = lin_buf(d0, spec);
  const int slot = threadIdx.x & 255;
  const bool jac = threadIdx.x >= 256;   // wave-uniform
  const int k = blockIdx.x * 256 + slot;
  double r0 = 0.0;
  int e = 0, pi = 0, li = 0, ci = 0;
  double jp[12], jl[6];
  bool live = k < d.nae;
  if (live) {
    e = d.aedge ? d.aedge[k] : k;
    if (d.elevel && d.elevel[e]) {   // level 1: outside the graph, terms stay zero
      live = false;
      if (!jac) d.rchi[k] = 0.0;
    }
  }
  if (live) {
    pi = d.e_pose[e]; li = d.e_point[e]; ci = d.e_cam[e];
    const double* pose = d.poses + 6 * pi;
    const double* X = d.points + 3 * li;
    if (!jac) {
      double er[2];
      edge_error(pose, X, d.mc + 6 * ci, d.cam + 17 * ci, d.e_meas + 2 * e, er);
      const double c2 = d.e_info[e] * (er[0] * er[0] + er[1] * er[1]);
      double r1;
      huber(c2, d.delta, d.dsqr, &r0, &r1);
      d.err[2 * e] = er[0]; d.err[2 * e + 1] = er[1];
      d.chi[e] = c2;
      d.rchi[k] = r0;
      if (spec) {
        const double w = r1 * d.e_info[e];
        d.w[e] = w;
        wsh[slot] = w;
      }
    } else if (spec) {
      edge_jac(pose, X, d.mc + 6 * ci, d.cam + 17 * ci, jp, jl);
      for (int i = 0; i < 12; i++) d.jp[12 * e + i] = jp[i];
      for (int i = 0; i < 6; i++) d.jl[6 * e + i] = jl[i];
    }
  }
  __syncthreads();
  if (jac && spec && live && d.hpl && d.pose_h[pi] >= 0 && d.point_h[li] >= 0) {
    const double w = wsh[slot];
    for (int a = 0; a < 6; a++)
      for (int bb = 0; bb < 3; bb++)
        d.hpl[18 * e + 3 * a + bb] = w * (jp[a] * jl[bb] + jp[6 + a] * jl[3 + bb]);
  }
  // block_sum256 over the error waves (0-3): the same butterfly and wave order
  {
    double v = r0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (!jac && (threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  }
  __syncthreads();
  // The partial goes write-through (sc1 store), its wait drains before the arrival add, and the
  // last workgroup reads every partial with sc1 loads (lm_end_body): the hand-off of
  // MI355X_MICROARCH.md's first table row, with no L2 write-back (a __threadfence per workgroup
  // wrote back the ~6 MB of Jacobians this kernel leaves dirty) and no acquire.
  if (threadIdx.x == 0) {
    __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)(d.part_chi + blockIdx.x),
                       (unsigned long long)__double_as_longlong(((sm[0] + sm[1]) + sm[2]) + sm[3]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(&c->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) __hip_atomic_store(&c->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next step
  lm_end_body(d0, q, le);
}

// chi2 of the starting point -> currentChi (the optimize() call's activeRobustChi2)
__device__ __forceinline__ void lm_start_body(LmCtl* c, double chi) {
  c->chi0 = chi;
  c->currentChi = chi;
  c->iniChi = chi;
}
__global__ void k_lm_start(LmCtl* c, const double* sc) {
  if (threadIdx.x != 0) return;
  lm_start_body(c, sc[0]);
}
// lambda of iteration 0: tau * max diagonal (computeLambdaInit,
// optimization_algorithm_levenberg.cpp:166-180); pt / pose = max |diagonal| of Hll / Hpp
__device__ __forceinline__ void lm_lambda0_body(LmCtl* c, double pt, double pose) {
  c->lambda = c->tau * fmax(pt, pose);
  c->ni = 2;
  c->nBad = 0;
}
// the LM control block of a run, by value (no pageable host copy on the stream)
// (+ the per-block chunk counters of k_schur's fused fin, zeroed)
__global__ void k_ctl_init(LmCtl h0, LmCtl* c, uint32_t* blk_arrive, int nblk) {
  constexpr int nw = (int)(sizeof(LmCtl) / 4);
  static_assert(sizeof(LmCtl) % 4 == 0, "word copy");
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&h0);
  uint32_t* dst = reinterpret_cast<uint32_t*>(c);
  for (int i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = src[i];
  if (blk_arrive)
    for (int i = threadIdx.x; i < nblk; i += blockDim.x) blk_arrive[i] = 0u;
}
__global__ void k_lm_lambda0(LmCtl* c, const double* sc) {
  if (threadIdx.x != 0 || c->done) return;
  lm_lambda0_body(c, sc[1], sc[2]);
}
// after a trial (k_edges_end's last workgroup, one thread): OptimizationAlgorithmLevenberg::solve's accept / reject
// (optimization_algorithm_levenberg.cpp:99-163) and, when the iteration ends, the terminate
// action (sparse_optimizer_terminate_action.cpp:43-72) -- the arithmetic of the host driver
// statement for statement.  sc = {robust chi2, points' model decrease, poses' model
// decrease}; flag = the solve failed (zero pivot).
__device__ void lm_control(LmCtl* c, const double* sc, int flag, LmSig* sig) {
  {
    const int stop = __hip_atomic_load(&sig->ext_stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    c->ext_stop = stop;
    if (flag & ldlt::kFlagTimeout) {   // x is garbage: no LM decision, the host reports MCS_ERR_HIP
      c->dev_err = 1;
      c->done = 1;
      c->restore = 1;                  // k_edges_end pops the trial's state
      return;
    }
    double tempChi = sc[0];
    if (flag & ldlt::kFlagZeroPivot) tempChi = 1.7976931348623157e308;
    double rho = c->currentChi - tempChi;
    double scale = sc[2] + sc[1];
    scale += 1e-3;
    rho /= scale;
    if (rho > 0 && isfinite(tempChi)) {
      double alpha = 1. - cube_rn(2 * rho - 1);
      alpha = fmin(alpha, 2. / 3.);
      c->lambda *= fmax(1. / 3., alpha);
      c->ni = 2;
      c->currentChi = tempChi;
      c->restore = 0;
      if (c->spec_lin) c->jbuf ^= 1;   // the trial's linearisation (k_edges_end) is current
    } else {
      c->lambda *= c->ni;
      c->ni *= 2;
      c->restore = 1;   // k_edges_end pops the state right after this decision
    }
    c->qmax++;
    if (rho < 0 && c->qmax < c->max_trials && !stop) {
      c->lin = 0;       // the next step retries the trial with the larger lambda
    } else {
      int result = 0;
      if (c->qmax == c->max_trials || rho == 0) result = 1;
      else {
        if ((c->iniChi - c->currentChi) * 1e3 < c->iniChi) c->nBad++;
        else c->nBad = 0;
        if (c->nBad >= 3) result = 1;
      }
      c->it++;
      const int i = c->iter;
      const double cur = c->currentChi;
      if (i < kLmTraceCap) c->trace[i] = cur;
      int stopOpt = 0;
      if (i == 0) c->lastChi = cur;
      else {
        if (i < c->terminate_max_iter) {
          const double gain = (c->lastChi - cur) / cur;
          c->lastChi = cur;
          if (gain >= 0 && gain < c->gain_threshold) stopOpt = 1;
        } else {
          stopOpt = 1;
        }
      }
      if (stopOpt) c->stop_out = 1;
      c->lambda_final = c->lambda;
      c->iter = i + 1;
      if (c->iter >= c->max_iterations || stop || stopOpt || result != 0) {
        c->done = 1;
      } else {
        c->lin = 1;
        c->qmax = 0;
        c->iniChi = c->currentChi;
      }
    }
  }
}

// Test hooks (mcs_ba_lm_replay, mcs_ba_huber_eval): the production device functions replayed on
// scripted inputs, so the LM control and the robust kernel can be checked statement for
// statement against the reference text (tests/golden/gen_g2o_solver.py).
// in = {chi0, maxdiag points, maxdiag poses}; trials [n][4] = {robust chi2 of the trial,
// points' model decrease, poses' model decrease, solve failed}; out [n][10] per trial =
// {lambda used, lambda after, ni, accepted, qmax, nBad, iterations done, done, stop_out,
// currentChi}.  One thread.
__global__ void k_lm_replay(LmCtl* c, LmSig* sig, const double* in, const double* trials, int n,
                            double* out, int* n_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  lm_start_body(c, in[0]);
  if (!c->done) lm_lambda0_body(c, in[1], in[2]);
  int t = 0;
  for (; t < n && !c->done; t++) {
    const double* tr = trials + 4 * t;
    const double sc[3] = {tr[0], tr[1], tr[2]};
    const double lam = c->lambda;
    lm_control(c, sc, tr[3] != 0.0 ? 1 : 0, sig);
    double* o = out + 10 * t;
    o[0] = lam; o[1] = c->lambda; o[2] = c->ni; o[3] = c->restore ? 0.0 : 1.0; o[4] = c->qmax;
    o[5] = c->nBad; o[6] = c->iter; o[7] = c->done; o[8] = c->stop_out; o[9] = c->currentChi;
  }
  *n_out = t;
}

__global__ void k_huber_eval(const double* e, int n, double delta, double dsqr, double* rho0, double* rho1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) huber(e[i], delta, dsqr, &rho0[i], &rho1[i]);
}

// launch helper: part = kRedPartMax doubles of scratch (stream-ordered reuse is safe)
template <bool MAX>
void reduce_dev(const double* v, int n, double* out, double* part, hipStream_t st) {
  if (n <= 32768) {
    hipLaunchKernelGGL(k_reduce<MAX>, dim3(1), dim3(1024), 0, st, v, n, out);
    return;
  }
  const int chunk = std::max(8 * 256, (n + kRedPartMax - 1) / kRedPartMax);
  const int g = (n + chunk - 1) / chunk;
  hipLaunchKernelGGL(k_reduce_part<MAX>, dim3(g), dim3(256), 0, st, v, n, chunk, part);
  hipLaunchKernelGGL(k_reduce<MAX>, dim3(1), dim3(1024), 0, st, (const double*)part, g, out);
}

// per active point: Hll (3x3), b_l over its edges in edge order; diag -> red (for lambda init)
// four lanes per point (edges q0 + sub, q0 + sub + 4, ...), the quad's partial sums combined
// in a fixed order ((l0 + l1) + (l2 + l3)): deterministic, and 4x the threads of one lane per
// point (config C: 3000 points would occupy 12 workgroups)
__device__ __forceinline__ double quad_sum(double v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  return v;
}
// D = Hll + lambda I -> Dinv = D.inverse() as the reference's Eigen 3.2.10 computes a fixed
// 3x3 inverse (ThirdParty/Eigen/Eigen/src/LU/Inverse.h:117-159): cofactor(i, j) =
// m(i1, j1) m(i2, j2) - m(i1, j2) m(i2, j1) with i1 = i+1, i2 = i+2, j1 = j+1, j2 = j+2 (mod 3);
// det = the column-0 cofactors times column 0, summed by redux_novec_unroller (Redux.h:77-106:
// a 3-vector of Matrix<double,3,1> is not packet-aligned in 3.2, so c0 + (c1 + c2)); row 0 of
// the inverse = the column-0 cofactors, entry (r, c) otherwise = cofactor(c, r), each times
// 1 / det.  Pinned by tests/golden/g2o_schur.npz.  (k_point_trial and k_build_trial share it.)
__host__ __device__ __forceinline__ void dinv_of(const double* H, double lam, double (&Di)[9]) {
  double m[9];
  for (int k = 0; k < 9; k++) m[k] = H[k];
  m[0] += lam; m[4] += lam; m[8] += lam;
  auto cof = [&](int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[3 * i1 + j1] * m[3 * i2 + j2] - m[3 * i1 + j2] * m[3 * i2 + j1];
  };
  const double k0 = cof(0, 0), k1 = cof(1, 0), k2 = cof(2, 0);
  const double det = k0 * m[0] + (k1 * m[3] + k2 * m[6]);
  const double id = 1.0 / det;
  Di[0] = k0 * id; Di[1] = k1 * id; Di[2] = k2 * id;
  Di[3] = cof(0, 1) * id; Di[4] = cof(1, 1) * id; Di[5] = cof(2, 1) * id;
  Di[6] = cof(0, 2) * id; Di[7] = cof(1, 2) * id; Di[8] = cof(2, 2) * id;
}
// db = Dinv * b_l (CoeffBasedProduct, CoeffBasedProduct.h:240-258: k ascending)
__host__ __device__ __forceinline__ void db_of(const double (&Di)[9], const double* b, double* db) {
  for (int a = 0; a < 3; a++) db[a] = Di[3 * a] * b[0] + Di[3 * a + 1] * b[1] + Di[3 * a + 2] * b[2];
}
// Y = Hpl * Dinv (BDinv = (*Bi) * Dinv, block_solver.hpp:403), same product order
__host__ __device__ __forceinline__ void ybl_of(const double* B, const double (&Di)[9], double* Y) {
  double bb[18];
  for (int k = 0; k < 18; k++) bb[k] = B[k];
  for (int a = 0; a < 6; a++)
    for (int c = 0; c < 3; c++)
      Y[3 * a + c] = bb[3 * a] * Di[c] + bb[3 * a + 1] * Di[3 + c] + bb[3 * a + 2] * Di[6 + c];
}
// Y_e = Hpl_e Dinv of one (point, edge) entry whose pose is active
__device__ __forceinline__ void y_of(const Dev& d, int e, const double (&Di)[9]) {
  ybl_of(d.hpl + 18 * e, Di, d.y + 18 * e);
}

// per landmark: Dinv, db and one edge's Y from the production helpers (mcs_ba_point_block_eval)
__global__ void k_point_block_eval(const double* H, double lam, const double* b, const double* hpl, int n,
                                   double* Dinv, double* db, double* Y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double Di[9];
  dinv_of(H + 9 * i, lam, Di);
  for (int k = 0; k < 9; k++) Dinv[9 * i + k] = Di[k];
  db_of(Di, b + 3 * i, db + 3 * i);
  ybl_of(hpl + 18 * i, Di, Y + 18 * i);
}


// TRIAL (k_build_trial): the same quad then carries k_point_trial's point part -- Dinv, db and
// the Y of the point's edges -- from the H and b it holds (LIN: just built; otherwise the
// iteration's stored Hll / b_l: a rejected trial re-solves the same linearisation)
template <bool TRIAL>
__device__ __forceinline__ void points_build_body(const Dev& d, int block, bool lin) {
  const int gt = block * kBuildNT + threadIdx.x;
  const int l = gt >> 2, sub = gt & 3;
  const bool act = l < d.nl;
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
  if (lin) {
    if (act) {
      auto term = [&](int e) {
        const double* jl = d.jl + 6 * e;
        const double w = d.w[e];
        const double we0 = -w * d.err[2 * e], we1 = -w * d.err[2 * e + 1];
        for (int a = 0; a < 3; a++) {
          for (int bb = 0; bb < 3; bb++) H[3 * a + bb] += w * (jl[a] * jl[bb] + jl[3 + a] * jl[3 + bb]);
          b[a] += jl[a] * we0 + jl[3 + a] * we1;
        }
      };
      // the quad lane's entries q and q + 4 with their index loads together, added in q order
      const int q1 = d.pt_ptr[l + 1];
      for (int q = d.pt_ptr[l] + sub; q < q1; q += 8) {
        const bool two = q + 4 < q1;
        const int ea = d.pt_edges[q], eb = d.pt_edges[two ? q + 4 : q];
        term(ea);
        if (two) term(eb);
      }
    }
#pragma unroll
    for (int i = 0; i < 9; i++) H[i] = quad_sum(H[i]);
#pragma unroll
    for (int i = 0; i < 3; i++) b[i] = quad_sum(b[i]);
    if (act && sub == 0) {
      for (int i = 0; i < 9; i++) d.Hll[9 * l + i] = H[i];
      for (int i = 0; i < 3; i++) d.bl[3 * l + i] = b[i];
      d.red[l] = fmax(fmax(fabs(H[0]), fabs(H[4])), fabs(H[8]));
    }
  } else if (TRIAL && act) {
    for (int i = 0; i < 9; i++) H[i] = d.Hll[9 * l + i];
    for (int i = 0; i < 3; i++) b[i] = d.bl[3 * l + i];
  }
  if (!TRIAL || !act) return;
  double Di[9];
  dinv_of(H, lam_of(d), Di);
  if (sub == 0) {
    for (int k = 0; k < 9; k++) d.Dinv[9 * l + k] = Di[k];
    db_of(Di, b, d.db + 3 * l);
  }
  for (int q = d.pt_ptr[l] + sub; q < d.pt_ptr[l + 1]; q += 4) {
    // pt_h[q] = pose_h[e_pose[pt_edges[q]]] (host-built): one load instead of a chain of three
    if (d.pt_h[q] >= 0) y_of(d, d.pt_edges[q], Di);
  }
}

// One level of a wave's recursive halving over N values (of NA slots): values [0, H) and
// [H, N) (zero-padded to H) split by lane bit O; the lane keeps one half in acc[0, H) and adds
// its partner's copy of that half.  Own + partner at every level is what a full xor butterfly
// forms for every value, bit for bit, with ~N exchanges instead of 6 N.
template <int NA, int N, int O>
__device__ __forceinline__ void wave_halve(double (&acc)[NA], int lane) {
  constexpr int H = (N + 1) / 2;
  const bool hi = (lane & O) != 0;
#pragma unroll
  for (int i = 0; i < H; i++) {
    const double a = acc[i], b = (H + i < N) ? acc[H + i] : 0.0;
    const double keep = hi ? b : a, give = hi ? a : b;
    acc[i] = keep + __shfl_xor(give, O);
  }
}
// the six levels (bits 32 .. 1) over N <= 64 values; returns the value whose wave sum the lane
// then holds in acc[0] (-1: a padding slot).  The split points are the static H of each level;
// a lane's real count shrinks to n - H on the high side, so some slots of the last levels are
// zero padding.
template <int N, int NA>
__device__ __forceinline__ int wave_halve_all(double (&acc)[NA], int lane) {
  static_assert(N <= 64 && N <= NA, "one value per lane at most");
  constexpr int N1 = (N + 1) / 2, N2 = (N1 + 1) / 2, N3 = (N2 + 1) / 2, N4 = (N3 + 1) / 2,
                N5 = (N4 + 1) / 2;
  wave_halve<NA, N, 32>(acc, lane);
  wave_halve<NA, N1, 16>(acc, lane);
  wave_halve<NA, N2, 8>(acc, lane);
  wave_halve<NA, N3, 4>(acc, lane);
  wave_halve<NA, N4, 2>(acc, lane);
  wave_halve<NA, N5, 1>(acc, lane);
  int idx = 0, n = N, nk = N;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const int h = (nk + 1) / 2;
    if (lane & (32 >> k)) { idx += h; n -= h; } else n = n < h ? n : h;
    nk = h;
  }
  return n > 0 ? idx : -1;
}

// Deterministic block sum of NV per-thread partials over a workgroup of NW waves: the fixed
// xor-butterfly's sums inside each wave, then the NW wave sums in wave order.  On return
// sm[v * NW] holds sum v (after the barrier).
template <int NV, int NW>
__device__ __forceinline__ void block_sum_vec(double (&acc)[NV], double* sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // the wave sums by recursive halving (the xor butterfly's sums, bit for bit); sum v ends in
  // one lane, which writes it
  const int mine = wave_halve_all<NV>(acc, lane);
  if (mine >= 0) sm[mine * NW + w] = acc[0];
  __syncthreads();
  if (threadIdx.x < NV) {
    const int v = threadIdx.x;
    double t = sm[v * NW];
#pragma unroll
    for (int k = 1; k < NW; k++) t += sm[v * NW + k];
    sm[v * NW] = t;
  }
  __syncthreads();
}

constexpr int kUpper6[21][2] = {{0, 0}, {0, 1}, {0, 2}, {0, 3}, {0, 4}, {0, 5}, {1, 1},
                                {1, 2}, {1, 3}, {1, 4}, {1, 5}, {2, 2}, {2, 3}, {2, 4},
                                {2, 5}, {3, 3}, {3, 4}, {3, 5}, {4, 4}, {4, 5}, {5, 5}};

// per active pose: Hpp (6x6, upper 21 mirrored), b_p; edges of the pose split over the
// workgroup's threads (fixed stride), block tree sum.  Also the diagonal and b_p into the
// exchange area.
__device__ __forceinline__ void poses_build_body(const Dev& d, int i) {
  __shared__ double sm[27 * (kBuildNT / 64)];
  const int t = threadIdx.x;
  double acc[27];
#pragma unroll
  for (int v = 0; v < 27; v++) acc[v] = 0.0;
  // a thread's edges t, t + 256, ... in that order; kU of them per pass with every load issued
  // before the first sum (the edge -> Jacobian gather is two dependent round trips, and a
  // pose has ~1500 edges at config C: one at a time the chain was the whole kernel).  Loads
  // past the list read the last edge (unconditional: no merge waits) and are not summed.
#ifndef MCS_BUILD_KU
#define MCS_BUILD_KU 4
#endif
  constexpr int kU = MCS_BUILD_KU;
  const int q0 = d.ps_ptr[i], q1 = d.ps_ptr[i + 1];
  for (int qb = q0 + t; qb < q1; qb += kU * kBuildNT) {
    int e[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) e[u] = d.ps_edges[min(qb + u * kBuildNT, q1 - 1)];
    double j0[kU][6], j1[kU][6], w[kU], er0[kU], er1[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const double* jp = d.jp + 12 * e[u];
#pragma unroll
      for (int a = 0; a < 6; a++) { j0[u][a] = jp[a]; j1[u][a] = jp[6 + a]; }
      w[u] = d.w[e[u]];
      er0[u] = d.err[2 * e[u]];
      er1[u] = d.err[2 * e[u] + 1];
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      if (qb + u * kBuildNT >= q1) break;
      const double we0 = -w[u] * er0[u], we1 = -w[u] * er1[u];
#pragma unroll
      for (int v = 0; v < 21; v++) {
        const int a = kUpper6[v][0], bb = kUpper6[v][1];
        acc[v] += w[u] * (j0[u][a] * j0[u][bb] + j1[u][a] * j1[u][bb]);
      }
#pragma unroll
      for (int a = 0; a < 6; a++) acc[21 + a] += j0[u][a] * we0 + j1[u][a] * we1;
    }
  }
  constexpr int NW = kBuildNT / 64;
  block_sum_vec<27, NW>(acc, sm);
  if (t < 21) {
    const int a = kUpper6[t][0], bb = kUpper6[t][1];
    const double h = sm[t * NW];
    d.Hpp[36 * i + 6 * a + bb] = h;
    d.Hpp[36 * i + 6 * bb + a] = h;
    if (a == bb) d.hdiag[6 * i + a] = h;
  } else if (t < 27) {
    d.bp[6 * i + t - 21] = sm[t * NW];
    d.bpf[6 * i + t - 21] = sm[t * NW];
  }
}
// both builds in one launch: workgroups [0, np) per pose, the rest four lanes per point
__global__ __launch_bounds__(kBuildNT) void k_build(Dev d0) {
  if (lm_done(d0) || (d0.ctl && !d0.ctl->lin)) return;
  const Dev d = lin_buf(d0, false);
  if ((int)blockIdx.x < d.np) poses_build_body(d, blockIdx.x);
  else points_build_body<false>(d, blockIdx.x - d.np, true);
}

// the trial's push (backup of every pose and point) and the solve-flag reset, grid-strided
__device__ __forceinline__ void trial_push(const Dev& d, int q, int stride) {
  for (int i = q; i < d.n_pose_dbl; i += stride) d.push_poses[i] = d.poses[i];
  for (int i = q; i < d.n_point_dbl; i += stride) d.push_points[i] = d.points[i];
  if (q == 0) *d.flag = 0;
}

// One thread per (point, edge) entry of the point CSR: D = Hll + lambda I -> Dinv (cofactors,
// recomputed per entry: identical bits), Y_e = Hpl_e Dinv; the first entry of each point
// also stores Dinv and db = Dinv b_l.
__global__ __launch_bounds__(256) void k_point_trial(Dev d0) {
  if (lm_done(d0)) return;
  const Dev d = lin_buf(d0, false);
  const int q = blockIdx.x * 256 + threadIdx.x;
  trial_push(d, q, gridDim.x * 256);
  if (q >= d.npe) return;
  const int e = d.pt_edges[q];
  const int l = d.point_h[d.e_point[e]];
  const bool first = (q == d.pt_ptr[l]);
  const bool pose_act = d.pt_h[q] >= 0;
  if (!first && !pose_act) return;
  double Di[9];
  dinv_of(d.Hll + 9 * l, lam_of(d), Di);
  if (first) {
    for (int k = 0; k < 9; k++) d.Dinv[9 * l + k] = Di[k];
    db_of(Di, d.bl + 3 * l, d.db + 3 * l);
  }
  if (pose_act) y_of(d, e, Di);
}

// Device-driven steps after the first: k_build (when the step linearises) and k_point_trial in
// one launch -- the point quads go on from their H / b to Dinv, db and Y (same arithmetic,
// same bits), every thread takes part in the push.  Step 0 keeps the two launches: lambda's
// initial value needs the built diagonal first.
__global__ __launch_bounds__(kBuildNT) void k_build_trial(Dev d0) {
  if (lm_done(d0)) return;
  const Dev d = lin_buf(d0, false);
  const bool lin = d.ctl->lin != 0;
  trial_push(d, blockIdx.x * kBuildNT + threadIdx.x, gridDim.x * kBuildNT);
  if ((int)blockIdx.x < d.np) { if (lin) poses_build_body(d, blockIdx.x); }
  else points_build_body<true>(d, blockIdx.x - d.np, lin);
}


// reduced camera system, lower blocks (i >= j): S_ij = [i==j](Hpp_i + lam0 I)
//   - sum over (e1 in pose i, e2 in pose j, same point) Y_e1 Hpl_e2^T;
// diagonal blocks also form bschur_i = b_i - sum_e Hpl_e db(point(e)).
// Work items (host-built, `build_schur_items`): item = (block, chunk c of nch); chunk c covers
// pairs [q0 + c*CH, ...) and, on a diagonal block, pose edges [e0 + c*CH, ...).  One wave per
// item: lane L accumulates entries L, L+64, ... in registers, a fixed recursive halving over
// the wave (wave_halve_all) leaves each of the 42 sums in one lane.  A block with one chunk (config E: ~90 pairs per
// block) writes S / bschur directly; otherwise the chunk's sums go to a partial slot and
// the wave that completes the block's last chunk adds the slots in chunk order (config C: 55
// blocks of thousands of pairs, so a
// block per wave would leave the GPU idle).  Every order is fixed: bitwise reproducible.
// lam0 = lambda on rank 0 and 0 elsewhere (the sharded sum then holds lambda once).

__device__ __forceinline__ void schur_write(const Dev& d, int bi, int bj, double lam0, int lane,
                                            double v) {
  if (lane < 36) {
    const int a = lane / 6, c = lane % 6;
    if (bi == bj && c > a) return;   // lower triangle of the diagonal block only
    double s0 = 0.0;
    if (bi == bj) { s0 = d.Hpp[36 * bi + 6 * a + c]; if (a == c) s0 += lam0; }
    d.S[ldlt::sidx(6 * bi + a, 6 * bj + c, d.T)] = s0 - v;
  } else if (lane < 42 && bi == bj) {
    const int a = lane - 36;
    d.bs[6 * bi + a] = d.bp[6 * bi + a] - v;
  }
}


__global__ __launch_bounds__(256) void k_schur(Dev d0) {
  if (lm_done(d0)) return;
  const Dev d = lin_buf(d0, false);
  const double lam0 = lam0_of(d);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int it = blockIdx.x * 4 + w;
  if (it >= *d.nitem) return;
  const int blk = d.it_blk[it], c = d.it_chunk[it], slot = d.it_slot[it];
  const int bi = d.blk_i[blk], bj = d.blk_j[blk];
  const int q0 = min(d.pr_ptr[blk] + c * kSchurChunk, d.pr_ptr[blk + 1]);
  const int q1 = min(q0 + kSchurChunk, d.pr_ptr[blk + 1]);
  double acc[42];
#pragma unroll
  for (int v = 0; v < 42; v++) acc[v] = 0.0;
  // the next pair's index is loaded ahead, so each pair costs one dependent round trip (its
  // rows), not two
  int q = q0 + lane;
  uint2 pqn = q < q1 ? d.pr[q] : make_uint2(0u, 0u);
  for (; q < q1; q += 64) {
    const uint2 pq = pqn;
    if (q + 64 < q1) pqn = d.pr[q + 64];
    const double* Y = d.y + 18 * pq.x;
    const double* B = d.hpl + 18 * pq.y;
    double y[18], bb[18];
#pragma unroll
    for (int k = 0; k < 18; k++) { y[k] = Y[k]; bb[k] = B[k]; }
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
      for (int cc = 0; cc < 6; cc++)
        acc[6 * a + cc] += y[3 * a] * bb[3 * cc] + y[3 * a + 1] * bb[3 * cc + 1] + y[3 * a + 2] * bb[3 * cc + 2];
  }
  int nact = q1 - q0;
  if (bi == bj) {
    const int e0 = min(d.ps_ptr[bi] + c * kSchurChunk, d.ps_ptr[bi + 1]);
    const int e1 = min(e0 + kSchurChunk, d.ps_ptr[bi + 1]);
    nact = max(nact, e1 - e0);
    auto term = [&](int e, int lh) {
      if (lh < 0) return;   // fixed point (pose-only BA): no Schur term
      const double* B = d.hpl + 18 * e;
      const double* g = d.db + 3 * lh;
      const double g0 = g[0], g1 = g[1], g2 = g[2];
#pragma unroll
      for (int a = 0; a < 6; a++) acc[36 + a] += B[3 * a] * g0 + B[3 * a + 1] * g1 + B[3 * a + 2] * g2;
    };
    // a lane's edges q and q + 64 (the chunk is 2 x 64) with their three-deep index chains
    // interleaved, then added in q order
    for (int q = e0 + lane; q < e1; q += 128) {
      const bool two = q + 64 < e1;
      const int ea = d.ps_edges[q], eb = d.ps_edges[two ? q + 64 : q];
      const int la = d.point_h[d.e_point[ea]], lb = d.point_h[d.e_point[eb]];
      term(ea, la);
      if (two) term(eb, lb);
    }
  }
  (void)nact;
  // the 42 wave sums by recursive halving: at level o a lane keeps the half of its values
  // selected by lane bit o and adds its partner's copy of that half (own + partner: the same
  // sum, bit for bit, as a full xor butterfly forms for every value), so 44 exchanges instead
  // of 6 x 42, and sum v ends in one lane (wave_halve_all), which writes it
  const int v = wave_halve_all<42>(acc, lane);
  if (slot < 0) {
    if (v >= 0) schur_write(d, bi, bj, lam0, v, acc[0]);
    return;
  }
  if (!d.blk_arrive) {   // k_schur_fin adds the slots
    if (v >= 0) d.schur_part[(size_t)slot * 42 + v] = acc[0];
    return;
  }
  // Fused fin (one-tile systems): the slot goes write-through (sc1), the wave's stores drain, one
  // lane counts the chunk in; the wave whose chunk arrives last adds the block's slots in chunk
  // order with sc1 loads (k_schur_fin's order and bits) and writes S / bschur.  Each wave hands
  // off for itself (MI355X_MICROARCH.md, first table row): no fence, no extra launch.
  if (v >= 0)
    __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)(d.schur_part + (size_t)slot * 42 + v),
                       (unsigned long long)__double_as_longlong(acc[0]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int n = d.blk_nch[blk];
  unsigned prev = 0;
  if (lane == 0) prev = __hip_atomic_fetch_add(&d.blk_arrive[blk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __builtin_amdgcn_readfirstlane(prev);
  if ((int)prev != n - 1) return;
  if (lane == 0) __hip_atomic_store(&d.blk_arrive[blk], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next step
  const int s0 = d.blk_slot0[blk];
  double sum = 0.0;
  if (lane < 42) {
    const __attribute__((address_space(1))) unsigned long long* P =
        (const __attribute__((address_space(1))) unsigned long long*)(d.schur_part + (size_t)s0 * 42 + lane);
    int cc = 0;
    for (; cc + 8 <= n; cc += 8) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 8; u++)
        t[u] = __longlong_as_double((long long)__hip_atomic_load(P + (size_t)(cc + u) * 42, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
      for (int u = 0; u < 8; u++) sum += t[u];
    }
    for (; cc < n; cc++)
      sum += __longlong_as_double((long long)__hip_atomic_load(P + (size_t)cc * 42, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  schur_write(d, bi, bj, lam0, lane, sum);
}

// blocks split into several chunks: sum the chunk slots in chunk order, then write (one wave
// per block; blocks of one chunk were written by k_schur).  Measured against finishing in
// k_schur by the wave whose chunk arrives last (agent release / atomic / acquire): equal at
// config C, 2.6x slower k_schur at config E, whose 199 diagonal blocks split 16 ways.
__global__ __launch_bounds__(256) void k_schur_fin(Dev d, int nblk) {
  if (lm_done(d) || d.blk_arrive) return;
  const double lam0 = lam0_of(d);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + w;
  if (b >= nblk) return;
  const int n = d.blk_nch[b];
  if (n <= 1) return;
  const int s0 = d.blk_slot0[b];
  double v = 0.0;
  if (lane < 42) {
    // eight slots' loads in flight, then added in chunk order (the same sum, bit for bit, as
    // one slot at a time, without a dependent round trip per slot)
    const double* P = d.schur_part + (size_t)s0 * 42 + lane;
    int c = 0;
    for (; c + 8 <= n; c += 8) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 8; u++) t[u] = P[(size_t)(c + u) * 42];
#pragma unroll
      for (int u = 0; u < 8; u++) v += t[u];
    }
    for (; c < n; c++) v += P[(size_t)c * 42];
  }
  schur_write(d, d.blk_i[b], d.blk_j[b], lam0, lane, v);
}


// x_l = Dinv (b_l - sum_e Hpl_e^T x_p); point = backup + x_l; model-decrease terms:
// red[k] (points, k < nl) and red[nl + i] (poses) summed separately (poses are replicated
// across shards, points are not).
__global__ __launch_bounds__(256) void k_update(Dev d0) {
  if (lm_done(d0)) return;
  const Dev d = lin_buf(d0, false);
  const int gt = blockIdx.x * 256 + threadIdx.x;
  const double lam = lam_of(d);
  double spt = 0.0, sps = 0.0;   // this thread's point / pose model-decrease term
  if (gt < 4 * d.nl) {   // points: four lanes per point, as the point build
    const int k = gt >> 2, sub = gt & 3;
    double c[3] = {0.0, 0.0, 0.0};
    auto term = [&](int e, int i1) {
      if (i1 < 0) return;
      const double* B = d.hpl + 18 * e;
      for (int b = 0; b < 3; b++)
        for (int a = 0; a < 6; a++) c[b] -= B[3 * a + b] * d.xp[6 * i1 + a];
    };
    // the quad lane's entries q and q + 4 with their index loads together, applied in q order
    const int q1 = d.pt_ptr[k + 1];
    for (int q = d.pt_ptr[k] + sub; q < q1; q += 8) {
      const bool two = q + 4 < q1;
      const int qb = two ? q + 4 : q;
      const int ea = d.pt_edges[q], eb = d.pt_edges[qb];
      const int ia = d.pt_h[q], ib = d.pt_h[qb];
      term(ea, ia);
      if (two) term(eb, ib);
    }
#pragma unroll
    for (int b = 0; b < 3; b++) c[b] = d.bl[3 * k + b] + quad_sum(c[b]);
    if (sub == 0) {
      const double* Di = d.Dinv + 9 * k;
      double s = 0;
      const int v = d.hpt_vtx[k];
      for (int a = 0; a < 3; a++) {
        const double xa = Di[3 * a] * c[0] + Di[3 * a + 1] * c[1] + Di[3 * a + 2] * c[2];
        d.points[3 * v + a] = d.points_bk[3 * v + a] + xa;
        s += xa * (lam * xa + d.bl[3 * k + a]);
      }
      d.red[k] = s;
      spt = s;
    }
  } else if (gt < 4 * d.nl + d.np) {
    const int i = gt - 4 * d.nl;
    const int v = d.hpose_vtx[i];
    double s = 0;
    for (int a = 0; a < 6; a++) {
      const double xa = d.xp[6 * i + a];
      d.poses[6 * v + a] = d.poses_bk[6 * v + a] + xa;
      s += xa * (lam * xa + d.bpf[6 * i + a]);
    }
    d.red[d.nl + i] = s;
    sps = s;
  }
  if (d.part_pt) {   // device-driven step: workgroup partials of both sums
    const double a = block_sum256(spt);
    const double b = block_sum256(sps);
    if (threadIdx.x == 0) { d.part_pt[blockIdx.x] = a; d.part_ps[blockIdx.x] = b; }
  }
}

// ---- device build of the Schur pair lists and the k_schur work items ---------------------
// BlockSolver::buildStructure's per-point product of pose groups (block_solver.hpp:143-295),
// in the order build_pairs_host (ba_structure.hpp) produces on the host: per point, groups of
// its edges by active pose in increasing pose order, for every group pair (P1 >= P2) the
// edges of P1 x the edges of P2 in edge order; points in order; then a stable radix sort by
// block id (rocPRIM) makes the lists block-major with that order kept inside every block.

// The pairs of a point are {(a, b) : h(a) >= h(b) >= 0} over its active edges; after the
// stable sort by block id only their order INSIDE a block matters, and there it is (a, b) in
// edge order -- exactly the order of the plain double loop over the point's edges (pt_edges is
// in edge order).  So every (point, edge a) entry counts and emits its own pairs in b order,
// one thread per entry, at the offset the scan over the entries gives it: no per-point sort.
__device__ __forceinline__ void entry_range(const Dev& d, int q, int* q0, int* q1) {
  const int l = d.point_h[d.e_point[d.pt_edges[q]]];
  *q0 = d.pt_ptr[l];
  *q1 = d.pt_ptr[l + 1];
}
__global__ __launch_bounds__(256) void k_pair_count(Dev d, int32_t* cnt) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q > d.npe) return;
  if (q == d.npe) { cnt[q] = 0; return; }   // the scan's total slot
  const int ha = d.pt_h[q];
  int n = 0;
  if (ha >= 0) {
    int q0, q1;
    entry_range(d, q, &q0, &q1);
    for (int b = q0; b < q1; b++) {
      const int hb = d.pt_h[b];
      n += (hb >= 0 && hb <= ha) ? 1 : 0;
    }
  }
  cnt[q] = n;
}

__global__ __launch_bounds__(256) void k_pair_emit(Dev d, const int32_t* off, uint32_t* keys,
                                                   uint2* vals, int64_t pmax, uint32_t pad_key) {
  const int64_t gt = (int64_t)blockIdx.x * 256 + threadIdx.x;
  // padding past the last pair: a key above every block, sorted to the end
  const int64_t total = off[d.npe];
  for (int64_t q = total + gt; q < pmax; q += (int64_t)gridDim.x * 256) {
    keys[q] = pad_key;
    vals[q] = make_uint2(0u, 0u);
  }
  const int q = (int)gt;
  if (q >= d.npe) return;
  const int ha = d.pt_h[q];
  if (ha < 0) return;
  int q0, q1;
  entry_range(d, q, &q0, &q1);
  const uint32_t ea = (uint32_t)d.pt_edges[q];
  int64_t o = off[q];
  for (int b = q0; b < q1; b++) {
    const int hb = d.pt_h[b];
    if (hb < 0 || hb > ha) continue;
    keys[o] = (uint32_t)((int64_t)ha * (ha + 1) / 2 + hb);
    vals[o] = make_uint2(ea, (uint32_t)d.pt_edges[b]);
    o++;
  }
}

// pr_ptr[b] = first sorted pair of block >= b (b = 0..nblk; the padding keys are nblk), and
// the block's chunk count (pairs, or on a diagonal block its pose's edges, per kSchurChunk)
__global__ __launch_bounds__(256) void k_block_ptr(Dev d, const uint32_t* keys, int64_t pmax,
                                                   int nblk, int32_t* pr_ptr, int32_t* nch,
                                                   int32_t* nslot) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b > nblk) return;
  auto lb = [&](uint32_t k) {
    int64_t lo = 0, hi = pmax;
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (keys[m] < k) lo = m + 1; else hi = m;
    }
    return lo;
  };
  const int64_t p0 = lb((uint32_t)b);
  pr_ptr[b] = (int32_t)p0;
  if (b == nblk) { nch[b] = 0; nslot[b] = 0; return; }
  const int np_ = (int)(lb((uint32_t)b + 1) - p0);
  const int bi = d.blk_i[b], bj = d.blk_j[b];
  const int ne = (bi == bj) ? d.ps_ptr[bi + 1] - d.ps_ptr[bi] : 0;
  const int n = max(1, (max(np_, ne) + kSchurChunk - 1) / kSchurChunk);
  nch[b] = n;
  nslot[b] = n > 1 ? n : 0;
}

__global__ __launch_bounds__(256) void k_block_items(int nblk, const int32_t* nch,
                                                     const int32_t* it_off, const int32_t* slot_off,
                                                     int32_t* it_blk, int32_t* it_chunk,
                                                     int32_t* it_slot, int32_t* it_nch,
                                                     int32_t* nitem) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b == nblk) *nitem = it_off[nblk];
  if (b >= nblk) return;
  const int n = nch[b], i0 = it_off[b];
  for (int c = 0; c < n; c++) {
    it_blk[i0 + c] = b;
    it_chunk[i0 + c] = c;
    it_slot[i0 + c] = n > 1 ? slot_off[b] + c : -1;
    it_nch[i0 + c] = n;
  }
}

// edges that left the active set (LocalBA culling, Optimizer::remask): zero every per-edge term
// a build kernel reads, so their contributions to Hll / b_l / Hpp / b_p / Schur are exact zeros
__device__ __forceinline__ void zero_edge_terms(const Dev& d, int e) {
  d.w[e] = 0.0;
  d.err[2 * e] = 0.0; d.err[2 * e + 1] = 0.0;
  for (int i = 0; i < 12; i++) d.jp[12 * e + i] = 0.0;
  for (int i = 0; i < 6; i++) d.jl[6 * e + i] = 0.0;
  for (int i = 0; i < 18; i++) { d.hpl[18 * e + i] = 0.0; d.y[18 * e + i] = 0.0; }
  if (d.alt_err) {   // both linearisation buffers (a later run may flip to either)
    d.alt_w[e] = 0.0;
    d.alt_err[2 * e] = 0.0; d.alt_err[2 * e + 1] = 0.0;
    for (int i = 0; i < 12; i++) d.alt_jp[12 * e + i] = 0.0;
    for (int i = 0; i < 6; i++) d.alt_jl[6 * e + i] = 0.0;
    for (int i = 0; i < 18; i++) d.alt_hpl[18 * e + i] = 0.0;
  }
}
__global__ __launch_bounds__(256) void k_zero_edges(Dev d, const int32_t* edges, int n) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  zero_edge_terms(d, edges[k]);
}

// ---- LocalBA's culling on the device (mcs_local_ba_ex) -----------------------------------
// The culling passes of LocalBundleAdjustment (src/cOptimizer.cpp:798-817 after round 1,
// :830-849 after round 2) walk the edges in vpEdges order with per-point state: observations
// left and the bad flag EraseObservation raises below two (src/cMapPoint.cpp:120-152).  A
// point's decisions depend only on its own edges, in edge order, so one thread per active point
// walks its point-CSR list (pt_edges is in edge order and, in round 1, holds every edge of the
// point) and decides exactly as the sequential pass does.  Round 1 also moves the culled edges to
// level 1 and zeroes their per-edge terms (what Optimizer::remask's k_zero_edges does), counts
// the culled edges per pose and the points left, and its last workgroup reports whether an
// active pose lost all its edges (g2o would drop it from the system: the host then rebuilds from
// scratch).  Round 2 keeps round 1's active list; k_edges / k_edges_end skip its level-1 edges
// (Dev::elevel), whose terms stay zero.  (A one-workgroup compaction of the list took 39 us.)
struct LbaState {
  int32_t* obs_left; int32_t* edges_left; int32_t* edges_all;   // per point vertex
  uint8_t* bad;                                                  // per point vertex
  uint8_t* inlier; uint8_t* level;                               // per edge
  const int32_t* extra;                                          // extra observations (nullable)
  double* chi;                                                   // chi2 of every edge
  double k2;                                                     // thHuber^2
  int32_t* pose_cnt;                                             // active edges per active pose
  uint32_t* ctr;                                                 // {culled edges, points left, arrivals}
  int32_t* res;                                                  // {nae, pose_left, nl_left} (host memory)
  uint8_t* pwrite;                                               // per point vertex (round 2)
};

__global__ __launch_bounds__(256) void k_lba_cull(Dev d, LbaState L, int round1) {
  const int l = blockIdx.x * 256 + threadIdx.x;
  if (l >= d.nl) return;
  const int v = d.hpt_vtx[l], q0 = d.pt_ptr[l], q1 = d.pt_ptr[l + 1];
  int ol, el;
  bool bad;
  if (round1) {
    el = q1 - q0;
    ol = el + (L.extra ? L.extra[v] : 0);
    bad = false;
    L.edges_all[v] = el;
  } else {
    ol = L.obs_left[v]; el = L.edges_left[v]; bad = L.bad[v] != 0;
  }
  // the point's edges eight at a time: their indices, then their flags and chi2 all in flight,
  // then the sequential decisions in edge order from registers
  for (int qb = q0; qb < q1; qb += 8) {
    int ev[8];
    bool in[8];
    double ch[8];
#pragma unroll
    for (int j = 0; j < 8; j++) ev[j] = d.pt_edges[min(qb + j, q1 - 1)];
#pragma unroll
    for (int j = 0; j < 8; j++) { in[j] = L.inlier[ev[j]] != 0; ch[j] = L.chi[ev[j]]; }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (qb + j >= q1) break;
      const int e = ev[j];
      if (!in[j] || bad || !(ch[j] > L.k2)) continue;
      L.inlier[e] = 0;
      if (round1) { L.level[e] = 1; zero_edge_terms(d, e); }
      el--;
      if (--ol < 2) bad = true;
    }
  }
  L.obs_left[v] = ol; L.edges_left[v] = el; L.bad[v] = bad ? 1 : 0;
  // cOptimizer.cpp:885-902: not bad, TotalNrObservations() > 1, >= 2 vertex edges
  if (!round1 && L.pwrite) L.pwrite[v] = !bad && el > 1 && L.edges_all[v] >= 2;
}

// round 1's bookkeeping after k_lba_cull's decisions: per-pose survivors (one atomic per culled
// edge, integer counts), culled edges and points left (one atomic per wave); the last
// workgroup writes the three counts into host memory
__global__ __launch_bounds__(256) void k_lba_count(Dev d, LbaState L) {
  __shared__ int last;
  const int l = blockIdx.x * 256 + threadIdx.x;
  int culled = 0, alive = 0;
  if (l < d.nl) {
    const int v = d.hpt_vtx[l];
    const int el = L.edges_left[v];
    alive = el > 0 ? 1 : 0;
    culled = L.edges_all[v] - el;
    if (culled) {
      for (int q = d.pt_ptr[l]; q < d.pt_ptr[l + 1]; q++) {
        const int e = d.pt_edges[q];
        const int h = d.pt_h[q];
        if (L.level[e] && h >= 0) atomicSub(&L.pose_cnt[h], 1);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { culled += __shfl_xor(culled, o); alive += __shfl_xor(alive, o); }
  if ((threadIdx.x & 63) == 0) {
    if (culled) atomicAdd(&L.ctr[0], (unsigned)culled);
    if (alive) atomicAdd(&L.ctr[1], (unsigned)alive);
  }
  // every count is an atomic (performed in device-coherent memory): each wave drains its own,
  // then one lane counts the workgroup in; the last one reads them with atomic loads
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(&L.ctr[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  int left = 0;
  for (int h = threadIdx.x; h < d.np; h += 256) left |= __hip_atomic_load(&L.pose_cnt[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= 0 ? 1 : 0;
  left = __syncthreads_or(left);
  if (threadIdx.x == 0) {
    const unsigned c0 = __hip_atomic_load(&L.ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned c1 = __hip_atomic_load(&L.ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    L.res[0] = d.nae - (int)c0;
    L.res[1] = left;
    L.res[2] = (int)c1;
  }
}

// the culling state before round 1: every edge an inlier at level 0, every point vertex clear
__global__ __launch_bounds__(256) void k_lba_init(Dev d, LbaState L, int ne, int npt) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < ne) { L.inlier[i] = 1; L.level[i] = 0; }
  if (i < d.np) L.pose_cnt[i] = d.ps_ptr[i + 1] - d.ps_ptr[i];
  if (i < 4) L.ctr[i] = 0u;
  if (i < npt) {
    L.obs_left[i] = 0; L.edges_left[i] = 0; L.edges_all[i] = 0; L.bad[i] = 0;
    if (L.pwrite) L.pwrite[i] = 0;
  }
}

// LocalBA's round-2 results into host memory: [poses | points | inlier flags | write-back flags]
__global__ __launch_bounds__(256) void k_lba_out(const double* poses, int npo, const double* points, int npt,
                                                 const uint8_t* inl, int ne, const uint8_t* pw, int npw,
                                                 uint8_t* host) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  double* hd = reinterpret_cast<double*>(host);
  if (i < npo) hd[i] = poses[i];
  else if (i < npo + npt) hd[i] = points[i - npo];
  uint8_t* hb = host + 8 * (size_t)(npo + npt);
  if (i < ne) hb[i] = inl[i];
  if (i < npw) hb[ne + i] = pw[i];
}

// the trial's pop (restore every pose and point from the backups) in one launch
__global__ __launch_bounds__(256) void k_restore(Dev d) {
  const int q = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  for (int i = q; i < d.n_pose_dbl; i += stride) d.poses[i] = d.push_poses[i];
  for (int i = q; i < d.n_point_dbl; i += stride) d.points[i] = d.push_points[i];
}

}  // namespace ba
}  // namespace mcs

using namespace mcs;
using namespace mcs::ba;


struct mcs_ba_ctx {
  int device = 0;
  HostStruct hs;
  // host threads for config-E-sized calls (structure build, staging copy); made on the first
  // call with at least kParMinEdges edges.  MCS_HOST_THREADS: their number (default 8, 1: off)
  std::unique_ptr<mcs::HostPool> pool;
  mcs::HostPool* pool_for(int n_edges) {
    if (n_edges < kParMinEdges) return nullptr;
    if (!pool) {
      const char* e = std::getenv("MCS_HOST_THREADS");
      int t = e ? std::atoi(e) : 8;
      const int hw = (int)std::thread::hardware_concurrency();
      if (hw > 0) t = std::min(t, hw);
      pool.reset(new mcs::HostPool(std::max(1, std::min(t, 16))));
    }
    return pool->size() > 1 ? pool.get() : nullptr;
  }
  hipStream_t st = nullptr;
  // Device buffers are cached across calls: the driver requests them in the same order
  // every call, so request k reuses slot k when it is large enough (grow-only).
  std::vector<void*> bufs;
  std::vector<size_t> caps;
  size_t next = 0;
  double* pinned = nullptr;   // host-pinned readback scalars
  int32_t* pinned_i = nullptr;
  TrialSig* sig = nullptr;    // host-coherent trial outcome (k_reduce3)
  uint64_t sig_seq = 0;
  LmSig* lsig = nullptr;      // host-coherent progress of the device-driven LM (k_edges_end)
  uint64_t lsig_seq = 0;
  void* pinned_ctl = nullptr; // host-pinned readback of the final LmCtl
  // host-pinned staging of a call's packed problem upload (grow-only)
  uint8_t* stage = nullptr;
  size_t stage_cap = 0;
  uint8_t* stage_get(size_t bytes) {
    if (bytes > stage_cap) {
      if (stage) (void)hipHostFree(stage);
      stage = nullptr; stage_cap = 0;
      const size_t cap = std::max(bytes, (size_t)1 << 20);
      // mapped: k_lba_out writes LocalBA's results into it directly
      if (hipHostMalloc((void**)&stage, cap, hipHostMallocMapped) != hipSuccess) return nullptr;
      stage_cap = cap;
    }
    return stage;
  }
  // second staging buffer (threaded calls): the structure arrays, filled while the problem
  // arrays' copy out of `stage` may still be in flight
  uint8_t* stage2 = nullptr;
  size_t stage2_cap = 0;
  uint8_t* stage2_get(size_t bytes) {
    if (bytes > stage2_cap) {
      if (stage2) (void)hipHostFree(stage2);
      stage2 = nullptr; stage2_cap = 0;
      const size_t cap = std::max(bytes, (size_t)1 << 20);
      if (hipHostMalloc((void**)&stage2, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
      stage2_cap = cap;
    }
    return stage2;
  }
  // optional stage timing (mcs_ba_enable_timing): HIP events on st around each stage,
  // accumulated after the per-trial synchronisation the LM control needs anyway
  bool timing = false;
  bool ldlt_pipe = true;   // pipelined LDL^T for multi-tile systems (2 <= T <= kPipeMaxT)
  hipEvent_t ev[8] = {};
  double acc_ms[MCS_BA_NSTAGES] = {};
  double host_ms[MCS_BA_NHOST] = {};   // host phases (mcs_ba_read_host_timing)
  int32_t host_calls = 0;
  int32_t n_iter = 0, n_trial = 0, last_n = 0;
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

// Wait for a stream by polling instead of a blocking synchronisation: the blocking wait may
// sleep and costs up to ~0.4 ms of wake-up latency at the end of a LocalBA call (measured in
// the bench's host phase "download": 0.12 - 0.52 ms for the same work).
static hipError_t spin_sync(hipStream_t st) {
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q != hipErrorNotReady) return q;
    for (int k = 0; k < 64; k++) __builtin_ia32_pause();
  }
}

// The problem arrays of a call, packed into one device block through one pinned staging
// buffer and ONE host-to-device copy (some thirty pageable copies cost ~0.4 ms per call on a
// config-C LocalBA round).  add() records where each array's device pointer goes; flush()
// fills the pointers.
struct Packer {
  struct Item { void** dst; const void* src; size_t bytes, off; };
  std::vector<Item> items;
  size_t total = 0;
  template <typename D, typename T>
  void add(D** dst, const T* src, size_t n) {
    static_assert(sizeof(D) == sizeof(T), "element type");
    items.push_back({reinterpret_cast<void**>(const_cast<void*>(static_cast<const void*>(dst))), src,
                     src ? n * sizeof(T) : 0, total});
    total += (std::max<size_t>(1, n) * sizeof(T) + 255) & ~(size_t)255;
  }
  template <typename D, typename T>
  void add(D** dst, const std::vector<T>& v) { add(dst, v.data(), v.size()); }
  // second: into stage2, behind a first flush of this call (whose spin_sync already found the
  // previous call's copies done; the first flush's own copy may still be running)
  hipError_t flush(mcs_ba_ctx* c, mcs::HostPool* pool = nullptr, bool second = false) {
    uint8_t* d = (uint8_t*)c->alloc(std::max<size_t>(total, 256));
    if (!d) return hipErrorOutOfMemory;
    if (!second) {
      const hipError_t e = spin_sync(c->st);   // the staging buffer is free again
      if (e != hipSuccess) return e;
    }
    uint8_t* h = second ? c->stage2_get(std::max<size_t>(total, 256)) : c->stage_get(std::max<size_t>(total, 256));
    if (!h) return hipErrorOutOfMemory;
    for (const Item& it : items) *it.dst = d + it.off;
    if (pool && total >= ((size_t)4 << 20)) {
      // config E packs ~20 MB: the staging copy split by byte range over the host threads
      const int T = pool->size();
      pool->run([&](int t) {
        const size_t lo = total * t / T, hi = total * (t + 1) / T;
        for (const Item& it : items) {
          const size_t a = std::max(lo, it.off), b = std::min(hi, it.off + it.bytes);
          if (a < b) std::memcpy(h + a, (const uint8_t*)it.src + (a - it.off), b - a);
        }
      });
    } else {
      for (const Item& it : items)
        if (it.bytes) std::memcpy(h + it.off, it.src, it.bytes);
    }
    return total ? hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, c->st) : hipSuccess;
  }
};

unsigned gb(int n) { return (unsigned)std::max(1, (n + 255) / 256); }

// Exchange-buffer layout (offsets in doubles) for T tiles and np active poses: [bs | S tiles |
// hdiag | bpf | scalars]; bs first so that bs and the leading (non-zero) diagonals of S are one
// range.  The head of the buffer is reused for the structure exchange (pose activity counts)
// before T is known.
struct XLayout {
  size_t S, bs, hdiag, bpf, sc, total;
  XLayout(int T, int np) {
    bs = 0;
    S = (size_t)ldlt::TB * T;
    hdiag = S + ldlt::tile_doubles(T);
    bpf = hdiag + 6 * (size_t)np;
    sc = bpf + 6 * (size_t)np;
    total = sc + 16;
  }
};

int64_t xchg_doubles(int32_t n_poses) {
  const int np = std::max(0, n_poses);
  const XLayout x(ldlt::tiles_for(std::max(1, 6 * np)), np);
  return (int64_t)std::max<size_t>(x.total, (size_t)np + 16);
}

struct Shard {
  int rank = 0, world = 1;
  double* xchg = nullptr;
  mcs_ba_allreduce_fn fn = nullptr;
  void* user = nullptr;
  bool ordered = false;   // stream_ordered: the callback enqueues on st, no host drain
};

// One optimize() call split in two so that LocalBA's second round can reuse the first
// round's device state: setup() = initializeOptimization + buildStructure + the problem
// upload; remask() = the same graph with more edges at level 1 (the culled ones: their
// per-edge terms are zeroed once and the active-edge list shrinks, nothing else moves);
// run() = SparseOptimizer::optimize (LM iterations) + the result download.
// host phase clock: add the time since the previous mark to c->host_ms[k]
struct HostClock {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(double* acc, int k) {
    const auto n = std::chrono::steady_clock::now();
    acc[k] += std::chrono::duration<double, std::milli>(n - t).count();
    t = n;
  }
};

struct Optimizer {
  mcs_ba_ctx* c;
  const mcs_ba_problem* p;
  bool points_fixed;
  Shard sh;
  bool sharded = false;
  hipStream_t st = nullptr;
  HostStruct& s;
  Dev d;
  int n = 0, T = 1, NE = 0;
  int band = 1;          // tile bandwidth of the reduced camera system (ldlt::Work::band)
  int64_t pmax = 0;      // upper bound of the Schur pairs (device-built lists)
  int items_max = 1;     // upper bound of the k_schur work items
  int32_t* it_nch_dev = nullptr;   // chunks of each item's block (checked by the test hook)
  int nblk = 0;
  XLayout X{1, 0};
  size_t xs_count = 0;   // doubles of the per-trial exchange: bs + the non-zero diagonals of S
  int nl_glob = 0, nae_glob = 0;
  double *d_poses = nullptr, *d_points = nullptr, *d_scalar = nullptr, *d_part = nullptr;
  int* d_flag = nullptr;
  ldlt::Work lw;
  unsigned g_state = 1;
  bool sig_path = false;
  hipError_t he = hipSuccess;
  // LocalBA culling on the device (mcs_local_ba_ex with the device-driven LM): set lba and
  // lba_extra before setup(); lba_tail picks what run_device does after the LM loop
  bool lba = false;
  const int32_t* lba_extra = nullptr;
  LbaState L{};
  int lba_tail = 0;   // 0 download; 1 round 1: cull + compaction, no download; 2 round 2: cull +
                      // results; 3 round 2 without the cull (empty graph)
  int32_t lba_res[3] = {0, 0, 0};   // round 1: active edges left, a pose left the system, points left
  uint8_t* lba_inlier_out = nullptr;
  uint8_t* lba_pwrite_out = nullptr;

  Optimizer(mcs_ba_ctx* c_, const mcs_ba_problem* p_, bool pf) : c(c_), p(p_), points_fixed(pf), s(c_->hs) {
    std::memset(&d, 0, sizeof(d));
  }
  double* dz(size_t cnt_) {
    double* q = (double*)c->alloc(std::max<size_t>(1, cnt_) * 8);
    if (!q) he = hipErrorOutOfMemory;
    return q;
  }
  // collective over xchg[off, off+cnt); no-op on one rank.  Stream-ordered shards get it
  // enqueued on st behind the producing kernels; otherwise the stream is drained first and the
  // callback completes it (its host time is the exchange stage).
  int allreduce(int op, size_t off, size_t cnt) {
    if (!sharded || cnt == 0) return MCS_OK;
    if (!sh.ordered) MCS_HIP_CHECK(hipStreamSynchronize(st));
    const auto t0 = std::chrono::steady_clock::now();
    if (sh.fn(sh.user, op, (int64_t)off, (int64_t)cnt, (void*)st) != 0) {
      set_error("BA: allreduce callback failed");
      return MCS_ERR_HIP;
    }
    if (c->timing && !sh.ordered)
      c->acc_ms[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MCS_OK;
  }
  // all-reduce host scalars through the tail of the exchange buffer
  int allreduce_host(double* v, int cnt, int op, size_t off) {
    if (!sharded) return MCS_OK;
    MCS_HIP_CHECK(hipMemcpyAsync(sh.xchg + off, v, 8 * (size_t)cnt, hipMemcpyHostToDevice, st));
    int rc = allreduce(op, off, cnt);
    if (rc) return rc;
    MCS_HIP_CHECK(hipMemcpyAsync(v, sh.xchg + off, 8 * (size_t)cnt, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipStreamSynchronize(st));
    return MCS_OK;
  }

  // the problem's own arrays (and the trial backups' space) into a packed upload
  void add_problem(Packer& pk, const double* poses, const double* points, double** poses_bk,
                   double** points_bk) {
    pk.add(&d.mc, p->mc, 6 * (size_t)p->n_cams);
    pk.add(&d.cam, p->cam, 17 * (size_t)p->n_cams);
    pk.add(&d.e_pose, p->edge_pose, (size_t)NE);
    pk.add(&d.e_point, p->edge_point, (size_t)NE);
    pk.add(&d.e_cam, p->edge_cam, (size_t)NE);
    pk.add(&d.e_meas, p->edge_meas, 2 * (size_t)NE);
    pk.add(&d.e_info, p->edge_info, (size_t)NE);
    pk.add(&d_poses, poses, 6 * (size_t)p->n_poses);
    pk.add(&d_points, points, 3 * (size_t)p->n_points);
    // the trial backups are written by every trial's push before anything reads them: space only
    pk.add(poses_bk, static_cast<const double*>(nullptr), 6 * (size_t)p->n_poses);
    pk.add(points_bk, static_cast<const double*>(nullptr), 3 * (size_t)p->n_points);
  }

  int setup(const double* poses, const double* points, const uint8_t* edge_level,
            const mcs_ba_shard* shard_in) {
    if (p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0 || p->n_cams < 1) return MCS_ERR_ARG;
    HostClock hc;
    c->host_calls++;
    // ---- structure, pass 1: the index checks, the active edges and their per-pose / per-point
    // counts (+ active point / edge counts), all-reduced over the shards below
    std::vector<double> cnt;
    mcs::HostPool* const pool = c->pool_for(p->n_edges);
    if (!scan_edges(*p, edge_level, points_fixed, s, cnt, pool)) {
      set_error("edge vertex index out of range");
      return MCS_ERR_ARG;
    }
    MCS_HIP_CHECK(hipSetDevice(c->device));
    if (shard_in && shard_in->world > 1) {
      if (!shard_in->xchg || !shard_in->allreduce || shard_in->rank < 0 || shard_in->rank >= shard_in->world ||
          shard_in->xchg_cap < xchg_doubles(p->n_poses)) {
        set_error("invalid mcs_ba_shard (exchange buffer too small or no allreduce callback)");
        return MCS_ERR_ARG;
      }
      sh.rank = shard_in->rank; sh.world = shard_in->world; sh.xchg = shard_in->xchg;
      sh.fn = shard_in->allreduce; sh.user = shard_in->user;
      sh.ordered = shard_in->stream_ordered != 0;
    }
    sharded = sh.world > 1;
    st = c->st;
    c->free_all();
    if (!sharded) {
      sh.xchg = (double*)c->alloc((size_t)xchg_doubles(p->n_poses) * 8);
      if (!sh.xchg) { set_error("BA: out of device memory"); return MCS_ERR_HIP; }
    }
    // ---- threaded (config-E-sized) calls: the problem arrays go up now, their copy
    // overlapping the structure build; the structure arrays follow from the second staging
    // buffer (GlobalBA 6.15 / 6.20 -> 5.86 / 5.47 ms per call, profiles/r06_split_ab.txt).  The
    // second flush relies on this first one's spin_sync (Packer::flush): split implies it ran.
    NE = p->n_edges;
    double *d_poses_bk = nullptr, *d_points_bk = nullptr;
    const bool split = pool != nullptr;
    if (split) {
      Packer pk;
      add_problem(pk, poses, points, &d_poses_bk, &d_points_bk);
      if ((he = pk.flush(c, pool)) != hipSuccess) MCS_HIP_CHECK(he);
    }
    // ---- global pose activity (+ active point / edge counts)
    int rc;
    if ((rc = allreduce_host(cnt.data(), p->n_poses + 2, MCS_REDUCE_SUM, 0))) return rc;
    hc.mark(c->host_ms, 0);
    build_structure(*p, points_fixed, cnt, s, pool);
    hc.mark(c->host_ms, 1);
    nl_glob = (int)cnt[p->n_poses];
    nae_glob = (int)cnt[p->n_poses + 1];
    n = 6 * s.np;
    T = ldlt::tiles_for(std::max(1, n));
    X = XLayout(T, s.np);
    xs_count = X.hdiag - X.bs;
    band = T;
    if (T > 1) {
      // Tiles of S below the widest tile diagonal any rank's points touch are zero on every
      // rank (their blocks have no pairs; the padding rows there are zero too), and LDL^T keeps
      // a banded matrix's L inside the same band: the factorisation runs on diagonals 0 .. w
      // only (ldlt::Work::band), and the sharded exchange stops at diagonal w too.
      std::vector<int> wpart(pool ? pool->size() : 1, 1);   // >= 1: pose blocks straddling a tile boundary
      auto span = [&](int t, int nt) {
        const int q0 = (int)((int64_t)s.nl * t / nt), q1 = (int)((int64_t)s.nl * (t + 1) / nt);
        int w = 1;
        for (int q = q0; q < q1; q++) {
          int lo = INT32_MAX, hi = -1;
          for (int e = s.pt_ptr[q]; e < s.pt_ptr[q + 1]; e++) {
            const int h = s.pt_h[e];
            if (h >= 0) { lo = std::min(lo, h); hi = std::max(hi, h); }
          }
          if (hi >= 0) w = std::max(w, (6 * hi + 5) / ldlt::TB - (6 * lo) / ldlt::TB);
        }
        wpart[t] = w;
      };
      if (pool && s.nl >= 4096) pool->run([&](int t) { span(t, (int)wpart.size()); });
      else span(0, 1);
      double wd = *std::max_element(wpart.begin(), wpart.end());
      if ((rc = allreduce_host(&wd, 1, MCS_REDUCE_MAX, X.sc))) return rc;
      band = ldlt::pipe_band(T, (int)wd + 1);
      if (sharded) xs_count = (size_t)ldlt::TB * T + ldlt::band_tiles((int)wd + 1, T) * ldlt::TB * ldlt::TB;
    }
    const bool pipelined = T >= 2 && c->ldlt_pipe && ldlt::pipe_supported(T, band);
    if (!pipelined && (size_t)T * ldlt::TB * 8 > 96 * 1024) {
      set_error("more than 2048 active poses with a reduced camera system too wide for the banded "
                "factorisation (its task table exceeds the pipeline's bound)");
      return MCS_ERR_UNSUPPORTED;
    }
    {
      Packer pk;
      if (!split) add_problem(pk, poses, points, &d_poses_bk, &d_points_bk);
      // every edge active (LocalBA round 1, GlobalBA): no list, the kernels index edges directly
      if ((int)s.aedge.size() != NE) pk.add(&d.aedge, s.aedge);
      else d.aedge = nullptr;
      pk.add(&d.pose_h, s.pose_h); pk.add(&d.point_h, s.point_h);
      pk.add(&d.hpose_vtx, s.hpose_vtx); pk.add(&d.hpt_vtx, s.hpt_vtx);
      pk.add(&d.pt_ptr, s.pt_ptr); pk.add(&d.pt_edges, s.pt_edges); pk.add(&d.pt_h, s.pt_h);
      pk.add(&d.ps_ptr, s.ps_ptr); pk.add(&d.ps_edges, s.ps_edges);
      pk.add(&d.blk_i, s.blk_i); pk.add(&d.blk_j, s.blk_j);
      if (lba && lba_extra) pk.add(&L.extra, lba_extra, (size_t)p->n_points);
      he = pk.flush(c, pool, split);
    }
    d.delta = p->huber_delta;
    d.dsqr = huber_dsqr(p->huber_delta);
    d.poses = d_poses; d.points = d_points; d.poses_bk = d_poses_bk; d.points_bk = d_points_bk;
    d.nae = (int)s.aedge.size();
    d.np = s.np; d.nl = s.nl;
    d.npe = (int)s.pt_edges.size();
    d.err = dz(2 * (size_t)NE); d.w = dz(NE); d.jp = dz(12 * (size_t)NE); d.jl = dz(6 * (size_t)NE);
    d.hpl = dz(18 * (size_t)NE); d.y = dz(18 * (size_t)NE); d.chi = dz(NE); d.rchi = dz(NE);
    // the second linearisation buffer (device-driven runs: speculative linearisation)
    if (!sharded) {
      d.alt_err = dz(2 * (size_t)NE); d.alt_w = dz(NE); d.alt_jp = dz(12 * (size_t)NE);
      d.alt_jl = dz(6 * (size_t)NE); d.alt_hpl = dz(18 * (size_t)NE);
    } else {
      d.alt_err = d.alt_w = d.alt_jp = d.alt_jl = d.alt_hpl = nullptr;
    }
    d.Hpp = dz(36 * (size_t)s.np); d.bp = dz(6 * (size_t)s.np);
    d.Hll = dz(9 * (size_t)s.nl); d.bl = dz(3 * (size_t)s.nl);
    d.Dinv = dz(9 * (size_t)s.nl); d.db = dz(3 * (size_t)s.nl);
    d.S = sh.xchg + X.S; d.bs = sh.xchg + X.bs; d.hdiag = sh.xchg + X.hdiag; d.bpf = sh.xchg + X.bpf;
    d.T = T;
    d.xp = dz((size_t)ldlt::TB * T);
    d.red = dz((size_t)NE + 6 * (size_t)s.np + s.nl + 16);
    // bounds of the device-built pair lists / items: a point with k active edges gives at most
    // k^2 pairs (k (k + 1) / 2 when its edges have distinct poses, as the reference's one
    // observation per keyframe makes them; the C-ABI takes any graph); a block at most
    // 1 + pairs / CH + pose edges / CH chunks
    nblk = s.np * (s.np + 1) / 2;
    pmax = 0;
    for (int l = 0; l < s.nl; l++) {
      const int64_t k = s.pt_ptr[l + 1] - s.pt_ptr[l];
      pmax += k * k;
    }
    if (pmax > INT32_MAX) { set_error("BA: more than 2^31 Schur pairs"); return MCS_ERR_UNSUPPORTED; }
    items_max = (int)std::min<int64_t>(INT32_MAX, 2 * (int64_t)nblk + pmax / kSchurChunk +
                                                       s.ps_ptr[s.np] / kSchurChunk + 1);
    d.schur_part = dz((size_t)items_max * 42);

    lw.L = dz(ldlt::tile_doubles(T));
    lw.Linv = dz((size_t)T * ldlt::TB * ldlt::TB);
    lw.z = dz((size_t)ldlt::TB * T);
    // pipelined factorisation (one launch per solve) for every multi-tile system
    lw.W = nullptr; lw.du = nullptr; lw.sync = nullptr; lw.tasks = nullptr; lw.ntasks = 0; lw.pipe_T = 0;
    if (pipelined) {
      const std::vector<int4>& tq = ldlt::pipe_tasks_host(T, band);
      lw.W = dz(ldlt::tile_doubles(T));
      lw.du = dz((size_t)T * 128);
      lw.sync = (unsigned*)dz((ldlt::pipe_sync_words(T, band) + 1) / 2);
      lw.tasks = (int4*)dz(2 * tq.size());
      if (he == hipSuccess && lw.tasks)
        he = hipMemcpyAsync(lw.tasks, tq.data(), tq.size() * sizeof(int4), hipMemcpyHostToDevice, st);
      lw.ntasks = (int)tq.size();
      lw.pipe_T = T;
      lw.band = band;
    }
    // scalars: [0] chi2 [1] point scale [2] pose scale [3] chi_now; the solve flag in [5] (one
    // 48-byte readback per trial)
    d_scalar = dz(8);
    d_part = dz(kRedPartMax);
    d_flag = reinterpret_cast<int*>(d_scalar + 5);
    if (lba) {
      const size_t npt = (size_t)std::max(1, p->n_points), ne = (size_t)std::max(1, NE);
      L.obs_left = (int32_t*)c->alloc(4 * npt);
      L.edges_left = (int32_t*)c->alloc(4 * npt);
      L.edges_all = (int32_t*)c->alloc(4 * npt);
      L.bad = (uint8_t*)c->alloc(npt);
      L.pwrite = (uint8_t*)c->alloc(npt);
      L.inlier = (uint8_t*)c->alloc(ne);
      L.level = (uint8_t*)c->alloc(ne);
      L.pose_cnt = (int32_t*)c->alloc(4 * (size_t)std::max(1, s.np));
      L.ctr = (uint32_t*)c->alloc(16);
      L.res = c->pinned_i;   // written by k_lba_count straight into host memory
      L.chi = d.chi;
      L.k2 = p->huber_delta * p->huber_delta;
      if (!L.obs_left || !L.edges_left || !L.edges_all || !L.bad || !L.pwrite || !L.inlier || !L.level ||
          !L.pose_cnt || !L.ctr)
        he = hipErrorOutOfMemory;
      else
        hipLaunchKernelGGL(k_lba_init, dim3(gb(std::max(NE, p->n_points))), dim3(256), 0, st, d, L, NE,
                           p->n_points);
    }
    if (he != hipSuccess) { set_hip_error(he, "BA upload", __FILE__, __LINE__); return MCS_ERR_HIP; }
    d.push_poses = d_poses_bk; d.push_points = d_points_bk;
    d.n_pose_dbl = 6 * p->n_poses; d.n_point_dbl = 3 * p->n_points;
    d.flag = d_flag;
    g_state = gb(std::max(d.n_pose_dbl, d.n_point_dbl));
    sig_path = !sharded && d.nae <= 32768 && s.nl <= 32768 && s.np <= 32768;
    const int rp = enqueue_pairs();
    hc.mark(c->host_ms, 2);
    return rp;
  }

  // The Schur pair lists and k_schur items, built on the device (the kernels above), stream
  // ordered after the upload: nothing is read back.
  int enqueue_pairs() {
    const int npe = (int)s.pt_edges.size();
    int32_t* cnt = (int32_t*)c->alloc(4 * (size_t)(npe + 1));
    int32_t* off = (int32_t*)c->alloc(4 * (size_t)(npe + 1));
    uint32_t* k_in = (uint32_t*)c->alloc(4 * (size_t)std::max<int64_t>(1, pmax));
    uint32_t* k_out = (uint32_t*)c->alloc(4 * (size_t)std::max<int64_t>(1, pmax));
    uint2* v_in = (uint2*)c->alloc(8 * (size_t)std::max<int64_t>(1, pmax));
    uint2* v_out = (uint2*)c->alloc(8 * (size_t)std::max<int64_t>(1, pmax));
    int32_t* pr_ptr = (int32_t*)c->alloc(4 * (size_t)(nblk + 1));
    int32_t* nch = (int32_t*)c->alloc(4 * (size_t)(nblk + 1));
    int32_t* nslot = (int32_t*)c->alloc(4 * (size_t)(nblk + 1));
    int32_t* it_off = (int32_t*)c->alloc(4 * (size_t)(nblk + 1));
    int32_t* slot_off = (int32_t*)c->alloc(4 * (size_t)(nblk + 1));
    int32_t* it_blk = (int32_t*)c->alloc(4 * (size_t)items_max);
    int32_t* it_chunk = (int32_t*)c->alloc(4 * (size_t)items_max);
    int32_t* it_slot = (int32_t*)c->alloc(4 * (size_t)items_max);
    int32_t* it_nch = (int32_t*)c->alloc(4 * (size_t)items_max);
    int32_t* nitem = (int32_t*)c->alloc(4);
    if (!cnt || !off || !k_in || !k_out || !v_in || !v_out || !pr_ptr || !nch || !nslot || !it_off ||
        !slot_off || !it_blk || !it_chunk || !it_slot || !it_nch || !nitem) {
      set_error("BA: out of device memory (pair lists)");
      return MCS_ERR_HIP;
    }
    const unsigned bits = nblk > 0 ? 32u - (unsigned)__builtin_clz((unsigned)nblk) : 1u;
    size_t b_scan1 = 0, b_scan2 = 0, b_sort = 0;
    auto plus = rocprim::plus<int32_t>();
    MCS_HIP_CHECK(rocprim::exclusive_scan(nullptr, b_scan1, cnt, off, 0, (size_t)npe + 1, plus, st));
    MCS_HIP_CHECK(rocprim::exclusive_scan(nullptr, b_scan2, nch, it_off, 0, (size_t)nblk + 1, plus, st));
    if (pmax > 0)
      MCS_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, b_sort, k_in, k_out, v_in, v_out, (size_t)pmax, 0u, bits, st));
    const size_t tb = std::max(std::max(b_scan1, b_scan2), b_sort) + 256;
    void* tmp = c->alloc(tb);
    if (!tmp) { set_error("BA: out of device memory (scan storage)"); return MCS_ERR_HIP; }
    size_t b = tb;
    hipLaunchKernelGGL(k_pair_count, dim3(gb(npe + 1)), dim3(256), 0, st, d, cnt);
    MCS_HIP_CHECK(rocprim::exclusive_scan(tmp, b, cnt, off, 0, (size_t)npe + 1, plus, st));
    if (pmax > 0) {
      const unsigned g = std::max(gb(npe), std::min(gb((int)std::min<int64_t>(pmax, INT32_MAX)), 4096u));
      hipLaunchKernelGGL(k_pair_emit, dim3(g), dim3(256), 0, st, d, (const int32_t*)off, k_in, v_in, pmax,
                         (uint32_t)nblk);
      b = tb;
      MCS_HIP_CHECK(rocprim::radix_sort_pairs(tmp, b, k_in, k_out, v_in, v_out, (size_t)pmax, 0u, bits, st));
    }
    hipLaunchKernelGGL(k_block_ptr, dim3(gb(nblk + 1)), dim3(256), 0, st, d, (const uint32_t*)k_out, pmax,
                       nblk, pr_ptr, nch, nslot);
    b = tb;
    MCS_HIP_CHECK(rocprim::exclusive_scan(tmp, b, nch, it_off, 0, (size_t)nblk + 1, plus, st));
    b = tb;
    MCS_HIP_CHECK(rocprim::exclusive_scan(tmp, b, nslot, slot_off, 0, (size_t)nblk + 1, plus, st));
    hipLaunchKernelGGL(k_block_items, dim3(gb(nblk + 1)), dim3(256), 0, st, nblk, (const int32_t*)nch,
                       (const int32_t*)it_off, (const int32_t*)slot_off, it_blk, it_chunk, it_slot, it_nch,
                       nitem);
    MCS_HIP_CHECK(hipGetLastError());
    d.pr_ptr = pr_ptr; d.pr = v_out;
    d.it_blk = it_blk; d.it_chunk = it_chunk; d.it_slot = it_slot;
    d.blk_nch = nch; d.blk_slot0 = slot_off;
    it_nch_dev = it_nch;
    d.nitem = nitem;
    return MCS_OK;
  }

  // More edges at level 1 (a subset of the active ones; unsharded only).  g2o re-runs
  // initializeOptimization: the culled edges leave the graph, and a vertex left without active
  // edges leaves the system.  Here the culled edges' per-edge terms (weight, Jacobians, Hpl,
  // error) are zeroed once and the active-edge list shrinks; every sum they took part in then
  // adds exact zeros, and a point left without edges keeps Hll = 0 (its update is Dinv * 0 = 0,
  // its Schur and model-decrease terms are 0).  Returns 1 (nothing changed on the device) when
  // an active pose would leave the system: the caller then rebuilds from scratch.
  int remask(const uint8_t* edge_level) {
    if (sharded) return 1;
    HostClock hc;
    std::vector<int32_t> keep;
    std::vector<int32_t> culled;
    keep.reserve(s.aedge.size());
    std::vector<int32_t> pose_left(s.np, 0);
    std::vector<char> pt_left(s.nl, 0);
    for (int e : s.aedge) {
      if (edge_level && edge_level[e]) { culled.push_back(e); continue; }
      keep.push_back(e);
      const int h = s.pose_h[p->edge_pose[e]];
      if (h >= 0) pose_left[h]++;
      const int l = s.point_h[p->edge_point[e]];
      if (l >= 0) pt_left[l] = 1;
    }
    for (int h = 0; h < s.np; h++)
      if (pose_left[h] == 0) return 1;
    int nl_left = 0;
    for (int l = 0; l < s.nl; l++) nl_left += pt_left[l];
    if (!culled.empty()) {
      const size_t nb = (keep.size() + culled.size()) * 4 + 512;
      uint8_t* h = c->stage_get(nb);   // the stream is idle: run() ended with a synchronise
      if (!h) { set_error("BA: out of pinned host memory"); return MCS_ERR_HIP; }
      int32_t* dk = (int32_t*)c->alloc(std::max<size_t>(1, keep.size()) * 4);
      int32_t* dc = (int32_t*)c->alloc(culled.size() * 4);
      if (!dk || !dc) { set_error("BA: out of device memory"); return MCS_ERR_HIP; }
      const size_t off_c = ((keep.size() * 4 + 255) & ~(size_t)255);
      std::memcpy(h, keep.data(), keep.size() * 4);
      std::memcpy(h + off_c, culled.data(), culled.size() * 4);
      if (!keep.empty()) MCS_HIP_CHECK(hipMemcpyAsync(dk, h, keep.size() * 4, hipMemcpyHostToDevice, st));
      MCS_HIP_CHECK(hipMemcpyAsync(dc, h + off_c, culled.size() * 4, hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_zero_edges, dim3(gb((int)culled.size())), dim3(256), 0, st, d, (const int32_t*)dc,
                         (int)culled.size());
      d.aedge = dk;
      d.nae = (int)keep.size();
    }
    s.aedge.swap(keep);
    nae_glob = d.nae;
    nl_glob = nl_left;
    sig_path = !sharded && d.nae <= 32768 && s.nl <= 32768 && s.np <= 32768;
    hc.mark(c->host_ms, 4);
    return MCS_OK;
  }

  // Round 2 of a device-culled LocalBA: round 1's active list with its level-1 edges skipped
  // (no host round trip: the culled edges' terms were zeroed by k_lba_cull)
  void remask_device() {
    d.elevel = L.level;   // round 1's list; its level-1 edges are skipped (terms zeroed)
    nae_glob = lba_res[0];
    nl_glob = lba_res[2];
    sig_path = !sharded && d.nae <= 32768 && s.nl <= 32768 && s.np <= 32768;
  }

  // run_device's tail for LocalBA (lba_tail 1..3): chi2 of every edge at the final estimate,
  // the culling pass, and either round 2's counts (round 1: nothing is downloaded; the host
  // reads three counts) or the results (round 2: poses, points, inlier flags, write-back)
  int lba_finish(double* poses, double* points) {
    HostClock hc;
    if (lba_tail <= 2) {
      Dev d2 = d;
      d2.ctl = nullptr;
      d2.aedge = nullptr;
      d2.elevel = nullptr;
      d2.nae = NE;
      d2.err = dz(2 * (size_t)NE);
      d2.rchi = dz(NE);
      if (he != hipSuccess) { set_hip_error(he, "BA chi2", __FILE__, __LINE__); return MCS_ERR_HIP; }
      hipLaunchKernelGGL(k_edges, dim3(gb(NE)), dim3(256), 0, st, d2, 0);
      hipLaunchKernelGGL(k_lba_cull, dim3(gb(s.nl)), dim3(256), 0, st, d, L, lba_tail == 1 ? 1 : 0);
    }
    if (lba_tail == 1) {
      hipLaunchKernelGGL(k_lba_count, dim3(gb(s.nl)), dim3(256), 0, st, d, L);
      MCS_HIP_CHECK(spin_sync(st));
      std::memcpy(lba_res, c->pinned_i, 12);
      hc.mark(c->host_ms, 3);
      MCS_HIP_CHECK(hipGetLastError());
      return MCS_OK;
    }
    const size_t b_po = 48 * (size_t)p->n_poses, b_pt = 24 * (size_t)p->n_points;
    const size_t b_in = (size_t)NE, b_pw = lba_pwrite_out ? (size_t)p->n_points : 0;
    const size_t total = b_po + b_pt + b_in + b_pw + 64;
    if (total > c->stage_cap) MCS_HIP_CHECK(hipStreamSynchronize(st));   // regrow
    uint8_t* hst = c->stage_get(total);
    if (!hst) { set_error("BA: out of pinned host memory"); return MCS_ERR_HIP; }
    // one kernel writes the four results into the pinned staging buffer (host memory the device
    // reaches directly): no readback copies
    const int nmax = (int)std::max<size_t>({b_po / 8 + b_pt / 8, b_in, b_pw, 1});
    hipLaunchKernelGGL(k_lba_out, dim3(gb(nmax)), dim3(256), 0, st, (const double*)d_poses,
                       (int)(b_po / 8), (const double*)d_points, (int)(b_pt / 8), (const uint8_t*)L.inlier,
                       (int)b_in, (const uint8_t*)L.pwrite, (int)b_pw, hst);
    MCS_HIP_CHECK(spin_sync(st));
    if (b_po) std::memcpy(poses, hst, b_po);
    if (b_pt) std::memcpy(points, hst + b_po, b_pt);
    if (b_in && lba_inlier_out) std::memcpy(lba_inlier_out, hst + b_po + b_pt, b_in);
    if (b_pw) std::memcpy(lba_pwrite_out, hst + b_po + b_pt + b_in, b_pw);
    hc.mark(c->host_ms, 3);
    MCS_HIP_CHECK(hipGetLastError());
    return MCS_OK;
  }

  // the round-1 state a host fallback needs (a pose left the system): the estimate, the levels
  // and the per-point culling state
  int lba_fetch(double* poses, double* points, uint8_t* level, uint8_t* inlier, int32_t* obs_left,
                int32_t* edges_left, uint8_t* bad) {
    const size_t npt = (size_t)p->n_points;
    MCS_HIP_CHECK(hipMemcpyAsync(poses, d_poses, 48 * (size_t)p->n_poses, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipMemcpyAsync(points, d_points, 24 * npt, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipMemcpyAsync(level, L.level, (size_t)NE, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipMemcpyAsync(inlier, L.inlier, (size_t)NE, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipMemcpyAsync(obs_left, L.obs_left, 4 * npt, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipMemcpyAsync(edges_left, L.edges_left, 4 * npt, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipMemcpyAsync(bad, L.bad, npt, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipStreamSynchronize(st));
    return MCS_OK;
  }

  // poses and points only (round 1 stopped by the caller's flag)
  int fetch_state(double* poses, double* points) {
    MCS_HIP_CHECK(hipMemcpyAsync(poses, d_poses, 48 * (size_t)p->n_poses, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipMemcpyAsync(points, d_points, 24 * (size_t)p->n_points, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(hipStreamSynchronize(st));
    return MCS_OK;
  }

  // the LM loop runs on the device (run_device) for these options
  bool device_driven(const mcs_ba_options* o, const mcs_ba_report* rep) const {
    const bool long_trace = rep && rep->trace_chi2 && rep->trace_cap > kLmTraceCap &&
                            o->max_iterations > kLmTraceCap;
    return !sharded && !c->timing && !long_trace;
  }

  int run(const mcs_ba_options* o, double* poses, double* points, double* edge_chi2,
          volatile int32_t* stop_flag, mcs_ba_report* rep) {
    // one GPU and no per-stage timing: the LM control runs on the device (no per-trial
    // host round trip); sharded runs agree on every decision through the host exchange
    // (the device loop records the chi2 trace of its first kLmTraceCap iterations only: a
    // caller asking for a longer trace of a longer run gets the host-driven loop, which fills
    // up to trace_cap like every other path)
    if (device_driven(o, rep))
      return run_device(o, poses, points, edge_chi2, stop_flag, rep);
    auto rec = [&](int k) { if (c->timing) (void)hipEventRecord(c->ev[k], st); };
    auto ms = [&](int a, int b) { float f = 0.f; (void)hipEventElapsedTime(&f, c->ev[a], c->ev[b]); return (double)f; };
    int rc;
    if (rep) {
      rep->n_active_edges = nae_glob;
      rep->n_active_poses = s.np;
      rep->n_active_points = nl_glob;
      rep->iterations = 0;
    }
    // control state agreed by all ranks: the caller's stop flag is folded into every scalar
    // exchange, so no rank leaves the LM loop alone
    volatile int32_t aux = 0;
    volatile int32_t* stop = stop_flag ? stop_flag : &aux;
    int agreed_stop = 0;
    const size_t sc = X.sc;

    auto chi_now = [&](double* out) -> int {   // robust chi2 of the current estimate (all ranks)
      hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, d, 0);
      reduce_dev<false>(d.rchi, d.nae, d_scalar, d_part, st);
      MCS_HIP_CHECK(hipMemcpyAsync(c->pinned + 3, d_scalar, 8, hipMemcpyDeviceToHost, st));
      MCS_HIP_CHECK(hipStreamSynchronize(st));
      double v[2] = {c->pinned[3], (double)(*stop != 0)};
      int r = allreduce_host(v, 2, MCS_REDUCE_SUM, sc);
      if (r) return r;
      *out = v[0];
      agreed_stop = v[1] > 0;
      return MCS_OK;
    };
    // one LM trial (push, Schur, solve, update, chi2), enqueued on st; lambda in d (by value)
    auto enqueue_trial = [&](bool stop_now) -> int {
      int rc2;
      rec(2);
      // also pushes the state (poses / points -> backups) and resets the solve flag
      hipLaunchKernelGGL(k_point_trial, dim3(std::max(gb(d.npe), g_state)), dim3(256), 0, st, d);
      if (s.np) {
        hipLaunchKernelGGL(k_schur, dim3((unsigned)((items_max + 3) / 4)), dim3(256), 0, st, d);
        hipLaunchKernelGGL(k_schur_fin, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, st, d, nblk);
        // one tile (LocalBA): the padding is applied inside the fused solve, after the exchange
        if (T > 1) MCS_HIP_CHECK(ldlt::pad(d.S, d.bs, n, T, sh.rank == 0 ? 1.0 : 0.0, st));
        rec(3);
        if ((rc2 = allreduce(MCS_REDUCE_SUM, X.bs, xs_count))) return rc2;   // bs | S band
        rec(4);
        if (T == 1) MCS_HIP_CHECK(ldlt::solve_one_tile(d.S, d.bs, d.xp, n, 1.0, d_flag, st));
        else MCS_HIP_CHECK(ldlt::solve(d.S, d.bs, d.xp, T, lw, d_flag, st));
      } else {
        rec(3); rec(4);
      }
      rec(5);
      hipLaunchKernelGGL(k_update, dim3(gb(4 * s.nl + s.np)), dim3(256), 0, st, d);
      hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, d, 0);
      if (sig_path) {
        Sum3 q{{d.rchi, d.red, d.red + s.nl}, {d.nae, s.nl, s.np}};
        hipLaunchKernelGGL(k_reduce3, dim3(3), dim3(1024), 0, st, q, (const int*)d_flag, c->sig, ++c->sig_seq);
      } else if (sharded) {
        // chi2 and the points' model decrease are partial sums: reduce them straight into the
        // exchange buffer next to the stop flag, all-reduce them there and read back once
        // (pinned[0..2] = the summed {chi2, points' decrease, stop}; pinned[3] = the poses'
        // decrease, replicated; pinned[5] = the solve flag, identical on every rank)
        reduce_dev<false>(d.rchi, d.nae, sh.xchg + X.sc, d_part, st);
        reduce_dev<false>(d.red, s.nl, sh.xchg + X.sc + 1, d_part, st);
        reduce_dev<false>(d.red + s.nl, s.np, d_scalar + 2, d_part, st);
        c->pinned[7] = stop_now ? 1.0 : 0.0;
        MCS_HIP_CHECK(hipMemcpyAsync(sh.xchg + X.sc + 2, c->pinned + 7, 8, hipMemcpyHostToDevice, st));
        if ((rc2 = allreduce(MCS_REDUCE_SUM, X.sc, 3))) return rc2;
        MCS_HIP_CHECK(hipMemcpyAsync(c->pinned, sh.xchg + X.sc, 24, hipMemcpyDeviceToHost, st));
        MCS_HIP_CHECK(hipMemcpyAsync(c->pinned + 3, d_scalar + 2, 8, hipMemcpyDeviceToHost, st));
        MCS_HIP_CHECK(hipMemcpyAsync(c->pinned + 5, d_scalar + 5, 8, hipMemcpyDeviceToHost, st));
      } else {
        reduce_dev<false>(d.red, s.nl, d_scalar + 1, d_part, st);
        reduce_dev<false>(d.red + s.nl, s.np, d_scalar + 2, d_part, st);
        reduce_dev<false>(d.rchi, d.nae, d_scalar, d_part, st);
        MCS_HIP_CHECK(hipMemcpyAsync(c->pinned, d_scalar, 48, hipMemcpyDeviceToHost, st));
      }
      rec(6);
      return MCS_OK;
    };
    // wait for the trial's outcome: spin on the released sequence number (sig_path), checking
    // the stream now and then so a failed launch cannot spin forever; else synchronise the
    // stream after the readback copy.  Fills pinned[0..2] and the solve flag.
    auto wait_trial = [&](int* fl) -> int {
      if (!sig_path) {
        MCS_HIP_CHECK(hipStreamSynchronize(st));
        std::memcpy(fl, c->pinned + 5, sizeof(*fl));
        return MCS_OK;
      }
      const uint64_t want = c->sig_seq;
      auto arrived = [&]() {
        return __atomic_load_n(&c->sig->seq[0], __ATOMIC_ACQUIRE) == want &&
               __atomic_load_n(&c->sig->seq[1], __ATOMIC_ACQUIRE) == want &&
               __atomic_load_n(&c->sig->seq[2], __ATOMIC_ACQUIRE) == want;
      };
      for (uint32_t k = 1;; k++) {
        if (arrived()) break;
        __builtin_ia32_pause();   // spin politely: other ranks' threads may share this core
        if ((k & 1023) == 0) {
          const hipError_t q = hipStreamQuery(st);
          if (q == hipSuccess) {
            if (arrived()) break;
            set_error("BA: trial signal missing after the stream drained");
            return MCS_ERR_HIP;
          }
          if (q != hipErrorNotReady) { set_hip_error(q, "BA trial", __FILE__, __LINE__); return MCS_ERR_HIP; }
        }
      }
      c->pinned[0] = c->sig->v[0]; c->pinned[1] = c->sig->v[1]; c->pinned[2] = c->sig->v[2];
      *fl = c->sig->flag;
      if (c->timing) MCS_HIP_CHECK(hipStreamSynchronize(st));   // events complete
      return MCS_OK;
    };
    double chi0 = 0;
    if ((s.np + nl_glob) == 0 || nae_glob == 0) {
      if (rep) rep->chi2_initial = rep->chi2_final = 0;
    } else {
      if ((rc = chi_now(&chi0))) return rc;
      if (rep) rep->chi2_initial = chi0;
      double lambda = 0, lastChi = 0;
      int ni = 2, nBad = 0, it = 0;
      bool ok = true;
      double currentChi = chi0;
      for (int i = 0; i < o->max_iterations && !agreed_stop && ok; i++) {
        // ---- OptimizationAlgorithmLevenberg::solve(i)
        // The robust chi2 of the linearisation point equals the chi2 the previous iteration
        // ended with (same kernel, same state: accepted trial or restored backup), so only
        // the first iteration reads anything back (the max diagonal for lambda's init).
        rec(0);
        hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, d, 1);
        hipLaunchKernelGGL(k_build, dim3((unsigned)s.np + (unsigned)((4 * s.nl + kBuildNT - 1) / kBuildNT)), dim3(kBuildNT), 0, st, d);
        rec(1);
        c->n_iter++;
        bool lin_pending = c->timing;
        if ((rc = allreduce(MCS_REDUCE_SUM, X.hdiag, 12 * (size_t)s.np))) return rc;   // hdiag | bpf
        if (i == 0) {
          reduce_dev<true>(d.red, s.nl, d_scalar + 1, d_part, st);
          reduce_dev<true>(d.hdiag, 6 * s.np, d_scalar + 2, d_part, st);
          MCS_HIP_CHECK(hipMemcpyAsync(c->pinned + 1, d_scalar + 1, 16, hipMemcpyDeviceToHost, st));
          MCS_HIP_CHECK(hipStreamSynchronize(st));
          double mx = std::max(c->pinned[1], c->pinned[2]);
          if ((rc = allreduce_host(&mx, 1, MCS_REDUCE_MAX, sc))) return rc;
          lambda = o->tau * mx; ni = 2; nBad = 0;
        }
        const double iniChi = currentChi;
        double rho = 0;
        int qmax = 0;
        do {
          // lambda reaches the kernels by value (Dev d), no upload; a captured graph of the trial
          // (replayed per trial) measured no faster than these direct launches
          d.lam = lambda;
          d.lam0 = sh.rank == 0 ? lambda : 0.0;
          if ((rc = enqueue_trial(*stop != 0))) return rc;
          int fl;   // identical on every rank (same reduced system)
          if ((rc = wait_trial(&fl))) return rc;
          if (fl & ldlt::kFlagTimeout) {
            set_error("BA: the LDL^T solve's hand-off wait timed out (ldlt kFlagTimeout); result discarded");
            return MCS_ERR_HIP;
          }
          if (c->timing) {
            if (lin_pending) { c->acc_ms[0] += ms(0, 1); lin_pending = false; }
            if (sh.ordered) c->acc_ms[2] += ms(3, 4);
            c->acc_ms[1] += ms(2, 3);
            c->acc_ms[3] += ms(4, 5);
            c->acc_ms[4] += ms(5, 6);
            c->n_trial++;
            c->last_n = n;
          }
          // sharded: summed on the device by enqueue_trial
          const double tr[3] = {c->pinned[0], c->pinned[1], sharded ? c->pinned[2] : 0.0};
          const double scale_pose = sharded ? c->pinned[3] : c->pinned[2];
          agreed_stop = sharded ? tr[2] > 0 : *stop != 0;
          double tempChi = tr[0];
          if (fl & ldlt::kFlagZeroPivot) tempChi = std::numeric_limits<double>::max();
          rho = currentChi - tempChi;
          double scale = scale_pose + tr[1];
          scale += 1e-3;
          rho /= scale;
          if (rho > 0 && std::isfinite(tempChi)) {
            double alpha = 1. - cube_rn(2 * rho - 1);
            alpha = std::min(alpha, 2. / 3.);
            lambda *= std::max(1. / 3., alpha);
            ni = 2;
            currentChi = tempChi;
          } else {
            lambda *= ni;
            ni *= 2;
            hipLaunchKernelGGL(k_restore, dim3(g_state), dim3(256), 0, st, d);  // pop
          }
          qmax++;
        } while (rho < 0 && qmax < o->max_trials && !agreed_stop);
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
        // current state == currentChi (see above); identical on every rank
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
          if (stopOpt) { *stop = 1; agreed_stop = 1; }
        }
        if (rep) rep->lambda_final = lambda;
      }
      if (rep) rep->iterations = it;
      if (rep) rep->chi2_final = currentChi;
    }
    if (rep) rep->stop_flag = *stop;
    return download(poses, points, edge_chi2);
  }

  // results through the pinned staging buffer (free again: the stream has been drained since
  // the upload), then one host copy each; edge_chi2 (nullable): chi2 of every edge
  int download(double* poses, double* points, double* edge_chi2) {
    HostClock hc;
    if (edge_chi2) {
      // chi2 of every edge (active or not) at the final estimate; a private view: d keeps its
      // active list for a later remask() + run()
      Dev d2 = d;
      d2.ctl = nullptr;
      d2.aedge = nullptr;
      d2.elevel = nullptr;
      d2.nae = NE;
      d2.err = dz(2 * (size_t)NE);
      d2.rchi = dz(NE);
      if (he != hipSuccess) { set_hip_error(he, "BA chi2", __FILE__, __LINE__); return MCS_ERR_HIP; }
      hipLaunchKernelGGL(k_edges, dim3(gb(NE)), dim3(256), 0, st, d2, 0);
    }
    const size_t b_po = 48 * (size_t)p->n_poses, b_pt = 24 * (size_t)p->n_points;
    const size_t b_ch = edge_chi2 ? 8 * (size_t)NE : 0;
    if (b_po + b_pt + b_ch + 64 > c->stage_cap) MCS_HIP_CHECK(hipStreamSynchronize(st));   // regrow
    uint8_t* hst = c->stage_get(b_po + b_pt + b_ch + 64);
    if (!hst) { set_error("BA: out of pinned host memory"); return MCS_ERR_HIP; }
    if (b_po) MCS_HIP_CHECK(hipMemcpyAsync(hst, d_poses, b_po, hipMemcpyDeviceToHost, st));
    if (b_pt) MCS_HIP_CHECK(hipMemcpyAsync(hst + b_po, d_points, b_pt, hipMemcpyDeviceToHost, st));
    if (b_ch) MCS_HIP_CHECK(hipMemcpyAsync(hst + b_po + b_pt, d.chi, b_ch, hipMemcpyDeviceToHost, st));
    MCS_HIP_CHECK(spin_sync(st));
    if (b_po) std::memcpy(poses, hst, b_po);
    if (b_pt) std::memcpy(points, hst + b_po, b_pt);
    if (b_ch) std::memcpy(edge_chi2, hst + b_po + b_pt, b_ch);
    hc.mark(c->host_ms, 3);
    MCS_HIP_CHECK(hipGetLastError());
    return MCS_OK;
  }

  // Device-driven SparseOptimizer::optimize: the host enqueues LM steps (restore if the last
  // trial was rejected, linearisation if it ended an iteration, one trial, k_edges_end) up to two
  // ahead of the device and watches the progress word only to stop enqueuing; the decisions
  // are k_edges_end's.  Kernels of steps past the end return at once.
  int run_device(const mcs_ba_options* o, double* poses, double* points, double* edge_chi2,
                 volatile int32_t* stop_flag, mcs_ba_report* rep) {
    if (rep) {
      rep->n_active_edges = nae_glob;
      rep->n_active_poses = s.np;
      rep->n_active_points = nl_glob;
      rep->iterations = 0;
    }
    volatile int32_t aux = 0;
    volatile int32_t* stop = stop_flag ? stop_flag : &aux;
    LmCtl* dctl = (LmCtl*)c->alloc(sizeof(LmCtl));
    if (!dctl) { set_error("BA: out of device memory"); return MCS_ERR_HIP; }
    LmCtl h0;
    std::memset(&h0, 0, sizeof(h0));
    h0.tau = o->tau; h0.gain_threshold = o->gain_threshold;
    h0.max_iterations = o->max_iterations; h0.max_trials = o->max_trials;
    h0.terminate_max_iter = o->terminate_max_iter;
    h0.lin = 1; h0.ni = 2;
    h0.spec_lin = d.alt_err ? 1 : 0;   // k_edges_end linearises every trial (see k_edges_end)
    h0.jbuf = 0;
    const bool empty = (s.np + nl_glob) == 0 || nae_glob == 0;
    h0.done = (empty || o->max_iterations <= 0 || *stop != 0) ? 1 : 0;
    c->lsig->ext_stop = *stop != 0;
    c->lsig->done = 0;   // this run's `done` (the previous run's stream has drained)
    Dev dd = d;
    dd.ctl = dctl;
    // one-tile systems (LocalBA): k_schur adds a split block's chunk slots itself (fused fin)
    // (multi-tile systems keep the k_schur_fin launch: fused, config E measured 7.07 against
    // 6.90 ms per GlobalBA call)
    const bool fuse = T == 1;
    dd.blk_arrive = (fuse && nblk > 0) ? (uint32_t*)c->alloc(4 * (size_t)nblk) : nullptr;
    hipLaunchKernelGGL(k_ctl_init, dim3(1), dim3(256), 0, st, h0, dctl, dd.blk_arrive, nblk);
    const int* skip = &dctl->done;
    const unsigned g_upd = gb(4 * s.nl + s.np), g_edg = gb(d.nae);
    dd.part_chi = dz(g_edg);
    dd.part_pt = dz(g_upd);
    dd.part_ps = dz(g_upd);
    if (he != hipSuccess) { set_hip_error(he, "BA partials", __FILE__, __LINE__); return MCS_ERR_HIP; }
    // the starting point's chi2 (activeRobustChi2 before the first iteration): from step 0's
    // linearising pass when the loop will run (the same errors), else a plain evaluation
    const bool lin0 = !empty && !h0.done;
    if (!empty) {
      if (lin0) {
        hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, dd, 1);
      } else {
        Dev d0 = d;
        hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, d0, 0);
      }
      reduce_dev<false>(d.rchi, d.nae, d_scalar, d_part, st);
      hipLaunchKernelGGL(k_lm_start, dim3(1), dim3(64), 0, st, dctl, (const double*)d_scalar);
    }
    auto enqueue_step = [&](int step) -> int {
      // the first step linearises at the start; later steps find the accepted trial's
      // linearisation (k_edges_end) already in place, or keep the iteration's after a reject
      if ((step == 0 && !lin0) || (step > 0 && !h0.spec_lin))
        hipLaunchKernelGGL(k_edges, dim3(gb(d.nae)), dim3(256), 0, st, dd, 1);
      const unsigned g_build = (unsigned)s.np + (unsigned)((4 * s.nl + kBuildNT - 1) / kBuildNT);
      if (step == 0) {   // iteration 0 is always step 0: lambda from the max diagonal
        hipLaunchKernelGGL(k_build, dim3(g_build), dim3(kBuildNT), 0, st, dd);
        reduce_dev<true>(d.red, s.nl, d_scalar + 1, d_part, st);
        reduce_dev<true>(d.hdiag, 6 * s.np, d_scalar + 2, d_part, st);
        hipLaunchKernelGGL(k_lm_lambda0, dim3(1), dim3(64), 0, st, dctl, (const double*)d_scalar);
        hipLaunchKernelGGL(k_point_trial, dim3(std::max(gb(d.npe), g_state)), dim3(256), 0, st, dd);
      } else {
        hipLaunchKernelGGL(k_build_trial, dim3(g_build), dim3(kBuildNT), 0, st, dd);
      }
      if (s.np) {
        hipLaunchKernelGGL(k_schur, dim3((unsigned)((items_max + 3) / 4)), dim3(256), 0, st, dd);
        if (!dd.blk_arrive)
          hipLaunchKernelGGL(k_schur_fin, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, st, dd, nblk);
        if (T == 1) MCS_HIP_CHECK(ldlt::solve_one_tile(d.S, d.bs, d.xp, n, 1.0, d_flag, st, skip));
        else {
          MCS_HIP_CHECK(ldlt::pad(d.S, d.bs, n, T, 1.0, st, skip));
          MCS_HIP_CHECK(ldlt::solve(d.S, d.bs, d.xp, T, lw, d_flag, st, skip));
        }
      }
      LmEnd le{d_scalar, (const int*)d_flag, c->lsig, ++c->lsig_seq, (LmCtl*)c->pinned_ctl};
      hipLaunchKernelGGL(k_update, dim3(gb(4 * s.nl + s.np)), dim3(256), 0, st, dd);
      // the trial's evaluation, then (last workgroup) its three sums from the workgroup
      // partials of k_edges_end / k_update (a fixed order: partials in workgroup order, each a
      // fixed in-workgroup tree), the LM decision and the pop of a rejected trial
      Sum3 q{{dd.part_chi, dd.part_pt, dd.part_ps}, {(int)g_edg, (int)g_upd, (int)g_upd}};
      hipLaunchKernelGGL(k_edges_end, dim3(g_edg), dim3(kEdgeEndNT), 0, st, dd, q, le);
      return hipGetLastError() == hipSuccess ? MCS_OK : MCS_ERR_HIP;
    };
    // progress word of the step whose k_edges_end published sequence `want`
    auto wait_seq = [&](uint64_t want) -> int {
      for (uint32_t k = 1;; k++) {
        if (__atomic_load_n(&c->lsig->seq, __ATOMIC_ACQUIRE) >= want) return MCS_OK;
        __builtin_ia32_pause();
        if ((k & 1023) == 0) {
          c->lsig->ext_stop = *stop != 0;   // the caller's abort flag reaches k_edges_end
          const hipError_t q = hipStreamQuery(st);
          if (q == hipSuccess) {
            if (__atomic_load_n(&c->lsig->seq, __ATOMIC_ACQUIRE) >= want) return MCS_OK;
            set_error("BA: LM progress word missing after the stream drained");
            return MCS_ERR_HIP;
          }
          if (q != hipErrorNotReady) { set_hip_error(q, "BA LM step", __FILE__, __LINE__); return MCS_ERR_HIP; }
        }
      }
    };
    int rc;
    if (!h0.done) {
      const uint64_t base = c->lsig_seq;
      const int max_steps = o->max_iterations * std::max(1, o->max_trials);
      for (int step = 0; step < max_steps; step++) {
        if (step >= MCS_LM_AHEAD) {   // keep MCS_LM_AHEAD steps in flight
          if ((rc = wait_seq(base + (uint64_t)step - (MCS_LM_AHEAD - 1)))) return rc;
          c->lsig->ext_stop = *stop != 0;
          if (c->lsig->done) break;
        }
        if ((rc = enqueue_step(step))) { set_error("BA: LM step launch failed"); return rc; }
      }
    }
    LmCtl* hc = (LmCtl*)c->pinned_ctl;
    // the step that ended the run wrote the control block to hc (k_edges_end); otherwise (no
    // step ran, or the host stopped at max_steps before seeing `done`) read it back
    const bool ctl_written = !h0.done && __atomic_load_n(&c->lsig->done, __ATOMIC_ACQUIRE) != 0;
    if (!ctl_written) MCS_HIP_CHECK(hipMemcpyAsync(hc, dctl, sizeof(LmCtl), hipMemcpyDeviceToHost, st));
    // per-edge chi2 of every edge at the final estimate, poses, points: the common tail (or
    // LocalBA's device culling)
    const int rtail = lba_tail ? lba_finish(poses, points) : download(poses, points, edge_chi2);
    if (rtail) return rtail;
    if (hc->dev_err) {
      set_error("BA: the LDL^T solve's hand-off wait timed out (ldlt kFlagTimeout); optimisation aborted");
      return MCS_ERR_HIP;
    }
    if (hc->stop_out) *stop = 1;   // the terminate action raised the flag (host-visible)
    if (rep) {
      rep->chi2_initial = empty ? 0.0 : hc->chi0;
      rep->chi2_final = empty ? 0.0 : hc->currentChi;
      rep->iterations = hc->it;
      rep->lambda_final = hc->lambda_final;
      if (rep->trace_chi2)
        for (int i = 0; i < std::min(hc->iter, std::min(rep->trace_cap, kLmTraceCap)); i++)
          rep->trace_chi2[i] = hc->trace[i];
      rep->stop_flag = *stop;
    }
    return MCS_OK;
  }
};

int optimize_impl(mcs_ba_ctx* c, const mcs_ba_problem* p, const mcs_ba_options* o, double* poses,
                  double* points, const uint8_t* edge_level, double* edge_chi2,
                  volatile int32_t* stop_flag, mcs_ba_report* rep, const mcs_ba_shard* shard_in,
                  bool points_fixed) {
  if (!c || !p || !o || !poses || !points) return MCS_ERR_ARG;
  Optimizer opt(c, p, points_fixed);
  int rc = opt.setup(poses, points, edge_level, shard_in);
  if (rc) return rc;
  return opt.run(o, poses, points, edge_chi2, stop_flag, rep);
}

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
  MCS_HIP_CHECK(hipHostMalloc((void**)&c->pinned_i, 64, hipHostMallocMapped));   // k_lba_count writes it
  MCS_HIP_CHECK(hipHostMalloc((void**)&c->sig, sizeof(TrialSig), hipHostMallocCoherent | hipHostMallocMapped));
  std::memset((void*)c->sig, 0, sizeof(TrialSig));
  MCS_HIP_CHECK(hipHostMalloc((void**)&c->lsig, sizeof(LmSig), hipHostMallocCoherent | hipHostMallocMapped));
  MCS_HIP_CHECK(hipHostMalloc((void**)&c->pinned_ctl, sizeof(LmCtl), hipHostMallocMapped));   // k_edges_end writes it
  std::memset((void*)c->lsig, 0, sizeof(LmSig));
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
  if (c->sig) (void)hipHostFree(c->sig);
  if (c->lsig) (void)hipHostFree(c->lsig);
  if (c->pinned_ctl) (void)hipHostFree(c->pinned_ctl);
  if (c->stage) (void)hipHostFree(c->stage);
  if (c->stage2) (void)hipHostFree(c->stage2);
  if (c->st) (void)hipStreamDestroy(c->st);
  for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
  delete c;
}

int mcs_ba_enable_timing(mcs_ba_ctx* c, int32_t on) {
  if (!c) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(c->device));
  if (on && !c->ev[0])
    for (auto& e : c->ev) MCS_HIP_CHECK(hipEventCreate(&e));
  c->timing = on != 0;
  return MCS_OK;
}

int mcs_ba_read_timing(mcs_ba_ctx* c, double* ms, int32_t* n_iterations, int32_t* n_trials,
                       int32_t* last_n, int32_t reset) {
  if (!c) return MCS_ERR_ARG;
  for (int k = 0; k < MCS_BA_NSTAGES; k++) if (ms) ms[k] = c->acc_ms[k];
  if (n_iterations) *n_iterations = c->n_iter;
  if (n_trials) *n_trials = c->n_trial;
  if (last_n) *last_n = c->last_n;
  if (reset) {
    for (double& v : c->acc_ms) v = 0.0;
    c->n_iter = c->n_trial = 0;
  }
  return MCS_OK;
}

int mcs_ba_check_structure(mcs_ba_ctx* c, const mcs_ba_problem* p, const uint8_t* edge_level) {
  if (!c || !p) return MCS_ERR_ARG;
  Optimizer opt(c, p, false);
  int rc = opt.setup(p->poses, p->points, edge_level, nullptr);
  if (rc) return rc;
  HostStruct h = c->hs;
  build_pairs_host(*p, h);
  const int nb = opt.nblk;
  std::vector<int32_t> pr_ptr(nb + 1), items;
  int32_t nitem = 0;
  MCS_HIP_CHECK(hipMemcpyAsync(pr_ptr.data(), opt.d.pr_ptr, 4 * (size_t)(nb + 1), hipMemcpyDeviceToHost, c->st));
  MCS_HIP_CHECK(hipMemcpyAsync(&nitem, opt.d.nitem, 4, hipMemcpyDeviceToHost, c->st));
  MCS_HIP_CHECK(hipStreamSynchronize(c->st));
  int64_t bad = 0;
  for (int b = 0; b <= nb; b++) bad += pr_ptr[b] != h.pr_ptr[b];
  if (bad) return (int)std::min<int64_t>(bad, INT32_MAX);
  const int np_ = pr_ptr[nb];
  std::vector<uint2> pr(std::max(1, np_));
  if (np_) MCS_HIP_CHECK(hipMemcpy(pr.data(), opt.d.pr, 8 * (size_t)np_, hipMemcpyDeviceToHost));
  for (int q = 0; q < np_; q++) bad += ((int)pr[q].x != h.pr_e1[q]) + ((int)pr[q].y != h.pr_e2[q]);
  bad += nitem != (int32_t)h.it_blk.size();
  if (!bad && nitem > 0) {
    std::vector<int32_t> v(nitem);
    const int32_t* src[4] = {opt.d.it_blk, opt.d.it_chunk, opt.d.it_slot, opt.it_nch_dev};
    const std::vector<int32_t>* ref[4] = {&h.it_blk, &h.it_chunk, &h.it_slot, &h.it_nch};
    for (int k = 0; k < 4; k++) {
      MCS_HIP_CHECK(hipMemcpy(v.data(), src[k], 4 * (size_t)nitem, hipMemcpyDeviceToHost));
      for (int i = 0; i < nitem; i++) bad += v[i] != (*ref[k])[i];
    }
  }
  return (int)std::min<int64_t>(bad, INT32_MAX);
}

int mcs_ba_read_host_timing(mcs_ba_ctx* c, double* ms, int32_t* n_calls, int32_t reset) {
  if (!c) return MCS_ERR_ARG;
  for (int k = 0; k < MCS_BA_NHOST; k++) if (ms) ms[k] = c->host_ms[k];
  if (n_calls) *n_calls = c->host_calls;
  if (reset) {
    for (double& v : c->host_ms) v = 0.0;
    c->host_calls = 0;
  }
  return MCS_OK;
}

int mcs_ba_optimize(mcs_ba_ctx* c, const mcs_ba_problem* p, const mcs_ba_options* o,
                    double* poses, double* points, const uint8_t* edge_level, double* edge_chi2,
                    volatile int32_t* stop_flag, mcs_ba_report* rep) {
  return optimize_impl(c, p, o, poses, points, edge_level, edge_chi2, stop_flag, rep, nullptr, false);
}

int64_t mcs_ba_xchg_doubles(int32_t n_poses) { return xchg_doubles(n_poses); }

int mcs_ba_optimize_sharded(mcs_ba_ctx* c, const mcs_ba_problem* p, const mcs_ba_options* o,
                            double* poses, double* points, const uint8_t* edge_level,
                            double* edge_chi2, volatile int32_t* stop_flag, mcs_ba_report* rep,
                            const mcs_ba_shard* shard) {
  return optimize_impl(c, p, o, poses, points, edge_level, edge_chi2, stop_flag, rep, shard, false);
}

int mcs_global_ba(mcs_ba_ctx* c, const mcs_ba_problem* p, int32_t pose_only, double* poses,
                  double* points, volatile int32_t* stop_flag, mcs_ba_report* rep,
                  const mcs_ba_shard* shard) {
  mcs_ba_options o;
  mcs_ba_default_options(&o);
  o.max_iterations = 15;   // optimizer.optimize(15) (src/cOptimizer.cpp:241)
  return optimize_impl(c, p, &o, poses, points, nullptr, nullptr, stop_flag, rep, shard, pose_only != 0);
}

int mcs_local_ba_ex(mcs_ba_ctx* c, const mcs_ba_problem* p, const int32_t* point_extra_obs,
                    double* poses, double* points, uint8_t* edge_inlier, uint8_t* point_write,
                    int32_t* write_back, volatile int32_t* stop_flag, mcs_ba_report* r1,
                    mcs_ba_report* r2) {
  if (!c || !p || !poses || !points || !edge_inlier || !write_back) return MCS_ERR_ARG;
  mcs_ba_options o;
  mcs_ba_default_options(&o);
  const double huberK2 = p->huber_delta * p->huber_delta;
  std::vector<uint8_t> level(p->n_edges, 0);
  std::vector<double> chi(p->n_edges);
  // cMapPoint bookkeeping: observations left (good-keyframe edges + observations from bad
  // keyframes) and the bad flag EraseObservation raises below two (src/cMapPoint.cpp:120-152)
  std::vector<int32_t> obs_left(p->n_points, 0), edges_left(p->n_points, 0);
  std::vector<uint8_t> pt_bad(p->n_points, 0);
  for (int e = 0; e < p->n_edges; e++) edges_left[p->edge_point[e]]++;
  for (int i = 0; i < p->n_points; i++)
    obs_left[i] = edges_left[i] + (point_extra_obs ? point_extra_obs[i] : 0);
  if (point_write) std::memset(point_write, 0, (size_t)p->n_points);
  // pbStopFlag == NULL: the terminate action raises its own auxiliary flag and g2o keeps it
  // installed as the force-stop flag, so a round 1 that converged leaves round 2 with zero
  // iterations (sparse_optimizer_terminate_action.cpp:64-72, sparse_optimizer.cpp:376)
  volatile int32_t aux = 0;
  volatile int32_t* sf = stop_flag ? stop_flag : &aux;
  mcs_ba_report t1{}, t2{};
  if (!r1) r1 = &t1;
  if (!r2) r2 = &t2;
  *write_back = 0;
  for (int e = 0; e < p->n_edges; e++) edge_inlier[e] = 1;
  if (stop_flag && *stop_flag) return MCS_OK;               // :771-773
  // culling pass (:798-817, :830-849): edges in vpEdges order, a bad point's edges skipped
  auto cull = [&](bool disable) {
    for (int e = 0; e < p->n_edges; e++) {
      const int pt = p->edge_point[e];
      if (!edge_inlier[e] || pt_bad[pt] || !(chi[e] > huberK2)) continue;
      edge_inlier[e] = 0;
      if (disable) level[e] = 1;
      edges_left[pt]--;
      if (--obs_left[pt] < 2) pt_bad[pt] = 1;
    }
  };
  o.max_iterations = 10;
  // round 1 builds the structure and uploads the problem; round 2 (the same graph with the
  // culled edges at level 1) reuses both (Optimizer::remask) unless a pose left the system
  Optimizer opt(c, p, false);
  if (opt.device_driven(&o, r1) && opt.device_driven(&o, r2)) {
    // The culling passes run on the device between and after the rounds (k_lba_cull): round 2
    // follows round 1 without a download, and only the results come back.
    opt.lba = true;
    opt.lba_extra = point_extra_obs;
    int rc = opt.setup(poses, points, level.data(), nullptr);
    if (rc) return rc;
    opt.lba_tail = 1;
    rc = opt.run(&o, poses, points, nullptr, sf, r1);
    if (rc) return rc;
    if (r1->n_active_poses + r1->n_active_points == 0) return MCS_OK;   // :784-788 (nothing moved)
    if (stop_flag && *stop_flag) return opt.fetch_state(poses, points);   // bDoMore = false (:790-794)
    o.max_iterations = 15;                                    // :819-820
    if (opt.lba_res[1]) {
      // an active pose lost every edge: g2o's initializeOptimization drops it from the system, so
      // round 2 rebuilds from scratch on the host's copy of round 1's state
      std::vector<int32_t> obs_d(p->n_points), el_d(p->n_points);
      if ((rc = opt.lba_fetch(poses, points, level.data(), edge_inlier, obs_d.data(), el_d.data(), pt_bad.data())))
        return rc;
      for (int i = 0; i < p->n_points; i++)
        if (edges_left[i] > 0) { obs_left[i] = obs_d[i]; edges_left[i] = el_d[i]; }
      rc = mcs_ba_optimize(c, p, &o, poses, points, level.data(), chi.data(), sf, r2);
      if (rc) return rc;
      if (r2->n_active_poses + r2->n_active_points == 0) return MCS_OK;
      cull(false);
    } else {
      opt.remask_device();
      // round 2's report counts (run_device) decide whether the final culling runs (:822-826)
      const bool empty2 = (opt.s.np + opt.nl_glob) == 0;
      opt.lba_tail = empty2 ? 3 : 2;
      opt.lba_inlier_out = edge_inlier;
      opt.lba_pwrite_out = empty2 ? nullptr : point_write;
      rc = opt.run(&o, poses, points, nullptr, sf, r2);
      if (rc) return rc;
      if (r2->n_active_poses + r2->n_active_points == 0) return MCS_OK;   // :822-826
      *write_back = 1;
      return MCS_OK;
    }
    *write_back = 1;
    if (point_write) {
      std::vector<int32_t> edges_all(p->n_points, 0);
      for (int e = 0; e < p->n_edges; e++) edges_all[p->edge_point[e]]++;
      for (int i = 0; i < p->n_points; i++)
        point_write[i] = !pt_bad[i] && edges_left[i] > 1 && edges_all[i] >= 2;
    }
    return MCS_OK;
  }
  int rc = opt.setup(poses, points, level.data(), nullptr);
  if (rc) return rc;
  rc = opt.run(&o, poses, points, chi.data(), sf, r1);
  if (rc) return rc;
  // optimize() returns -1 == OptimizationAlgorithm::Fail only for an empty active graph
  if (r1->n_active_poses + r1->n_active_points == 0) return MCS_OK;   // :784-788
  if (stop_flag && *stop_flag) return MCS_OK;               // bDoMore = false (:790-794)
  {
    HostClock hc;
    cull(true);
    hc.mark(c->host_ms, 4);
  }
  o.max_iterations = 15;                                    // :819-820
  rc = opt.remask(level.data());
  if (rc < 0) return rc;
  if (rc == 0) rc = opt.run(&o, poses, points, chi.data(), sf, r2);
  else rc = mcs_ba_optimize(c, p, &o, poses, points, level.data(), chi.data(), sf, r2);
  if (rc) return rc;
  if (r2->n_active_poses + r2->n_active_points == 0) return MCS_OK;   // :822-826
  cull(false);
  *write_back = 1;
  if (point_write) {   // :885-902: not bad, TotalNrObservations() > 1, >= 2 vertex edges
    std::vector<int32_t> edges_all(p->n_points, 0);
    for (int e = 0; e < p->n_edges; e++) edges_all[p->edge_point[e]]++;
    for (int i = 0; i < p->n_points; i++)
      point_write[i] = !pt_bad[i] && edges_left[i] > 1 && edges_all[i] >= 2;
  }
  return MCS_OK;
}

int mcs_local_ba(mcs_ba_ctx* c, const mcs_ba_problem* p, double* poses, double* points,
                 uint8_t* edge_inlier, int32_t* write_back, volatile int32_t* stop_flag,
                 mcs_ba_report* r1, mcs_ba_report* r2) {
  return mcs_local_ba_ex(c, p, nullptr, poses, points, edge_inlier, nullptr, write_back, stop_flag,
                         r1, r2);
}

int mcs_pose_optimization(mcs_ba_ctx* c, const mcs_ba_problem* p, double* pose, uint8_t* outlier,
                          int32_t* n_good, double* bad_ratio, mcs_ba_report* r1, mcs_ba_report* r2) {
  if (!c || !p || !pose || !n_good || (p->n_edges > 0 && !outlier)) return MCS_ERR_ARG;
  if (p->n_poses != 1) {
    set_error("PoseOptimization: the problem must hold exactly one pose vertex");
    return MCS_ERR_ARG;
  }
  mcs_ba_problem q = *p;
  const uint8_t not_fixed = 0;
  q.pose_fixed = &not_fixed;                                // vSE3->setFixed(false) (:299)
  mcs_ba_options o;
  mcs_ba_default_options(&o);                               // gain 1e-6, max 15 (:290-291)
  o.max_iterations = 10;                                    // optimize(10) (:434, :457)
  const double th2 = p->huber_delta * p->huber_delta;      // thHuber = 1.345 * mult (:344)
  const int N = p->n_edges;
  std::vector<uint8_t> level(N, 0);
  std::vector<double> chi(N), pts(p->points, p->points + 3 * (size_t)p->n_points);
  // no setForceStopFlag: the terminate action's own flag is shared by both optimize() calls
  volatile int32_t aux = 0;
  mcs_ba_report t1{}, t2{};
  int rc = optimize_impl(c, &q, &o, pose, pts.data(), level.data(), chi.data(), &aux,
                         r1 ? r1 : &t1, nullptr, true);    // map points fixed (:382)
  if (rc) return rc;
  int nBad = 0;
  for (int e = 0; e < N; e++) {                             // :439-454
    if (chi[e] > th2) { outlier[e] = 1; level[e] = 1; nBad++; }
    else outlier[e] = 0;
  }
  rc = optimize_impl(c, &q, &o, pose, pts.data(), level.data(), chi.data(), &aux,
                     r2 ? r2 : &t2, nullptr, true);
  if (rc) return rc;
  for (int e = 0; e < N; e++) {                             // :460-474
    if (level[e]) continue;
    if (chi[e] > th2) { outlier[e] = 1; nBad++; }
    else outlier[e] = 0;
  }
  *n_good = N - nBad;                                       // return value (:485)
  if (bad_ratio) *bad_ratio = N > 0 ? (double)nBad / N : 0.0;   // `inliers` (:481-483)
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
  d.delta = p->huber_delta; d.dsqr = huber_dsqr(p->huber_delta);
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

int mcs_ba_lm_replay(int32_t device, const mcs_ba_options* o, const double* in3, const double* trials,
                     int32_t n, double* out, int32_t* n_out) {
  if (!o || !in3 || (n > 0 && (!trials || !out)) || !n_out || n < 0) {
    set_error("lm_replay: null argument or n < 0");
    return MCS_ERR_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  MCS_HIP_CHECK(hipSetDevice(device));
  LmCtl h0;
  std::memset(&h0, 0, sizeof(h0));
  h0.tau = o->tau; h0.gain_threshold = o->gain_threshold;      // as run_device sets them
  h0.max_iterations = o->max_iterations; h0.max_trials = o->max_trials;
  h0.terminate_max_iter = o->terminate_max_iter;
  h0.lin = 1; h0.ni = 2;
  h0.done = o->max_iterations <= 0 ? 1 : 0;
  LmCtl* dc = nullptr; LmSig* ds = nullptr; double *din = nullptr, *dtr = nullptr, *dout = nullptr; int* dn = nullptr;
  int rc = MCS_OK;
  auto chk = [&](hipError_t e, const char* w) { if (e != hipSuccess && rc == MCS_OK) { set_hip_error(e, w, __FILE__, __LINE__); rc = MCS_ERR_HIP; } };
  chk(hipMalloc(&dc, sizeof(LmCtl)), "malloc"); chk(hipMalloc(&ds, sizeof(LmSig)), "malloc");
  chk(hipMalloc(&din, 3 * 8), "malloc"); chk(hipMalloc(&dtr, std::max(1, n) * 32), "malloc");
  chk(hipMalloc(&dout, std::max(1, n) * 80), "malloc"); chk(hipMalloc(&dn, 4), "malloc");
  if (rc == MCS_OK) {
    chk(hipMemcpy(dc, &h0, sizeof(h0), hipMemcpyHostToDevice), "h2d");
    chk(hipMemset(ds, 0, sizeof(LmSig)), "memset");
    chk(hipMemcpy(din, in3, 3 * 8, hipMemcpyHostToDevice), "h2d");
    if (n) chk(hipMemcpy(dtr, trials, (size_t)n * 32, hipMemcpyHostToDevice), "h2d");
    chk(hipMemset(dn, 0, 4), "memset");
    hipLaunchKernelGGL(k_lm_replay, dim3(1), dim3(64), 0, 0, dc, ds, (const double*)din, (const double*)dtr, n, dout, dn);
    chk(hipGetLastError(), "launch");
    chk(hipDeviceSynchronize(), "sync");
    int32_t m = 0;
    chk(hipMemcpy(&m, dn, 4, hipMemcpyDeviceToHost), "d2h");
    if (rc == MCS_OK && m) chk(hipMemcpy(out, dout, (size_t)m * 80, hipMemcpyDeviceToHost), "d2h");
    *n_out = m;
  }
  for (void* q : {(void*)dc, (void*)ds, (void*)din, (void*)dtr, (void*)dout, (void*)dn})
    if (q) (void)hipFree(q);
  return rc;
}

int mcs_ba_huber_eval(int32_t device, const double* e, int32_t n, double delta, double* rho0, double* rho1) {
  if (n < 0 || (n > 0 && (!e || !rho0 || !rho1))) {
    set_error("huber_eval: null argument or n < 0");
    return MCS_ERR_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  if (n == 0) return MCS_OK;
  MCS_HIP_CHECK(hipSetDevice(device));
  double *de = nullptr, *d0 = nullptr, *d1 = nullptr;
  int rc = MCS_OK;
  auto chk = [&](hipError_t x, const char* w) { if (x != hipSuccess && rc == MCS_OK) { set_hip_error(x, w, __FILE__, __LINE__); rc = MCS_ERR_HIP; } };
  chk(hipMalloc(&de, (size_t)n * 8), "malloc"); chk(hipMalloc(&d0, (size_t)n * 8), "malloc");
  chk(hipMalloc(&d1, (size_t)n * 8), "malloc");
  if (rc == MCS_OK) {
    chk(hipMemcpy(de, e, (size_t)n * 8, hipMemcpyHostToDevice), "h2d");
    hipLaunchKernelGGL(k_huber_eval, dim3((n + 255) / 256), dim3(256), 0, 0, (const double*)de, n, delta,
                       huber_dsqr(delta), d0, d1);
    chk(hipGetLastError(), "launch");
    chk(hipMemcpy(rho0, d0, (size_t)n * 8, hipMemcpyDeviceToHost), "d2h");
    chk(hipMemcpy(rho1, d1, (size_t)n * 8, hipMemcpyDeviceToHost), "d2h");
  }
  for (void* q : {(void*)de, (void*)d0, (void*)d1})
    if (q) (void)hipFree(q);
  return rc;
}

int mcs_ba_point_block_eval(int32_t device, const double* H, double lambda, const double* b, const double* hpl,
                            int32_t n, double* Dinv, double* db, double* Y) {
  if (n < 0 || (n > 0 && (!H || !b || !hpl || !Dinv || !db || !Y))) {
    set_error("point_block_eval: null argument or n < 0");
    return MCS_ERR_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  if (n == 0) return MCS_OK;
  MCS_HIP_CHECK(hipSetDevice(device));
  double* dv = nullptr;
  const size_t N = (size_t)n, tot = N * (9 + 3 + 18 + 9 + 3 + 18);
  int rc = MCS_OK;
  auto chk = [&](hipError_t x, const char* w) { if (x != hipSuccess && rc == MCS_OK) { set_hip_error(x, w, __FILE__, __LINE__); rc = MCS_ERR_HIP; } };
  chk(hipMalloc(&dv, tot * 8), "malloc");
  if (rc == MCS_OK) {
    double *dH = dv, *dB = dH + 9 * N, *dP = dB + 3 * N, *dDi = dP + 18 * N, *dDb = dDi + 9 * N, *dY = dDb + 3 * N;
    chk(hipMemcpy(dH, H, 9 * N * 8, hipMemcpyHostToDevice), "h2d");
    chk(hipMemcpy(dB, b, 3 * N * 8, hipMemcpyHostToDevice), "h2d");
    chk(hipMemcpy(dP, hpl, 18 * N * 8, hipMemcpyHostToDevice), "h2d");
    if (rc == MCS_OK)
      hipLaunchKernelGGL(k_point_block_eval, dim3((n + 255) / 256), dim3(256), 0, 0, (const double*)dH, lambda,
                         (const double*)dB, (const double*)dP, n, dDi, dDb, dY);
    chk(hipGetLastError(), "launch");
    chk(hipMemcpy(Dinv, dDi, 9 * N * 8, hipMemcpyDeviceToHost), "d2h");
    chk(hipMemcpy(db, dDb, 3 * N * 8, hipMemcpyDeviceToHost), "d2h");
    chk(hipMemcpy(Y, dY, 18 * N * 8, hipMemcpyDeviceToHost), "d2h");
  }
  if (dv) (void)hipFree(dv);
  return rc;
}

int mcs_ldlt_set_wait_ticks(int64_t ticks) {
  ldlt::set_wait_ticks((long long)ticks);
  return MCS_OK;
}

int mcs_dense_ldlt_solve(int32_t device, const double* S, int32_t n, const double* b, double* x,
                         int32_t* zero_pivot) {
  return mcs_dense_ldlt_solve_ex(device, S, n, b, x, zero_pivot, 0);
}

int mcs_dense_ldlt_solve_ex(int32_t device, const double* S, int32_t n, const double* b, double* x,
                            int32_t* zero_pivot, int32_t path) {
  if (!S || !b || !x || n < 1 || path < 0 || path > 3) return MCS_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  MCS_HIP_CHECK(hipSetDevice(device));
  const int T = ldlt::tiles_for(n);
  const size_t NT = ldlt::tile_doubles(T), Np = (size_t)ldlt::TB * T;
  // path 0: the tile band of S (the widest tile diagonal holding a non-zero), as the BA derives
  // it from its structure; the other paths factor densely
  int band = T;
  if (path == 0 && T > 1) {
    int w = 1;
    for (int r = 0; r < n; r++)
      for (int c = 0; c < r; c++)
        if (S[(size_t)r * n + c] != 0.0) { w = std::max(w, r / ldlt::TB - c / ldlt::TB); break; }
    band = ldlt::pipe_band(T, w + 1);
  }
  const bool pipelined = path != 3 && T >= 2 && ldlt::pipe_supported(T, band);
  if (!pipelined && T > 1 && (size_t)T * ldlt::TB * 8 > 96 * 1024) return MCS_ERR_UNSUPPORTED;
  std::vector<double> hA(NT, 0.0), hb(Np, 0.0);
  for (int r = 0; r < n; r++)
    for (int c = 0; c <= r; c++) hA[ldlt::sidx(r, c, T)] = S[(size_t)r * n + c];
  for (int r = 0; r < n; r++) hb[r] = b[r];
  double *dA = nullptr, *db = nullptr, *dx = nullptr, *dL = nullptr, *dI = nullptr, *dz = nullptr;
  int* dflag = nullptr;
  hipStream_t st = nullptr;
  int rc = MCS_OK;
  auto chk = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && rc == MCS_OK) { set_hip_error(e, what, __FILE__, __LINE__); rc = MCS_ERR_HIP; }
  };
  chk(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
  chk(hipMalloc(&dA, NT * 8), "malloc"); chk(hipMalloc(&dL, NT * 8), "malloc");
  chk(hipMalloc(&dI, (size_t)T * 4096 * 8), "malloc");
  chk(hipMalloc(&db, Np * 8), "malloc"); chk(hipMalloc(&dx, Np * 8), "malloc"); chk(hipMalloc(&dz, Np * 8), "malloc");
  chk(hipMalloc(&dflag, 16), "malloc");
  if (rc == MCS_OK) {
    chk(hipMemcpyAsync(dA, hA.data(), NT * 8, hipMemcpyHostToDevice, st), "h2d");
    chk(hipMemcpyAsync(db, hb.data(), Np * 8, hipMemcpyHostToDevice, st), "h2d");
    chk(hipMemsetAsync(dflag, 0, 4, st), "memset");
    if (T == 1 && path == 0) {
      chk(ldlt::solve_one_tile(dA, db, dx, n, 1.0, dflag, st), "ldlt");
    } else {
      chk(ldlt::pad(dA, db, n, T, 1.0, st), "pad");
      ldlt::Work w{dL, dI, dz};
      // path 0 (banded) and 2 (dense): the pipelined factorisation (one launch); path 1: one
      // launch per step; all with the multi-workgroup backward substitution.  Path 3, and a
      // system the pipeline does not take (as in the BA): one launch per step + the
      // one-workgroup backward substitution, without the pipeline's sync words.
      if (rc == MCS_OK && pipelined) chk(ldlt::pipe_prepare(w, T, st, path == 0 ? band : 0), "pipe_prepare");
      w.per_step = (path == 1);
      chk(ldlt::solve(dA, db, dx, T, w, dflag, st), "ldlt");
      chk(hipStreamSynchronize(st), "sync");
      ldlt::pipe_release(w);
    }
    std::vector<double> hx(Np);
    int32_t fl = 0;
    chk(hipMemcpyAsync(hx.data(), dx, Np * 8, hipMemcpyDeviceToHost, st), "d2h");
    chk(hipMemcpyAsync(&fl, dflag, 4, hipMemcpyDeviceToHost, st), "d2h");
    chk(hipStreamSynchronize(st), "sync");
    for (int r = 0; r < n; r++) x[r] = hx[r];
    if (rc == MCS_OK && (fl & ldlt::kFlagTimeout)) {
      set_error("dense LDL^T: a hand-off wait of the pipelined solve timed out; x discarded");
      rc = MCS_ERR_HIP;
    }
    if (zero_pivot) *zero_pivot = fl & ldlt::kFlagZeroPivot;
  }
  for (void* q : {(void*)dA, (void*)dL, (void*)dI, (void*)db, (void*)dx, (void*)dz, (void*)dflag})
    if (q) (void)hipFree(q);
  if (st) (void)hipStreamDestroy(st);
  return rc;
}

}  // extern "C"
