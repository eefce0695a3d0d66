// cMultiFrame work around the extractor on the device (C-ABI of include/mcs_frame.h): bearing
// rays (ImgToWorld), the camera concatenation with PosInGrid, and isInFrustum.
//
// Reference: cMultiFrame::cMultiFrame src/cMultiFrame.cpp:128-184, PosInGrid :342-353,
// isInFrustum :218-270; cCamModelGeneral_::ImgToWorld src/cam_model_omni.cpp:49-67,
// WorldToImg :147-163, isPointInMirrorMask :165-180; cMultiCamSys_::WorldToCamHom_fast
// src/cam_system_omni.cpp:92-112, Get_MtMc include/cam_system_omni.h:162-168;
// cayley2rot include/misc.h:134-162, cConverter::invMat src/cConverter.cpp:31-44.
// Compiled with -ffp-contract=off; double ops spelled with _rn intrinsics where an FMA could
// otherwise be formed, so every rounding follows the reference's expression order.
#include "common.hpp"
#include "../../include/mcs_frame.h"

namespace mcs {
namespace frm {

constexpr int kGridCols = 64, kGridRows = 48;   // FRAME_GRID_COLS / ROWS (include/cMultiFrame.h:47-48)

__device__ __forceinline__ double horner_n(const double* c, int s, double x) {   // misc.h:117-124
  double r = 0.0;
  for (int i = s - 1; i >= 0; i--) r = __dadd_rn(__dmul_rn(r, x), c[i]);
  return r;
}

// ImgToWorld (cam_model_omni.cpp:49-67)
__device__ void img_to_world(const mcs_cam_model& m, double u, double v, double* X) {
  const double invAffine = __dsub_rn(m.c, __dmul_rn(m.d, m.e));
  const double u_t = __dsub_rn(u, m.u0), v_t = __dsub_rn(v, m.v0);
  double x = __ddiv_rn(__dsub_rn(u_t, __dmul_rn(m.d, v_t)), invAffine);
  double y = __ddiv_rn(__dadd_rn(__dmul_rn(-m.e, u_t), __dmul_rn(m.c, v_t)), invAffine);
  const double X2 = __dmul_rn(x, x), Y2 = __dmul_rn(y, y);
  double z = -horner_n(m.p, m.p_deg, __dsqrt_rn(__dadd_rn(X2, Y2)));
  const double norm = __dsqrt_rn(__dadd_rn(__dadd_rn(X2, Y2), __dmul_rn(z, z)));
  X[0] = __ddiv_rn(x, norm); X[1] = __ddiv_rn(y, norm); X[2] = __ddiv_rn(z, norm);
}

// cayley2rot (misc.h:134-162): R = (1 / scale) * R
__device__ void cay2rot(const double* c, double* R) {
  const double c1 = c[0], c2 = c[1], c3 = c[2];
  const double c1s = __dmul_rn(c1, c1), c2s = __dmul_rn(c2, c2), c3s = __dmul_rn(c3, c3);
  const double scale = __dadd_rn(__dadd_rn(__dadd_rn(1.0, c1s), c2s), c3s);
  const double inv = __ddiv_rn(1.0, scale);
  R[0] = __dmul_rn(inv, __dsub_rn(__dsub_rn(__dadd_rn(1.0, c1s), c2s), c3s));
  R[1] = __dmul_rn(inv, __dmul_rn(2.0, __dsub_rn(__dmul_rn(c1, c2), c3)));
  R[2] = __dmul_rn(inv, __dmul_rn(2.0, __dadd_rn(__dmul_rn(c1, c3), c2)));
  R[3] = __dmul_rn(inv, __dmul_rn(2.0, __dadd_rn(__dmul_rn(c1, c2), c3)));
  R[4] = __dmul_rn(inv, __dsub_rn(__dadd_rn(__dsub_rn(1.0, c1s), c2s), c3s));
  R[5] = __dmul_rn(inv, __dmul_rn(2.0, __dsub_rn(__dmul_rn(c2, c3), c1)));
  R[6] = __dmul_rn(inv, __dmul_rn(2.0, __dsub_rn(__dmul_rn(c1, c3), c2)));
  R[7] = __dmul_rn(inv, __dmul_rn(2.0, __dadd_rn(__dmul_rn(c2, c3), c1)));
  R[8] = __dmul_rn(inv, __dadd_rn(__dsub_rn(__dsub_rn(1.0, c1s), c2s), c3s));
}

// M = M_t * M_c as 4x4 products (Matx sum over k = 0..3 left to right): R [9], t [3]
__device__ void mtmc(const double* pose, const double* mc, double* R, double* t) {
  double Rt[9], Rc[9];
  cay2rot(pose, Rt);
  cay2rot(mc, Rc);
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) {
      double s = __dmul_rn(Rt[3 * i], Rc[j]);
      s = __dadd_rn(s, __dmul_rn(Rt[3 * i + 1], Rc[3 + j]));
      s = __dadd_rn(s, __dmul_rn(Rt[3 * i + 2], Rc[6 + j]));
      s = __dadd_rn(s, __dmul_rn(pose[3 + i], 0.0));
      R[3 * i + j] = s;
    }
    double s = __dmul_rn(Rt[3 * i], mc[3]);
    s = __dadd_rn(s, __dmul_rn(Rt[3 * i + 1], mc[4]));
    s = __dadd_rn(s, __dmul_rn(Rt[3 * i + 2], mc[5]));
    s = __dadd_rn(s, __dmul_rn(pose[3 + i], 1.0));
    t[i] = s;
  }
}

// WorldToCamHom_fast (cam_system_omni.cpp:92-112): invMat(M_t M_c) * [X 1], then WorldToImg
__device__ void world_to_cam_img(const double* R, const double* t, const double* cam,
                                 const double* X, double& u, double& v) {
  double ti[3];   // invMat: R' = R^T, t' = -R' t (cConverter.cpp:31-44)
  for (int i = 0; i < 3; i++) {
    double s = __dmul_rn(-R[i], t[0]);
    s = __dadd_rn(s, __dmul_rn(-R[3 + i], t[1]));
    s = __dadd_rn(s, __dmul_rn(-R[6 + i], t[2]));
    ti[i] = s;
  }
  double Xc[3];
  for (int i = 0; i < 3; i++) {
    double s = __dmul_rn(R[i], X[0]);
    s = __dadd_rn(s, __dmul_rn(R[3 + i], X[1]));
    s = __dadd_rn(s, __dmul_rn(R[6 + i], X[2]));
    s = __dadd_rn(s, __dmul_rn(ti[i], 1.0));
    Xc[i] = s;
  }
  const double x = Xc[0], y = Xc[1], z = Xc[2];   // WorldToImg (cam_model_omni.cpp:147-163)
  double norm = __dsqrt_rn(__dadd_rn(__dmul_rn(x, x), __dmul_rn(y, y)));
  if (norm == 0.0) norm = 1e-14;
  const double theta = atan(__ddiv_rn(-z, norm));
  const double rho = horner_n(cam + 5, 12, theta);
  const double uu = __dmul_rn(__ddiv_rn(x, norm), rho), vv = __dmul_rn(__ddiv_rn(y, norm), rho);
  u = __dadd_rn(__dadd_rn(__dmul_rn(uu, cam[0]), __dmul_rn(vv, cam[1])), cam[3]);
  v = __dadd_rn(__dadd_rn(__dmul_rn(uu, cam[2]), vv), cam[4]);
}

__global__ __launch_bounds__(256) void k_keypoint_rays(const mcs_keypoint* __restrict__ kps,
                                                       const int32_t* __restrict__ counts, int F,
                                                       int cap, const int32_t* __restrict__ cam_index,
                                                       const mcs_cam_model* __restrict__ cams,
                                                       double* __restrict__ rays) {
  const int f = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F || i >= counts[f]) return;
  const mcs_keypoint kp = kps[(int64_t)f * cap + i];
  const mcs_cam_model& m = cams[cam_index ? cam_index[f] : 0];
  double X[3];
  img_to_world(m, (double)kp.x, (double)kp.y, X);
  double* o = rays + ((int64_t)f * cap + i) * 3;
  o[0] = X[0]; o[1] = X[1]; o[2] = X[2];
}

// one workgroup per multi-frame: camera prefix offsets, then every keypoint slot of every camera
__global__ __launch_bounds__(256) void k_mf_concat(const int32_t* __restrict__ counts, int C, int cap,
                                                   const mcs_keypoint* __restrict__ kps,
                                                   const double* __restrict__ rays,
                                                   const uint8_t* __restrict__ desc, int B,
                                                   const double* __restrict__ gp,
                                                   mcs_keypoint* __restrict__ keys,
                                                   double* __restrict__ keys_rays,
                                                   uint8_t* __restrict__ descs,
                                                   int32_t* __restrict__ k2c, int32_t* __restrict__ k2l,
                                                   int32_t* __restrict__ grid, int32_t* __restrict__ total) {
  const int m = blockIdx.x;
  const int64_t in0 = (int64_t)m * C * cap, out0 = (int64_t)m * C * cap;
  int off = 0;
  for (int c = 0; c < C; c++) {
    const int n = counts[(int64_t)m * C + c];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int64_t src = in0 + (int64_t)c * cap + i, dst = out0 + off + i;
      const mcs_keypoint kp = kps[src];
      keys[dst] = kp;
      k2c[dst] = c;
      k2l[dst] = i;
      if (rays && keys_rays)
        for (int k = 0; k < 3; k++) keys_rays[dst * 3 + k] = rays[src * 3 + k];
      if (desc && descs)
        for (int k = 0; k < B; k++) descs[dst * B + k] = desc[src * B + k];
      if (grid) {   // PosInGrid: cvRound((kp.pt.x - mnMinX) * mfGridElementWidthInv)
        const double* g = gp + 4 * c;
        const int px = (int)rint(__dmul_rn(__dsub_rn((double)kp.x, g[0]), g[2]));
        const int py = (int)rint(__dmul_rn(__dsub_rn((double)kp.y, g[1]), g[3]));
        grid[dst] = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : (px | (py << 8));
      }
    }
    off += n;
  }
  if (threadIdx.x == 0) total[m] = off;
}

__global__ __launch_bounds__(256) void k_in_frustum(const double* __restrict__ pose,
                                                    const double* __restrict__ mc,
                                                    const double* __restrict__ camv, int C,
                                                    const uint8_t* __restrict__ masks, int mw,
                                                    int mh, const double* __restrict__ pts,
                                                    const double* __restrict__ nrm,
                                                    const double* __restrict__ dist, int n,
                                                    const double* __restrict__ scale, int L,
                                                    uint8_t* __restrict__ in_view,
                                                    double* __restrict__ proj,
                                                    int32_t* __restrict__ level,
                                                    double* __restrict__ view_cos) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)n * C) return;
  const int p = (int)(q / C), c = (int)(q - (int64_t)p * C);
  in_view[q] = 0;   // pMP->mbTrackInView[cam] = false
  double R[9], t[3];
  mtmc(pose, mc + 6 * c, R, t);
  const double* P = pts + 3 * (int64_t)p;
  double u, v;
  world_to_cam_img(R, t, camv + 17 * c, P, u, v);
  // isPointInMirrorMask(u, v, 0): cvRound, bounds (> 0 and < size), mask > 0
  const int ur = (int)rint(u), vr = (int)rint(v);
  if (ur >= mw || ur <= 0 || vr >= mh || vr <= 0) return;
  if (masks[(int64_t)c * mw * mh + (int64_t)vr * mw + ur] == 0) return;
  // distance to the camera centre (Get_MtMc translation) inside the invariance region
  const double maxD = __dmul_rn(1.2, dist[2 * (int64_t)p + 1]);
  const double minD = __dmul_rn(0.8, dist[2 * (int64_t)p]);
  const double PO[3] = {__dsub_rn(P[0], t[0]), __dsub_rn(P[1], t[1]), __dsub_rn(P[2], t[2])};
  const double d = __dsqrt_rn(__dadd_rn(__dadd_rn(__dmul_rn(PO[0], PO[0]), __dmul_rn(PO[1], PO[1])),
                                        __dmul_rn(PO[2], PO[2])));
  if (d < minD || d > maxD) return;
  const double* Pn = nrm + 3 * (int64_t)p;
  const double vc = __ddiv_rn(__dadd_rn(__dadd_rn(__dmul_rn(PO[0], Pn[0]), __dmul_rn(PO[1], Pn[1])),
                                        __dmul_rn(PO[2], Pn[2])), d);
  // nPredictedLevel = lower_bound(mvScaleFactors, dist / minDistance), capped
  const double ratio = __ddiv_rn(d, minD);
  int lv = 0;
  while (lv < L && scale[lv] < ratio) lv++;
  if (lv >= L) lv = L - 1;
  in_view[q] = 1;
  proj[2 * q] = u;
  proj[2 * q + 1] = v;
  level[q] = lv;
  view_cos[q] = vc;
}

}  // namespace frm
}  // namespace mcs

using namespace mcs;

extern "C" {

int mcs_keypoint_rays_device(const mcs_keypoint* d_kps, const int32_t* d_counts, int32_t n_frames,
                             int32_t cap, const int32_t* d_cam_index, const mcs_cam_model* d_cams,
                             double* d_rays, void* stream) {
  if (n_frames < 0 || cap < 0 || (n_frames > 0 && (!d_kps || !d_counts || !d_cams || !d_rays))) {
    set_error("mcs_keypoint_rays_device: bad argument");
    return MCS_ERR_ARG;
  }
  if (n_frames == 0 || cap == 0) return MCS_OK;
  hipLaunchKernelGGL(frm::k_keypoint_rays, dim3((cap + 255) / 256, n_frames), dim3(256), 0,
                     (hipStream_t)stream, d_kps, d_counts, n_frames, cap, d_cam_index, d_cams, d_rays);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_multiframe_concat_device(const int32_t* d_counts, int32_t n_mf, int32_t n_cams, int32_t cap,
                                 const mcs_keypoint* d_kps, const double* d_rays,
                                 const uint8_t* d_desc, int32_t desc_bytes,
                                 const double* d_grid_params, mcs_keypoint* d_keys,
                                 double* d_keys_rays, uint8_t* d_descs, int32_t* d_kp_to_cam,
                                 int32_t* d_cont_to_local, int32_t* d_grid_pos, int32_t* d_total,
                                 void* stream) {
  if (n_mf < 0 || n_cams < 1 || cap < 0 || desc_bytes < 0 ||
      (n_mf > 0 && (!d_counts || !d_kps || !d_keys || !d_kp_to_cam || !d_cont_to_local || !d_total)) ||
      (d_grid_pos && !d_grid_params)) {
    set_error("mcs_multiframe_concat_device: bad argument");
    return MCS_ERR_ARG;
  }
  if (n_mf == 0) return MCS_OK;
  hipLaunchKernelGGL(frm::k_mf_concat, dim3(n_mf), dim3(256), 0, (hipStream_t)stream, d_counts,
                     n_cams, cap, d_kps, d_rays, d_desc, desc_bytes, d_grid_params, d_keys,
                     d_keys_rays, d_descs, d_kp_to_cam, d_cont_to_local, d_grid_pos, d_total);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_is_in_frustum_device(const double* d_pose, const double* d_mc, const double* d_cam,
                             int32_t n_cams, const uint8_t* d_masks, int32_t mask_w,
                             int32_t mask_h, const double* d_pts, const double* d_normals,
                             const double* d_dist, int32_t n, const double* d_scale,
                             int32_t n_levels, uint8_t* d_in_view, double* d_proj,
                             int32_t* d_level, double* d_view_cos, void* stream) {
  if (n < 0 || n_cams < 1 || n_levels < 1 || mask_w < 1 || mask_h < 1 ||
      (n > 0 && (!d_pose || !d_mc || !d_cam || !d_masks || !d_pts || !d_normals || !d_dist ||
                 !d_scale || !d_in_view || !d_proj || !d_level || !d_view_cos))) {
    set_error("mcs_is_in_frustum_device: bad argument");
    return MCS_ERR_ARG;
  }
  const int64_t q = (int64_t)n * n_cams;
  if (q == 0) return MCS_OK;
  hipLaunchKernelGGL(frm::k_in_frustum, dim3((unsigned)((q + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, d_pose, d_mc, d_cam, n_cams, d_masks, mask_w, mask_h,
                     d_pts, d_normals, d_dist, n, d_scale, n_levels, d_in_view, d_proj, d_level,
                     d_view_cos);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

}  // extern "C"
