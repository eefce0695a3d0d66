// Projection-guided (windowed) matching: the cMultiFrame feature grid on the host, then
// GetFeaturesInArea and the Hamming distance of every window candidate on the device, then the
// reference's sequential best / second-best selection rules on the host.
//
// Reference (billamiable/MultiCol-SLAM-Annotation):
//   grid build (part of the cMultiFrame ctor)            src/cMultiFrame.cpp:154-184
//   PosInGrid                                            src/cMultiFrame.cpp:342-353
//   GetFeaturesInArea                                    src/cMultiFrame.cpp:272-340
//   SearchByProjection(F, MPs)       (rule 0)            src/cORBmatcher.cpp:67-166
//   SearchByProjection(Cur, Last)    (rule 1)            src/cORBmatcher.cpp:1991-2123
//   SearchForInitialization          (rule 2)            src/cORBmatcher.cpp:579-726
//   WindowSearch                     (rule 3)            src/cORBmatcher.cpp:326-473
//   DescriptorDistance64[Masked]                         src/cORBmatcher.cpp:2443-2477
// checkOrientation is false in the reference (include/cORBmatcher.h:40), so no rotation
// histograms.  GetFeaturesInArea's abs(kp.pt.x - x) is the double overload (the operand is a
// double), i.e. fabs.
#include "common.hpp"
#include "../../include/mcs_matcher.h"
#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

namespace mcs {
namespace win {

constexpr int kCols = MCS_GRID_COLS, kRows = MCS_GRID_ROWS;
constexpr int kQPB = 4;   // queries (waves) per 256-thread workgroup

struct SearchArgs {
  const int32_t* cell_ptr; const int32_t* cell_kp; const double* gp; int n_cams;
  const float* kp_xy; const int32_t* kp_oct; const uint8_t* kp_desc; const uint8_t* kp_mask;
  int bytes; int nq;
  const double* q_xyr; const int32_t* q_cl; const uint8_t* q_desc; const uint8_t* q_mask;
  int32_t* cand_ptr; int32_t* cand_kp; int32_t* cand_dist;
};

// window cell range of GetFeaturesInArea (:280-298); false = empty window
__device__ __forceinline__ bool cell_range(const SearchArgs& a, int cam, double x, double y,
                                           double r, int* x0, int* x1, int* y0, int* y1) {
  const double mnx = a.gp[4 * cam], mny = a.gp[4 * cam + 1];
  const double wi = a.gp[4 * cam + 2], hi = a.gp[4 * cam + 3];
  int nx0 = (int)floor((x - mnx - r) * wi);
  nx0 = max(0, nx0);
  if (nx0 >= kCols) return false;
  int nx1 = (int)ceil((x - mnx + r) * wi);
  nx1 = min(kCols - 1, nx1);
  if (nx1 < 0) return false;
  int ny0 = (int)floor((y - mny - r) * hi);
  ny0 = max(0, ny0);
  if (ny0 >= kRows) return false;
  int ny1 = (int)ceil((y - mny + r) * hi);
  ny1 = min(kRows - 1, ny1);
  if (ny1 < 0) return false;
  *x0 = nx0; *x1 = nx1; *y0 = ny0; *y1 = ny1;
  return true;
}

// DescriptorDistance64 / ...Masked over 32-bit words (the masked total is halved once, as
// the reference does over its 64-bit words)
__device__ __forceinline__ int ham(const uint8_t* q, const uint8_t* t, const uint8_t* mq,
                                  const uint8_t* mt, int bytes) {
  const uint32_t* a = reinterpret_cast<const uint32_t*>(q);
  const uint32_t* b = reinterpret_cast<const uint32_t*>(t);
  int d = 0;
  if (!mq) {
    for (int w = 0; w < bytes / 4; w++) d += __popc(a[w] ^ b[w]);
    return d;
  }
  const uint32_t* ma = reinterpret_cast<const uint32_t*>(mq);
  const uint32_t* mb = reinterpret_cast<const uint32_t*>(mt);
  for (int w = 0; w < bytes / 4; w++) {
    const uint32_t x = a[w] ^ b[w];
    d += __popc(x & ma[w]) + __popc(x & mb[w]);
  }
  return d / 2;
}

// One wave per query.  The window's cells are taken 64 at a time, one per lane in the
// reference's loop order (ix outer, iy inner); a wave prefix sum over the cell sizes flattens
// their keypoints (insertion order within a cell), so a step costs two dependent loads for 64
// cells instead of a chain per cell.  Candidates passing the level and |dx|, |dy| <= r tests
// are compacted by ballot rank, which keeps the reference's order.
// COUNT: count only; else write (keypoint, distance) from cand_ptr[q].
template <bool COUNT>
__global__ __launch_bounds__(256) void k_window(SearchArgs a) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * kQPB + (threadIdx.x >> 6);
  if (q >= a.nq) return;
  const double x = a.q_xyr[3 * q], y = a.q_xyr[3 * q + 1], r = a.q_xyr[3 * q + 2];
  const int cam = a.q_cl[3 * q], minL = a.q_cl[3 * q + 1], maxL = a.q_cl[3 * q + 2];
  int cnt = 0;
  int x0, x1, y0, y1;
  if (cam >= 0 && cam < a.n_cams && cell_range(a, cam, x, y, r, &x0, &x1, &y0, &y1)) {
    const bool check = !(minL == -1 && maxL == -1);
    const bool same = check && (minL == maxL);
    const uint8_t* qd = a.q_desc + (int64_t)q * a.bytes;
    const uint8_t* qm = a.q_mask ? a.q_mask + (int64_t)q * a.bytes : nullptr;
    const int base = COUNT ? 0 : a.cand_ptr[q];
    const int ncy = y1 - y0 + 1, ncell = (x1 - x0 + 1) * ncy;
    for (int cb = 0; cb < ncell; cb += 64) {
      const int ci = cb + lane;
      int start = 0, len = 0;
      if (ci < ncell) {
        const int cell = (cam * kCols + x0 + ci / ncy) * kRows + y0 + ci % ncy;
        start = a.cell_ptr[cell];
        len = a.cell_ptr[cell + 1] - start;
      }
      const int incl = dev::wave_incl_scan(len);
      const int off = incl - len;
      const int tot = __shfl(incl, 63);
      for (int e0 = 0; e0 < tot; e0 += 64) {
        const int e = e0 + lane;
        // owning cell = the last lane whose offset is <= e (an empty cell shares its offset
        // with the next cell, lanes past the window hold tot)
        int o = 0;
#pragma unroll
        for (int s = 32; s > 0; s >>= 1)
          if (__shfl(off, o + s) <= e) o += s;
        const int so = __shfl(start, o), oo = __shfl(off, o);
        bool ok = false;
        int k = 0;
        if (e < tot) {
          k = a.cell_kp[so + (e - oo)];
          const int oc = a.kp_oct[k];
          ok = true;
          if (check && !same) ok = !(oc < minL || oc > maxL);
          else if (same) ok = (oc == minL);
          if (ok) {
            const double dx = (double)a.kp_xy[2 * k] - x, dy = (double)a.kp_xy[2 * k + 1] - y;
            ok = !(fabs(dx) > r || fabs(dy) > r);
          }
        }
        const uint64_t bal = __ballot(ok);
        if (!COUNT && ok) {
          const int pos = base + cnt + __popcll(bal & dev::lanemask_lt());
          a.cand_kp[pos] = k;
          a.cand_dist[pos] = ham(qd, a.kp_desc + (int64_t)k * a.bytes, qm,
                                 a.kp_mask ? a.kp_mask + (int64_t)k * a.bytes : nullptr, a.bytes);
        }
        cnt += __popcll(bal);
      }
    }
  }
  if (COUNT && lane == 0) a.cand_ptr[q + 1] = cnt;
}

// in-place inclusive scan of cand_ptr[1..nq] (cand_ptr[0] = 0), one workgroup, fixed order
__global__ __launch_bounds__(1024) void k_scan(int32_t* p, int nq, int64_t* total) {
  __shared__ int64_t carry;
  __shared__ int part[1024 / 64 + 1];
  if (threadIdx.x == 0) { carry = 0; p[0] = 0; }
  __syncthreads();
  for (int b = 0; b < nq; b += 1024) {
    const int i = b + (int)threadIdx.x;
    const int v = i < nq ? p[i + 1] : 0;
    int tot;
    const int ex = dev::block_excl_scan<1024>(v, part, &tot);
    if (i < nq) p[i + 1] = (int32_t)(carry + ex + v);
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

// device allocations of one host-buffer call, released on every return path
struct DevBufs {
  std::vector<void*> p;
  hipError_t err = hipSuccess;
  template <class T> T* alloc(size_t n) {
    void* q = nullptr;
    if (err == hipSuccess) err = hipMalloc(&q, std::max<size_t>(1, n) * sizeof(T));
    if (q) p.push_back(q);
    return static_cast<T*>(q);
  }
  template <class T> T* up(const T* h, size_t n) {
    T* d = alloc<T>(n);
    if (err == hipSuccess && h && n) err = hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice);
    return d;
  }
  ~DevBufs() { for (void* q : p) (void)hipFree(q); }
};

}  // namespace win
}  // namespace mcs

using namespace mcs;

extern "C" {

int mcs_frame_grid_build(const float* kp_xy, const int32_t* kp_cam, int32_t n_kp, int32_t n_cams,
                         const double* gp, int32_t* cell_ptr, int32_t* cell_kp,
                         int32_t* n_in_grid) {
  if (n_kp < 0 || n_cams < 1 || !gp || !cell_ptr || (n_kp > 0 && (!kp_xy || !kp_cam || !cell_kp)))
    return MCS_ERR_ARG;
  const int ncell = n_cams * win::kCols * win::kRows;
  std::vector<int32_t> cell(n_kp, -1), cnt(ncell + 1, 0);
  for (int i = 0; i < n_kp; i++) {
    const int c = kp_cam[i];
    if (c < 0 || c >= n_cams) continue;
    // PosInGrid: cvRound((kp.pt.x - mnMinX) * inv); float - int (mnMinX is an int) is a float
    const float fx = kp_xy[2 * i] - (float)gp[4 * c], fy = kp_xy[2 * i + 1] - (float)gp[4 * c + 1];
    const int px = cv_round((double)fx * gp[4 * c + 2]);
    const int py = cv_round((double)fy * gp[4 * c + 3]);
    if (px < 0 || px >= win::kCols || py < 0 || py >= win::kRows) continue;
    cell[i] = (c * win::kCols + px) * win::kRows + py;
    cnt[cell[i] + 1]++;
  }
  for (int k = 0; k < ncell; k++) cnt[k + 1] += cnt[k];
  for (int k = 0; k <= ncell; k++) cell_ptr[k] = cnt[k];
  for (int i = 0; i < n_kp; i++)     // keypoints in index order = push_back order (:180-181)
    if (cell[i] >= 0) cell_kp[cnt[cell[i]]++] = i;
  if (n_in_grid) *n_in_grid = cell_ptr[ncell];
  return MCS_OK;
}

int mcs_window_search_device(const int32_t* d_cell_ptr, const int32_t* d_cell_kp,
                             const double* d_grid_params, int32_t n_cams, const float* d_kp_xy,
                             const int32_t* d_kp_octave, const uint8_t* d_kp_desc,
                             const uint8_t* d_kp_mask, int32_t bytes, int32_t nq,
                             const double* d_q_xyr, const int32_t* d_q_cam_lvl,
                             const uint8_t* d_q_desc, const uint8_t* d_q_mask,
                             int32_t* d_cand_ptr, int32_t* d_cand_kp, int32_t* d_cand_dist,
                             int64_t cap, int64_t* total, void* stream) {
  if (!total || nq < 0 || n_cams < 1 || (bytes != 16 && bytes != 32 && bytes != 64)) return MCS_ERR_ARG;
  if (!d_cand_ptr || (nq > 0 && (!d_q_xyr || !d_q_cam_lvl || !d_q_desc || !d_grid_params ||
                                 !d_cell_ptr))) return MCS_ERR_ARG;
  if ((d_q_mask == nullptr) != (d_kp_mask == nullptr)) {
    set_error("window search: query and keypoint masks must both be given or both be null");
    return MCS_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  win::SearchArgs a{d_cell_ptr, d_cell_kp, d_grid_params, n_cams, d_kp_xy, d_kp_octave, d_kp_desc,
                    d_kp_mask, bytes, nq, d_q_xyr, d_q_cam_lvl, d_q_desc, d_q_mask, d_cand_ptr,
                    d_cand_kp, d_cand_dist};
  int64_t* d_total = nullptr;
  MCS_HIP_CHECK(hipMalloc((void**)&d_total, sizeof(int64_t)));
  const unsigned g = (unsigned)((nq + win::kQPB - 1) / win::kQPB);
  if (nq > 0) hipLaunchKernelGGL(win::k_window<true>, dim3(g), dim3(256), 0, st, a);
  hipLaunchKernelGGL(win::k_scan, dim3(1), dim3(1024), 0, st, d_cand_ptr, nq, d_total);
  int64_t tot = 0;
  hipError_t e = hipMemcpyAsync(&tot, d_total, sizeof(int64_t), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d_total);
  MCS_HIP_CHECK(e);
  *total = tot;
  if (tot > cap || (tot > 0 && (!d_cand_kp || !d_cand_dist))) {
    set_error("window search: candidate capacity too small (required size in *total)");
    return MCS_ERR_CAPACITY;
  }
  if (nq > 0 && tot > 0) hipLaunchKernelGGL(win::k_window<false>, dim3(g), dim3(256), 0, st, a);
  MCS_HIP_CHECK(hipGetLastError());
  return MCS_OK;
}

int mcs_window_select(int32_t rule, int32_t nq, const int32_t* cand_ptr, const int32_t* cand_kp,
                      const int32_t* cand_dist, const int32_t* kp_octave, int32_t n_kp,
                      int32_t th, double nnratio, uint8_t* kp_assigned, int32_t* match,
                      int32_t* n_matches) {
  if (rule < 0 || rule > 3 || nq < 0 || n_kp < 0 || !cand_ptr || !match || !n_matches) return MCS_ERR_ARG;
  if (rule != 2 && n_kp > 0 && !kp_assigned) return MCS_ERR_ARG;
  if (rule == 0 && n_kp > 0 && !kp_octave) return MCS_ERR_ARG;
  if (nq > 0 && cand_ptr[nq] > 0 && (!cand_kp || !cand_dist)) return MCS_ERR_ARG;
  for (int q = 0; q < nq; q++) match[q] = -1;
  int nm = 0;
  if (rule == 2) {
    // SearchForInitialization (:596-690): a train keypoint keeps the closest query so far
    std::vector<int> matched_dist(n_kp, INT_MAX), m21(n_kp, -1);
    for (int q = 0; q < nq; q++) {
      int best = INT_MAX, best2 = INT_MAX, bi = -1;
      for (int c = cand_ptr[q]; c < cand_ptr[q + 1]; c++) {
        const int k = cand_kp[c], d = cand_dist[c];
        if (matched_dist[k] <= d) continue;
        if (d < best) { best2 = best; best = d; bi = k; }
        else if (d < best2) best2 = d;
      }
      if (best <= th && best < (double)best2 * nnratio) {
        if (m21[bi] >= 0) { match[m21[bi]] = -1; nm--; }
        match[q] = bi;
        m21[bi] = q;
        matched_dist[bi] = best;
        nm++;
      }
    }
    *n_matches = nm;
    return MCS_OK;
  }
  for (int q = 0; q < nq; q++) {
    int best = INT_MAX, best2 = INT_MAX, bi = -1, lvl = -1, lvl2 = -1;
    for (int c = cand_ptr[q]; c < cand_ptr[q + 1]; c++) {
      const int k = cand_kp[c], d = cand_dist[c];
      if (kp_assigned[k]) continue;
      if (d < best) {
        best2 = best; best = d;
        lvl2 = lvl; lvl = rule == 0 ? kp_octave[k] : 0;
        bi = k;
      } else if (d < best2) {
        lvl2 = rule == 0 ? kp_octave[k] : 0;
        best2 = d;
      }
    }
    bool accept;
    if (rule == 0) accept = best <= th && !(lvl == lvl2 && best > nnratio * best2);   // :154-157
    else if (rule == 1) accept = best <= th;                                          // :2078
    else accept = best <= best2 * nnratio && best <= th;                              // :416
    if (accept) {
      kp_assigned[bi] = 1;
      match[q] = bi;
      nm++;
    }
  }
  *n_matches = nm;
  return MCS_OK;
}

int mcs_window_match(int32_t device, int32_t rule, const mcs_window_frame* f, int32_t nq,
                     const double* q_xyr, const int32_t* q_cam_lvl, const uint8_t* q_desc,
                     const uint8_t* q_mask, int32_t th, double nnratio, uint8_t* kp_assigned,
                     int32_t* match, int32_t* n_matches) {
  if (!f || f->n_cams < 1 || f->n_kp < 0 || nq < 0 || !f->grid_params || !match || !n_matches)
    return MCS_ERR_ARG;
  if (f->n_kp > 0 && (!f->kp_xy || !f->kp_cam || !f->kp_octave || !f->desc)) return MCS_ERR_ARG;
  if (nq > 0 && (!q_xyr || !q_cam_lvl || !q_desc)) return MCS_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("no HIP device visible (no CPU fallback)");
    return MCS_ERR_NO_DEVICE;
  }
  if (device < 0 || device >= ndev) return MCS_ERR_ARG;
  MCS_HIP_CHECK(hipSetDevice(device));
  const int ncell = f->n_cams * win::kCols * win::kRows;
  std::vector<int32_t> cell_ptr(ncell + 1), cell_kp(std::max(1, f->n_kp));
  int rc = mcs_frame_grid_build(f->kp_xy, f->kp_cam, f->n_kp, f->n_cams, f->grid_params,
                                cell_ptr.data(), cell_kp.data(), nullptr);
  if (rc) return rc;
  const size_t nk = (size_t)f->n_kp, nb = (size_t)f->bytes, nqs = (size_t)nq;
  win::DevBufs B;
  const double* d_gp = B.up(f->grid_params, 4 * (size_t)f->n_cams);
  const int32_t* d_cptr = B.up(cell_ptr.data(), cell_ptr.size());
  const int32_t* d_ckp = B.up(cell_kp.data(), (size_t)cell_ptr[ncell]);
  const float* d_xy = B.up(f->kp_xy, 2 * nk);
  const int32_t* d_oct = B.up(f->kp_octave, nk);
  const uint8_t* d_desc = B.up(f->desc, nk * nb);
  const uint8_t* d_mask = f->desc_mask ? B.up(f->desc_mask, nk * nb) : nullptr;
  const double* d_q = B.up(q_xyr, 3 * nqs);
  const int32_t* d_ql = B.up(q_cam_lvl, 3 * nqs);
  const uint8_t* d_qd = B.up(q_desc, nqs * nb);
  const uint8_t* d_qm = q_mask ? B.up(q_mask, nqs * nb) : nullptr;
  int32_t* d_cp = B.alloc<int32_t>(nqs + 1);
  int64_t cap = std::max<int64_t>(1024, 32 * (int64_t)nq), total = 0;
  int32_t* d_ck = B.alloc<int32_t>((size_t)cap);
  int32_t* d_cd = B.alloc<int32_t>((size_t)cap);
  if (B.err != hipSuccess) { set_hip_error(B.err, "window match upload", __FILE__, __LINE__); return MCS_ERR_HIP; }
  rc = mcs_window_search_device(d_cptr, d_ckp, d_gp, f->n_cams, d_xy, d_oct, d_desc, d_mask, f->bytes,
                                nq, d_q, d_ql, d_qd, d_qm, d_cp, d_ck, d_cd, cap, &total, nullptr);
  if (rc == MCS_ERR_CAPACITY) {
    cap = total;
    d_ck = B.alloc<int32_t>((size_t)cap);
    d_cd = B.alloc<int32_t>((size_t)cap);
    if (B.err != hipSuccess) { set_hip_error(B.err, "window match alloc", __FILE__, __LINE__); return MCS_ERR_HIP; }
    rc = mcs_window_search_device(d_cptr, d_ckp, d_gp, f->n_cams, d_xy, d_oct, d_desc, d_mask, f->bytes,
                                  nq, d_q, d_ql, d_qd, d_qm, d_cp, d_ck, d_cd, cap, &total, nullptr);
  }
  if (rc) return rc;
  std::vector<int32_t> cp(nqs + 1), ck(std::max<int64_t>(1, total)), cd(std::max<int64_t>(1, total));
  MCS_HIP_CHECK(hipMemcpy(cp.data(), d_cp, 4 * (nqs + 1), hipMemcpyDeviceToHost));
  if (total > 0) {
    MCS_HIP_CHECK(hipMemcpy(ck.data(), d_ck, 4 * (size_t)total, hipMemcpyDeviceToHost));
    MCS_HIP_CHECK(hipMemcpy(cd.data(), d_cd, 4 * (size_t)total, hipMemcpyDeviceToHost));
  }
  std::vector<uint8_t> fresh;
  if (!kp_assigned) { fresh.assign(std::max(1, f->n_kp), 0); kp_assigned = fresh.data(); }
  return mcs_window_select(rule, nq, cp.data(), ck.data(), cd.data(), f->kp_octave, f->n_kp, th,
                           nnratio, kp_assigned, match, n_matches);
}

}  // extern "C"
