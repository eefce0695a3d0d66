// C++ host program (no Python, no torch) driving the round-3 C-ABI the way the reference's
// host code would after LocalBundleAdjustment's write-back and before triangulation:
//   mcs_compute_e_rig                   <- SearchForTriangulationRaw's Es[i][j] = ComputeE(
//                                          KF1.Get_MtMc_inv(i), KF2.Get_MtMc(j))
//                                          (src/cORBmatcher.cpp:985-998)
//   mcs_distinctive_descriptors_device  <- cMapPoint::ComputeDistinctiveDescriptors
//                                          (src/cMapPoint.cpp:297-390), after :899-901
//   mcs_update_normal_depth_device      <- cMapPoint::UpdateNormalAndDepth (:453-496)
// Input file (little-endian, written by tests/test_host_cpp.py):
//   i32 nrig, i32 ncams, f64 mt1[nrig][6], f64 mt2[nrig][6], f64 mc[ncams][6]
//   i32 nb, i32 nrows, i32 npts_d, u8 desc[nrows][nb], i32 ptr[npts_d+1], i32 rows[ptr[npts_d]]
//   i32 npts, i32 nkf, i32 nlev, f64 pts[npts][3], i32 optr[npts+1], i32 okf[optr[npts]],
//   f64 kfc[nkf][3], i32 ref[npts], i32 lvl[npts], f64 scale[nlev]
// Output file: f64 E[nrig][ncams][ncams][9], i32 best[npts_d], u8 outdesc[npts_d][nb],
//   f64 normal[npts][3], f64 dmin[npts], f64 dmax[npts]
#include <hip/hip_runtime_api.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mcs_matcher.h"
#include "mcs_mappoint.h"

template <typename T>
static std::vector<T> rd(FILE* f, size_t n) {
  std::vector<T> v(n);
  if (n && std::fread(v.data(), sizeof(T), n, f) != n) { std::fprintf(stderr, "short read\n"); std::exit(2); }
  return v;
}
static int32_t rdi(FILE* f) { return rd<int32_t>(f, 1)[0]; }

template <typename T>
static T* up(const std::vector<T>& v) {
  T* d = nullptr;
  if (hipMalloc((void**)&d, std::max<size_t>(1, v.size()) * sizeof(T)) != hipSuccess) std::exit(3);
  if (!v.empty()) (void)hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  return d;
}
template <typename T>
static std::vector<T> down(const T* d, size_t n) {
  std::vector<T> v(n);
  if (n) (void)hipMemcpy(v.data(), d, n * sizeof(T), hipMemcpyDeviceToHost);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 3) { std::fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 1; }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 1;
  const int nrig = rdi(f), ncams = rdi(f);
  auto mt1 = rd<double>(f, 6 * (size_t)nrig), mt2 = rd<double>(f, 6 * (size_t)nrig);
  auto mc = rd<double>(f, 6 * (size_t)ncams);
  const int nb = rdi(f), nrows = rdi(f), npd = rdi(f);
  auto desc = rd<uint8_t>(f, (size_t)nrows * nb);
  auto ptr = rd<int32_t>(f, (size_t)npd + 1);
  auto rows = rd<int32_t>(f, (size_t)ptr[npd]);
  const int np = rdi(f), nkf = rdi(f), nlev = rdi(f);
  auto pts = rd<double>(f, 3 * (size_t)np);
  auto optr = rd<int32_t>(f, (size_t)np + 1);
  auto okf = rd<int32_t>(f, (size_t)optr[np]);
  auto kfc = rd<double>(f, 3 * (size_t)nkf);
  auto ref = rd<int32_t>(f, (size_t)np), lvl = rd<int32_t>(f, (size_t)np);
  auto scale = rd<double>(f, (size_t)nlev);
  std::fclose(f);

  // essential matrices of every camera pair, per rig pose pair (host entry point)
  std::vector<double> E((size_t)nrig * ncams * ncams * 9);
  for (int k = 0; k < nrig; k++) {
    const int rc = mcs_compute_e_rig(&mt1[6 * k], &mt2[6 * k], mc.data(), ncams, &E[(size_t)k * ncams * ncams * 9]);
    if (rc != MCS_OK) { std::fprintf(stderr, "compute_e_rig: %d %s\n", rc, mcs_last_error()); return 4; }
  }
  // map-point refresh (device entry points, default stream)
  uint8_t* d_desc = up(desc);
  int32_t *d_ptr = up(ptr), *d_rows = up(rows);
  int32_t* d_best = up(std::vector<int32_t>(npd, -7));
  uint8_t* d_od = up(std::vector<uint8_t>((size_t)npd * nb, 0));
  int rc = mcs_distinctive_descriptors_device(d_desc, nullptr, nb, d_ptr, d_rows, npd, d_best, d_od, nullptr, nullptr);
  if (rc != MCS_OK) { std::fprintf(stderr, "distinctive: %d %s\n", rc, mcs_last_error()); return 5; }
  double* d_pts = up(pts);
  int32_t *d_optr = up(optr), *d_okf = up(okf), *d_ref = up(ref), *d_lvl = up(lvl);
  double *d_kfc = up(kfc), *d_scale = up(scale);
  double* d_n = up(std::vector<double>(3 * (size_t)np, 0.0));
  double *d_min = up(std::vector<double>(np, 0.0)), *d_max = up(std::vector<double>(np, 0.0));
  rc = mcs_update_normal_depth_device(d_pts, np, d_optr, d_okf, d_kfc, d_ref, d_lvl, d_scale, nlev, d_n, d_min,
                                      d_max, nullptr);
  if (rc != MCS_OK) { std::fprintf(stderr, "normal/depth: %d %s\n", rc, mcs_last_error()); return 6; }
  if (hipDeviceSynchronize() != hipSuccess) return 7;
  // an argument error must come back as a status with a message, never a crash
  const int bad = mcs_distinctive_descriptors_device(d_desc, nullptr, 24, d_ptr, d_rows, npd, d_best, d_od, nullptr,
                                                     nullptr);
  std::printf("bad_bytes_status %d %s\n", bad, mcs_last_error());

  FILE* o = std::fopen(argv[2], "wb");
  if (!o) return 8;
  std::fwrite(E.data(), 8, E.size(), o);
  auto best = down(d_best, npd);
  auto od = down(d_od, (size_t)npd * nb);
  auto nrm = down(d_n, 3 * (size_t)np);
  auto mn = down(d_min, np), mx = down(d_max, np);
  std::fwrite(best.data(), 4, best.size(), o);
  std::fwrite(od.data(), 1, od.size(), o);
  std::fwrite(nrm.data(), 8, nrm.size(), o);
  std::fwrite(mn.data(), 8, mn.size(), o);
  std::fwrite(mx.data(), 8, mx.size(), o);
  std::fclose(o);
  std::printf("ok %d %d %d\n", nrig, npd, np);
  return 0;
}
