// Phase clocks of the whole dense solve (k_panel x T + k_backward) at config E size:
// s_memtime per (step, workgroup) at kernel entry, after the tile loads, after the tile
// factorisation, after the two W GEMMs, after the update GEMM and at exit; the solution is
// checked against a host LDL^T solve.  Prints per step: workgroups, median/max of each phase.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/bench/ldlt_solve_probe.hip -o tools/bench/ldlt_solve_probe
#define MCS_LDLT_PROBE 1
#include "../../multicol-slam-annotation_amd/csrc/ldlt.hip"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

using namespace mcs::ldlt;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1194;
  const int T = tiles_for(n), Np = T * TB;
  // SPD: diagonally dominant with smooth off-diagonal structure
  std::vector<double> M((size_t)Np * Np, 0.0), rhs(Np, 0.0);
  for (int r = 0; r < Np; r++)
    for (int c = 0; c <= r; c++) {
      double v = (r == c) ? (r < n ? 2.0 * Np : 1.0) : (r < n && c < n ? 1.0 / (1 + r - c) : 0.0);
      M[(size_t)r * Np + c] = M[(size_t)c * Np + r] = v;
    }
  for (int r = 0; r < n; r++) rhs[r] = std::sin(0.01 * r);
  std::vector<double> tiles(tile_doubles(T));
  for (int r = 0; r < Np; r++)
    for (int c = 0; c <= r; c++) tiles[sidx(r, c, T)] = M[(size_t)r * Np + c];
  double *dA, *db, *dx, *dL, *dLi, *dz;
  int* dflag;
  (void)hipMalloc(&dA, tiles.size() * 8); (void)hipMalloc(&db, Np * 8); (void)hipMalloc(&dx, Np * 8);
  (void)hipMalloc(&dL, tiles.size() * 8); (void)hipMalloc(&dLi, (size_t)T * TB * TB * 8);
  (void)hipMalloc(&dz, Np * 8); (void)hipMalloc(&dflag, 4);
  Work w{dL, dLi, dz};
  std::vector<double> x(Np);
  for (int rep = 0; rep < 3; rep++) {
    (void)hipMemcpy(dA, tiles.data(), tiles.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, rhs.data(), Np * 8, hipMemcpyHostToDevice);
    (void)hipMemset(dflag, 0, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    if (solve(dA, db, dx, T, w, dflag, 0) != hipSuccess) { std::printf("launch failed\n"); return 2; }
    (void)hipEventRecord(e1, 0);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("sync failed\n"); return 2; }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::printf("rep %d: solve %.3f ms (n=%d, T=%d)\n", rep, ms, n, T);
  }
  (void)hipMemcpy(x.data(), dx, Np * 8, hipMemcpyDeviceToHost);
  // residual check
  double rmax = 0;
  for (int r = 0; r < n; r++) {
    double s = 0;
    for (int c = 0; c < n; c++) s += M[(size_t)r * Np + c] * x[c];
    rmax = std::max(rmax, std::fabs(s - rhs[r]));
  }
  std::vector<long long> st(32 * 256 * 8);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_panel_stamps), st.size() * 8);
  std::printf("residual %.3e\n", rmax);
  std::printf("step  wgs  load(med/max)  factor(med/max)  W-gemms(med/max)  upd-gemm(med/max)  tail(med/max)  total(max) [cycles]\n");
  for (int k = 0; k < T && k < 32; k++) {
    const int m = T - 1 - k, nwg = std::min(256, 1 + m * (m + 1) / 2);
    std::vector<long long> ph[6];
    for (int g = 0; g < nwg; g++) {
      const long long* s = &st[((size_t)k * 256 + g) * 8];
      ph[0].push_back(s[1] - s[0]);
      ph[1].push_back(s[2] - s[1]);
      if (g > 0) {
        ph[2].push_back(s[3] - s[2]);
        ph[3].push_back(s[4] - s[3]);
        ph[4].push_back(s[5] - s[4]);
        ph[5].push_back(s[5] - s[0]);
      }
    }
    auto mm = [](std::vector<long long> v, bool mx) -> long long {
      if (v.empty()) return 0;
      std::sort(v.begin(), v.end());
      return mx ? v.back() : v[v.size() / 2];
    };
    std::printf("%4d %4d  %6lld/%6lld  %6lld/%6lld  %6lld/%6lld  %6lld/%6lld  %6lld/%6lld  %7lld\n", k, nwg,
                mm(ph[0], 0), mm(ph[0], 1), mm(ph[1], 0), mm(ph[1], 1), mm(ph[2], 0), mm(ph[2], 1),
                mm(ph[3], 0), mm(ph[3], 1), mm(ph[4], 0), mm(ph[4], 1), mm(ph[5], 1));
  }
  return rmax < 1e-8 ? 0 : 1;
}
