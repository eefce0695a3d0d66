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
#include <chrono>
#include <unistd.h>

using namespace mcs::ldlt;

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int n = argc > 1 ? atoi(argv[1]) : 1194;
  const int mode = argc > 2 ? atoi(argv[2]) : 0;   // 0 both, 1 launch-per-step only, 2 pipelined only
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
  if (mode != 3) {   // mode 3: the legacy path (no sync words: single-workgroup k_backward)
    if (pipe_prepare(w, T, 0) != hipSuccess) { std::printf("pipe_prepare (per-step) failed\n"); return 2; }
    w.per_step = true;
  }
  std::vector<double> x(Np), xp(Np);
  // pipelined path first (its own Work), then the launch-per-step path below; x must agree
  // bitwise
  if (mode != 1 && mode != 3) {
    double *pA, *pb, *px, *pL, *pLi, *pz;
    (void)hipMalloc(&pA, tiles.size() * 8); (void)hipMalloc(&pb, Np * 8); (void)hipMalloc(&px, Np * 8);
    (void)hipMalloc(&pL, tiles.size() * 8); (void)hipMalloc(&pLi, (size_t)T * TB * TB * 8);
    (void)hipMalloc(&pz, Np * 8);
    Work wp{pL, pLi, pz};
    std::printf("pipe_prepare T=%d\n", T);
    if (pipe_prepare(wp, T, 0) != hipSuccess) { std::printf("pipe_prepare failed\n"); return 2; }
    std::printf("prepared: %d tasks\n", wp.ntasks);
    for (int rep = 0; rep < 5; rep++) {
      (void)hipMemcpy(pA, tiles.data(), tiles.size() * 8, hipMemcpyHostToDevice);
      (void)hipMemcpy(pb, rhs.data(), Np * 8, hipMemcpyHostToDevice);
      (void)hipMemset(dflag, 0, 4);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0, 0);
      if (rep == 0) std::printf("copies done\n");
      if (solve(pA, pb, px, T, wp, dflag, 0) != hipSuccess) { std::printf("pipe launch failed\n"); return 2; }
      (void)hipEventRecord(e1, 0);
      if (rep == 0) std::printf("launched\n");
      {
        auto t0 = std::chrono::steady_clock::now();
        while (hipEventQuery(e1) != hipSuccess) {
          if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3)) {
            unsigned hs0[2];
            std::printf("pipe rep %d did not finish\n", rep);
            fflush(stdout);
            _exit(4);
          }
        }
      }
      if (hipDeviceSynchronize() != hipSuccess) { std::printf("pipe sync failed\n"); return 2; }
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned hs[2];
      int fl = 0;
      (void)hipMemcpy(hs, wp.sync, 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(&fl, dflag, 4, hipMemcpyDeviceToHost);
      std::printf("pipe rep %d: solve %.3f ms (tickets %u, err %u, flag %d, tasks %d)\n", rep, ms, hs[0], hs[1], fl, wp.ntasks);
      if (hs[1]) {
        const int nt = T * (T + 1) / 2;
        std::vector<unsigned> sw(pipe_sync_words(T));
        (void)hipMemcpy(sw.data(), wp.sync, sw.size() * 4, hipMemcpyDeviceToHost);
        std::printf("cnt:");
        for (int q = 0; q < nt; q++) std::printf(" %u", sw[4 + q]);
        std::printf("\npan:");
        for (int q = 0; q < nt; q++) std::printf(" %u", sw[4 + nt + q]);
        std::printf("\ndg:");
        for (int q = 0; q < T; q++) std::printf(" %u", sw[4 + 2 * nt + q]);
        std::printf("\n");
        return 3;
      }
    }
    (void)hipMemcpy(xp.data(), px, Np * 8, hipMemcpyDeviceToHost);
    {
      // timeline of the last rep (microseconds from the diag workgroup's first stamp)
      std::vector<long long> ds(128 * 8), ts((size_t)(wp.ntasks + 1) * 4);
      (void)hipMemcpyFromSymbol(ds.data(), HIP_SYMBOL(g_diag_stamps), ds.size() * 8);
      (void)hipMemcpyFromSymbol(ts.data(), HIP_SYMBOL(g_task_stamps), ts.size() * 8);
      const long long z0 = ds[0];
      auto us = [&](long long v) { return (v - z0) / 100.0; };
      std::printf("diag k: start waitA+ loaded factored published waitB+ trsm-published (us)\n");
      for (int k = 0; k < T && k < 128; k++) {
        const long long* d = &ds[k * 8];
        std::printf("%3d %8.2f %8.2f %8.2f %8.2f %8.2f %8.2f %8.2f\n", k, us(d[0]), us(d[1]), us(d[2]), us(d[3]),
                    us(d[4]), k + 1 < T ? us(d[5]) : 0.0, k + 1 < T ? us(d[6]) : 0.0);
      }
      std::vector<int4> tasks(wp.ntasks);
      (void)hipMemcpy(tasks.data(), wp.tasks, tasks.size() * 16, hipMemcpyDeviceToHost);
      double wsum = 0, csum = 0;
      for (int q = 1; q <= wp.ntasks; q++) {
        const long long* t4 = &ts[(size_t)q * 4];
        wsum += (t4[1] - t4[0]) / 100.0;
        csum += (t4[3] - t4[1]) / 100.0;
      }
      std::printf("tasks: mean wait %.2f us, mean run %.2f us\n", wsum / wp.ntasks, csum / wp.ntasks);
      for (int q = 1; q <= wp.ntasks && q < 80; q++) {
        const long long* t4 = &ts[(size_t)q * 4];
        const int4 tq = tasks[q - 1];
        std::printf("  task %4d %s (%d,%d,%d): start %8.2f ready %8.2f loaded %8.2f end %8.2f\n", q,
                    tq.x ? "UPD " : "TRSM", tq.y, tq.z, tq.w, us(t4[0]), us(t4[1]), us(t4[2]), us(t4[3]));
      }
    }
    if (mode == 2) return 0;
  }
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
  size_t ndiff = 0;
  for (int r = 0; r < Np; r++) ndiff += (x[r] != xp[r]);
  if (mode == 0) {
    std::printf("pipelined vs launch-per-step: %zu of %d entries differ\n", ndiff, Np);
    if (ndiff) return 1;
  }
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
