// Cycle probe + correctness check of the dense LDL^T tile factorisation (one workgroup, one
// 64x64 tile): s_memtime (shader clock) and s_memrealtime (100 MHz) around the phases, and
// L, D, L^-1 compared with a host LDL^T of the same tile.  Exit status 1 on a mismatch.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/bench/ldlt_probe.hip -o tools/bench/ldlt_probe
#define MCS_LDLT_PROBE 1
#include "../../multicol-slam-annotation_amd/csrc/ldlt.hip"
#include <cmath>
#include <cstdio>
#include <vector>

using namespace mcs::ldlt;

__global__ __launch_bounds__(256) void k_probe(const double* A, double* outL, double* outI,
                                               long long* stamps) {
  extern __shared__ double sm[];
  double* sK = sm;
  double* sI = sK + TB * LS;
  int& fail = *reinterpret_cast<int*>(sI + TB * LS);
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) fail = 0;
  load_tile_lower(sK, A);
  __syncthreads();
  long long t1 = __builtin_amdgcn_s_memtime();
#ifdef MCS_LDLT_FACTOR_V0
  factor_tile_v0(sK, sI, &fail);
#else
  factor_tile(sK, sI, &fail);
#endif
  long long t2 = __builtin_amdgcn_s_memtime(), r2 = __builtin_amdgcn_s_memrealtime();
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int r = e >> 6, c = e & 63;
    outL[e] = c <= r ? sK[r * LS + c] : 0.0;
    outI[e] = sI[r * LS + c];
  }
  if (threadIdx.x == 0) {
    stamps[0] = t1 - t0; stamps[1] = t2 - t1; stamps[2] = t2 - t0; stamps[3] = r2 - r0;
    stamps[4] = fail;
    for (int i = 0; i < 9; i++) stamps[5 + i] = g_ldlt_stamps[i] - t1;
  }
}

int main(int argc, char** argv) {
  std::vector<double> h(4096);
  for (int i = 0; i < 64; i++)
    for (int j = 0; j < 64; j++) h[i * 64 + j] = (i == j) ? 70.0 : 1.0 / (1 + i + j);
  // host reference: unblocked LDL^T, then X = L^-1 (unit lower)
  std::vector<double> L(4096, 0.0), D(64), X(4096, 0.0);
  for (int j = 0; j < 64; j++) {
    double d = h[j * 64 + j];
    for (int k = 0; k < j; k++) d -= L[j * 64 + k] * L[j * 64 + k] * D[k];
    D[j] = d;
    for (int i = j + 1; i < 64; i++) {
      double s = h[i * 64 + j];
      for (int k = 0; k < j; k++) s -= L[i * 64 + k] * L[j * 64 + k] * D[k];
      L[i * 64 + j] = s / d;
    }
  }
  for (int c = 0; c < 64; c++)
    for (int r = 0; r < 64; r++) {
      double s = (r == c) ? 1.0 : 0.0;
      for (int k = 0; k < r; k++) s -= L[r * 64 + k] * X[k * 64 + c];
      X[r * 64 + c] = s;
    }
  double *dA, *dL, *dI;
  long long* dS;
  (void)hipMalloc(&dA, 4096 * 8); (void)hipMalloc(&dL, 4096 * 8); (void)hipMalloc(&dI, 4096 * 8);
  (void)hipMalloc(&dS, 16 * 8);
  (void)hipMemcpy(dA, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  const size_t lds = 2 * 64 * LS * 8 + 16;
  (void)hipFuncSetAttribute((const void*)k_probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  bool ok = true;
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(256), lds, 0, dA, dL, dI, dS);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("launch failed\n"); return 2; }
    long long s[14];
    std::vector<double> oL(4096), oI(4096);
    (void)hipMemcpy(s, dS, 14 * 8, hipMemcpyDeviceToHost);
    std::printf("phase stamps (cyc from factor start): panel/update p0..p3, Linv diag:");
    for (int i = 0; i < 9; i++) std::printf(" %lld", s[5 + i]);
    std::printf("\n");
    (void)hipMemcpy(oL.data(), dL, 4096 * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(oI.data(), dI, 4096 * 8, hipMemcpyDeviceToHost);
    double eL = 0, eD = 0, eI = 0, eU = 0;
    for (int r = 0; r < 64; r++)
      for (int c = 0; c < 64; c++) {
        const int e = r * 64 + c;
        if (c < r) eL = std::fmax(eL, std::fabs(oL[e] - L[e]));
        if (c == r) eD = std::fmax(eD, std::fabs(oL[e] - D[r]) / std::fabs(D[r]));
        if (c <= r) eI = std::fmax(eI, std::fabs(oI[e] - X[e]));
        else eU = std::fmax(eU, std::fabs(oI[e]));
      }
    ok = ok && s[4] == 0 && eL < 1e-12 && eD < 1e-12 && eI < 1e-11 && eU == 0.0;
    std::printf("{\"load_cyc\": %lld, \"factor_cyc\": %lld, \"total_cyc\": %lld, \"total_us\": %.2f, "
                "\"clock_mhz\": %.0f, \"fail\": %lld, \"err_L\": %.3e, \"err_D\": %.3e, "
                "\"err_Linv\": %.3e, \"upper_Linv\": %.3e}\n",
                s[0], s[1], s[2], s[3] / 100.0, s[2] / (s[3] / 100.0), s[4], eL, eD, eI, eU);
  }
  if (argc > 1) {   // dump L (with D) and L^-1 of the last rep for a bitwise comparison
    std::vector<double> oL(4096), oI(4096);
    (void)hipMemcpy(oL.data(), dL, 4096 * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(oI.data(), dI, 4096 * 8, hipMemcpyDeviceToHost);
    FILE* f = std::fopen(argv[1], "wb");
    if (f) { std::fwrite(oL.data(), 8, 4096, f); std::fwrite(oI.data(), 8, 4096, f); std::fclose(f); }
  }
  std::printf(ok ? "LDLT PROBE OK\n" : "LDLT PROBE MISMATCH\n");
  return ok ? 0 : 1;
}
