// Cycle probe of the dense LDL^T building blocks (one workgroup, one 64x64 tile):
// s_memtime (shader clock) and s_memrealtime (100 MHz) around each phase.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/bench/ldlt_probe.hip -o tools/bench/ldlt_probe
#include "../../multicol-slam-annotation_amd/csrc/ldlt.hip"
#include <cstdio>
#include <vector>

using namespace mcs::ldlt;

template <int V>
__global__ __launch_bounds__(256) void k_probe(const double* A, double* out, long long* stamps, long long* ts) {
  extern __shared__ double sm[];
  double* sK = sm;
  double* sI = sK + TB * 65;
  double* scol = sI + TB * 65;
  __shared__ int fail;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) fail = 0;
  load_tile_lower(sK, A);
  __syncthreads();
  long long t1 = __builtin_amdgcn_s_memtime();
  factor_tile(sK, sI, scol, &fail);
  long long t2 = __builtin_amdgcn_s_memtime(), r2 = __builtin_amdgcn_s_memrealtime();
  for (int e = threadIdx.x; e < 4096; e += 256) out[e] = sK[(e >> 6) * 65 + (e & 63)] + sI[(e >> 6) * 65 + (e & 63)];
  if (threadIdx.x == 0) {
    stamps[0] = t1 - t0; stamps[1] = t2 - t1; stamps[2] = t2 - t0; stamps[3] = r2 - r0;
  }
}

int main() {
  std::vector<double> h(4096);
  for (int i = 0; i < 64; i++)
    for (int j = 0; j < 64; j++) h[i * 64 + j] = (i == j) ? 70.0 : 1.0 / (1 + i + j);
  double *dA, *dO;
  long long* dS;
  (void)hipMalloc(&dA, 4096 * 8); (void)hipMalloc(&dO, 4096 * 8); (void)hipMalloc(&dS, 64);
  (void)hipMemcpy(dA, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  const size_t lds = (2 * 64 * 65 + 512) * 8;
  long long* dT; (void)hipMalloc(&dT, 4 * 64 * 4 * 8);
  void (*ks[8])(const double*, double*, long long*, long long*) = {k_probe<0>, k_probe<0>, k_probe<0>, k_probe<0>, k_probe<0>, k_probe<0>, k_probe<0>, k_probe<0>};
  const char* names[8] = {"full", "full", "full", "full", "full", "full", "full", "full"};
  for (int v = 0; v < 8; v++) (void)hipFuncSetAttribute((const void*)ks[v], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int rep = 0; rep < 4; rep++) {
    const int v = rep / 2;
    printf("%s ", names[v]);
    hipLaunchKernelGGL(ks[v], dim3(1), dim3(256), lds, 0, dA, dO, dS, dT);
    (void)hipDeviceSynchronize();
    long long s[4];
    (void)hipMemcpy(s, dS, 32, hipMemcpyDeviceToHost);
    std::vector<double> o(4096);
    (void)hipMemcpy(o.data(), dO, 4096 * 8, hipMemcpyDeviceToHost);
    printf("out00=%.6f ", o[0]);
    printf("{\"load_cyc\": %lld, \"factor_cyc\": %lld, \"total_cyc\": %lld, \"total_us\": %.2f, \"clock_mhz\": %.0f}\n",
           s[0], s[1], s[2], s[3] / 100.0, s[2] / (s[3] / 100.0));
  }
  return 0;
}
