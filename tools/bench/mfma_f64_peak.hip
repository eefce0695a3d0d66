// Measures the FP64 matrix-core rate of the device: every wave issues back-to-back
// v_mfma_f64_16x16x4_f64 on 4 independent accumulators (2048 flop each).  Prints TFLOP/s.
// Build: hipcc --offload-arch=gfx950 -O3 tools/bench/mfma_f64_peak.hip -o tools/bench/mfma_f64_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_peak(double* out, int iters, double a0) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  const double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
  for (int i = 0; i < iters; i++) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  const d4 s = c0 + c1 + c2 + c3;
  if (s[0] == 12345.678) out[threadIdx.x] = s[1];   // keep the chain alive
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double* d = nullptr;
  hipMalloc(&d, 4096);
  const int iters = 4096, blocks = cus * 8;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_peak<<<blocks, 256>>>(d, 16, 1.0);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  k_peak<<<blocks, 256>>>(d, iters, 1.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)blocks * 4 /*waves*/ * iters * 4 /*mfma*/ * 2048.0;
  printf("{\"cus\": %d, \"ms\": %.4f, \"fp64_mfma_tflops\": %.3f}\n", cus, ms, flops / (ms * 1e-3) / 1e12);
  hipFree(d);
  return 0;
}
