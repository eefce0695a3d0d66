// Issue/latency probe for one 256-thread workgroup (1 wave per SIMD): FP64 FMA chains,
// LDS broadcast reads, f64 division, readlane and barrier, in shader-clock cycles.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_lat(double* out, long long* cyc, int n) {
  __shared__ double lds[1024];
  const int t = threadIdx.x;
  for (int k = t; k < 1024; k += 256) lds[k] = 1.0 + k * 1e-6;
  __syncthreads();
  double a[16];
#pragma unroll
  for (int q = 0; q < 16; q++) a[q] = t * 1e-3 + q;
  long long t0 = __builtin_amdgcn_s_memtime();
  // (1) 16 independent FMA chains, n iterations
  for (int k = 0; k < n; k++) {
#pragma unroll
    for (int q = 0; q < 16; q++) a[q] = __builtin_fma(a[q], 0.999999, 1e-7);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  // (2) one dependent FMA chain
  double x = a[0];
  for (int k = 0; k < n; k++) {
#pragma unroll
    for (int q = 0; q < 16; q++) x = __builtin_fma(x, 0.999999, 1e-7);
  }
  long long t2 = __builtin_amdgcn_s_memtime();
  // (3) LDS broadcast reads: 8 x b128 per iteration + FMAs consuming them
  double y = 0.0;
  for (int k = 0; k < n; k++) {
    const double2* p = reinterpret_cast<const double2*>(lds + ((k * 16) & 1023));
#pragma unroll
    for (int q = 0; q < 8; q++) { double2 v = p[q]; y = __builtin_fma(v.x, v.y, y); }
  }
  long long t3 = __builtin_amdgcn_s_memtime();
  // (4) f64 division chain
  double z = 1.0 + t;
  for (int k = 0; k < n; k++) {
#pragma unroll
    for (int q = 0; q < 16; q++) z = 1.000001 / z;
  }
  long long t4 = __builtin_amdgcn_s_memtime();
  // (5) barriers
  for (int k = 0; k < n * 16; k++) __syncthreads();
  long long t5 = __builtin_amdgcn_s_memtime();
  // (6) LDS write + barrier + read round trip
  double w = 0.0;
  for (int k = 0; k < n * 16; k++) {
    if (t < 64) lds[(k & 1) * 64 + t] = w + k;
    __syncthreads();
    w += lds[(k & 1) * 64 + (t & 63)];
  }
  long long t6 = __builtin_amdgcn_s_memtime();
  double s = x + y + z + w;
#pragma unroll
  for (int q = 0; q < 16; q++) s += a[q];
  out[t] = s;
  if (t == 0) {
    const double m = 16.0 * n;
    cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4; cyc[5] = t6 - t5;
    (void)m;
  }
}

int main() {
  double* d; long long* c;
  (void)hipMalloc(&d, 256 * 8); (void)hipMalloc(&c, 64);
  const int n = 64;
  for (int r = 0; r < 2; r++) {
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(256), 0, 0, d, c, n);
    (void)hipDeviceSynchronize();
    long long h[6];
    (void)hipMemcpy(h, c, 48, hipMemcpyDeviceToHost);
    const double m = 16.0 * n;
    printf("{\"fma_indep_cyc_per_op\": %.2f, \"fma_dep_latency\": %.2f, \"lds_b128_bcast_per_read\": %.2f, "
           "\"div_f64_dep\": %.2f, \"barrier\": %.2f, \"lds_write_barrier_read\": %.2f}\n",
           h[0] / m, h[1] / m, h[2] / (8.0 * n), h[3] / m, h[4] / m, h[5] / m);
  }
  return 0;
}
