// Latency / issue probe for the LDL^T column chain (one wave, shader cycles), unrolled x16 so
// loop overhead is amortised:
//   fma_dep      dependent v_fma_f64 chain (cycles per link)
//   rcp_dep      dependent v_rcp_f64 chain
//   ldexp_dep    dependent v_ldexp_f64 chain
//   rl_fma_dep   readlane pair -> v_fma_f64 with SGPR operand, dependent
//   lds_dep      ds_write_b64 -> uniform ds_read_b64 -> v_fma_f64, dependent
//   rl_issue     independent readlane pairs (cycles per pair), results summed into 16 accumulators
//   fma_issue    independent v_fma_f64 (cycles per instruction)
//   fmas_issue   independent v_fma_f64 with an SGPR-pair operand
// Build: hipcc --offload-arch=gfx950 -O3 tools/bench/lat_probe2.hip -o tools/bench/lat_probe2
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

#define U16(X) X X X X X X X X X X X X X X X X

__global__ __launch_bounds__(64) void k_lat(double* out, long long* cyc, int n, int lane) {
  __shared__ double lds[128];
  const int t = threadIdx.x;
  double x = 1.0 + t * 1e-3;
  const double c1 = 0.999999 + 1e-9 * n, c2 = 1e-7 * n;
  long long ts[9];
  ts[0] = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; k++) { U16(x = __builtin_fma(x, c1, c2);) }
  ts[1] = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; k++) { U16(x = __builtin_amdgcn_rcp(x);) }
  ts[2] = __builtin_amdgcn_s_memtime();
  int sh = n & 1;
  for (int k = 0; k < n; k++) { U16(x = __builtin_ldexp(x, sh);) }
  ts[3] = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; k++) { U16(x = __builtin_fma(readlane_d(x, lane), c1, x);) }
  ts[4] = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; k++) {
    U16(lds[t] = x; __builtin_amdgcn_wave_barrier(); x = __builtin_fma(lds[lane], c1, x); __builtin_amdgcn_wave_barrier();)
  }
  ts[5] = __builtin_amdgcn_s_memtime();
  double acc[16];
#pragma unroll
  for (int q = 0; q < 16; q++) acc[q] = x + q;
  for (int k = 0; k < n; k++) {
#pragma unroll
    for (int q = 0; q < 16; q++) acc[q] = acc[q] + readlane_d(x, q);
    x = acc[k & 15] * 1e-3;
  }
  ts[6] = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; k++) {
#pragma unroll
    for (int q = 0; q < 16; q++) acc[q] = __builtin_fma(acc[q], c1, c2);
  }
  ts[7] = __builtin_amdgcn_s_memtime();
  const double s1 = readlane_d(x, 3);
  for (int k = 0; k < n; k++) {
#pragma unroll
    for (int q = 0; q < 16; q++) acc[q] = __builtin_fma(acc[q], s1, c2);
  }
  ts[8] = __builtin_amdgcn_s_memtime();
  double s = x;
#pragma unroll
  for (int q = 0; q < 16; q++) s += acc[q];
  out[t] = s;
  if (t == 0)
    for (int i = 0; i < 8; i++) cyc[i] = ts[i + 1] - ts[i];
}

int main() {
  double* d; long long* c;
  (void)hipMalloc(&d, 64 * 8); (void)hipMalloc(&c, 64);
  const int n = 64;
  for (int r = 0; r < 2; r++) {
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, c, n, 5);
    (void)hipDeviceSynchronize();
    long long h[8];
    (void)hipMemcpy(h, c, 64, hipMemcpyDeviceToHost);
    const double m = 16.0 * n;
    printf("{\"fma_dep\": %.1f, \"rcp_dep\": %.1f, \"ldexp_dep\": %.1f, \"rl_fma_dep\": %.1f, \"lds_dep\": %.1f, "
           "\"rl_issue_pair\": %.1f, \"fma_issue\": %.1f, \"fmas_issue\": %.1f}\n",
           h[0] / m, h[1] / m, h[2] / m, h[3] / m, h[4] / m, h[5] / m, h[6] / m, h[7] / m);
  }
  return 0;
}
