// LDS read throughput for one 256-thread workgroup: broadcast vs lane-consecutive, b32/b64/b128.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k_lds(double* out, long long* cyc, int n) {
  __shared__ double lds[4096];
  const int t = threadIdx.x, l = t & 63;
  for (int k = t; k < 4096; k += 256) lds[k] = 1.0 + k * 1e-6;
  __syncthreads();
  double y0 = 0, y1 = 0, y2 = 0, y3 = 0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; k++) {
    const int base = (k * 32) & 2047;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      if (MODE == 0) {        // b128 broadcast
        const double2 v = reinterpret_cast<const double2*>(lds + base)[q];
        y0 += v.x; y1 += v.y;
      } else if (MODE == 1) { // b64 broadcast (x2 to move the same bytes)
        y0 += lds[base + 2 * q]; y1 += lds[base + 2 * q + 1];
      } else if (MODE == 2) { // b128 lane-consecutive
        const double2 v = reinterpret_cast<const double2*>(lds + base + 128 * q)[l];
        y0 += v.x; y1 += v.y;
      } else if (MODE == 3) { // b64 lane-consecutive (x2)
        y0 += lds[base + 128 * q + l]; y1 += lds[base + 128 * q + 64 + l];
      } else {                // b32 broadcast (x4)
        const float* f = reinterpret_cast<const float*>(lds + base);
        y0 += f[4 * q]; y1 += f[4 * q + 1]; y2 += f[4 * q + 2]; y3 += f[4 * q + 3];
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[t] = y0 + y1 + y2 + y3;
  if (t == 0) cyc[MODE] = t1 - t0;
}

int main() {
  double* d; long long* c;
  (void)hipMalloc(&d, 256 * 8); (void)hipMalloc(&c, 64);
  const int n = 256;
  for (int r = 0; r < 2; r++) {
    hipLaunchKernelGGL(k_lds<0>, dim3(1), dim3(256), 0, 0, d, c, n);
    hipLaunchKernelGGL(k_lds<1>, dim3(1), dim3(256), 0, 0, d, c, n);
    hipLaunchKernelGGL(k_lds<2>, dim3(1), dim3(256), 0, 0, d, c, n);
    hipLaunchKernelGGL(k_lds<3>, dim3(1), dim3(256), 0, 0, d, c, n);
    hipLaunchKernelGGL(k_lds<4>, dim3(1), dim3(256), 0, 0, d, c, n);
    (void)hipDeviceSynchronize();
    long long h[5];
    (void)hipMemcpy(h, c, 40, hipMemcpyDeviceToHost);
    const double m = 8.0 * n;   // per 16 bytes/lane moved
    printf("{\"b128_bcast\": %.1f, \"2xb64_bcast\": %.1f, \"b128_lane\": %.1f, \"2xb64_lane\": %.1f, \"4xb32_bcast\": %.1f}  cycles per 16 B/lane\n",
           h[0] / m, h[1] / m, h[2] / m, h[3] / m, h[4] / m);
  }
  return 0;
}
