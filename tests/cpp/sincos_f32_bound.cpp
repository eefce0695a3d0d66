// Exhaustive check of mcs::sincos_f32 (multicol-slam-annotation_amd/csrc/desc_math.hpp): the
// largest |error| against double-precision sin / cos over EVERY float t in [0, 2 pi + 1e-3]
// (k_orient_desc's angle range).  Prints "maxerr <e> count <n>"; the test requires
// e <= kSinCosErr, the bound the kernel's near-half margin is derived from.
// Build: g++ -O2 -std=c++17 -ffp-contract=off -pthread (no fast-math: fma and rint are IEEE).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../multicol-slam-annotation_amd/csrc/desc_math.hpp"

int main(int argc, char** argv) {
  const int nt = argc > 1 ? std::atoi(argv[1]) : 8;
  const float hi = 6.2841853f;   // 2 pi + 1e-3
  uint32_t end;
  std::memcpy(&end, &hi, 4);
  std::vector<double> mx(nt, 0.0);
  std::vector<uint64_t> cnt(nt, 0);
  std::vector<std::thread> th;
  for (int k = 0; k < nt; k++)
    th.emplace_back([&, k] {
      const uint64_t lo = (uint64_t)end * k / nt, up = (uint64_t)end * (k + 1) / nt;
      double m = 0.0;
      for (uint64_t b = lo; b < up; b++) {
        float t;
        const uint32_t bb = (uint32_t)b;
        std::memcpy(&t, &bb, 4);
        float s, c;
        mcs::sincos_f32(t, s, c);
        double sd, cd;
        ::sincos((double)t, &sd, &cd);
        const double es = std::fabs((double)s - sd), ec = std::fabs((double)c - cd);
        if (es > m) m = es;
        if (ec > m) m = ec;
      }
      mx[k] = m;
      cnt[k] = up - lo;
    });
  for (auto& t : th) t.join();
  double m = 0.0;
  uint64_t n = 0;
  for (int k = 0; k < nt; k++) { if (mx[k] > m) m = mx[k]; n += cnt[k]; }
  std::printf("maxerr %.9e count %llu bound %.9e\n", m, (unsigned long long)n, (double)mcs::kSinCosErr);
  return 0;
}
