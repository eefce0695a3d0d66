// HostPool (csrc/host_pool.hpp): every run(f) calls f(0) .. f(n-1) exactly once each and
// returns only after all of them finished; repeated runs, pools of 1..16 workers, and a pool
// destroyed right after its last run.  Prints "ok" or the first failure.
#include <atomic>
#include <cstdio>
#include <vector>
#include "../../multicol-slam-annotation_amd/csrc/host_pool.hpp"

int main() {
  for (int n = 1; n <= 16; n++) {
    mcs::HostPool pool(n);
    if (pool.size() != n) { std::printf("size %d != %d\n", pool.size(), n); return 1; }
    std::vector<int> hits(n, 0);
    for (int rep = 0; rep < 2000; rep++) {
      std::vector<std::atomic<int>> seen(n);
      for (auto& s : seen) s = 0;
      pool.run([&](int t) { seen[t].fetch_add(1); hits[t]++; });
      for (int t = 0; t < n; t++)
        if (seen[t].load() != 1) { std::printf("n %d rep %d: index %d ran %d times\n", n, rep, t, seen[t].load()); return 1; }
    }
    for (int t = 0; t < n; t++)
      if (hits[t] != 2000) { std::printf("n %d: index %d hits %d\n", n, t, hits[t]); return 1; }
  }
  { mcs::HostPool p0(0); if (p0.size() != 1) { std::printf("size of HostPool(0) %d\n", p0.size()); return 1; } }
  std::printf("ok\n");
  return 0;
}
