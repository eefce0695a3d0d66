// CPU timing of the BA host structure build (ba_structure.hpp) on a dumped problem:
//   python tools/bench/dump_problem.py /tmp/cfgc && g++ -O3 -std=c++17 \
//     -pthread tools/bench/structure_bench.cpp -o /tmp/sb && /tmp/sb /tmp/cfgc [threads]
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "../../multicol-slam-annotation_amd/csrc/ba_structure.hpp"

template <typename T>
std::vector<T> load(const std::string& f) {
  std::ifstream in(f, std::ios::binary | std::ios::ate);
  const size_t n = (size_t)in.tellg() / sizeof(T);
  in.seekg(0);
  std::vector<T> v(n);
  in.read(reinterpret_cast<char*>(v.data()), n * sizeof(T));
  return v;
}

int main(int argc, char** argv) {
  const std::string d = argc > 1 ? argv[1] : "/tmp/cfgc";
  auto ep = load<int32_t>(d + "/edge_pose.bin"), el = load<int32_t>(d + "/edge_point.bin");
  auto pf = load<uint8_t>(d + "/pose_fixed.bin");
  auto np = load<int32_t>(d + "/sizes.bin");
  mcs_ba_problem p{};
  p.n_poses = np[0]; p.n_points = np[1]; p.n_edges = (int)ep.size(); p.n_cams = 3;
  std::vector<int32_t> ec(ep.size(), 0);   // camera indices: only range-checked here
  p.edge_pose = ep.data(); p.edge_point = el.data(); p.pose_fixed = pf.data(); p.edge_cam = ec.data();
  const int threads = argc > 2 ? std::atoi(argv[2]) : 1;
  mcs::HostPool pool(threads);
  mcs::ba::HostStruct s;
  double best = 1e9, best_sb = 1e9;
  using clk = std::chrono::steady_clock;
  for (int r = 0; r < 50; r++) {
    const auto t0 = clk::now();
    std::vector<double> cnt;
    mcs::ba::scan_edges(p, nullptr, false, s, cnt, &pool);
    mcs::ba::build_structure(p, false, cnt, s, &pool);
    const auto t1 = clk::now();
    mcs::ba::build_pairs_host(p, s);
    const auto t2 = clk::now();
    best_sb = std::min(best_sb, std::chrono::duration<double, std::milli>(t1 - t0).count());
    best = std::min(best, std::chrono::duration<double, std::milli>(t2 - t0).count());
  }
  std::printf("edges %d points %d poses %d threads %d: np %d nl %d pairs %zu items %zu  scan+structure %.3f ms, "
              "with pairs %.3f ms (best of 50)\n", p.n_edges, p.n_points, p.n_poses, threads, s.np, s.nl,
              s.pr_e1.size(), s.it_blk.size(), best_sb, best);
  return 0;
}
