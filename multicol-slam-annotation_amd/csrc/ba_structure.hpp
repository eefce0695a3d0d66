// Host side of one bundle-adjustment call: g2o's initializeOptimization(0) +
// buildIndexMapping + BlockSolver<6,3>::buildStructure over the flat problem of
// include/mcs_ba.h (the active set, the Hessian index of every vertex, CSR edge lists and the
// edge pairs of every lower block of the Schur complement, cut into k_schur work items).
// Host-only C++ (also compiled by tools/bench/structure_bench.cpp on the CPU).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/mcs_ba.h"
#include "host_pool.hpp"

namespace mcs {
namespace ba {

#ifndef MCS_SCHUR_CHUNK
#define MCS_SCHUR_CHUNK 128
#endif
constexpr int kSchurChunk = MCS_SCHUR_CHUNK;   // pairs per k_schur wave (config C: 128 beat 32 / 64 / 256)

// host-side structure of one optimize() call (build_structure); owned by the context so its
// capacity is reused across that context's calls and released with it
struct HostStruct {
  std::vector<int32_t> aedge, pose_h, point_h, hpose_vtx, hpt_vtx, pt_ptr, pt_edges, ps_ptr,
      ps_edges, blk_i, blk_j, pr_ptr, pr_e1, pr_e2, it_blk, it_chunk, it_slot, it_nch;
  std::vector<int32_t> pt_h;   // Hessian index of the pose of every pt_edges entry (-1: fixed)
  std::vector<int32_t> cnt_pt, cnt_pose, cursor;     // scan_edges / build_structure scratch
  // the threaded path (HostPool): edge chunk bounds, per-chunk active counts and their
  // compacted edges, per-chunk per-vertex counts (turned into per-chunk fill cursors)
  std::vector<int32_t> par_begin, par_nae, par_off, par_ae, par_pt, par_pose;
  int par_T = 0;   // chunks of the last scan_edges (0: the one-thread path ran)
  // the edges come in non-decreasing point order (LocalBA and GlobalBA build them so): the
  // point lists are then the active-edge list itself, and the fill pass needs no point cursors
  bool pt_sorted = false;
  std::vector<int32_t> tmp_e, tmp_g, tmp_p, tmp_f;   // build_pairs_host scratch
  int n_slots = 0;
  int np = 0, nl = 0;
};

// SparseOptimizer::initializeOptimization(0) + buildIndexMapping + BlockSolver::buildStructure
// (sparse_optimizer.cpp:166-267, block_solver.hpp:143-295) in two passes over the edges.
//
// scan_edges: the vertex-index checks, the active edges (level 0 and not allVerticesFixed) in
// edge order, and per pose / per point their numbers (cnt = the per-pose counts, then the
// active point and edge counts: what the shards all-reduce).  Branch-free in the loop: the
// edges come grouped by point, so a per-edge branch on the data mispredicts and a counter
// chain through memory is the loop's critical path; one pass instead of the four of the
// first version (config C: 0.35 -> 0.11 ms on this build host with build_structure).
// Returns false when an edge names a vertex or camera out of range.
inline bool scan_edges_par(const mcs_ba_problem& p, const uint8_t* level, bool points_fixed,
                           HostStruct& s, std::vector<double>& cnt, HostPool& pool);
// systems at least this large take the threaded path when a pool is given
constexpr int kParMinEdges = 65536;

inline bool scan_edges(const mcs_ba_problem& p, const uint8_t* level, bool points_fixed,
                       HostStruct& s, std::vector<double>& cnt, HostPool* pool = nullptr,
                       int par_min = kParMinEdges) {
  if (pool && pool->size() > 1 && p.n_edges >= par_min)
    return scan_edges_par(p, level, points_fixed, s, cnt, *pool);
  s.par_T = 0;
  const int NE = p.n_edges, NP = p.n_poses, NL = p.n_points;
  s.aedge.resize(NE);
  s.cnt_pt.assign(NL, 0);
  s.cnt_pose.assign(NP, 0);
  int32_t* const ae = s.aedge.data();
  int32_t* const cp = s.cnt_pt.data();
  int32_t* const cpo = s.cnt_pose.data();
  unsigned bad = 0, uns = 0;
  int nae = 0, prev = 0;
  for (int e = 0; e < NE; e++) {
    const int pi = p.edge_pose[e], li = p.edge_point[e], ci = p.edge_cam[e];
    const unsigned b = ((unsigned)pi >= (unsigned)NP) | ((unsigned)li >= (unsigned)NL) |
                       ((unsigned)ci >= (unsigned)p.n_cams);
    bad |= b;
    uns |= (unsigned)(li < prev);
    prev = li;
    if (b) continue;
    const int act = !(level && level[e]) && !(points_fixed && p.pose_fixed[pi]);
    ae[nae] = e;
    nae += act;
    cpo[pi] += act;
    cp[li] += act;
  }
  if (bad) return false;
  s.pt_sorted = uns == 0;
  s.aedge.resize(nae);
  cnt.assign((size_t)NP + 2, 0.0);
  for (int i = 0; i < NP; i++) cnt[i] = cpo[i];
  int nl = 0;
  if (!points_fixed)
    for (int i = 0; i < NL; i++) nl += cp[i] > 0;
  cnt[NP] = nl;
  cnt[NP + 1] = nae;
  return true;
}

// build_structure (after scan_edges on the same HostStruct): active non-fixed poses in vertex
// order (pose_cnt: active edges per pose over ALL shards), active points in vertex order, CSR
// lists point -> edges and pose -> edges in edge order (one fill pass, counting-sort cursors;
// the fixed poses' edges go to a dropped tail run instead of a branch) and the lower pose
// blocks of the Schur complement.  The block pairs themselves: build_pairs_host / the device.
inline void build_structure_fill_par(const mcs_ba_problem& p, bool points_fixed, HostStruct& s,
                                    HostPool& pool);

inline void build_structure(const mcs_ba_problem& p, bool points_fixed,
                            const std::vector<double>& pose_cnt, HostStruct& s, HostPool* pool = nullptr) {
  const int NP = p.n_poses, NL = p.n_points;
  const int nae = (int)s.aedge.size();
  s.pose_h.resize(NP);
  s.hpose_vtx.resize(NP);
  int np = 0;
  for (int i = 0; i < NP; i++) {
    const bool a = pose_cnt[i] > 0 && !p.pose_fixed[i];
    s.pose_h[i] = a ? np : -1;
    if (a) s.hpose_vtx[np++] = i;
  }
  s.np = np;
  s.hpose_vtx.resize(np);
  const int32_t* const poh = s.pose_h.data();
  const int32_t* const ae = s.aedge.data();
  int32_t* const cp = s.cnt_pt.data();
  // pose runs 0 .. np-1, then run np: the edges of fixed poses
  s.ps_ptr.assign(np + 2, 0);
  int32_t* const sp = s.ps_ptr.data();
  for (int i = 0; i < NP; i++) sp[(poh[i] >= 0 ? poh[i] : np) + 1] += s.cnt_pose[i];
  for (int h = 0; h <= np; h++) sp[h + 1] += sp[h];
  s.point_h.resize(NL);
  s.hpt_vtx.resize(NL);
  s.pt_ptr.resize(NL + 1);
  s.pt_ptr[0] = 0;
  int nl = 0;
  int32_t* const ph = s.point_h.data();
  int32_t* const pp = s.pt_ptr.data();
  int32_t* const hv = s.hpt_vtx.data();
  if (!points_fixed) {
    for (int i = 0; i < NL; i++) {
      const int c = cp[i];
      ph[i] = c > 0 ? nl : -1;
      hv[nl] = i;                       // overwritten by the next point unless this one counts
      pp[nl + 1] = pp[nl] + c;
      cp[i] = pp[nl];                   // the point's fill cursor
      nl += c > 0;
    }
  } else {
    for (int i = 0; i < NL; i++) ph[i] = -1;
  }
  s.nl = nl;
  s.hpt_vtx.resize(nl);
  s.pt_ptr.resize(nl + 1);
  s.pt_edges.resize(pp[nl]);
  s.pt_h.resize(pp[nl]);
  s.ps_edges.resize(nae);
  int32_t* const pe = s.pt_edges.data();
  int32_t* const pth = s.pt_h.data();
  int32_t* const pse = s.ps_edges.data();
  if (pool && s.par_T > 0 && s.par_T == pool->size()) {
    build_structure_fill_par(p, points_fixed, s, *pool);
  } else {
  s.cursor.assign(sp, sp + np + 1);
  int32_t* const fs = s.cursor.data();
  if (!points_fixed && s.pt_sorted) {
    // point order = edge order: pt_edges is the active-edge list (no counter chain through
    // the point cursors, which consecutive edges of one point would serialise on)
    if (nae) std::memcpy(pe, ae, (size_t)nae * 4);
    for (int k = 0; k < nae; k++) {
      const int e = ae[k];
      const int h = poh[p.edge_pose[e]];
      pth[k] = h;
      pse[fs[h >= 0 ? h : np]++] = e;
    }
  } else if (!points_fixed) {
    for (int k = 0; k < nae; k++) {
      const int e = ae[k];
      const int h = poh[p.edge_pose[e]];
      const int r = cp[p.edge_point[e]]++;
      pe[r] = e;
      pth[r] = h;                       // the pose's Hessian index per entry (-1: fixed)
      pse[fs[h >= 0 ? h : np]++] = e;
    }
  } else {
    for (int k = 0; k < nae; k++) {
      const int e = ae[k];
      const int h = poh[p.edge_pose[e]];
      pse[fs[h >= 0 ? h : np]++] = e;
    }
  }
  }
  s.ps_edges.resize(sp[np]);
  s.ps_ptr.resize(np + 1);
  const size_t nblk = (size_t)np * (np + 1) / 2;
  s.blk_i.resize(nblk); s.blk_j.resize(nblk);
  for (int i = 0, b = 0; i < np; i++)
    for (int j = 0; j <= i; j++, b++) { s.blk_i[b] = i; s.blk_j[b] = j; }
}

// ---- the threaded path (config-E-sized systems) ----------------------------------------
// scan_edges over T contiguous edge chunks: each chunk compacts its active edges and counts
// them per pose and per point on its own; the chunks' lists are then concatenated in chunk
// order (= edge order) and the counts summed.  build_structure's fill pass runs over the same
// chunks with per-chunk cursors: chunk t's edges of a vertex go after those of chunks < t, so
// every list is in edge order exactly as the one-thread pass leaves it (the outputs are equal,
// tests/test_ba_structure_host.py).
inline bool scan_edges_par(const mcs_ba_problem& p, const uint8_t* level, bool points_fixed,
                           HostStruct& s, std::vector<double>& cnt, HostPool& pool) {
  const int NE = p.n_edges, NP = p.n_poses, NL = p.n_points, T = pool.size();
  s.par_T = T;
  s.par_begin.resize(T + 1);
  for (int t = 0; t <= T; t++) s.par_begin[t] = (int)((int64_t)NE * t / T);
  s.par_nae.assign(T, 0);
  s.par_off.assign(T + 1, 0);
  s.par_ae.resize(NE);
  s.par_pt.resize((size_t)T * NL);
  s.par_pose.resize((size_t)T * NP);
  std::vector<unsigned> bad(T, 0u);
  const int32_t* const epo = p.edge_pose;
  const int32_t* const ept = p.edge_point;
  const int32_t* const eca = p.edge_cam;
  const uint8_t* const pfx = p.pose_fixed;
  const unsigned ncam = (unsigned)p.n_cams;
  pool.run([&, epo, ept, eca, pfx, ncam, level, points_fixed, NP, NL](int t) {
    int32_t* const cp = s.par_pt.data() + (size_t)t * NL;
    int32_t* const cpo = s.par_pose.data() + (size_t)t * NP;
    std::memset(cp, 0, (size_t)NL * 4);
    std::memset(cpo, 0, (size_t)NP * 4);
    const int e0 = s.par_begin[t], e1 = s.par_begin[t + 1];
    int32_t* const out = s.par_ae.data() + e0;
    unsigned b = 0, uns = 0;
    int n = 0, prev = e0 > 0 ? ept[e0 - 1] : 0;
    for (int e = e0; e < e1; e++) {
      const int pi = epo[e], li = ept[e], ci = eca[e];
      const unsigned bb = ((unsigned)pi >= (unsigned)NP) | ((unsigned)li >= (unsigned)NL) |
                          ((unsigned)ci >= ncam);
      b |= bb;
      uns |= (unsigned)(li < prev);
      prev = li;
      if (bb) continue;
      const int act = !(level && level[e]) && !(points_fixed && pfx[pi]);
      out[n] = e;
      n += act;
      cpo[pi] += act;
      cp[li] += act;
    }
    s.par_nae[t] = n;
    bad[t] = b | (uns << 1);
  });
  unsigned uns_all = 0;
  for (int t = 0; t < T; t++) {
    if (bad[t] & 1u) return false;
    uns_all |= bad[t];
  }
  s.pt_sorted = uns_all == 0;
  for (int t = 0; t < T; t++) s.par_off[t + 1] = s.par_off[t] + s.par_nae[t];
  const int nae = s.par_off[T];
  s.aedge.resize(nae);
  s.cnt_pt.resize(NL);
  s.cnt_pose.resize(NP);
  std::vector<int> nl_part(T, 0);
  pool.run([&](int t) {
    std::memcpy(s.aedge.data() + s.par_off[t], s.par_ae.data() + s.par_begin[t], (size_t)s.par_nae[t] * 4);
    // per-vertex totals over the chunks, vertices split over the threads
    const int v0 = (int)((int64_t)NL * t / T), v1 = (int)((int64_t)NL * (t + 1) / T);
    int nl = 0;
    for (int v = v0; v < v1; v++) {
      int c = 0;
      for (int u = 0; u < T; u++) c += s.par_pt[(size_t)u * NL + v];
      s.cnt_pt[v] = c;
      nl += c > 0;
    }
    nl_part[t] = nl;
  });
  for (int i = 0; i < NP; i++) {
    int c = 0;
    for (int u = 0; u < T; u++) c += s.par_pose[(size_t)u * NP + i];
    s.cnt_pose[i] = c;
  }
  cnt.assign((size_t)NP + 2, 0.0);
  for (int i = 0; i < NP; i++) cnt[i] = s.cnt_pose[i];
  int nl = 0;
  if (!points_fixed)
    for (int t = 0; t < T; t++) nl += nl_part[t];
  cnt[NP] = nl;
  cnt[NP + 1] = nae;
  return true;
}

// build_structure's fill pass over scan_edges_par's chunks (pose_h, point_h, pt_ptr and ps_ptr
// are already set): per-chunk cursors from the per-chunk counts, then each chunk writes its
// active edges into the point and pose lists
inline void build_structure_fill_par(const mcs_ba_problem& p, bool points_fixed, HostStruct& s,
                                     HostPool& pool) {
  const int NP = p.n_poses, NL = p.n_points, T = s.par_T;
  const int np = s.np;
  const int32_t* const poh = s.pose_h.data();
  const int32_t* const ph = s.point_h.data();
  const int32_t* const pp = s.pt_ptr.data();
  const int32_t* const sp = s.ps_ptr.data();
  // pose cursors per (chunk, pose vertex): active poses fill their run, fixed poses the dropped
  // tail run np
  {
    int tail = sp[np];
    for (int i = 0; i < NP; i++) {
      int base = poh[i] >= 0 ? sp[poh[i]] : tail;
      for (int u = 0; u < T; u++) {
        int32_t& c = s.par_pose[(size_t)u * NP + i];
        const int n = c;
        c = base;
        base += n;
      }
      if (poh[i] < 0) tail = base;
    }
  }
  int32_t* const pe = s.pt_edges.data();
  int32_t* const pth = s.pt_h.data();
  int32_t* const pse = s.ps_edges.data();
  const bool sorted = s.pt_sorted;
  if (!sorted) pool.run([&](int t) {
    if (!points_fixed) {   // point cursors per (chunk, point vertex), vertices split over threads
      const int v0 = (int)((int64_t)NL * t / T), v1 = (int)((int64_t)NL * (t + 1) / T);
      for (int v = v0; v < v1; v++) {
        if (ph[v] < 0) continue;
        int base = pp[ph[v]];
        for (int u = 0; u < T; u++) {
          int32_t& c = s.par_pt[(size_t)u * NL + v];
          const int n = c;
          c = base;
          base += n;
        }
      }
    }
  });
  pool.run([&](int t) {
    int32_t* const cp = s.par_pt.data() + (size_t)t * NL;
    int32_t* const cpo = s.par_pose.data() + (size_t)t * NP;
    const int32_t* const ae = s.aedge.data() + s.par_off[t];
    const int n = s.par_nae[t];
    if (!points_fixed && sorted) {
      int32_t* const pek = pe + s.par_off[t];
      int32_t* const phk = pth + s.par_off[t];
      if (n) std::memcpy(pek, ae, (size_t)n * 4);
      for (int k = 0; k < n; k++) {
        const int e = ae[k];
        const int pv = p.edge_pose[e];
        phk[k] = poh[pv];
        pse[cpo[pv]++] = e;
      }
    } else if (!points_fixed) {
      for (int k = 0; k < n; k++) {
        const int e = ae[k];
        const int pv = p.edge_pose[e];
        const int r = cp[p.edge_point[e]]++;
        pe[r] = e;
        pth[r] = poh[pv];
        pse[cpo[pv]++] = e;
      }
    } else {
      for (int k = 0; k < n; k++) {
        const int e = ae[k];
        const int pv = p.edge_pose[e];
        pse[cpo[pv]++] = e;
      }
    }
  });
  (void)np;
}

// The edge pairs of every lower block in (point, e1, e2) order and the k_schur work items, on
// the host.  The product builds both on the device (ba.hip, enqueue_pairs); this restatement
// is the checker of that build (mcs_ba_check_structure) and the CPU timing reference
// (tools/bench/structure_bench.cpp).
inline void build_pairs_host(const mcs_ba_problem& p, HostStruct& s) {
  const size_t nblk = (size_t)s.np * (s.np + 1) / 2;
  s.pr_ptr.assign(nblk + 1, 0);
  // Per point, its edges with an active pose, grouped by pose (stable, so edge order inside
  // a group): the pairs of block (i1, i2), i2 <= i1, that a point contributes are then the
  // product group(i1) x group(i2) in (e1, e2) order -- the order of the plain double loop over
  // the point's edges, without visiting the pairs that fall above the diagonal.
  std::vector<int32_t>& ge = s.tmp_e;   // grouped edges, point by point
  std::vector<int32_t>& gr = s.tmp_g;   // groups: (pose, begin, end) triples
  std::vector<int32_t>& gp = s.tmp_p;   // per point: first group (nl + 1 entries)
  ge.clear(); gr.clear(); gp.assign(s.nl + 1, 0);
  for (int l = 0; l < s.nl; l++) {
    const size_t b0 = ge.size();
    for (int a = s.pt_ptr[l]; a < s.pt_ptr[l + 1]; a++) {
      const int e = s.pt_edges[a];
      const int h = s.pose_h[p.edge_pose[e]];
      if (h < 0) continue;
      // insertion into (pose, edge order), stable
      ge.push_back(e);
      size_t q = ge.size() - 1;
      while (q > b0 && s.pose_h[p.edge_pose[ge[q - 1]]] > h) { ge[q] = ge[q - 1]; q--; }
      ge[q] = e;
    }
    for (size_t q = b0; q < ge.size();) {
      const int h = s.pose_h[p.edge_pose[ge[q]]];
      size_t r = q + 1;
      while (r < ge.size() && s.pose_h[p.edge_pose[ge[r]]] == h) r++;
      gr.push_back(h); gr.push_back((int32_t)q); gr.push_back((int32_t)r);
      q = r;
    }
    gp[l + 1] = (int32_t)(gr.size() / 3);
  }
  auto for_blocks = [&](auto&& f) {   // f(block, group of i1, group of i2), point by point
    for (int l = 0; l < s.nl; l++)
      for (int gi = gp[l]; gi < gp[l + 1]; gi++) {
        const int h1 = gr[3 * gi];
        for (int gj = gp[l]; gj <= gi; gj++)
          f((size_t)h1 * (h1 + 1) / 2 + gr[3 * gj], gi, gj);
      }
  };
  for_blocks([&](size_t blk, int gi, int gj) {
    s.pr_ptr[blk + 1] += (gr[3 * gi + 2] - gr[3 * gi + 1]) * (gr[3 * gj + 2] - gr[3 * gj + 1]);
  });
  for (size_t b = 0; b < nblk; b++) s.pr_ptr[b + 1] += s.pr_ptr[b];
  s.pr_e1.assign(s.pr_ptr[nblk], 0);
  s.pr_e2.assign(s.pr_ptr[nblk], 0);
  std::vector<int32_t>& fill = s.tmp_f;
  fill.assign(s.pr_ptr.begin(), s.pr_ptr.end() - 1);
  for_blocks([&](size_t blk, int gi, int gj) {
    int q = fill[blk];
    for (int a = gr[3 * gi + 1]; a < gr[3 * gi + 2]; a++)
      for (int b = gr[3 * gj + 1]; b < gr[3 * gj + 2]; b++, q++) {
        s.pr_e1[q] = ge[a];
        s.pr_e2[q] = ge[b];
      }
    fill[blk] = q;
  });
  // k_schur work items: chunks of kSchurChunk pairs (and, on diagonal blocks, pose edges)
  s.it_blk.clear(); s.it_chunk.clear(); s.it_slot.clear(); s.it_nch.clear();
  s.n_slots = 0;
  for (size_t b = 0; b < nblk; b++) {
    const int np_ = s.pr_ptr[b + 1] - s.pr_ptr[b];
    int ne = 0;
    if (s.blk_i[b] == s.blk_j[b]) ne = s.ps_ptr[s.blk_i[b] + 1] - s.ps_ptr[s.blk_i[b]];
    const int nch = std::max(1, (std::max(np_, ne) + kSchurChunk - 1) / kSchurChunk);
    for (int c = 0; c < nch; c++) {
      s.it_blk.push_back((int32_t)b);
      s.it_chunk.push_back(c);
      s.it_slot.push_back(nch > 1 ? s.n_slots + c : -1);
      s.it_nch.push_back(nch);
    }
    if (nch > 1) s.n_slots += nch;
  }
}

}  // namespace ba
}  // namespace mcs
