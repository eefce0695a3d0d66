// BundleAdjustment and PoseOptimization graph assembly on the host (C-ABI of include/mcs_ba.h):
// cOptimizer::BundleAdjustment src/cOptimizer.cpp:101-259 and cOptimizer::PoseOptimization
// :294-430 over flat map / frame descriptions.  g2o's vertex table (id -> vertex) becomes an
// id -> (kind, slot) hash map, so the id rules of the reference -- including its maxKF quirk and
// what a repeated id does -- are decided exactly as g2o's addVertex / vertex(id) would decide
// them.  Pure integer bookkeeping, no device work: the graph goes to mcs_global_ba /
// mcs_pose_optimization.
#include <cstdio>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "../../include/mcs_ba.h"

namespace {

enum VertexKind : int32_t { V_POSE = 0, V_MC = 1, V_IO = 2, V_POINT = 3 };
struct VertexRef { int32_t kind, slot; };

// g2o::OptimizableGraph::addVertex (optimizable_graph.cpp:243-262): a second vertex with a
// registered id is refused and the first one stays
bool add_vertex(std::unordered_map<int64_t, VertexRef>& ids, int64_t id, int32_t kind, int32_t slot) {
  return ids.emplace(id, VertexRef{kind, slot}).second;
}

}  // namespace

extern "C" int mcs_global_ba_select(const mcs_gba_map* m, mcs_gba_graph* g) {
  using mcs::set_error;
  if (!m || !g || m->n_kf < 0 || m->n_points < 0 || m->n_cams <= 0 || !m->kf_id || !m->kf_bad ||
      (m->n_points > 0 && (!m->pt_id || !m->pt_bad || !m->pt_obs_off)) ||
      !g->pose_kf || !g->pose_fixed || !g->kf_slot || (m->n_points > 0 && (!g->points || !g->pt_slot)) ||
      (g->edge_cap > 0 && (!g->edge_obs || !g->edge_pose || !g->edge_point))) {
    set_error("mcs_global_ba_select: null or invalid argument");
    return MCS_ERR_ARG;
  }
  if (m->n_points > 0 && m->pt_obs_off[m->n_points] > 0 && !m->obs_kf) {
    set_error("mcs_global_ba_select: null argument (obs_kf)");
    return MCS_ERR_ARG;
  }
  g->n_poses = g->n_points = g->n_edges = 0;
  g->collision_id = -1;
  g->mc_vertex_id0 = g->io_vertex_id0 = -1;
  if (m->n_kf == 0) {             // the reference reads vpKFs[0]->camSystem (:134)
    set_error("mcs_global_ba_select: empty keyframe list");
    return MCS_ERR_ARG;
  }
  const int nkf = m->n_kf, npt = m->n_points, nc = m->n_cams;
  std::unordered_map<int64_t, VertexRef> ids;
  ids.reserve((size_t)nkf + 2 * nc + npt);
  auto collide = [&](int64_t id) {
    g->collision_id = id;
    char buf[160];
    std::snprintf(buf, sizeof buf, "mcs_global_ba_select: a vertex with ID %lld has already been "
                  "registered with this graph (g2o addVertex FATAL, optimizable_graph.cpp:247)", (long long)id);
    set_error(buf);
    return MCS_ERR_ARG;
  };

  // ---- keyframe vertices (:110-130); maxKF follows the last good keyframe with mnId > 0
  int64_t maxKF = 0;
  const int64_t maxKFid = 0;      // declared and never updated by the reference (:105)
  for (int i = 0; i < nkf; i++) {
    g->kf_slot[i] = -1;
    if (m->kf_bad[i]) continue;
    const int64_t id = m->kf_id[i];
    const int s = g->n_poses;
    if (!add_vertex(ids, id, V_POSE, s)) return collide(id);
    g->pose_kf[s] = i;
    g->pose_fixed[s] = id == 0 ? 1 : 0;
    g->n_poses++;
    if (id > maxKFid) maxKF = id;
  }
  int64_t cur = maxKF + 1;        // currVertexIdx (:132)
  // ---- Mc and IO vertices (:136-159)
  g->mc_vertex_id0 = cur;
  for (int c = 0; c < nc; c++, cur++)
    if (!add_vertex(ids, cur, V_MC, c)) return collide(cur);
  g->io_vertex_id0 = cur;
  for (int c = 0; c < nc; c++, cur++)
    if (!add_vertex(ids, cur, V_IO, c)) return collide(cur);

  // ---- point vertices (:165-182) and the mnId -> vertex map
  std::unordered_map<int64_t, int32_t> pt_of_id;
  pt_of_id.reserve((size_t)npt);
  for (int i = 0; i < npt; i++) {
    if (m->pt_bad[i]) continue;
    const int s = g->n_points;
    if (!add_vertex(ids, cur, V_POINT, s)) return collide(cur);
    g->points[s] = i;
    if (g->point_vertex_id) g->point_vertex_id[s] = cur;
    pt_of_id[m->pt_id[i]] = s;     // mapPointId_to_cont_g2oId[pMP->mnId] = currVertexIdx (:176)
    g->n_points++;
    cur++;
  }

  // ---- edges (:184-231): vertex(pKF->mnId) for the pose
  int ne = 0;
  for (int s = 0; s < g->n_points; s++) {
    const int p = g->points[s];
    for (int o = m->pt_obs_off[p]; o < m->pt_obs_off[p + 1]; o++) {
      const int k = m->obs_kf[o];
      if (k < 0 || k >= nkf) { set_error("mcs_global_ba_select: observation keyframe out of range"); return MCS_ERR_ARG; }
      if (m->kf_bad[k]) continue;
      auto it = ids.find(m->kf_id[k]);
      if (it == ids.end() || it->second.kind != V_POSE) {
        set_error("mcs_global_ba_select: an observing keyframe has no pose vertex");
        return MCS_ERR_ARG;
      }
      if (ne < g->edge_cap) {
        g->edge_obs[ne] = o;
        g->edge_pose[ne] = it->second.slot;
        g->edge_point[ne] = s;
      }
      ne++;
    }
  }
  g->n_edges = ne;

  // ---- write-back slots (:242-259)
  for (int i = 0; i < nkf; i++) {
    auto it = ids.find(m->kf_id[i]);
    g->kf_slot[i] = (it != ids.end() && it->second.kind == V_POSE) ? it->second.slot : -1;
  }
  for (int i = 0; i < npt; i++) {
    auto it = pt_of_id.find(m->pt_id[i]);
    g->pt_slot[i] = it != pt_of_id.end() ? it->second : -1;
  }
  if (ne > g->edge_cap) { set_error("mcs_global_ba_select: edge_cap too small"); return MCS_ERR_CAPACITY; }
  return MCS_OK;
}

extern "C" int mcs_pose_optimization_select(const mcs_po_frame* f, mcs_po_graph* g) {
  using mcs::set_error;
  if (!f || !g || f->n_keys < 0 || f->n_mp < 0 || f->n_cams <= 0 ||
      (f->n_keys > 0 && !f->key_mp) || (f->n_mp > 0 && (!f->pt_id || !g->points)) ||
      (g->edge_cap > 0 && (!g->edge_obs || !g->edge_point))) {
    set_error("mcs_pose_optimization_select: null or invalid argument");
    return MCS_ERR_ARG;
  }
  g->n_points = g->n_edges = 0;
  // vertex 0 = Mt, 1..nc = Mc, nc+1..2nc = IO (:296-342); points from 2nc + 1 on
  int64_t cur = 1 + 2 * (int64_t)f->n_cams;
  std::unordered_map<int64_t, int32_t> slot_of_id;     // mapPt_2_obs_idx / mapPointId_to_cont_g2oId
  slot_of_id.reserve((size_t)f->n_mp);
  int ne = 0;
  for (int i = 0; i < f->n_keys; i++) {
    const int p = f->key_mp[i];
    if (p < 0) continue;         // NULL association (:370)
    if (p >= f->n_mp) { set_error("mcs_pose_optimization_select: map point index out of range"); return MCS_ERR_ARG; }
    auto it = slot_of_id.find(f->pt_id[p]);
    int s;
    if (it == slot_of_id.end()) {
      s = g->n_points++;
      slot_of_id.emplace(f->pt_id[p], s);
      g->points[s] = p;
      if (g->point_vertex_id) g->point_vertex_id[s] = cur;
      cur++;
    } else {
      s = it->second;
    }
    if (ne < g->edge_cap) {
      g->edge_obs[ne] = i;
      g->edge_point[ne] = s;
    }
    ne++;
  }
  g->n_edges = ne;
  if (ne > g->edge_cap) { set_error("mcs_pose_optimization_select: edge_cap too small"); return MCS_ERR_CAPACITY; }
  return MCS_OK;
}
