// LocalBundleAdjustment graph assembly on the host (C-ABI of include/mcs_ba.h):
// cOptimizer::LocalBundleAdjustment src/cOptimizer.cpp:503-769 over a flat map description.
// The reference marks keyframes / points with mnBALocalForKF / mnBAFixedForKF = pKF->mnId;
// here those marks are per-call arrays.  Pure integer bookkeeping, no device work: the
// resulting graph goes to mcs_local_ba_ex.
#include <cstring>
#include <vector>

#include "common.hpp"
#include "../../include/mcs_ba.h"

extern "C" int mcs_local_ba_select(const mcs_lba_map* m, int32_t cur_kf, const int32_t* covis,
                                   int32_t n_covis, mcs_lba_graph* g) {
  using mcs::set_error;
  if (!m || !g || cur_kf < 0 || cur_kf >= m->n_kf || n_covis < 0 || (n_covis > 0 && !covis) ||
      !m->kf_id || !m->kf_bad || !m->kf_mp_off || !m->pt_bad || !m->pt_obs_off ||
      !g->local_kf || !g->fixed_kf || !g->pose_fixed || !g->points || !g->point_extra_obs ||
      (g->edge_cap > 0 && (!g->edge_obs || !g->edge_pose || !g->edge_point)) ||
      (m->kf_mp_off[m->n_kf] > 0 && !m->kf_mp)) {
    set_error("mcs_local_ba_select: null argument");
    return MCS_ERR_ARG;
  }
  if (m->n_points > 0 && m->pt_obs_off[m->n_points] > 0 && !m->obs_kf) {
    set_error("mcs_local_ba_select: null argument (obs_kf)");
    return MCS_ERR_ARG;
  }
  const int nkf = m->n_kf, npt = m->n_points;
  g->n_local = g->n_fixed = g->n_points = g->n_edges = 0;
  std::vector<uint8_t> local_mark(nkf, 0), fixed_mark(nkf, 0), pt_mark(npt, 0);
  std::vector<int32_t> slot(nkf, -1);

  // ---- local keyframes: pKF, then every covisible (marked even when bad, added when not)
  g->local_kf[g->n_local++] = cur_kf;
  local_mark[cur_kf] = 1;
  // GetVectorCovisibleKeyFrames holds each neighbour once and never pKF itself; a list that
  // does not would make pose slots and local_kf disagree, so it is rejected
  for (int i = 0; i < n_covis; i++) {
    const int k = covis[i];
    if (k < 0 || k >= nkf) { set_error("mcs_local_ba_select: covisible index out of range"); return MCS_ERR_ARG; }
    if (local_mark[k]) {
      set_error(k == cur_kf ? "mcs_local_ba_select: covisible list holds the current keyframe"
                            : "mcs_local_ba_select: duplicate covisible keyframe");
      return MCS_ERR_ARG;
    }
    local_mark[k] = 1;
    if (!m->kf_bad[k] && g->n_local < nkf) g->local_kf[g->n_local++] = k;
  }
  if (g->n_local <= 1) return MCS_LBA_EMPTY;   // :519-520

  // ---- local map points in order of first appearance (:521-537)
  for (int i = 0; i < g->n_local; i++) {
    const int k = g->local_kf[i];
    for (int q = m->kf_mp_off[k]; q < m->kf_mp_off[k + 1]; q++) {
      const int p = m->kf_mp[q];
      if (p < 0) continue;
      if (p >= npt) { set_error("mcs_local_ba_select: map point index out of range"); return MCS_ERR_ARG; }
      if (m->pt_bad[p] || pt_mark[p]) continue;
      pt_mark[p] = 1;
      g->points[g->n_points++] = p;
    }
  }

  // ---- fixed keyframes: observers of local points that are neither local nor fixed (:540-558)
  for (int i = 0; i < g->n_points; i++) {
    const int p = g->points[i];
    for (int o = m->pt_obs_off[p]; o < m->pt_obs_off[p + 1]; o++) {
      const int k = m->obs_kf[o];
      if (k < 0 || k >= nkf) { set_error("mcs_local_ba_select: observation keyframe out of range"); return MCS_ERR_ARG; }
      if (!local_mark[k] && !fixed_mark[k]) {
        fixed_mark[k] = 1;
        if (!m->kf_bad[k]) g->fixed_kf[g->n_fixed++] = k;
      }
    }
  }

  // ---- vertex fixed flags (:585-612, 615-627): oneFixed holds the LAST local keyframe's test
  bool oneFixed = false;
  for (int i = 0; i < g->n_local; i++) {
    const int k = g->local_kf[i];
    oneFixed = m->kf_id[k] == 0;
    g->pose_fixed[i] = oneFixed ? 1 : 0;
    slot[k] = i;
  }
  if (!oneFixed && g->n_fixed == 0) g->pose_fixed[0] = 1;   // pKF
  for (int i = 0; i < g->n_fixed; i++) {
    g->pose_fixed[g->n_local + i] = 1;
    slot[g->fixed_kf[i]] = g->n_local + i;
  }

  // ---- one edge per observation of a local point from a good keyframe (:688-766)
  int ne = 0;
  for (int i = 0; i < g->n_points; i++) {
    const int p = g->points[i];
    int extra = 0;
    for (int o = m->pt_obs_off[p]; o < m->pt_obs_off[p + 1]; o++) {
      const int k = m->obs_kf[o];
      if (m->kf_bad[k]) { extra++; continue; }
      if (ne < g->edge_cap) {
        g->edge_obs[ne] = o;
        g->edge_pose[ne] = slot[k];
        g->edge_point[ne] = i;
      }
      ne++;
    }
    g->point_extra_obs[i] = extra;
  }
  g->n_edges = ne;
  if (ne > g->edge_cap) { set_error("mcs_local_ba_select: edge_cap too small"); return MCS_ERR_CAPACITY; }
  return MCS_OK;
}
