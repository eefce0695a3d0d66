"""GlobalBundleAdjustment / PoseOptimization against the reference's OWN text.

tests/golden/globalba_ref.npz holds cOptimizer::BundleAdjustment (src/cOptimizer.cpp:73-261) and
cOptimizer::PoseOptimization (:264-486) evaluated from the reference text by
tests/golden/gen_globalba_ref.py: the vertices with their g2o ids (keyframe mnId, the maxKF rule
for the Mc / IO / point ids, mnId 0 fixed, poseOnly), the collision of two vertex ids when vpKFs
is not id-ordered, the edges (keyframe, point vertex, camera, measurement, information I,
Huber sqrt(5.991)), the optimize calls, the write-back (and which list entries have no vertex to
read back: undefined in the reference), and for PoseOptimization the point vertex per distinct
mnId, one edge per non-NULL match, invSigma2(octave) information, 1.345 * huberMultiplier, the
two rounds, the outlier flags and the returned counts.

  * CPU: the product's graph assembly (mcs_global_ba_select / mcs_pose_optimization_select)
    reproduces every vertex id, fixed flag, edge and write-back slot; the oracle's optimisation
    of the assembled problem reproduces the fixture's results bit for bit (the fixture's
    optimize() calls ran the same restated g2o rounds);
  * GPU: select -> mcs_global_ba / mcs_pose_optimization: iterations equal, poses abs 1e-6,
    points 1e-5 of their scale, PoseOptimization's outlier flags and counts identical.
"""
import os

import numpy as np
import pytest

FIX = os.path.join(os.path.dirname(__file__), "golden", "globalba_ref.npz")


def _fix():
    return np.load(FIX, allow_pickle=False)


def _gba_names():
    return [str(n) for n in _fix()["gba_names"]]


def _po_names():
    return [str(n) for n in _fix()["po_names"]]


def _gba_case(name):
    z = _fix()
    p = name + "_"
    m = {k[len(p) + 4:]: z[k] for k in z.files if k.startswith(p + "map_")}
    pose_only, stop, collision = [int(v) for v in z[p + "meta"]]
    return z, p, m, pose_only, (None if stop < 0 else stop), collision


def _select(m):
    from mcs_amd import ba
    return ba.global_ba_select(dict(m), raise_on_error=False)


def test_fixture_basics():
    z = _fix()
    assert int(z["n_statements"]) > 150
    assert len(_gba_names()) >= 6 and len(_po_names()) >= 3
    assert any(int(z[n + "_meta"][2]) >= 0 for n in _gba_names())       # a collision case


@pytest.mark.parametrize("name", _gba_names())
def test_select_matches_reference_text(built, name):
    """Vertex ids / kinds / fixed flags, the maxKF rule, collisions, edges and write-back slots."""
    z, p, m, pose_only, stop, collision = _gba_case(name)
    g = _select(m)
    verts = z[p + "vertices"]                     # (id, kind, fixed, refused) in addVertex order
    if collision >= 0:
        assert g["status"] < 0 and g["collision_id"] == collision
        return
    assert g["status"] == 0 and g["collision_id"] == -1
    assert not verts[:, 3].any()
    mt = verts[verts[:, 1] == 0]
    assert np.array_equal(m["kf_id"][g["pose_kf"]], mt[:, 0])
    assert np.array_equal(g["pose_fixed"], mt[:, 2])
    nc = len(m["mc"])
    assert np.array_equal(verts[verts[:, 1] == 1, 0], g["mc_vertex_id0"] + np.arange(nc))
    assert np.array_equal(verts[verts[:, 1] == 2, 0], g["io_vertex_id0"] + np.arange(nc))
    pv = z[p + "point_vertices"]                  # (vertex id, vpMP index)
    assert np.array_equal(g["point_vertex_id"], pv[:, 0]) and np.array_equal(g["points"], pv[:, 1])
    assert np.array_equal(verts[verts[:, 1] == 3, 2], np.full(len(pv), pose_only))
    e = z[p + "edges"]                            # (vpKFs index, point vertex id, camera)
    assert np.array_equal(g["pose_kf"][g["edge_pose"]], e[:, 0])
    assert np.array_equal(g["point_vertex_id"][g["edge_point"]], e[:, 1])
    assert np.array_equal(m["obs_cam"][g["edge_obs"]], e[:, 2])
    assert np.array_equal(m["obs_meas"][g["edge_obs"]], z[p + "edge_meas"])
    assert np.all(z[p + "edge_info"] == 1.0) and np.all(z[p + "edge_delta"] == np.sqrt(5.991))
    # write-back: the text wrote exactly the entries with a slot, in list order
    pw, ub = z[p + "pose_write"], z[p + "pose_ub"]
    assert np.array_equal(np.nonzero(g["kf_slot"] >= 0)[0], pw[:, 0].astype(int))
    assert np.array_equal(np.nonzero(g["kf_slot"] < 0)[0], ub)
    qw, qub = z[p + "point_write"], z[p + "point_ub"]
    assert np.array_equal(np.nonzero(g["pt_slot"] >= 0)[0], qw[:, 0].astype(int))
    assert np.array_equal(np.nonzero(g["pt_slot"] < 0)[0], qub)


def _gba_problem(m, g, pose_only):
    from mcs_amd import ba
    pr = ba.problem_from_gba_graph(m, g)
    return pr


@pytest.mark.parametrize("name", _gba_names())
def test_oracle_global_ba_matches_reference_text(built, name):
    from mcs_amd import ba
    from tests import oracle_bind as ob
    z, p, m, pose_only, stop, collision = _gba_case(name)
    if collision >= 0:
        return
    g = _select(m)
    pr = _gba_problem(m, g, pose_only)
    o = ba.BAOptions(max_iterations=15, gain_threshold=1e-6, terminate_max_iter=15)
    r = ob.ba_optimize(pr, o, stop_flag=0 if stop is None else stop, points_fixed=bool(pose_only))
    log = z[p + "optimize_log"]
    assert r["report"].iterations == int(log[0, 1])
    kp, pp = ba.global_ba_write_back(m, g, r["poses"], r["points"])
    pw, qw = z[p + "pose_write"], z[p + "point_write"]
    assert np.array_equal(kp[pw[:, 0].astype(int)], pw[:, 1:])
    assert np.array_equal(pp[qw[:, 0].astype(int)], qw[:, 1:])


@pytest.mark.gpu
@pytest.mark.parametrize("name", _gba_names())
def test_gpu_global_ba_matches_reference_text(gpu, name):
    from mcs_amd import ba
    z, p, m, pose_only, stop, collision = _gba_case(name)
    if collision >= 0:
        return
    g = _select(m)
    pr = _gba_problem(m, g, pose_only)
    r = ba.Solver().global_ba(pr, pose_only=bool(pose_only), stop_flag=stop)
    log = z[p + "optimize_log"]
    assert r["report"].iterations == int(log[0, 1])
    kp, pp = ba.global_ba_write_back(m, g, r["poses"], r["points"])
    pw, qw = z[p + "pose_write"], z[p + "point_write"]
    assert np.abs(kp[pw[:, 0].astype(int)] - pw[:, 1:]).max() < 1e-6
    want = qw[:, 1:]
    scale = np.maximum(1.0, np.linalg.norm(want, axis=1))
    rel = np.abs(pp[qw[:, 0].astype(int)] - want).max(axis=1) / scale
    assert rel.max() < 1e-5, rel.max()
    if stop is not None:
        assert r["stop_flag"] == int(z[p + "stop_after"])


# ---------------------------------------------------------------------------- PoseOptimization
def _po_case(name):
    z = _fix()
    p = name + "_"
    return z, p


def _po_problem(z, p, g):
    """The mcs_ba_problem PoseOptimization builds (:364-430) from the select's lists."""
    k = g["edge_obs"]
    oct_ = z[p + "key_oct"][k]
    return dict(poses=z[p + "pose"].reshape(1, 6).copy(), pose_fixed=np.zeros(1, np.uint8),
                points=np.ascontiguousarray(z[p + "pt_pos"][g["points"]]), mc=z[p + "mc"], cam=z[p + "cam"],
                edge_pose=np.zeros(len(k), np.int32), edge_point=g["edge_point"].astype(np.int32),
                edge_cam=z[p + "key_cam"][k].astype(np.int32), edge_meas=np.ascontiguousarray(z[p + "key_pt"][k]),
                edge_info=z[p + "inv_sigma2"][oct_].copy(), huber_delta=1.345 * float(z[p + "huber_mult"]))


def _po_select(z, p):
    from mcs_amd import ba
    return ba.pose_optimization_select(z[p + "key_mp"], z[p + "pt_id"], len(z[p + "mc"]))


def _outlier_of_keys(z, p, g, edge_outlier):
    out = np.zeros(len(z[p + "key_mp"]), np.uint8)
    out[g["edge_obs"]] = edge_outlier
    return out


@pytest.mark.parametrize("name", _po_names())
def test_pose_select_matches_reference_text(built, name):
    z, p = _po_case(name)
    g = _po_select(z, p)
    verts = z[p + "vertices"]
    nc = len(z[p + "mc"])
    assert np.array_equal(verts[:1 + 2 * nc, 0], np.arange(1 + 2 * nc))
    pv = z[p + "point_vertices"]
    assert np.array_equal(g["point_vertex_id"], pv[:, 0]) and np.array_equal(g["points"], pv[:, 1])
    assert np.all(verts[verts[:, 1] == 3, 2] == 1)          # every point vertex fixed (:382)
    e = z[p + "edges"]                                     # (map point index, camera)
    assert np.array_equal(g["points"][g["edge_point"]], e[:, 0])
    assert np.array_equal(z[p + "key_cam"][g["edge_obs"]], e[:, 1])
    pr = _po_problem(z, p, g)
    assert np.array_equal(pr["edge_meas"], z[p + "edge_meas"])
    assert np.array_equal(pr["edge_info"], z[p + "edge_info"])
    assert np.all(z[p + "edge_delta"] == pr["huber_delta"])


@pytest.mark.parametrize("name", _po_names())
def test_oracle_pose_optimization_matches_reference_text(built, name):
    from tests import oracle_bind as ob
    z, p = _po_case(name)
    g = _po_select(z, p)
    r = ob.pose_optimization(_po_problem(z, p, g))
    assert np.array_equal(_outlier_of_keys(z, p, g, r["outlier"]), z[p + "outlier"])
    assert r["n_good"] == int(z[p + "ret"])
    assert r["bad_ratio"] == float(z[p + "inliers"])
    assert np.array_equal(r["pose"], z[p + "pose_out"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", _po_names())
def test_gpu_pose_optimization_matches_reference_text(gpu, name):
    from mcs_amd import ba
    z, p = _po_case(name)
    g = _po_select(z, p)
    r = ba.Solver().pose_optimization(_po_problem(z, p, g))
    assert np.array_equal(_outlier_of_keys(z, p, g, r["outlier"]), z[p + "outlier"])
    assert r["n_good"] == int(z[p + "ret"])
    assert r["bad_ratio"] == float(z[p + "inliers"])
    assert np.abs(r["pose"] - z[p + "pose_out"]).max() < 1e-6
    log = z[p + "optimize_log"]
    assert r["report1"].iterations == int(log[0, 1]) and r["report2"].iterations == int(log[1, 1])


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs the reference checkout")
def test_fixture_regenerates_from_reference_text(tmp_path):
    """In the build container the generator re-derives the fixture from the reference text."""
    import subprocess
    import sys
    out = tmp_path / "g.npz"
    gen = os.path.join(os.path.dirname(__file__), "golden", "gen_globalba_ref.py")
    subprocess.check_call([sys.executable, gen, "--out", str(out)], timeout=900)
    q, z = np.load(out), _fix()
    assert sorted(q.files) == sorted(z.files)
    for k in q.files:
        assert np.array_equal(q[k], z[k]), k
