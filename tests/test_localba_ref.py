"""LocalBundleAdjustment's assembly and bookkeeping against the reference's OWN text.

tests/golden/localba_ref.npz holds cOptimizer::LocalBundleAdjustment (src/cOptimizer.cpp:
489-908) and cMapPoint's isBad / GetObservations / EraseObservation / TotalNrObservations /
SetBadFlag (src/cMapPoint.cpp:120-206, 259-264) evaluated from the reference text by
tests/golden/gen_localba_ref.py on scripted maps, with g2o's optimizer as a recording stand-in
whose optimize(n) runs one round of this project's g2o restatement (the LM control it uses is
pinned to the g2o text, tests/test_g2o_golden.py).  Recorded: local keyframes, vertices (pose
order, fixed flags, the oneFixed quirk), every edge in vpEdges order, the edges culled in both
passes, the written-back points and the final estimates.

CPU: the product's mcs_local_ba_select (host code) reproduces the selection, vertex flags and
edge list exactly; the oracle's select + local_ba_ex reproduce the culling, write-back sets and
estimates bit for bit (they run the same restated g2o rounds).  GPU: select -> mcs_local_ba_ex
reproduces the culled edges and written-back points exactly, poses abs 1e-6, points with >= 3
observations abs 1e-5, 2-observation points 1e-5 of their scale (as tests/test_ba.py).
"""
import os

import numpy as np
import pytest

from tests import oracle_bind as ob

FIX = os.path.join(os.path.dirname(__file__), "golden", "localba_ref.npz")
_Z = {}


def _fix():
    if "z" not in _Z:
        _Z["z"] = dict(np.load(FIX, allow_pickle=False))
    return _Z["z"]


def _names():
    return sorted({k.split("_")[0] for k in _fix() if k.startswith("s") and k[1].isdigit()})


def _case(name):
    z = _fix()
    p = name + "_"
    m = {k[len(p) + 4:]: z[k] for k in z if k.startswith(p + "map_")}
    cur, ncov, stop = [int(v) for v in z[p + "meta"]]
    return z, p, m, cur, z[p + "covis"], (None if stop < 0 else stop)


def _select(m, cur, cv):
    from mcs_amd import ba
    return ba.local_ba_select(m, cur, cv)


def _expected_slots(z, p, m):
    """Pose slots (keyframe indices) and fixed flags from the recorded vertex sequence."""
    vs = z[p + "vertices"]
    id2kf = {int(i): k for k, i in enumerate(m["kf_id"])}
    mt = vs[vs[:, 1] == 0]
    return np.array([id2kf[int(i)] for i in mt[:, 0]], np.int32), mt[:, 2].astype(np.uint8)


@pytest.mark.parametrize("name", _names())
def test_select_matches_reference_text(name):
    from mcs_amd import ba
    z, p, m, cur, cv, stop = _case(name)
    g = _select(m, cur, cv)
    local = z[p + "local"]
    assert g["status"] == 0 and np.array_equal(g["local_kf"], local)
    if p + "vertices" not in z:
        return
    slots, fixed = _expected_slots(z, p, m)
    assert np.array_equal(np.concatenate([g["local_kf"], g["fixed_kf"]]), slots)
    assert np.array_equal(g["pose_fixed"], fixed)
    pv = z[p + "point_vertices"]
    assert np.array_equal(g["points"], pv[:, 1])
    # every edge in vpEdges order: keyframe slot, point slot, camera, measurement, information
    e = z[p + "edges"]
    slot_of = {int(k): i for i, k in enumerate(slots)}
    pslot = {int(v): i for i, v in enumerate(pv[:, 0])}
    assert len(g["edge_obs"]) == len(e)
    assert np.array_equal(g["edge_pose"], [slot_of[int(k)] for k in e[:, 0]])
    assert np.array_equal(g["edge_point"], [pslot[int(v)] for v in e[:, 1]])
    o = g["edge_obs"]
    assert np.array_equal(m["obs_cam"][o], e[:, 2])
    assert np.array_equal(m["obs_meas"][o], z[p + "edge_meas"])
    assert np.array_equal(m["obs_info"][o], z[p + "edge_info"])
    assert np.all(z[p + "edge_delta"] == 1.345 * float(z["std_recon"]))
    assert np.array_equal(g["point_extra_obs"] >= 0, np.ones(len(g["points"]), bool))


def _problem(z, p, m, g):
    from mcs_amd import ba
    return ba.problem_from_graph(m, g, huber_delta=float(z[p + "edge_delta"][0]))


def _expected_outcome(z, p, n_points):
    e = z[p + "edges"]
    inlier = (e[:, 3] == 0).astype(np.uint8)
    pw = np.zeros(n_points, np.uint8)
    pv = z[p + "point_vertices"]
    slot = {int(pt): i for i, pt in enumerate(pv[:, 1])}
    for row in z[p + "point_write"]:
        pw[slot[int(row[0])]] = 1
    return inlier, pw, len(z[p + "pose_write"]) > 0


@pytest.mark.parametrize("name", _names())
def test_oracle_local_ba_matches_reference_text(name):
    """The oracle's select + LocalBA rounds (restatement) against the text: same culling,
    write-back and (same restated g2o rounds) the same estimates bit for bit."""
    z, p, m, cur, cv, stop = _case(name)
    g = ob.local_ba_select(m, cur, cv)
    if p + "vertices" not in z:
        return
    pr = _problem(z, p, m, g)
    o = ob.local_ba_ex(pr, g["point_extra_obs"], stop_flag=stop)
    inl, pw, wb = _expected_outcome(z, p, len(g["points"]))
    if not z[p + "optimize_log"].size:
        assert o["write_back"] == 0
        return
    assert o["write_back"] == int(wb)
    assert np.array_equal(o["edge_inlier"], inl)
    assert np.array_equal(o["point_write"], pw)
    assert np.array_equal(o["poses"], z[p + "est_poses"])
    assert np.array_equal(o["points"], z[p + "est_points"])
    if stop is not None:
        assert o["stop_flag"] == int(z[p + "stop_after"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", _names())
def test_gpu_local_ba_matches_reference_text(gpu, name):
    from mcs_amd import ba
    z, p, m, cur, cv, stop = _case(name)
    g = _select(m, cur, cv)
    if p + "vertices" not in z:
        return
    pr = _problem(z, p, m, g)
    r = ba.Solver().local_ba_ex(pr, g["point_extra_obs"], stop_flag=stop)
    inl, pw, wb = _expected_outcome(z, p, len(g["points"]))
    if not z[p + "optimize_log"].size:
        assert r["write_back"] == 0
        return
    assert r["write_back"] == int(wb)
    assert np.array_equal(r["edge_inlier"], inl)
    assert np.array_equal(r["point_write"], pw)
    assert np.abs(r["poses"] - z[p + "est_poses"]).max() < 1e-6
    cnt = np.bincount(pr["edge_point"], minlength=len(pr["points"]))
    w3 = (pw == 1) & (cnt >= 3)
    w2 = (pw == 1) & (cnt == 2)
    assert np.abs(r["points"][w3] - z[p + "est_points"][w3]).max() < 1e-5
    if w2.any():
        # two-observation points are weakly constrained along their rays: the same 1e-5 of the
        # point's own scale (distance from the origin) as tests/test_ba.py
        scale = np.maximum(1.0, np.linalg.norm(z[p + "est_points"][w2], axis=1))
        rel = np.abs(r["points"][w2] - z[p + "est_points"][w2]).max(axis=1) / scale
        assert rel.max() < 1e-5, rel.max()


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs the reference checkout")
def test_fixture_regenerates_from_reference_text(tmp_path):
    """In the build container the generator re-derives the fixture from the reference text."""
    import subprocess
    import sys
    out = tmp_path / "l.npz"
    gen = os.path.join(os.path.dirname(__file__), "golden", "gen_localba_ref.py")
    subprocess.check_call([sys.executable, gen, "--out", str(out)], timeout=900)
    q, z = np.load(out), _fix()
    assert sorted(q.files) == sorted(z.keys())
    for k in q.files:
        assert np.array_equal(q[k], z[k]), k
