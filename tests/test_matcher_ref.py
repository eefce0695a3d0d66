"""The matcher against the reference's OWN text.

tests/golden/matcher_ref.npz holds, evaluated from the reference's text by
tests/golden/gen_matcher_ref.py (tests/golden/cxx_eval.py translator):
  * a11 DescriptorDistance64 / DescriptorDistance64Masked (src/cORBmatcher.cpp:2443-2477) and the
    ctor's TH_HIGH_ / TH_LOW_ (:46-65);
  * a10 the cMultiFrame ctor's feature grid (src/cMultiFrame.cpp:154-184, PosInGrid :342-353)
    and scale tables (:193-209) on scripted extractor outputs;
  * a13 the four windowed searches (SearchByProjection(F, MPs) :67-166, SearchByProjection
    (Current, Last) :1991-2123, SearchForInitialization :579-726, WindowSearch :326-473) with
    GetFeaturesInArea (:272-340): every GetFeaturesInArea call, its index list, the query
    descriptor the caller read, and the rule's final assignment;
  * a12 SearchForTriangulationRaw (:968-1155) on scripted keyframes (rig poses, rays,
    descriptors, map-point matches; ComputeE / CheckDistEpipolarLine from the reference text).
Map points / keyframes / the rig are scripted stand-ins (orientation check off, as the
reference's matchers run).  Index / distance / match outputs: exact.

CPU: the product's host pieces (mcs_frame_grid_build, mcs_window_select, the distance entry
points) and the oracle against the fixture.  GPU: mcs_window_search_device candidate lists and
distances, mcs_window_match, mcs_search_for_triangulation_raw[_masked].
"""
import ctypes
import os

import numpy as np
import pytest

from tests import oracle_bind as ob

FIX = os.path.join(os.path.dirname(__file__), "golden", "matcher_ref.npz")
RULES = [(0, "th1", 0.8), (0, "th3", 0.8), (3, "ws40", 0.7), (3, "ws80", 0.7), (2, "ws50", 0.9),
         (2, "ws100", 0.9), (1, "th7", 0.9), (1, "th15", 0.9)]
NC = 3


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


_Z = {}


def _fix():
    if "z" not in _Z:
        _Z["z"] = dict(np.load(FIX, allow_pickle=False))
    return _Z["z"]


def _popc(x):
    return np.unpackbits(np.ascontiguousarray(x, np.uint8), axis=-1).sum(axis=-1).astype(np.int32)


def _dist(q, d, qm=None, dm=None):
    x = np.bitwise_xor(q, d)
    if qm is None:
        return _popc(x)
    return (_popc(x & qm) + _popc(x & dm)) // 2


def _frame(z, sc, tag):
    p = "w%d_%s_" % (sc, tag)
    return dict(xy=z[p + "xy"], oct=z[p + "oct"], cam=z[p + "cam"], loc=z[p + "loc"], desc=z[p + "desc"],
                dmask=z.get(p + "dmask"), gp=z[p + "gp"], grid=z[p + "grid"])


def _queries(z, sc, rule, key):
    """The recorded GetFeaturesInArea calls as product queries (x, y, r), (cam, lo, hi) and the
    query descriptors (+ masks) the caller read."""
    p = "w%d_r%d_%s_" % (sc, rule, key)
    calls = z[p + "calls"]
    src = z[p + "qsrc"]
    masked = bool(z["w%d_meta" % sc][1])
    nb = int(z["w%d_meta" % sc][2])
    nq = len(calls)
    xyr = np.ascontiguousarray(calls[:, 1:4])
    cl = np.ascontiguousarray(np.stack([calls[:, 0], calls[:, 4], calls[:, 5]], 1).astype(np.int32))
    qd = np.zeros((nq, nb), np.uint8)
    qm = np.zeros((nq, nb), np.uint8) if masked else None
    f1 = _frame(z, sc, "f1")
    glob = {(int(c), int(l)): i for i, (c, l) in enumerate(zip(f1["cam"], f1["loc"]))}
    qid = np.full(nq, -1, np.int64)
    for q in range(nq):
        kind, a, b = src[q]
        if kind == 0:            # a map point's descriptor (rule 0)
            qd[q] = z["w%d_mp_desc" % sc][a]
            if masked:
                qm[q] = z["w%d_mp_mask" % sc][a]
            qid[q] = a
        elif kind == 1:          # a row of the query frame (F1 / LastFrame): global keypoint index
            g = glob[(a, b)]
            qd[q] = f1["desc"][g]
            if masked:
                qm[q] = f1["dmask"][g]
            qid[q] = g
    lists = (z[p + "list_ptr"], z[p + "list_idx"])
    return xyr, cl, qd, qm, qid, lists


def _th(z, sc, rule):
    masked, nb = bool(z["w%d_meta" % sc][1]), int(z["w%d_meta" % sc][2])
    hi, lo = z["th_%d_%d" % (nb, int(masked))] if ("th_%d_%d" % (nb, int(masked))) in z else (None, None)
    if hi is None:
        from mcs_amd import window as mw
        hi, lo = mw.matcher_thresholds(nb, masked)
    return int(lo) if rule == 2 else int(hi)


def _initial_assigned(z, sc, rule):
    n2 = int(z["w%d_meta" % sc][4])
    a = np.zeros(n2, np.uint8)
    if rule == 0:
        a[z["w%d_r0_pre_assigned" % sc]] = 1
    elif rule == 1:
        a[z["w%d_r0_pre_assigned" % sc][:20]] = 1
    return a


def _expected(z, sc, rule, key):
    p = "w%d_r%d_%s_" % (sc, rule, key)
    return z[p + ("m12" if rule == 2 else "assign")]


def _assemble(z, sc, rule, m, qid):
    """The rule's final output from the product's per-query matches."""
    n1, n2 = int(z["w%d_meta" % sc][3]), int(z["w%d_meta" % sc][4])
    if rule == 2:
        return np.asarray(m, np.int32)      # vnMatches12: query q is F1 keypoint q
    a = np.full(n2, -1, np.int32)
    pre = _initial_assigned(z, sc, rule)
    a[pre.astype(bool)] = 10 ** 6 if rule == 0 else -2
    for q, k in enumerate(m):
        if k >= 0:
            a[k] = qid[q]
    return a


def _rename(z):
    """Rules 0 / 1 store the assignment as <key>_assign next to the call records."""
    for sc in range(3):
        for rule, key, _ in RULES:
            p = "w%d_r%d_%s_" % (sc, rule, key)
            if rule in (0, 1) and p + "assign" not in z:
                z[p + "assign"] = z["w%d_r%d_%s_assign" % (sc, rule, key)]
    return z


def test_distances_and_thresholds_match_reference_text():
    import mcs_amd
    z = _fix()
    for nb in (16, 32, 64):
        A, B, MA, MB = z["d%d_a" % nb], z["d%d_b" % nb], z["d%d_ma" % nb], z["d%d_mb" % nb]
        assert np.array_equal(_dist(A, B), z["d%d_dist" % nb])
        assert np.array_equal(_dist(A, B, MA, MB), z["d%d_dist_masked" % nb])
        got = np.array([mcs_amd.descriptor_distance64(A[i], B[i]) for i in range(len(A))])
        assert np.array_equal(got, z["d%d_dist" % nb])
        fn = ob.lib().oracle_descriptor_distance64_masked
        om = [fn(_p(A[i]), _p(B[i]), _p(MA[i]), _p(MB[i]), nb) for i in range(len(A))]
        assert np.array_equal(om, z["d%d_dist_masked" % nb])
    from mcs_amd import window as mw
    for nb, masks in ((32, False), (32, True), (16, False), (64, False)):
        assert tuple(z["th_%d_%d" % (nb, int(masks))]) == mw.matcher_thresholds(nb, masks)


@pytest.mark.parametrize("sc", [0, 1, 2])
def test_frame_grid_matches_reference_ctor(sc):
    """mcs_frame_grid_build (host) against the grid the reference ctor filled, cell by cell."""
    from mcs_amd import window as mw
    z = _fix()
    for tag in ("f1", "f2"):
        f = _frame(z, sc, tag)
        ptr, cells = mw.grid_build(f["xy"], f["cam"], f["gp"])
        want = [[] for _ in range(NC * 64 * 48)]
        for c, ix, iy, idx in f["grid"]:
            want[(c * 64 + ix) * 48 + iy].append(idx)
        wptr = np.cumsum([0] + [len(v) for v in want])
        assert np.array_equal(ptr, wptr), (sc, tag)
        assert np.array_equal(cells, np.array([i for v in want for i in v], np.int32)), (sc, tag)
        # the grid constants of the ctor (:154-157) are the product's grid_params
        assert np.array_equal(f["gp"], mw.grid_params([(0, 0)] * NC, [(754, 480)] * NC))


def _cands_numpy(z, sc, rule, key, qd, qm):
    """Distances of the recorded candidate lists (the reference's DescriptorDistance64[Masked])."""
    xyr, cl, _, _, _, (ptr, idx) = _queries(z, sc, rule, key)
    f2 = _frame(z, sc, "f2")
    dist = np.zeros(len(idx), np.int32)
    for q in range(len(ptr) - 1):
        ks = idx[ptr[q]:ptr[q + 1]]
        if len(ks):
            dist[ptr[q]:ptr[q + 1]] = _dist(qd[q][None], f2["desc"][ks],
                                            None if qm is None else qm[q][None],
                                            None if qm is None else f2["dmask"][ks])
    return ptr, idx, dist


@pytest.mark.parametrize("sc", [0, 1, 2])
@pytest.mark.parametrize("rule,key,ratio", RULES)
def test_window_select_matches_reference_text(sc, rule, key, ratio):
    """mcs_window_select (the product's host selection) over the reference's own candidate
    lists gives the reference text's final assignment, for every rule."""
    from mcs_amd import window as mw
    z = _rename(_fix())
    xyr, cl, qd, qm, qid, _ = _queries(z, sc, rule, key)
    ptr, idx, dist = _cands_numpy(z, sc, rule, key, qd, qm)
    f2 = _frame(z, sc, "f2")
    a0 = _initial_assigned(z, sc, rule)
    m, n, _ = mw.window_select(rule, ptr, idx, dist, f2["oct"], _th(z, sc, rule), ratio, a0)
    assert n == int(z["w%d_r%d_%s_nmatches" % (sc, rule, key)])
    assert np.array_equal(_assemble(z, sc, rule, m, qid), _expected(z, sc, rule, key))


@pytest.mark.parametrize("sc", [0, 1, 2])
def test_oracle_window_candidates_match_reference_text(sc):
    """The oracle's GetFeaturesInArea (oracle/matcher_oracle.cpp) returns the reference lists."""
    z = _rename(_fix())
    f2 = _frame(z, sc, "f2")
    nb = f2["desc"].shape[1]
    for rule, key, _ in RULES:
        xyr, cl, qd, qm, _, (ptr, idx) = _queries(z, sc, rule, key)
        nq = len(xyr)
        cap = len(idx) + 16
        optr = np.zeros(nq + 1, np.int32)
        okp = np.zeros(cap, np.int32)
        od = np.zeros(cap, np.int32)
        tot = ob.lib().oracle_window_candidates(NC, _p(f2["gp"]), _p(f2["xy"]), _p(f2["cam"]), _p(f2["oct"]),
                                                _p(f2["desc"]), _p(f2["dmask"]), len(f2["xy"]), nb, nq,
                                                _p(xyr), _p(cl), _p(qd), _p(qm), _p(optr), _p(okp), _p(od), cap)
        assert tot == len(idx)
        assert np.array_equal(optr, ptr) and np.array_equal(okp[:tot], idx), (rule, key)


def _tri(z, sc):
    p = "t%d_" % sc
    seed, masked, nb, th_low = [int(v) for v in z[p + "meta"]]
    k = [dict(rays=np.ascontiguousarray(z[p + "k%d_rays" % i]), cam=z[p + "k%d_cam" % i],
              desc=z[p + "k%d_desc" % i], has=z[p + "k%d_has" % i],
              dmask=z.get(p + "k%d_dmask" % i)) for i in (0, 1)]
    return k, np.ascontiguousarray(z[p + "E"]), masked, nb, th_low, z[p + "m12"], int(z[p + "nmatches"])


FIX_BIG = os.path.join(os.path.dirname(__file__), "golden", "matcher_ref_big.npz")


def _fix_tri(sc):
    """Scenarios 0-3 from matcher_ref.npz; 4 = config-B density (3 cameras x 2000 keypoints per
    keyframe, clutter groups that overflow the device kernel's candidate slots) from
    matcher_ref_big.npz (gen_matcher_ref.py --big)."""
    return np.load(FIX_BIG, allow_pickle=False) if sc >= 4 else _fix()


@pytest.mark.parametrize("sc", [0, 1, 2, 3, 4])
def test_oracle_triangulation_matches_reference_text(sc):
    z = _fix_tri(sc)
    k, E, masked, nb, th_low, m12, nm = _tri(z, sc)
    ref = np.zeros(len(k[0]["rays"]), np.int32)
    n = ob.lib().oracle_search_for_triangulation_raw_ex(
        _p(k[0]["desc"]), _p(k[0]["dmask"]) if masked else None, len(k[0]["rays"]), _p(k[1]["desc"]),
        _p(k[1]["dmask"]) if masked else None, len(k[1]["rays"]), nb, _p(k[0]["cam"]), _p(k[1]["cam"]),
        _p(k[0]["has"]), _p(k[1]["has"]), _p(k[0]["rays"]), _p(k[1]["rays"]), _p(E), 1e-2, NC, _p(ref))
    assert n == nm and np.array_equal(ref, m12)


@pytest.mark.gpu
@pytest.mark.parametrize("sc", [0, 1, 2, 3, 4])
def test_gpu_triangulation_matches_reference_text(gpu, sc):
    import mcs_amd
    z = _fix_tri(sc)
    k, E, masked, nb, th_low, m12, nm = _tri(z, sc)
    got = np.zeros(len(k[0]["rays"]), np.int32)
    n = ctypes.c_int32()
    L = mcs_amd.lib()
    if masked:
        rc = L.mcs_search_for_triangulation_raw_masked(
            _p(k[0]["desc"]), _p(k[0]["dmask"]), _p(k[0]["cam"]), _p(k[0]["has"]), _p(k[0]["rays"]),
            len(k[0]["rays"]), _p(k[1]["desc"]), _p(k[1]["dmask"]), _p(k[1]["cam"]), _p(k[1]["has"]),
            _p(k[1]["rays"]), len(k[1]["rays"]), NC, _p(E), nb, th_low, 1e-2, _p(got), ctypes.byref(n))
    else:
        rc = L.mcs_search_for_triangulation_raw(
            _p(k[0]["desc"]), _p(k[0]["cam"]), _p(k[0]["has"]), _p(k[0]["rays"]), len(k[0]["rays"]),
            _p(k[1]["desc"]), _p(k[1]["cam"]), _p(k[1]["has"]), _p(k[1]["rays"]), len(k[1]["rays"]), NC,
            _p(E), nb, th_low, 1e-2, _p(got), ctypes.byref(n))
    assert rc == 0
    assert n.value == nm and np.array_equal(got, m12)


@pytest.mark.gpu
@pytest.mark.parametrize("sc", [0, 1, 2])
def test_gpu_window_search_and_match_reference_text(gpu, sc):
    """Device GetFeaturesInArea lists (order included) and distances equal the reference's, and
    the device search + host selection (FrameGrid path and the one-call mcs_window_match) give
    the reference text's final assignment, for every rule."""
    from mcs_amd import window as mw
    z = _rename(_fix())
    f2 = _frame(z, sc, "f2")
    frame = mw.FrameGrid(f2["xy"], f2["cam"], f2["oct"], f2["desc"], f2["gp"], f2["dmask"])
    for rule, key, ratio in RULES:
        xyr, cl, qd, qm, qid, _ = _queries(z, sc, rule, key)
        ptr, idx, dist = _cands_numpy(z, sc, rule, key, qd, qm)
        gptr, gkp, gdist = mw.window_search(frame, xyr, cl, qd, qm)
        assert np.array_equal(gptr, ptr) and np.array_equal(gkp, idx), (rule, key)
        assert np.array_equal(gdist, dist), (rule, key)
        a0 = _initial_assigned(z, sc, rule)
        th = _th(z, sc, rule)
        m, n, _ = mw.window_match(rule, frame, xyr, cl, qd, th, ratio, q_mask=qm, kp_assigned=a0)
        assert n == int(z["w%d_r%d_%s_nmatches" % (sc, rule, key)]), (rule, key)
        assert np.array_equal(_assemble(z, sc, rule, m, qid), _expected(z, sc, rule, key)), (rule, key)
        m2, n2, _ = mw.window_match_host(rule, f2["gp"], f2["xy"], f2["cam"], f2["oct"], f2["desc"], xyr, cl,
                                         qd, th, ratio, desc_mask=f2["dmask"], q_mask=qm, kp_assigned=a0)
        assert n2 == n and np.array_equal(m2, m), (rule, key)


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs the reference checkout")
def test_fixture_regenerates_from_reference_text(tmp_path):
    """In the build container the generator re-derives the fixture from the reference text."""
    import subprocess
    import sys
    out = tmp_path / "m.npz"
    gen = os.path.join(os.path.dirname(__file__), "golden", "gen_matcher_ref.py")
    subprocess.check_call([sys.executable, gen, "--out", str(out)], timeout=900)
    q, z = np.load(out), _fix()
    assert sorted(q.files) == sorted(z.keys())
    for k in q.files:
        assert np.array_equal(q[k], z[k]), k


@pytest.mark.skipif(not (os.path.isdir("/root/reference") and os.environ.get("MCS_REGEN_BIG") == "1"),
                    reason="needs the reference checkout and MCS_REGEN_BIG=1 (several minutes)")
def test_big_fixture_regenerates_from_reference_text(tmp_path):
    import subprocess
    import sys
    out = tmp_path / "mb.npz"
    gen = os.path.join(os.path.dirname(__file__), "golden", "gen_matcher_ref.py")
    subprocess.check_call([sys.executable, gen, "--big", "--out", str(out)], timeout=3000)
    q, z = np.load(out), np.load(FIX_BIG, allow_pickle=False)
    assert sorted(q.files) == sorted(z.files)
    for k in q.files:
        assert np.array_equal(q[k], z[k]), k
