"""Generate tests/golden/globalba_ref.npz: cOptimizer::BundleAdjustment's and
cOptimizer::PoseOptimization's OWN graph assembly, optimisation calls and write-back, evaluated
from the reference TEXT (no reference source is stored: numbers only).

Translated from /root/reference by tests/golden/cxx_eval.py (safe_exec, no builtins):
  cOptimizer::BundleAdjustment      src/cOptimizer.cpp:73-261 (the whole body: keyframe vertices
      with the maxKF / maxKFid rule, Mc / IO vertices, point vertices and the mnId -> vertex map,
      one edge per observation from a good keyframe, optimize(15), the write-back loops)
  cOptimizer::PoseOptimization      src/cOptimizer.cpp:264-486 (the whole body: vertices, one
      edge per non-NULL map-point match with the first vertex of its mnId, both optimize(10)
      rounds, the outlier classification, the returned count and ratio)
  cMapPoint::isBad, GetObservations src/cMapPoint.cpp (via gen_localba_ref)
Stand-ins (as gen_localba_ref.py):
  * keyframes / map points / the frame are scripted objects;
  * g2o's SparseOptimizer records vertices and edges with g2o's addVertex rule (a second vertex
    with a registered id is refused and reported, optimizable_graph.cpp:243-262) and runs
    optimize(n) through this project's g2o restatement (oracle_ba_optimize_ex, pinned to the
    g2o text by g2o_solver.npz); a graph with a refused vertex is not optimised (its edges
    would bind vertices of the wrong type: undefined behaviour), the scenario records the
    collision instead;
  * hom2cayley(GetPose()) / cayley2hom(estimate) exchange the scripted Cayley vectors (the
    pose conversion itself is pinned in refmath.npz);
  * a write-back through a vertex that does not exist (a bad keyframe: vertex(mnId) == NULL;
    a bad point: mapPointId_to_cont_g2oId.find(mnId) == end()) is undefined in the reference;
    it is recorded as "no write" (the product's kf_slot / pt_slot = -1).

    python tests/golden/gen_globalba_ref.py [--ref /root/reference]
"""
import argparse
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multicol-slam-annotation_amd"))
import cxx_rt as rt  # noqa: E402
import gen_localba_ref as L  # noqa: E402
from cxx_eval import (BOOL, DOUBLE, INT, VOID, ClassSpec, Cls, Fn, PtrT, Unsupported,  # noqa: E402
                      build_env, translate_function)
from safe_exec import safe_exec  # noqa: E402

V = L.V
KP, MP, MKF = L.KP, L.MP, L.MKF
c_ref, m_ref, val = L.c_ref, L.m_ref, L.val
_sig = L._sig
UB = -(10 ** 12)          # the id a UB lookup yields (never a vertex)


def setup(ref):
    ctx, ocpp, mcpp, mp, opt, enum, std_recon = L.setup(ref)
    # keyframe / frame accessors BundleAdjustment and PoseOptimization read
    kf = ctx.classes["cMultiKeyFrame"]
    kf.methods["GetPose"] = _sig([], Cls("Matx44d"))
    kf.methods["SetPose"] = _sig([c_ref(Cls("Matx44d"))], VOID)
    ctx.add_class(ClassSpec("Matx44d"))
    ctx.add_class(ClassSpec("cMultiFrame", {
        "camSystem": Cls("cMultiCamSys_"), "mvpMapPoints": V(PtrT(MP)), "mvbOutlier": V(BOOL),
        "keypoint_to_cam": Cls("unordered_map", (INT, INT)), "mvKeys": V(KP),
        "mvInvLevelSigma2": V(DOUBLE)}, {"GetPoseMin": _sig([], Cls("Matx61d"))}))
    ctx.funcs["hom2cayley"] = Fn("s_hom2cayley", None, Cls("Matx61d"))
    ctx.funcs["cayley2hom"] = Fn("s_cayley2hom", None, Cls("Matx44d"))
    ctx.funcs["Vector2d"] = Fn("s_Vector2d", None, Cls("Vector2d"))
    ctx.funcs["chrono::steady_clock::now"] = Fn("s_now", None, Cls("chrono::steady_clock::time_point"))
    ctx.add_class(ClassSpec("Vector2d"))
    ctx.add_class(ClassSpec("chrono::steady_clock::time_point", ctor="s_timepoint"))
    for vc in ("Matx44d", "Vector2d", "chrono::steady_clock::time_point"):
        L.cxx_eval.VALUE_CLASSES.add(vc)
    for name in L.G2O_VERTEX:
        ctx.classes[name].methods["dimension"] = _sig([], INT)
    ctx.classes["EdgeProjectXYZ2MCS"].methods["computeError"] = _sig([], VOID)
    ctx.classes["SparseOptimizer"].methods["initializeOptimization"] = Fn(None, [val(INT)], BOOL, defaults=["0"])
    for name in ("LinearSolverDense", "BlockSolverX", "BlockSolverX::LinearSolverType"):
        ctx.add_class(ClassSpec(name, {}, {}, ctor="G2O_Solver"))
    return ctx, ocpp, mcpp, mp, opt, enum, std_recon


def translate_all(ref):
    ctx, ocpp, mcpp, mp, opt, enum, std_recon = setup(ref)
    srcs, n_stmt = [], [0]

    def fn(pyname, src, pattern, this=None, ret=VOID):
        params, init, body = L.find_fn(src, pattern)
        n_stmt[0] += body.count(";")
        srcs.append(translate_function(ctx, pyname, params, body, this_cls=this, ret=ret))
    fn("f_mp_isBad", mcpp, r"bool cMapPoint::isBad\(\)", this=mp, ret=BOOL)
    fn("f_mp_GetObservations", mcpp, r"std::map<cMultiKeyFrame\*, std::vector<size_t>> cMapPoint::GetObservations\(\)",
       this=mp, ret=Cls("map", (PtrT(MKF), V(INT))))
    fn("f_ba", ocpp, r"void cOptimizer::BundleAdjustment\(const std::vector<cMultiKeyFrame\*> &vpKFs", this=opt)
    fn("f_po", ocpp, r"int cOptimizer::PoseOptimization\(", this=opt, ret=INT)
    return ctx, srcs, n_stmt[0], enum


# ------------------------------------------------------------------------------ g2o stand-ins
class Collision(Exception):
    pass


class GOptimizerG(L.GOptimizer):
    """SparseOptimizer with g2o's duplicate-id rule and point-fixed rounds."""

    def __init__(self, ob, log):
        L.GOptimizer.__init__(self, ob, log)
        self.collisions = []

    def m_addVertex(self, vp):
        v = L.rt.deref(vp)
        self.order.append(v)
        if v.id in self.vertices:                 # addVertex FATAL: the first vertex stays
            self.collisions.append(v.id)
            v.refused = True
            return False
        self.vertices[v.id] = v
        return True

    def m_vertex(self, i):
        v = self.vertices.get(int(i))
        return rt.Ptr(obj=NULL_VERTEX) if v is None else rt.Ptr(obj=v)

    def m_initializeOptimization(self, level=0):
        self.level = int(level)
        return True

    def m_optimize(self, n):
        if self.collisions:
            raise Collision(self.collisions[0])
        from mcs_amd import ba
        ta = self.actions[0]
        order = [v for v in self.order if not getattr(v, "refused", False)]
        mt = [v for v in order if v.kind == "Mt"]
        mcs = [v for v in order if v.kind == "Mc"]
        ios = [v for v in order if v.kind == "IO"]
        pts = [v for v in order if v.kind == "P"]
        pidx = {id(v): i for i, v in enumerate(mt)}
        lidx = {id(v): i for i, v in enumerate(pts)}
        cidx = {id(v): i for i, v in enumerate(mcs)}
        E = self.edges
        for e in E:
            assert e.v[0].kind == "Mt" and e.v[1].kind == "P" and e.v[2].kind == "Mc" and e.v[3].kind == "IO"
            assert ios.index(e.v[3]) == cidx[id(e.v[2])]
        deltas = {e.kernel.delta for e in E}
        assert len(deltas) <= 1
        pfix = {v.fix for v in pts}
        assert len(pfix) <= 1
        info = [e.info for e in E]
        assert all(i[0] == "I" for i in info)
        pr = dict(poses=np.array([v.est for v in mt]).reshape(-1, 6),
                  pose_fixed=np.array([v.fix for v in mt], np.uint8),
                  points=np.array([v.est for v in pts]).reshape(-1, 3), mc=np.array([v.est for v in mcs]),
                  cam=np.array([v.est for v in ios]),
                  edge_pose=np.array([pidx[id(e.v[0])] for e in E], np.int32),
                  edge_point=np.array([lidx[id(e.v[1])] for e in E], np.int32),
                  edge_cam=np.array([cidx[id(e.v[2])] for e in E], np.int32),
                  edge_meas=np.array([e.meas for e in E]).reshape(-1, 2),
                  edge_info=np.array([i[1] for i in info], np.float64),
                  huber_delta=deltas.pop() if deltas else 1.0)
        lvl = np.array([0 if e.level == self.level else 1 for e in E], np.uint8)
        before = self._flag()
        opts = ba.BAOptions(max_iterations=int(n), gain_threshold=ta.gain, terminate_max_iter=ta.maxit)
        r = self.ob.ba_optimize(pr, opts, edge_level=lvl, stop_flag=int(before),
                                points_fixed=bool(pfix and pfix.pop()))
        after = bool(r["stop_flag"])
        if self.force is not None:
            self.force[0] = after
        elif after or self.aux is not None:
            self.aux = after
        rep = r["report"]
        for i, v in enumerate(mt):
            v.est = [float(x) for x in r["poses"][i]]
        for i, v in enumerate(pts):
            v.est = [float(x) for x in r["points"][i]]
        for e, c in zip(E, r["edge_chi2"]):
            e.chi = float(c)
        empty = rep.n_active_poses + rep.n_active_points == 0
        self.log.append((int(n), int(rep.iterations), int(before), int(self._flag()), int(empty)))
        return -1 if empty else int(rep.iterations)


class _NullVertex(L.GVertex):
    """vertex(id) of an id without a vertex: g2o returns NULL; reading its estimate is UB."""

    def __init__(self):
        L.GVertex.__init__(self, "NULL")

    def m_estimate(self):
        return None


NULL_VERTEX = _NullVertex()


class UBMap(rt.Map):
    """unordered_map whose find() of a missing key (then ->second) yields UB (a recorded
    undefined lookup, never a vertex id) instead of raising."""
    __slots__ = ()

    def m_find(self, k):
        return rt.MapIt(self, k if k in self.d else _UB_KEY)

    def pair(self, k):
        if k is _UB_KEY:
            return rt.Pair(k, UB)
        return rt.Map.pair(self, k)


_UB_KEY = ("undefined",)


# ------------------------------------------------------------------------------ scenarios
def gba_world(m, rec, order=None):
    """vpKFs / vpMP over a map dict: keyframe objects in creation order (pointer order) with
    mnId, isBad, GetPose/SetPose, camSystem; map points with mnId, isBad, GetWorldPos /
    SetWorldPos and observations in keyframe order."""
    nk, npt = len(m["kf_id"]), len(m["pt_bad"])
    kfs = [rt.Struct("cMultiKeyFrame", {}) for _ in range(nk)]
    mps = [rt.Struct("cMapPoint", {}) for _ in range(npt)]
    obs_of_kf = [[] for _ in range(nk)]
    for p in range(npt):
        for o in range(m["pt_obs_off"][p], m["pt_obs_off"][p + 1]):
            obs_of_kf[m["obs_kf"][o]].append(o)
    for k, kf in enumerate(kfs):
        kf.f["_idx"] = k
        k2c = rt.Map(lambda: 0)
        for o in obs_of_kf[k]:
            k2c.d[o] = int(m["obs_cam"][o])

        def gkp(idx):
            kp = rt.KeyPoint()
            kp["pt"] = rt.Point2f(m["obs_meas"][idx, 0], m["obs_meas"][idx, 1])
            return kp
        cams = L.Standin()
        cams.m_GetNrCams = lambda: len(m["mc"])
        cams.m_Get_M_c_min = lambda c: [float(x) for x in m["mc"][c]]
        cams.m_GetCamModelObj = lambda c: L._CamObj(m["cam"][c])
        kf.f.update(mnId=int(m["kf_id"][k]), camSystem=cams, keypoint_to_cam=k2c,
                    isBad=(lambda k=k: bool(m["kf_bad"][k])), GetKeyPoint=gkp,
                    GetPose=(lambda k=k: ("pose", k)),
                    SetPose=(lambda T, k=k: rec["pose_write"].append((k, list(T[1]))) if T is not None else
                             rec["pose_ub"].append(k)))
    for p, mpt in enumerate(mps):
        obs = rt.Map(lambda: rt.Vector(lambda: 0), ordered=True)
        for o in range(m["pt_obs_off"][p], m["pt_obs_off"][p + 1]):
            key = rt.Ptr(obj=kfs[m["obs_kf"][o]])
            if key not in obs.d:
                obs.d[key] = rt.Vector(lambda: 0)
            obs.d[key].v.append(int(o))
        mpt.f.update(_idx=p, mnId=int(m["pt_id"][p]), mObservations=obs, mbBad=bool(m["pt_bad"][p]),
                     mMutexFeatures=None, mMutexPos=None,
                     GetWorldPos=(lambda p=p: L._world_pos(p, m)),
                     SetWorldPos=(lambda x, p=p: rec["point_write"].append((p, [float(v) for v in x]))
                                  if x is not None and getattr(x, "kind", "P") == "P" else
                                  rec["point_ub"].append(p)),
                     UpdateNormalAndDepth=lambda: None)
    return kfs, mps


def gba_map(n_kf, n_points, target_edges, seed, bad_kf=(), bad_points=0.0, kf_order=None, ids=None,
            dup_pt_ids=()):
    """A BundleAdjustment map: make_map geometry, keyframe ids (default 0..n-1 in list order,
    so keyframe 0 is fixed), point ids 1000 + index (optionally duplicated), list order of vpKFs
    optionally permuted (pointer order != id order)."""
    from mcs_amd import ba
    m = ba.make_map(n_kf=n_kf, n_points=n_points, target_edges=target_edges, seed=seed, bad_kf=bad_kf,
                    bad_points=bad_points)
    nk = n_kf
    m["kf_id"] = np.arange(nk, dtype=np.int64) if ids is None else np.asarray(ids, np.int64)
    m["pt_id"] = 1000 + np.arange(len(m["pt_bad"]), dtype=np.int64)
    for a, b in dup_pt_ids:
        m["pt_id"][b] = m["pt_id"][a]
    m["obs_meas"] = m["obs_meas"].astype(np.float32).astype(np.float64)   # kp.pt is float
    if kf_order is not None:
        perm = np.asarray(kf_order)
        inv = np.argsort(perm)
        for k in ("kf_id", "kf_bad", "kf_pose"):
            m[k] = np.asarray(m[k])[perm]
        m["obs_kf"] = inv[m["obs_kf"]].astype(np.int32)
        # observations per point stay in std::map order = keyframe (list/pointer) order
        for p in range(len(m["pt_bad"])):
            lo, hi = m["pt_obs_off"][p], m["pt_obs_off"][p + 1]
            o = np.argsort(m["obs_kf"][lo:hi], kind="stable") + lo
            for k in ("obs_kf", "obs_cam", "obs_meas", "obs_info"):
                m[k][lo:hi] = np.asarray(m[k])[o]
    return m


GBA_SCENARIOS = [
    # name, gba_map kwargs, poseOnly, stop flag (None = no pbStopFlag)
    ("g0", dict(n_kf=8, n_points=300, target_edges=1800, seed=21), 0, None),
    ("g1", dict(n_kf=10, n_points=400, target_edges=2600, seed=22, bad_kf=(3,), bad_points=0.04), 0, None),
    # vpKFs not in id order, last keyframe with the largest id: no collision
    ("g2", dict(n_kf=9, n_points=350, target_edges=2200, seed=23, kf_order=[0, 2, 1, 4, 3, 6, 5, 7, 8]), 0, 0),
    ("g3", dict(n_kf=8, n_points=300, target_edges=1800, seed=24, dup_pt_ids=((5, 9), (20, 21))), 1, None),
    # sparse ids; the last keyframe in the list is bad: maxKF = the last GOOD keyframe's id
    ("g4", dict(n_kf=8, n_points=300, target_edges=1800, seed=25, ids=[0, 3, 7, 12, 13, 20, 26, 31],
                bad_kf=(7,)), 0, None),
    ("g5", dict(n_kf=6, n_points=120, target_edges=700, seed=26), 0, 1),
    # collisions: the list's last good keyframe is not the largest id -> Mc / point ids hit keyframes
    ("c0", dict(n_kf=8, n_points=200, target_edges=1200, seed=27, kf_order=[0, 1, 2, 3, 4, 7, 6, 5]), 0, None),
    ("c1", dict(n_kf=8, n_points=200, target_edges=1200, seed=28, ids=[0, 1, 2, 40, 4, 5, 6, 7]), 0, None),
]


def run_gba(G, ob, name, kw, pose_only, stop, out):
    log, rec = [], dict(pose_write=[], point_write=[], pose_ub=[], point_ub=[])
    m = gba_map(**kw)
    _POSES[0] = m["kf_pose"]
    kfs, mps = gba_world(m, rec)
    opt_obj = G["Optimizer_"]()
    captured = {}
    orig = GOptimizerG.m_addVertex

    def add_vertex(self, vp, _orig=orig):
        captured.setdefault("opt", self)
        return _orig(self, vp)
    GOptimizerG.m_addVertex = add_vertex
    G["_gba_log"][0] = log
    cell = None if stop is None else [bool(stop)]
    collision = -1
    try:
        G["f_ba"](opt_obj, rt.Vector(lambda: None, [rt.Ptr(obj=k) for k in kfs]),
                  rt.Vector(lambda: None, [rt.Ptr(obj=q) for q in mps]), bool(pose_only), 10, cell)
    except Collision as c:
        collision = int(c.args[0])
    finally:
        GOptimizerG.m_addVertex = orig
    p = name + "_"
    opt = captured["opt"]
    out[p + "meta"] = np.array([int(pose_only), -1 if stop is None else int(stop), collision], np.int64)
    for k in ("kf_id", "kf_bad", "pt_id", "pt_bad", "pt_obs_off", "obs_kf", "obs_cam", "obs_meas",
              "kf_pose", "pt_pos", "mc", "cam"):
        out[p + "map_" + k] = np.asarray(m[k])
    kinds = {"Mt": 0, "Mc": 1, "IO": 2, "P": 3}
    out[p + "vertices"] = np.array([(v.id, kinds[v.kind], int(v.fix), int(getattr(v, "refused", False)))
                                    for v in opt.order], np.int64).reshape(-1, 4)
    out[p + "point_vertices"] = np.array([(v.id, v.point) for v in opt.order if v.kind == "P"],
                                         np.int64).reshape(-1, 2)
    if collision >= 0:
        print("%s: collision at vertex id %d (%d vertices added)" % (name, collision, len(opt.order)), flush=True)
        return
    kf_of = {k.f["mnId"]: k.f["_idx"] for k in kfs if not m["kf_bad"][k.f["_idx"]]}
    mc_ids = [v.id for v in opt.order if v.kind == "Mc"]
    pt_vid = {v.id: v.point for v in opt.order if v.kind == "P"}
    ev = [(kf_of[e.v[0].id], e.v[1].id, mc_ids.index(e.v[2].id)) for e in opt.edges]
    out[p + "edges"] = np.array(ev, np.int64).reshape(-1, 3)
    out[p + "edge_meas"] = np.array([e.meas for e in opt.edges]).reshape(-1, 2)
    out[p + "edge_info"] = np.array([e.info[1] for e in opt.edges])
    out[p + "edge_delta"] = np.array([e.kernel.delta for e in opt.edges])
    out[p + "optimize_log"] = np.array(log, np.int64).reshape(-1, 5)
    out[p + "pose_write"] = np.array([[k] + x for k, x in rec["pose_write"]]).reshape(-1, 7)
    out[p + "point_write"] = np.array([[q] + x for q, x in rec["point_write"]]).reshape(-1, 4)
    out[p + "pose_ub"] = np.array(rec["pose_ub"], np.int64)
    out[p + "point_ub"] = np.array(rec["point_ub"], np.int64)
    out[p + "stop_after"] = -1 if cell is None else int(cell[0])
    assert all(pt_vid[e.v[1].id] == e.v[1].point for e in opt.edges)
    print("%s: %d poses, %d points, %d edges, optimize %s, %d / %d written (%d / %d undefined)" % (
        name, sum(v.kind == "Mt" for v in opt.order), len(pt_vid), len(ev), log, len(rec["pose_write"]),
        len(rec["point_write"]), len(rec["pose_ub"]), len(rec["point_ub"])), flush=True)


# ---- PoseOptimization
def po_frame(seed, n_points, n_keys, null_frac, dup_frac, outlier_frac, huber_mult):
    """A cMultiFrame for PoseOptimization: make_pose_problem geometry; mvpMapPoints with NULLs and
    repeated map points (one point matched by two keypoints), keypoint_to_cam, mvKeys (pt as
    float, octave), mvInvLevelSigma2."""
    from mcs_amd import ba
    pr = ba.make_pose_problem(seed=seed, n_points=n_points, target_edges=n_keys, outlier_frac=outlier_frac)
    rng = np.random.default_rng(seed + 5)
    ne = len(pr["edge_pose"])
    inv = L.inv_sigma2_table()
    octv = rng.integers(0, 8, ne)
    keys = []
    for e in range(ne):
        keys.append((int(pr["edge_point"][e]), int(pr["edge_cam"][e]), pr["edge_meas"][e], int(octv[e])))
    # NULL matches (keypoints without a map point) and duplicates (a map point seen twice)
    out = []
    for k in keys:
        r = rng.random()
        if r < null_frac:
            out.append((-1, k[1], k[2], k[3]))
        out.append(k)
        if rng.random() < dup_frac:
            out.append((k[0], k[1], k[2] + rng.normal(0, 0.5, 2), k[3]))
    n = len(out)
    key_mp = np.array([k[0] for k in out], np.int32)
    key_cam = np.array([k[1] for k in out], np.int32)
    key_pt = np.array([k[2] for k in out]).astype(np.float32).astype(np.float64)
    key_oct = np.array([k[3] for k in out], np.int32)
    pt_id = 5000 + np.arange(len(pr["points"]), dtype=np.int64)
    return dict(key_mp=key_mp, key_cam=key_cam, key_pt=key_pt, key_oct=key_oct, pt_id=pt_id,
                pt_pos=pr["points"], pose=pr["poses"][0], mc=pr["mc"], cam=pr["cam"],
                inv_sigma2=np.array(inv), huber_mult=float(huber_mult), n=n)


def _po_world_pos(p, f):
    L.GVertex.last_point[0] = p
    return rt.Vector(lambda: 0.0, [float(x) for x in f["pt_pos"][p]])


def po_world(f, rec):
    mps = []
    for p in range(len(f["pt_id"])):
        q = rt.Struct("cMapPoint", {})
        q.f.update(_idx=p, mnId=int(f["pt_id"][p]), mbBad=False, mMutexPos=None,
                   GetWorldPos=(lambda p=p: _po_world_pos(p, f)))
        mps.append(q)
    cams = L.Standin()
    cams.m_GetNrCams = lambda: len(f["mc"])
    cams.m_Get_M_c_min = lambda c: [float(x) for x in f["mc"][c]]
    cams.m_GetCamModelObj = lambda c: L._CamObj(f["cam"][c])
    cams.m_Set_M_t_from_min = lambda x: rec["pose"].append([float(v) for v in x])
    k2c = rt.Map(lambda: 0)
    keys = []
    for i in range(f["n"]):
        k2c.d[i] = int(f["key_cam"][i])
        kp = rt.KeyPoint()
        kp["pt"] = rt.Point2f(f["key_pt"][i, 0], f["key_pt"][i, 1])
        kp["octave"] = int(f["key_oct"][i])
        keys.append(kp)
    frame = rt.Struct("cMultiFrame", {})
    frame.f.update(camSystem=cams, keypoint_to_cam=k2c,
                   mvpMapPoints=rt.Vector(lambda: None, [rt.Ptr(obj=mps[j]) if j >= 0 else None for j in f["key_mp"]]),
                   mvbOutlier=rt.Vector(lambda: False, [True] * f["n"]),     # the text resets every entry
                   mvKeys=rt.Vector(rt.KeyPoint, keys),
                   mvInvLevelSigma2=rt.Vector(lambda: 0.0, [float(x) for x in f["inv_sigma2"]]),
                   GetPoseMin=lambda: [float(x) for x in f["pose"]])
    return frame


PO_SCENARIOS = [
    # name, seed, map points, keypoints with a map point, NULL fraction, duplicate fraction, outliers, huberMultiplier
    ("p0", 31, 900, 1200, 0.1, 0.03, 0.05, 1.0),
    ("p1", 32, 600, 800, 0.2, 0.05, 0.15, 2.0),
    ("p2", 33, 300, 400, 0.0, 0.0, 0.0, 1.0),
    ("p3", 34, 1500, 2500, 0.05, 0.02, 0.08, 1.5),
]


def run_po(G, name, args, out):
    seed, npt, nk, nullf, dupf, outf, hm = args
    f = po_frame(seed, npt, nk, nullf, dupf, outf, hm)
    log, rec = [], dict(pose=[])
    G["_gba_log"][0] = log
    frame = po_world(f, rec)
    opt_obj = G["Optimizer_"]()
    captured = {}
    orig = GOptimizerG.m_addVertex

    def add_vertex(self, vp, _orig=orig):
        captured.setdefault("opt", self)
        return _orig(self, vp)
    GOptimizerG.m_addVertex = add_vertex
    inl = [0.0]
    try:
        ret = G["f_po"](opt_obj, rt.Ptr(obj=frame), inl, hm)
    finally:
        GOptimizerG.m_addVertex = orig
    opt = captured["opt"]
    p = name + "_"
    for k in ("key_mp", "key_cam", "key_pt", "key_oct", "pt_id", "pt_pos", "pose", "mc", "cam", "inv_sigma2"):
        out[p + k] = np.asarray(f[k])
    out[p + "huber_mult"] = hm
    kinds = {"Mt": 0, "Mc": 1, "IO": 2, "P": 3}
    out[p + "vertices"] = np.array([(v.id, kinds[v.kind], int(v.fix)) for v in opt.order], np.int64)
    out[p + "point_vertices"] = np.array([(v.id, v.point) for v in opt.order if v.kind == "P"],
                                         np.int64).reshape(-1, 2)
    vid_pt = {v.id: v.point for v in opt.order if v.kind == "P"}
    mc_ids = [v.id for v in opt.order if v.kind == "Mc"]
    out[p + "edges"] = np.array([(vid_pt[e.v[1].id], mc_ids.index(e.v[2].id)) for e in opt.edges], np.int64).reshape(-1, 2)
    out[p + "edge_meas"] = np.array([e.meas for e in opt.edges]).reshape(-1, 2)
    out[p + "edge_info"] = np.array([e.info[1] for e in opt.edges])
    out[p + "edge_delta"] = np.array([e.kernel.delta for e in opt.edges])
    out[p + "outlier"] = np.array([bool(x) for x in frame.f["mvbOutlier"].v], np.uint8)
    out[p + "ret"] = int(ret)
    out[p + "inliers"] = float(inl[0])
    out[p + "pose_out"] = np.array(rec["pose"][-1])
    out[p + "optimize_log"] = np.array(log, np.int64).reshape(-1, 5)
    print("%s: %d keypoints, %d point vertices, %d edges, optimize %s, return %d, ratio %.4f" % (
        name, f["n"], len(vid_pt), len(opt.edges), log, ret, inl[0]), flush=True)


def load(ref):
    from tests import oracle_bind as ob
    ctx, srcs, n_stmt, enum = translate_all(ref)
    log_box = [[]]

    extra = {"s_Identity2": lambda: ("I", 1.0), "s_mscale": lambda I, s: (I[0], I[1] * s),
             "Lock_": lambda *x: None,
             "G2O_VertexMt_cayley": lambda: L.GVertex("Mt"), "G2O_VertexMc_cayley": lambda: L.GVertex("Mc"),
             "G2O_VertexOmniCameraParameters": lambda cam: L.GVertex("IO"),
             "G2O_VertexPointXYZ": lambda: L.GVertex("P"), "G2O_Edge": L.GEdge, "G2O_Huber": L.GHuber,
             "G2O_Terminate": L.GTerminate, "G2O_Solver": lambda *x: L.Standin(),
             "G2O_Optimizer": lambda: GOptimizerG(ob, log_box[0]),
             "s_hom2cayley": lambda T: None if T is None else list(_POSES[0][T[1]]),
             "s_cayley2hom": _cayley2hom,
             "s_Vector2d": lambda x, y: rt.Vector(lambda: 0.0, [float(x), float(y)]),
             "s_now": lambda: 0.0, "s_timepoint": lambda: 0.0, "_gba_log": log_box,
             "_Map": lambda fac, ordered: rt.Map(fac, ordered) if ordered else UBMap(fac, ordered)}
    for k, v in enum.items():
        extra["c_SR_" + k] = v
    env = build_env(ctx, rt, extra)
    G = safe_exec("\n".join(srcs), env, "<ref:cOptimizer.cpp / cMapPoint.cpp>")
    G["_gba_log"] = log_box
    return G, ob, n_stmt


_POSES = [None]


class _Est(list):
    """A vertex estimate that remembers the vertex kind it was read from: the write-back's
    static_cast<VertexMt_cayley*>(optimizer.vertex(mnId)) of a bad keyframe whose mnId is held by
    a Mc / IO / point vertex reads a vertex of another type (undefined)."""
    __slots__ = ("kind",)


def _estimate(self):
    e = _Est(self.est)
    e.kind = self.kind
    return e


def _cayley2hom(x):
    if x is None or getattr(x, "kind", "Mt") != "Mt":
        return None
    return ("hom", list(x))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "globalba_ref.npz"))
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    G, ob, n_stmt = load(a.ref)
    out = {"n_statements": n_stmt}

    # vertex dimension() (g2o BaseVertex<D, T>): 6 for the Cayley poses, 3 for points
    def dim(self):
        return {"Mt": 6, "Mc": 6, "IO": 17, "P": 3}[self.kind]
    L.GVertex.m_dimension = dim
    # every edge's computeError() at construction is a no-op here (its value is not read before
    # the optimisation recomputes it)
    L.GEdge.m_computeError = lambda self: None
    L.GVertex.m_estimate = _estimate
    for name, kw, pose_only, stop in GBA_SCENARIOS:
        if a.only and not re.fullmatch(a.only, name):
            continue
        run_gba(G, ob, name, kw, pose_only, stop, out)
    for name, *args in PO_SCENARIOS:
        if a.only and not re.fullmatch(a.only, name):
            continue
        run_po(G, name, args, out)
    out["gba_names"] = np.array([s[0] for s in GBA_SCENARIOS if not a.only or re.fullmatch(a.only, s[0])])
    out["po_names"] = np.array([s[0] for s in PO_SCENARIOS if not a.only or re.fullmatch(a.only, s[0])])
    np.savez_compressed(a.out, **out)
    print("wrote %s (%d statements translated)" % (a.out, n_stmt))


if __name__ == "__main__":
    main()
