"""Bundle adjustment binding (include/mcs_ba.h) + synthetic MultiCol BA problems.

Host mirror of cOptimizer::LocalBundleAdjustment (reference src/cOptimizer.cpp:489-908):
`local_ba(problem)` runs the GPU solver through mcs_local_ba; `optimize(problem, ...)` is one
initializeOptimization(0) + optimize(n) (the g2o call pair).

Synthetic problems follow SURVEY.md §8(d): Lafida 3-camera rig (M_c from
MultiCamSys_Calibration.yaml), MultiKeyFrames along a smooth trajectory, points sampled on
camera rays, observations = WorldToImg of visible points, octave ~ per-level budget,
pixel noise sigma = 0.5*1.2^octave, a few outliers, perturbed initial poses / points.
"""
import ctypes
import os
import threading
import weakref

import numpy as np

from . import synth

_D = ctypes.POINTER(ctypes.c_double)


class BAProblem(ctypes.Structure):
    _fields_ = [("n_poses", ctypes.c_int32), ("n_points", ctypes.c_int32),
                ("n_edges", ctypes.c_int32), ("n_cams", ctypes.c_int32),
                ("poses", ctypes.c_void_p), ("pose_fixed", ctypes.c_void_p),
                ("points", ctypes.c_void_p), ("mc", ctypes.c_void_p), ("cam", ctypes.c_void_p),
                ("edge_pose", ctypes.c_void_p), ("edge_point", ctypes.c_void_p),
                ("edge_cam", ctypes.c_void_p), ("edge_meas", ctypes.c_void_p),
                ("edge_info", ctypes.c_void_p), ("huber_delta", ctypes.c_double)]


class BAOptions(ctypes.Structure):
    _fields_ = [("max_iterations", ctypes.c_int32), ("gain_threshold", ctypes.c_double),
                ("terminate_max_iter", ctypes.c_int32), ("max_trials", ctypes.c_int32),
                ("tau", ctypes.c_double)]

    def __init__(self, max_iterations=10, gain_threshold=1e-6, terminate_max_iter=15,
                 max_trials=10, tau=1e-5):
        super().__init__(max_iterations, gain_threshold, terminate_max_iter, max_trials, tau)


class BAReport(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int32), ("stop_flag", ctypes.c_int32),
                ("chi2_initial", ctypes.c_double), ("chi2_final", ctypes.c_double),
                ("lambda_final", ctypes.c_double), ("n_active_edges", ctypes.c_int32),
                ("n_active_poses", ctypes.c_int32), ("n_active_points", ctypes.c_int32),
                ("trace_chi2", ctypes.c_void_p), ("trace_cap", ctypes.c_int32)]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


_PROBLEM_FIELDS = (("poses", np.float64), ("pose_fixed", np.uint8), ("points", np.float64),
                   ("mc", np.float64), ("cam", np.float64), ("edge_pose", np.int32),
                   ("edge_point", np.int32), ("edge_cam", np.int32), ("edge_meas", np.float64),
                   ("edge_info", np.float64))


_STRUCT_CACHE = []   # (weakrefs to the arrays, huber_delta, BAProblem), most recent last
_STRUCT_CACHE_LOCK = threading.Lock()
_STRUCT_CACHE_SIZE = 2


def as_struct(pr):
    """numpy problem dict -> BAProblem (keeps references alive in the dict).  A dict whose
    arrays are the same objects as at an earlier call (values may have changed in place) gets
    that call's struct back: the addresses are the same, and reading ten array addresses cost
    ~30 us of a ~2.3 ms LocalBA call.  The cache holds weak references only, so a problem the
    caller drops is freed (a dead reference never matches: a new array at a reused address is
    a cache miss), and at most two entries."""
    arrs = tuple(pr[k] for k, _ in _PROBLEM_FIELDS)
    hd = float(pr["huber_delta"])
    with _STRUCT_CACHE_LOCK:
        for ent in _STRUCT_CACHE:
            if ent[1] == hd and all(r() is y for r, y in zip(ent[0], arrs)):
                return ent[2]
    addr = []
    for k, dt in _PROBLEM_FIELDS:
        a = pr[k]
        if not (isinstance(a, np.ndarray) and a.dtype == dt and a.flags.c_contiguous):
            a = pr[k] = np.ascontiguousarray(a, dtype=dt)
        addr.append(a.__array_interface__["data"][0])
    s = BAProblem(len(pr["poses"]), len(pr["points"]), len(pr["edge_pose"]), len(pr["mc"]),
                  *addr, hd)
    refs = tuple(weakref.ref(pr[k]) for k, _ in _PROBLEM_FIELDS)
    with _STRUCT_CACHE_LOCK:
        _STRUCT_CACHE[:] = [e for e in _STRUCT_CACHE if all(r() is not None for r in e[0])]
        _STRUCT_CACHE.append((refs, hd, s))
        del _STRUCT_CACHE[:-_STRUCT_CACHE_SIZE]
    return s


# ---------------------------------------------------------------------------
# numpy restatement of the projection (generator only)
# ---------------------------------------------------------------------------
def cay2rot(c):
    c = np.asarray(c, np.float64)
    c1, c2, c3 = c[..., 0], c[..., 1], c[..., 2]
    s = 1 + c1 * c1 + c2 * c2 + c3 * c3
    R = np.stack([1 + c1 * c1 - c2 * c2 - c3 * c3, 2 * (c1 * c2 - c3), 2 * (c1 * c3 + c2),
                  2 * (c1 * c2 + c3), 1 - c1 * c1 + c2 * c2 - c3 * c3, 2 * (c2 * c3 - c1),
                  2 * (c1 * c3 - c2), 2 * (c2 * c3 + c1), 1 - c1 * c1 - c2 * c2 + c3 * c3], -1)
    return (R / s[..., None]).reshape(c.shape[:-1] + (3, 3))


def rot2cay(R):
    C = (R - np.eye(3)) @ np.linalg.inv(R + np.eye(3))
    return np.array([-C[1, 2], C[0, 2], -C[0, 1]])


def cam_vec(cam):
    return np.array([cam["c"], cam["d"], cam["e"], cam["u0"], cam["v0"]] + list(cam["pol"]))


def project(pose, mc, camv, X):
    """X_c = (M_t M_c)^-1 X, then WorldToImg; vectorised over X [...,3]."""
    Rt, Rc = cay2rot(pose[:3]), cay2rot(mc[:3])
    R = Rt @ Rc
    t = Rt @ mc[3:] + pose[3:]
    Xc = (X - t) @ R
    x, y, z = Xc[..., 0], Xc[..., 1], Xc[..., 2]
    rho = np.sqrt(x * x + y * y)
    rho = np.where(rho == 0, 1e-14, rho)
    th = np.arctan(-z / rho)
    r = np.zeros_like(th)
    for a in camv[5:][::-1]:
        r = r * th + a
    uu, vv = x / rho * r, y / rho * r
    return np.stack([uu * camv[0] + vv * camv[1] + camv[3], uu * camv[2] + vv + camv[4]], -1), Xc


def make_problem(n_local=10, n_fixed=3, n_points=3000, target_edges=20000, seed=0,
                 outlier_frac=0.02, noise_scale=0.5, pose_noise=(0.005, 0.02),
                 point_noise=0.05, cams=None, mcs=None, nfeatures=2000, huber_delta=1.345 * 2):
    """Config C-style LocalBA problem (10 local MKF + fixed observers, ~3k points, ~20k edges)."""
    rng = np.random.default_rng(seed)
    cams = cams or synth.LAFIDA_CAMS
    mcs = np.array(mcs or synth.LAFIDA_MC, np.float64)
    ncam = len(cams)
    camv = np.stack([cam_vec(c) for c in cams])
    masks = [synth.mirror_mask(c) for c in cams]
    nk = n_fixed + n_local
    # smooth trajectory: yaw sweep + forward motion
    gt_poses = np.zeros((nk, 6))
    for k in range(nk):
        yaw = 0.02 * k
        R = np.array([[np.cos(yaw), -np.sin(yaw), 0], [np.sin(yaw), np.cos(yaw), 0], [0, 0, 1]])
        gt_poses[k, :3] = rot2cay(R)
        gt_poses[k, 3:] = [0.12 * k, 0.02 * np.sin(k), 0.01 * k]
    # points on rays of random (kf, cam, pixel)
    pts = np.zeros((n_points, 3))
    i = 0
    while i < n_points:
        k = rng.integers(nk)
        c = rng.integers(ncam)
        u = rng.uniform(40, cams[c]["Iw"] - 40)
        v = rng.uniform(40, cams[c]["Ih"] - 40)
        if masks[c][int(v), int(u)] == 0:
            continue
        x, y, z = synth.img_to_world(cams[c], np.array(u), np.array(v))
        d = rng.uniform(1.5, 8.0)
        Rt, Rc = cay2rot(gt_poses[k, :3]), cay2rot(mcs[c, :3])
        R = Rt @ Rc
        t = Rt @ mcs[c, 3:] + gt_poses[k, 3:]
        pts[i] = R @ (np.array([float(x), float(y), float(z)]) * d) + t
        i += 1
    # visibility of every point in every (kf, cam)
    vis = []
    for k in range(nk):
        for c in range(ncam):
            uv, Xc = project(gt_poses[k], mcs[c], camv[c], pts)
            ok = np.isfinite(uv).all(-1)
            ui = np.round(uv[:, 0]).astype(int)
            vi = np.round(uv[:, 1]).astype(int)
            ok &= (ui > 30) & (vi > 30) & (ui < cams[c]["Iw"] - 30) & (vi < cams[c]["Ih"] - 30)
            idx = np.where(ok)[0]
            ok2 = np.zeros(n_points, bool)
            if len(idx):
                ok2[idx] = masks[c][vi[idx], ui[idx]] > 0
                # ray consistency: ImgToWorld(uv) must point along X_c
                rx, ry, rz = synth.img_to_world(cams[c], uv[idx, 0], uv[idx, 1])
                dirn = Xc[idx] / np.linalg.norm(Xc[idx], axis=1, keepdims=True)
                cosang = rx * dirn[:, 0] + ry * dirn[:, 1] + rz * dirn[:, 2]
                ok2[idx] &= cosang > 0.9999
            vis.append((k, c, ok2, uv))
    V = np.stack([v[2] for v in vis], 1)  # [n_points, nk*ncam]
    # subsample observations to hit the target edge count (keep >= 2 per point)
    nobs = V.sum(1)
    keep_p = np.minimum(1.0, target_edges / max(1, V.sum()))
    sel = V & (rng.random(V.shape) < keep_p)
    for p in range(n_points):
        if sel[p].sum() < 2 and V[p].sum() >= 2:
            cand = np.where(V[p])[0]
            sel[p, rng.choice(cand, 2, replace=False)] = True
    good = sel.sum(1) >= 2
    # octave distribution ~ per-level budget
    lev = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)
    lev /= lev.sum()
    e_pose, e_pt, e_cam, e_meas, e_info = [], [], [], [], []
    new_id = -np.ones(n_points, int)
    npts = 0
    for p in range(n_points):
        if not good[p]:
            continue
        new_id[p] = npts
        for j in np.where(sel[p])[0]:
            k, c = divmod(j, ncam)
            uv = vis[j][3][p]
            o = rng.choice(8, p=lev)
            sig = noise_scale * 1.2 ** o
            meas = uv + rng.normal(0, sig, 2)
            if rng.random() < outlier_frac:
                meas = np.array([rng.uniform(40, cams[c]["Iw"] - 40), rng.uniform(40, cams[c]["Ih"] - 40)])
            e_pose.append(k)
            e_pt.append(npts)
            e_cam.append(c)
            e_meas.append(meas)
            e_info.append(1.0 / (1.2 ** (2 * o)))
        npts += 1
    gt_pts = pts[good]
    poses0 = gt_poses.copy()
    pose_fixed = np.zeros(nk, np.uint8)
    pose_fixed[:n_fixed] = 1
    for k in range(n_fixed, nk):
        poses0[k, :3] += rng.normal(0, pose_noise[0], 3)
        poses0[k, 3:] += rng.normal(0, pose_noise[1], 3)
    pts0 = gt_pts + rng.normal(0, point_noise, gt_pts.shape)
    return dict(poses=poses0, pose_fixed=pose_fixed, points=pts0, mc=mcs, cam=camv,
                edge_pose=np.array(e_pose, np.int32), edge_point=np.array(e_pt, np.int32),
                edge_cam=np.array(e_cam, np.int32), edge_meas=np.array(e_meas, np.float64),
                edge_info=np.array(e_info, np.float64), huber_delta=huber_delta,
                gt_poses=gt_poses, gt_points=gt_pts)


def make_pose_problem(seed=0, n_points=1500, target_edges=5000, outlier_frac=0.05,
                      noise_scale=0.5, pose_noise=(0.01, 0.05), huber_multiplier=2.0):
    """PoseOptimization problem (src/cOptimizer.cpp:264-486): the current MultiFrame's pose
    (perturbed) and its 2D-3D correspondences to fixed map points (true positions), with
    information invSigma2(octave) and Huber delta 1.345 * huberMultiplier (:344)."""
    pr = make_problem(n_local=2, n_fixed=0, n_points=n_points, target_edges=target_edges,
                      seed=seed, outlier_frac=outlier_frac, noise_scale=noise_scale,
                      pose_noise=pose_noise, point_noise=0.0)
    sel = pr["edge_pose"] == 0
    used = np.unique(pr["edge_point"][sel])
    remap = -np.ones(len(pr["points"]), np.int64)
    remap[used] = np.arange(len(used))
    return dict(poses=pr["poses"][:1].copy(), pose_fixed=np.zeros(1, np.uint8),
                points=pr["gt_points"][used].copy(), mc=pr["mc"], cam=pr["cam"],
                edge_pose=np.zeros(int(sel.sum()), np.int32),
                edge_point=remap[pr["edge_point"][sel]].astype(np.int32),
                edge_cam=pr["edge_cam"][sel].copy(), edge_meas=pr["edge_meas"][sel].copy(),
                edge_info=pr["edge_info"][sel].copy(), huber_delta=1.345 * huber_multiplier,
                gt_pose=pr["gt_poses"][0].copy())


# ---------------------------------------------------------------------------
# LocalBundleAdjustment graph assembly (mcs_local_ba_select, src/cOptimizer.cpp:503-769)
# ---------------------------------------------------------------------------
class LbaMap(ctypes.Structure):
    _fields_ = [("n_kf", ctypes.c_int32), ("kf_id", ctypes.c_void_p), ("kf_bad", ctypes.c_void_p),
                ("kf_mp_off", ctypes.c_void_p), ("kf_mp", ctypes.c_void_p),
                ("n_points", ctypes.c_int32), ("pt_bad", ctypes.c_void_p),
                ("pt_obs_off", ctypes.c_void_p), ("obs_kf", ctypes.c_void_p)]


class LbaGraph(ctypes.Structure):
    _fields_ = [("local_kf", ctypes.c_void_p), ("n_local", ctypes.c_int32),
                ("fixed_kf", ctypes.c_void_p), ("n_fixed", ctypes.c_int32),
                ("pose_fixed", ctypes.c_void_p), ("points", ctypes.c_void_p),
                ("n_points", ctypes.c_int32), ("point_extra_obs", ctypes.c_void_p),
                ("edge_obs", ctypes.c_void_p), ("edge_pose", ctypes.c_void_p),
                ("edge_point", ctypes.c_void_p), ("n_edges", ctypes.c_int32),
                ("edge_cap", ctypes.c_int32)]


MCS_LBA_EMPTY = 1


def lba_map_struct(m):
    """numpy map dict (make_map) -> LbaMap (arrays kept alive in the dict)."""
    for k, dt in (("kf_id", np.int64), ("kf_bad", np.uint8), ("kf_mp_off", np.int32),
                  ("kf_mp", np.int32), ("pt_bad", np.uint8), ("pt_obs_off", np.int32),
                  ("obs_kf", np.int32)):
        m[k] = np.ascontiguousarray(m[k], dt)
    return LbaMap(len(m["kf_id"]), _p(m["kf_id"]), _p(m["kf_bad"]), _p(m["kf_mp_off"]),
                  _p(m["kf_mp"]), len(m["pt_bad"]), _p(m["pt_bad"]), _p(m["pt_obs_off"]),
                  _p(m["obs_kf"]))


def lba_graph_buffers(m):
    nk, npt, nobs = len(m["kf_id"]), len(m["pt_bad"]), len(m["obs_kf"])
    b = dict(local_kf=np.zeros(nk, np.int32), fixed_kf=np.zeros(nk, np.int32),
             pose_fixed=np.zeros(nk, np.uint8), points=np.zeros(npt, np.int32),
             point_extra_obs=np.zeros(npt, np.int32), edge_obs=np.zeros(max(1, nobs), np.int32),
             edge_pose=np.zeros(max(1, nobs), np.int32), edge_point=np.zeros(max(1, nobs), np.int32))
    g = LbaGraph(_p(b["local_kf"]), 0, _p(b["fixed_kf"]), 0, _p(b["pose_fixed"]), _p(b["points"]),
                 0, _p(b["point_extra_obs"]), _p(b["edge_obs"]), _p(b["edge_pose"]),
                 _p(b["edge_point"]), 0, nobs)
    return g, b


def lba_graph_result(rc, g, b):
    nl, nf, npt, ne = g.n_local, g.n_fixed, g.n_points, g.n_edges
    return dict(status=rc, local_kf=b["local_kf"][:nl].copy(), fixed_kf=b["fixed_kf"][:nf].copy(),
                pose_fixed=b["pose_fixed"][:nl + nf].copy(), points=b["points"][:npt].copy(),
                point_extra_obs=b["point_extra_obs"][:npt].copy(),
                edge_obs=b["edge_obs"][:ne].copy(), edge_pose=b["edge_pose"][:ne].copy(),
                edge_point=b["edge_point"][:ne].copy())


def local_ba_select(m, cur, covis):
    """mcs_local_ba_select: local / fixed keyframes, local points and edges of
    LocalBundleAdjustment for keyframe `cur` with covisibles `covis` (ordered)."""
    from . import lib
    st = lba_map_struct(m)
    cv = np.ascontiguousarray(covis, np.int32)
    g, b = lba_graph_buffers(m)
    rc = lib().mcs_local_ba_select(ctypes.byref(st), int(cur), _p(cv), len(cv), ctypes.byref(g))
    if rc < 0:
        from . import McsError, lib as _l
        raise McsError(rc, _l().mcs_last_error().decode())
    return lba_graph_result(rc, g, b)


def problem_from_graph(m, g, huber_delta=1.345 * 2):
    """mcs_ba_problem of one LocalBundleAdjustment call (vertices :585-711, edges :712-766):
    pose slots = local then fixed keyframes, points = local points, one edge per selected
    observation (measurement kp.pt, information invSigma2(octave))."""
    slots = np.concatenate([g["local_kf"], g["fixed_kf"]]).astype(np.int64)
    o = g["edge_obs"]
    return dict(poses=m["kf_pose"][slots].copy(), pose_fixed=g["pose_fixed"].copy(),
                points=m["pt_pos"][g["points"]].copy(), mc=m["mc"], cam=m["cam"],
                edge_pose=g["edge_pose"].astype(np.int32), edge_point=g["edge_point"].astype(np.int32),
                edge_cam=m["obs_cam"][o].astype(np.int32), edge_meas=m["obs_meas"][o].copy(),
                edge_info=m["obs_info"][o].copy(), huber_delta=huber_delta)


class GbaMap(ctypes.Structure):
    """Mirror of mcs_gba_map (include/mcs_ba.h)."""
    _fields_ = [("n_kf", ctypes.c_int32), ("kf_id", ctypes.c_void_p), ("kf_bad", ctypes.c_void_p),
                ("n_points", ctypes.c_int32), ("pt_id", ctypes.c_void_p), ("pt_bad", ctypes.c_void_p),
                ("pt_obs_off", ctypes.c_void_p), ("obs_kf", ctypes.c_void_p), ("n_cams", ctypes.c_int32)]


class GbaGraph(ctypes.Structure):
    """Mirror of mcs_gba_graph."""
    _fields_ = [("pose_kf", ctypes.c_void_p), ("pose_fixed", ctypes.c_void_p), ("n_poses", ctypes.c_int32),
                ("points", ctypes.c_void_p), ("point_vertex_id", ctypes.c_void_p), ("n_points", ctypes.c_int32),
                ("mc_vertex_id0", ctypes.c_int64), ("io_vertex_id0", ctypes.c_int64),
                ("kf_slot", ctypes.c_void_p), ("pt_slot", ctypes.c_void_p),
                ("edge_obs", ctypes.c_void_p), ("edge_pose", ctypes.c_void_p), ("edge_point", ctypes.c_void_p),
                ("n_edges", ctypes.c_int32), ("edge_cap", ctypes.c_int32), ("collision_id", ctypes.c_int64)]


class PoFrame(ctypes.Structure):
    """Mirror of mcs_po_frame."""
    _fields_ = [("n_keys", ctypes.c_int32), ("key_mp", ctypes.c_void_p), ("n_mp", ctypes.c_int32),
                ("pt_id", ctypes.c_void_p), ("n_cams", ctypes.c_int32)]


class PoGraph(ctypes.Structure):
    """Mirror of mcs_po_graph."""
    _fields_ = [("points", ctypes.c_void_p), ("point_vertex_id", ctypes.c_void_p), ("n_points", ctypes.c_int32),
                ("edge_obs", ctypes.c_void_p), ("edge_point", ctypes.c_void_p), ("n_edges", ctypes.c_int32),
                ("edge_cap", ctypes.c_int32)]


def global_ba_select(m, raise_on_error=True):
    """mcs_global_ba_select: the vertices and edges cOptimizer::BundleAdjustment builds from
    (vpKFs, vpMP) = the map dict's keyframes and points in list order (src/cOptimizer.cpp:101-234),
    and the write-back slots of :240-259.  m needs kf_id, kf_bad, pt_id, pt_bad, pt_obs_off,
    obs_kf and mc (n_cams)."""
    from . import lib, McsError
    for k, dt in (("kf_id", np.int64), ("kf_bad", np.uint8), ("pt_id", np.int64), ("pt_bad", np.uint8),
                  ("pt_obs_off", np.int32), ("obs_kf", np.int32)):
        m[k] = np.ascontiguousarray(m[k], dt)
    nk, npt, nobs = len(m["kf_id"]), len(m["pt_bad"]), len(m["obs_kf"])
    st = GbaMap(nk, _p(m["kf_id"]), _p(m["kf_bad"]), npt, _p(m["pt_id"]), _p(m["pt_bad"]),
                _p(m["pt_obs_off"]), _p(m["obs_kf"]), len(m["mc"]))
    b = dict(pose_kf=np.zeros(max(1, nk), np.int32), pose_fixed=np.zeros(max(1, nk), np.uint8),
             points=np.zeros(max(1, npt), np.int32), point_vertex_id=np.zeros(max(1, npt), np.int64),
             kf_slot=np.zeros(max(1, nk), np.int32), pt_slot=np.zeros(max(1, npt), np.int32),
             edge_obs=np.zeros(max(1, nobs), np.int32), edge_pose=np.zeros(max(1, nobs), np.int32),
             edge_point=np.zeros(max(1, nobs), np.int32))
    g = GbaGraph(_p(b["pose_kf"]), _p(b["pose_fixed"]), 0, _p(b["points"]), _p(b["point_vertex_id"]), 0,
                 -1, -1, _p(b["kf_slot"]), _p(b["pt_slot"]), _p(b["edge_obs"]), _p(b["edge_pose"]),
                 _p(b["edge_point"]), 0, nobs, -1)
    rc = lib().mcs_global_ba_select(ctypes.byref(st), ctypes.byref(g))
    if rc < 0 and raise_on_error:
        raise McsError(rc, lib().mcs_last_error().decode())
    npo, npp, ne = g.n_poses, g.n_points, g.n_edges
    return dict(status=rc, collision_id=g.collision_id, pose_kf=b["pose_kf"][:npo].copy(),
                pose_fixed=b["pose_fixed"][:npo].copy(), points=b["points"][:npp].copy(),
                point_vertex_id=b["point_vertex_id"][:npp].copy(), mc_vertex_id0=g.mc_vertex_id0,
                io_vertex_id0=g.io_vertex_id0, kf_slot=b["kf_slot"][:nk].copy(),
                pt_slot=b["pt_slot"][:npt].copy(), edge_obs=b["edge_obs"][:ne].copy(),
                edge_pose=b["edge_pose"][:ne].copy(), edge_point=b["edge_point"][:ne].copy())


def problem_from_gba_graph(m, g):
    """mcs_ba_problem of one BundleAdjustment call: poses = the keyframe vertices (mnId 0
    fixed), points = the point vertices, one edge per selected observation with measurement
    kp.pt, information I (:209) and Huber sqrt(5.991) (:161)."""
    o = g["edge_obs"]
    return dict(poses=np.ascontiguousarray(m["kf_pose"][g["pose_kf"]]), pose_fixed=g["pose_fixed"].copy(),
                points=np.ascontiguousarray(m["pt_pos"][g["points"]]), mc=m["mc"], cam=m["cam"],
                edge_pose=g["edge_pose"].astype(np.int32), edge_point=g["edge_point"].astype(np.int32),
                edge_cam=np.asarray(m["obs_cam"])[o].astype(np.int32),
                edge_meas=np.ascontiguousarray(np.asarray(m["obs_meas"])[o]), edge_info=np.ones(len(o)),
                huber_delta=HUBER_GLOBAL)


def global_ba_write_back(m, g, poses, points):
    """The reference's recovery loops (:242-259) over the select's slots: new keyframe poses
    and point positions for every list entry with a vertex (others keep their values)."""
    kp = np.array(m["kf_pose"], np.float64, copy=True)
    pp = np.array(m["pt_pos"], np.float64, copy=True)
    ks, ps = g["kf_slot"], g["pt_slot"]
    kp[ks >= 0] = poses[ks[ks >= 0]]
    pp[ps >= 0] = points[ps[ps >= 0]]
    return kp, pp


def global_map_from_problem(pr):
    """Config E as the map GlobalBundleAdjustment reads: keyframe i = pose i (mnId = i, so
    keyframe 0 is the fixed one), point j = point j (mnId = j), observations = the problem's
    edges in point order (each point's edges are in keyframe order, the std::map order)."""
    ep = np.asarray(pr["edge_point"])
    order = np.argsort(ep, kind="stable")
    npt, nk = len(pr["points"]), len(pr["poses"])
    off = np.zeros(npt + 1, np.int64)
    np.add.at(off, ep + 1, 1)
    return dict(kf_id=np.arange(nk, dtype=np.int64), kf_bad=np.zeros(nk, np.uint8),
                pt_id=np.arange(npt, dtype=np.int64), pt_bad=np.zeros(npt, np.uint8),
                pt_obs_off=np.cumsum(off).astype(np.int32),
                obs_kf=np.asarray(pr["edge_pose"])[order].astype(np.int32),
                obs_cam=np.asarray(pr["edge_cam"])[order], obs_meas=np.asarray(pr["edge_meas"])[order],
                kf_pose=pr["poses"], pt_pos=pr["points"], mc=pr["mc"], cam=pr["cam"])


def pose_optimization_select(key_mp, pt_id, n_cams):
    """mcs_pose_optimization_select: PoseOptimization's point vertices (one per distinct
    mnId, first appearance) and edges (one per non-NULL keypoint), src/cOptimizer.cpp:364-430."""
    from . import lib, McsError
    km = np.ascontiguousarray(key_mp, np.int32)
    pid = np.ascontiguousarray(pt_id, np.int64)
    f = PoFrame(len(km), _p(km), len(pid), _p(pid), int(n_cams))
    b = dict(points=np.zeros(max(1, len(pid)), np.int32), point_vertex_id=np.zeros(max(1, len(pid)), np.int64),
             edge_obs=np.zeros(max(1, len(km)), np.int32), edge_point=np.zeros(max(1, len(km)), np.int32))
    g = PoGraph(_p(b["points"]), _p(b["point_vertex_id"]), 0, _p(b["edge_obs"]), _p(b["edge_point"]), 0, len(km))
    rc = lib().mcs_pose_optimization_select(ctypes.byref(f), ctypes.byref(g))
    if rc < 0:
        raise McsError(rc, lib().mcs_last_error().decode())
    return dict(points=b["points"][:g.n_points].copy(), point_vertex_id=b["point_vertex_id"][:g.n_points].copy(),
                edge_obs=b["edge_obs"][:g.n_edges].copy(), edge_point=b["edge_point"][:g.n_edges].copy())


def make_map(n_kf=16, n_points=2500, target_edges=14000, seed=0, bad_kf=(), bad_points=0.01,
             zero_id_kf=None, unmatched_frac=0.1, covis_th=15):
    """Synthetic MultiKeyFrame map for LocalBundleAdjustment assembly: keyframes with mnId,
    isBad, map-point matches (with NULL entries), points with isBad and observations in
    keyframe order (the std::map iteration order of the reference with pointer order taken as
    keyframe order).  Geometry and observations from make_problem.  Returns the map dict;
    covisibles(m, k) gives GetVectorCovisibleKeyFrames (shared >= covis_th, weight order)."""
    rng = np.random.default_rng(seed + 17)
    pr = make_problem(n_local=n_kf, n_fixed=0, n_points=n_points, target_edges=target_edges,
                      seed=seed)
    nk, npt = len(pr["poses"]), len(pr["points"])
    ids = np.sort(rng.choice(np.arange(1, 10 * nk), nk, replace=False)).astype(np.int64)
    if zero_id_kf is not None:
        ids[zero_id_kf] = 0
    kf_bad = np.zeros(nk, np.uint8)
    kf_bad[list(bad_kf)] = 1
    pt_bad = (rng.random(npt) < bad_points).astype(np.uint8)
    order = np.lexsort((np.arange(len(pr["edge_pose"])), pr["edge_pose"], pr["edge_point"]))
    e_kf, e_pt = pr["edge_pose"][order], pr["edge_point"][order]
    obs_kf = e_kf.astype(np.int32)
    pt_obs_off = np.zeros(npt + 1, np.int32)
    np.add.at(pt_obs_off, e_pt + 1, 1)
    pt_obs_off = np.cumsum(pt_obs_off).astype(np.int32)
    # keyframe map-point matches: each observation is a keypoint of its keyframe, plus NULLs
    kf_lists = [[] for _ in range(nk)]
    for k, p in zip(e_kf, e_pt):
        kf_lists[k].append(int(p))
    kf_mp, kf_mp_off = [], [0]
    for k in range(nk):
        lst = kf_lists[k] + [-1] * int(unmatched_frac * len(kf_lists[k]))
        rng.shuffle(lst)
        kf_mp += lst
        kf_mp_off.append(len(kf_mp))
    return dict(kf_id=ids, kf_bad=kf_bad, kf_mp_off=np.array(kf_mp_off, np.int32),
                kf_mp=np.array(kf_mp, np.int32), pt_bad=pt_bad, pt_obs_off=pt_obs_off,
                obs_kf=obs_kf, obs_cam=pr["edge_cam"][order], obs_meas=pr["edge_meas"][order],
                obs_info=pr["edge_info"][order], kf_pose=pr["poses"], pt_pos=pr["points"],
                mc=pr["mc"], cam=pr["cam"], covis_th=covis_th)


def covisibles(m, k):
    """GetVectorCovisibleKeyFrames of keyframe k: keyframes sharing >= covis_th good map
    points, by decreasing weight (ties by index)."""
    nk = len(m["kf_id"])
    w = np.zeros(nk, np.int64)
    for p in range(len(m["pt_bad"])):
        if m["pt_bad"][p]:
            continue
        ks = set(m["obs_kf"][m["pt_obs_off"][p]:m["pt_obs_off"][p + 1]].tolist())
        if k in ks:
            for j in ks:
                if j != k:
                    w[j] += 1
    cand = [j for j in range(nk) if w[j] >= m["covis_th"]]
    return np.array(sorted(cand, key=lambda j: (-w[j], j)), np.int32)


# ---------------------------------------------------------------------------
# GPU solver binding
# ---------------------------------------------------------------------------
class Solver:
    """mcs_ba_ctx wrapper (device context reused across calls)."""

    def __init__(self, device=0):
        from . import lib, _check
        self._lib = lib()
        h = ctypes.c_void_p()
        _check(self._lib.mcs_ba_create(int(device), ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.mcs_ba_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def optimize(self, pr, options=None, edge_level=None, stop_flag=None, trace=0):
        from . import _check
        s = as_struct(pr)
        poses = pr["poses"].copy()
        points = pr["points"].copy()
        lvl = np.zeros(len(pr["edge_pose"]), np.uint8) if edge_level is None else \
            np.ascontiguousarray(edge_level, np.uint8)
        chi = np.zeros(len(pr["edge_pose"]), np.float64)
        o = options or BAOptions()
        tr = np.zeros(max(trace, 1), np.float64)
        rep = BAReport(0, 0, 0, 0, 0, 0, 0, 0, _p(tr) if trace else None, trace)
        sf = None if stop_flag is None else ctypes.c_int32(int(stop_flag))
        _check(self._lib.mcs_ba_optimize(self._h, ctypes.byref(s), ctypes.byref(o), _p(poses),
                                         _p(points), _p(lvl), _p(chi),
                                         ctypes.byref(sf) if sf is not None else None,
                                         ctypes.byref(rep)))
        return dict(poses=poses, points=points, edge_chi2=chi, report=rep,
                    stop_flag=None if sf is None else sf.value, trace=tr[:min(trace, rep.iterations)])

    def local_ba_ex(self, pr, extra_obs=None, stop_flag=0):
        """mcs_local_ba_ex: LocalBA rounds with the map-point bookkeeping (bad points, write-back
        mask).  extra_obs: observations of each point from bad keyframes (or None)."""
        from . import _check
        s = as_struct(pr)
        poses = pr["poses"].copy()
        points = pr["points"].copy()
        n = len(pr["edge_pose"])
        inl = np.zeros(max(1, n), np.uint8)
        pw = np.zeros(max(1, len(points)), np.uint8)
        ex = None if extra_obs is None else np.ascontiguousarray(extra_obs, np.int32)
        wb = ctypes.c_int32()
        sf = None if stop_flag is None else ctypes.c_int32(int(stop_flag))
        r1, r2 = BAReport(), BAReport()
        _check(self._lib.mcs_local_ba_ex(self._h, ctypes.byref(s), None if ex is None else _p(ex),
                                         _p(poses), _p(points), _p(inl), _p(pw), ctypes.byref(wb),
                                         None if sf is None else ctypes.byref(sf),
                                         ctypes.byref(r1), ctypes.byref(r2)))
        return dict(poses=poses, points=points, edge_inlier=inl[:n].copy(),
                    point_write=pw[:len(points)].copy(), write_back=wb.value,
                    stop_flag=None if sf is None else sf.value, report1=r1, report2=r2)

    def local_ba(self, pr, stop_flag=0):
        """mcs_local_ba; stop_flag None = pbStopFlag NULL (g2o's auxiliary terminate flag)."""
        from . import _check
        s = as_struct(pr)
        poses = pr["poses"].copy()
        points = pr["points"].copy()
        inl = np.zeros(len(pr["edge_pose"]), np.uint8)
        wb = ctypes.c_int32()
        sf = None if stop_flag is None else ctypes.c_int32(int(stop_flag))
        r1 = BAReport()
        r2 = BAReport()
        _check(self._lib.mcs_local_ba(self._h, ctypes.byref(s), _p(poses), _p(points), _p(inl),
                                      ctypes.byref(wb), None if sf is None else ctypes.byref(sf),
                                      ctypes.byref(r1), ctypes.byref(r2)))
        return dict(poses=poses, points=points, edge_inlier=inl, write_back=wb.value,
                    stop_flag=None if sf is None else sf.value, report1=r1, report2=r2)

    def pose_optimization(self, pr, trace=0):
        """cOptimizer::PoseOptimization (src/cOptimizer.cpp:264-486) via mcs_pose_optimization;
        pr holds one pose and fixed map points (make_pose_problem)."""
        from . import _check
        s = as_struct(pr)
        pose = np.ascontiguousarray(pr["poses"][0], np.float64).copy()
        n = len(pr["edge_pose"])
        out = np.zeros(max(n, 1), np.uint8)
        ngood = ctypes.c_int32()
        bad = ctypes.c_double()
        t1 = np.zeros(max(trace, 1))
        t2 = np.zeros(max(trace, 1))
        r1 = BAReport(0, 0, 0, 0, 0, 0, 0, 0, _p(t1) if trace else None, trace)
        r2 = BAReport(0, 0, 0, 0, 0, 0, 0, 0, _p(t2) if trace else None, trace)
        _check(self._lib.mcs_pose_optimization(self._h, ctypes.byref(s), _p(pose), _p(out),
                                               ctypes.byref(ngood), ctypes.byref(bad),
                                               ctypes.byref(r1), ctypes.byref(r2)))
        return dict(pose=pose, outlier=out[:n].copy(), n_good=ngood.value, bad_ratio=bad.value,
                    report1=r1, report2=r2, trace1=t1[:min(trace, r1.iterations)],
                    trace2=t2[:min(trace, r2.iterations)])

    def linearize(self, pr):
        from . import _check
        s = as_struct(pr)
        n = len(pr["edge_pose"])
        err = np.zeros((n, 2))
        jp = np.zeros((n, 2, 6))
        jl = np.zeros((n, 2, 3))
        _check(self._lib.mcs_ba_linearize(self._h, ctypes.byref(s), _p(err), _p(jp), _p(jl)))
        return err, jp, jl


# ---------------------------------------------------------------------------
# Global BA (config E) and point sharding
# ---------------------------------------------------------------------------
HUBER_GLOBAL = float(np.sqrt(5.991))     # cOptimizer::BundleAdjustment thHuber (src/cOptimizer.cpp:161)

# (user, op, offset, count, hipStream_t of the library)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                ctypes.c_int64, ctypes.c_void_p)


class BAShard(ctypes.Structure):
    """Mirror of mcs_ba_shard (include/mcs_ba.h)."""
    _fields_ = [("rank", ctypes.c_int32), ("world", ctypes.c_int32), ("xchg", ctypes.c_void_p),
                ("xchg_cap", ctypes.c_int64), ("allreduce", ALLREDUCE_FN),
                ("user", ctypes.c_void_p), ("stream_ordered", ctypes.c_int32)]


def ring_rig(ncams=8, size=1024, radius=0.12, phase_deg=10.0):
    """Config D/E rig: `ncams` Lafida-polynomial fisheyes scaled to size x size, optical axes
    horizontal and evenly spread in yaw, mounted on a ring of the given radius."""
    cam = synth.scaled_cam(synth.LAFIDA_CAMS[0], size, size)
    cams, mcs = [], []
    for c in range(ncams):
        ph = np.deg2rad(phase_deg + 360.0 * c / ncams)
        ax = np.array([np.cos(ph), np.sin(ph), 0.0])
        xc = np.array([-np.sin(ph), np.cos(ph), 0.0])
        yc = np.array([0.0, 0.0, -1.0])
        R = np.stack([xc, yc, -ax], 1)           # columns: camera axes in the body frame
        mcs.append(np.concatenate([rot2cay(R), radius * ax]))
        cams.append(dict(cam))
    return cams, np.array(mcs)


def make_global_problem(n_kf=200, n_points=50000, target_edges=400000, ncams=8, size=1024,
                        seed=0, outlier_frac=0.02, noise_scale=0.5, pose_noise=(0.003, 0.01),
                        point_noise=0.05, step=0.15, max_range=8.0):
    """Config E: GlobalBA over n_kf MultiKeyFrames of an ncams ring rig, ~n_points points and
    ~target_edges observations (vectorised generator).  BundleAdjustment semantics:
    information = I (:209), Huber sqrt(5.991) (:161), keyframe 0 fixed (:119-120)."""
    rng = np.random.default_rng(seed)
    cams, mcs = ring_rig(ncams, size)
    camv = np.stack([cam_vec(c) for c in cams])
    cam = cams[0]
    mask = synth.mirror_mask(cam)
    # smooth planar trajectory (slow yaw drift), body z up
    k = np.arange(n_kf)
    yaw = 0.6 * np.sin(k / 40.0)
    gt_poses = np.zeros((n_kf, 6))
    pos = np.zeros(3)
    for i in range(n_kf):
        R = np.array([[np.cos(yaw[i]), -np.sin(yaw[i]), 0], [np.sin(yaw[i]), np.cos(yaw[i]), 0],
                      [0, 0, 1]])
        gt_poses[i, :3] = rot2cay(R)
        gt_poses[i, 3:] = pos
        pos = pos + step * np.array([np.cos(yaw[i]), np.sin(yaw[i]), 0.02 * np.sin(i / 7.0)])
    # points on rays of random (kf, cam, pixel inside the mirror mask)
    ys, xs = np.nonzero(mask[40:-40, 40:-40])
    pick = rng.integers(len(xs), size=n_points)
    u = xs[pick] + 40 + rng.uniform(0, 1, n_points)
    v = ys[pick] + 40 + rng.uniform(0, 1, n_points)
    rx, ry, rz = synth.img_to_world(cam, u, v)
    depth = rng.uniform(1.5, max_range, n_points)
    kk = rng.integers(n_kf, size=n_points)
    cc = rng.integers(ncams, size=n_points)
    Xc = np.stack([rx, ry, rz], 1) * depth[:, None]
    Rt = cay2rot(gt_poses[kk, :3])
    Rc = cay2rot(mcs[cc, :3])
    Rw = Rt @ Rc
    tw = np.einsum("nij,nj->ni", Rt, mcs[cc, 3:]) + gt_poses[kk, 3:]
    pts = np.einsum("nij,nj->ni", Rw, Xc) + tw
    # visibility of every point in every (kf, cam): in range, inside the mask, ray-consistent
    rows, cols, uvs = [], [], []
    for i in range(n_kf):
        near = np.nonzero(np.linalg.norm(pts - gt_poses[i, 3:], axis=1) < max_range)[0]
        if len(near) == 0:
            continue
        for c in range(ncams):
            uv, Xc_ = project(gt_poses[i], mcs[c], camv[c], pts[near])
            ok = np.isfinite(uv).all(-1)
            ui = np.round(np.nan_to_num(uv[:, 0], nan=-1e6)).astype(np.int64)
            vi = np.round(np.nan_to_num(uv[:, 1], nan=-1e6)).astype(np.int64)
            ok &= (ui > 30) & (vi > 30) & (ui < size - 30) & (vi < size - 30)
            idx = np.nonzero(ok)[0]
            if len(idx) == 0:
                continue
            ok2 = mask[vi[idx], ui[idx]] > 0
            rx, ry, rz = synth.img_to_world(cam, uv[idx, 0], uv[idx, 1])
            d = Xc_[idx] / np.linalg.norm(Xc_[idx], axis=1, keepdims=True)
            ok2 &= (rx * d[:, 0] + ry * d[:, 1] + rz * d[:, 2]) > 0.9999
            idx = idx[ok2]
            rows.append(near[idx])
            cols.append(np.full(len(idx), i * ncams + c))
            uvs.append(uv[idx])
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    uvs = np.concatenate(uvs)
    # subsample observations towards the target (keep >= 2 per point when possible)
    order = np.argsort(rows, kind="stable")
    rows, cols, uvs = rows[order], cols[order], uvs[order]
    cnt_all = np.bincount(rows, minlength=n_points)
    forced = 2 * int((cnt_all >= 2).sum())
    keep = rng.random(len(rows)) < min(1.0, max(0, target_edges - forced) / max(1, len(rows) - forced))
    start = np.concatenate([[0], np.cumsum(cnt_all)[:-1]])
    for j in (0, 1):   # force the first two observations of points that have >= 2
        sel = cnt_all >= 2
        keep[start[sel] + j] = True
    rows, cols, uvs = rows[keep], cols[keep], uvs[keep]
    cnt = np.bincount(rows, minlength=n_points)
    good = cnt >= 2
    m = good[rows]
    rows, cols, uvs = rows[m], cols[m], uvs[m]
    new_id = -np.ones(n_points, np.int64)
    new_id[good] = np.arange(good.sum())
    ne = len(rows)
    lev = np.array([869, 724, 603, 503, 419, 349, 291, 242], np.float64)
    octv = rng.choice(8, size=ne, p=lev / lev.sum())
    meas = uvs + rng.normal(0, 1, (ne, 2)) * (noise_scale * 1.2 ** octv)[:, None]
    out = rng.random(ne) < outlier_frac
    meas[out] = rng.uniform(60, size - 60, (int(out.sum()), 2))
    poses0 = gt_poses.copy()
    pose_fixed = np.zeros(n_kf, np.uint8)
    pose_fixed[0] = 1
    poses0[1:, :3] += rng.normal(0, pose_noise[0], (n_kf - 1, 3))
    poses0[1:, 3:] += rng.normal(0, pose_noise[1], (n_kf - 1, 3))
    gt_pts = pts[good]
    pts0 = gt_pts + rng.normal(0, point_noise, gt_pts.shape)
    return dict(poses=poses0, pose_fixed=pose_fixed, points=pts0, mc=mcs, cam=camv,
                edge_pose=(cols // ncams).astype(np.int32), edge_point=new_id[rows].astype(np.int32),
                edge_cam=(cols % ncams).astype(np.int32), edge_meas=meas,
                edge_info=np.ones(ne), huber_delta=HUBER_GLOBAL, gt_poses=gt_poses,
                gt_points=gt_pts)


def config_e_problem(n_kf=200, n_points=50000, target_edges=400000, seed=7, **kw):
    """Config E through the reference-side boundary: the generated map (make_global_problem as
    GlobalBundleAdjustment's keyframe / map-point lists) assembled by mcs_global_ba_select into
    the problem mcs_global_ba takes (src/cOptimizer.cpp:101-234).  Ground truth kept."""
    pr = make_global_problem(n_kf=n_kf, n_points=n_points, target_edges=target_edges, seed=seed, **kw)
    m = global_map_from_problem(pr)
    g = global_ba_select(m)
    out = problem_from_gba_graph(m, g)
    out["gt_poses"], out["gt_points"] = pr["gt_poses"], pr["gt_points"]
    return out


def shard_points(pr, world):
    """Contiguous point ranges with balanced edge counts -> list of (point_lo, point_hi)."""
    npts = len(pr["points"])
    cnt = np.bincount(pr["edge_point"], minlength=npts)
    cum = np.cumsum(cnt)
    tot = cum[-1] if npts else 0
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(np.searchsorted(cum, tot * r / world, side="left")) + 1 if npts else 0)
    bounds.append(npts)
    bounds = np.maximum.accumulate(np.minimum(np.array(bounds), npts))
    return [(int(bounds[r]), int(bounds[r + 1])) for r in range(world)]


def shard_problem(pr, rank, world):
    """This rank's BA shard: the points [lo, hi) with ALL their edges (edge order kept),
    every pose (replicated).  Returns (sub_problem, (lo, hi), edge_ids)."""
    lo, hi = shard_points(pr, world)[rank]
    ep = np.asarray(pr["edge_point"])
    eids = np.nonzero((ep >= lo) & (ep < hi))[0]
    sub = dict(pr)
    sub["points"] = np.ascontiguousarray(pr["points"][lo:hi])
    for k in ("edge_pose", "edge_cam", "edge_meas", "edge_info"):
        sub[k] = np.ascontiguousarray(np.asarray(pr[k])[eids])
    sub["edge_point"] = np.ascontiguousarray(ep[eids] - lo, dtype=np.int32)
    return sub, (lo, hi), eids


class TorchExchange:
    """mcs_ba_shard backed by torch.distributed: the exchange buffer is a torch tensor on the
    rank's GPU and the callback all-reduces a slice of it (backend "nccl" = RCCL over xGMI).

    Default (stream_ordered = 0): the library drains its stream before each call and the
    callback returns only once the reduction is complete (the all-reduce is followed by a
    device synchronisation), which is correct whatever ProcessGroupNCCL does with streams.

    stream_ordered = 1 (opt-in: argument, or MCS_BA_STREAM_ORDERED=1): the callback issues the
    all-reduce with the library's stream as torch's current stream, so RCCL starts after the
    kernels that produced the slice and the library's next kernels wait for it on the device --
    no host synchronisation per exchange.  This relies on ProcessGroupNCCL making the external
    stream wait for the collective; it has run only on gloo and on the single-GPU ThreadExchange
    mock, never on real RCCL with world > 1, so it stays off until a 2-GPU run has shown ordered
    == unordered (identical poses and iteration counts).  A CPU buffer (gloo) is always reduced
    synchronously."""

    def __init__(self, n_poses, device, group=None, stream_ordered=None):
        import torch
        import torch.distributed as dist
        from . import lib
        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        cap = int(lib().mcs_ba_xchg_doubles(int(n_poses)))
        self.buf = torch.zeros(cap, dtype=torch.float64, device=device)
        self._cb = ALLREDUCE_FN(self._allreduce)
        if stream_ordered is None:
            stream_ordered = os.environ.get("MCS_BA_STREAM_ORDERED", "0") == "1"
        self.ordered = bool(stream_ordered) and self.buf.is_cuda
        self.shard = BAShard(self.rank, self.world, self.buf.data_ptr(), cap, self._cb, None,
                             1 if self.ordered else 0)
        self._streams = {}
        self.calls = 0

    def _stream(self, handle):
        s = self._streams.get(handle)
        if s is None:
            s = self.torch.cuda.ExternalStream(handle, device=self.buf.device)
            self._streams[handle] = s
        return s

    def _allreduce(self, user, op, off, cnt, stream=None):
        try:
            t = self.buf[off:off + cnt]
            rop = self.dist.ReduceOp.SUM if op == 0 else self.dist.ReduceOp.MAX
            if self.ordered:
                # the NCCL process group orders the collective after the current stream's work
                # and makes the current stream wait for it (no host wait)
                with self.torch.cuda.stream(self._stream(stream)):
                    self.dist.all_reduce(t, op=rop, group=self.group)
            elif self.buf.is_cuda:
                # the library drained its stream; complete the reduction before returning
                self.dist.all_reduce(t, op=rop, group=self.group)
                self.torch.cuda.synchronize(self.buf.device)
            else:
                self.dist.all_reduce(t, op=rop, group=self.group)
            self.calls += 1
            return 0
        except Exception:   # never raise through the C stack
            return 1


def _solver_global_ba(self, pr, pose_only=False, stop_flag=None, exchange=None, trace=0):
    """cOptimizer::BundleAdjustment (src/cOptimizer.cpp:73-261) on this rank's problem."""
    from . import _check
    s = as_struct(pr)
    poses = pr["poses"].copy()
    points = pr["points"].copy()
    tr = np.zeros(max(trace, 1), np.float64)
    rep = BAReport(0, 0, 0, 0, 0, 0, 0, 0, _p(tr) if trace else None, trace)
    sf = None if stop_flag is None else ctypes.c_int32(int(stop_flag))
    sh = ctypes.byref(exchange.shard) if exchange is not None else None
    _check(self._lib.mcs_global_ba(self._h, ctypes.byref(s), 1 if pose_only else 0, _p(poses),
                                   _p(points), ctypes.byref(sf) if sf is not None else None,
                                   ctypes.byref(rep), sh))
    return dict(poses=poses, points=points, report=rep,
                stop_flag=None if sf is None else sf.value, trace=tr[:min(trace, rep.iterations)])


def _solver_optimize_sharded(self, pr, exchange, options=None, edge_level=None, stop_flag=None,
                             trace=0):
    from . import _check
    s = as_struct(pr)
    poses = pr["poses"].copy()
    points = pr["points"].copy()
    lvl = np.zeros(len(pr["edge_pose"]), np.uint8) if edge_level is None else \
        np.ascontiguousarray(edge_level, np.uint8)
    chi = np.zeros(len(pr["edge_pose"]), np.float64)
    o = options or BAOptions()
    tr = np.zeros(max(trace, 1), np.float64)
    rep = BAReport(0, 0, 0, 0, 0, 0, 0, 0, _p(tr) if trace else None, trace)
    sf = None if stop_flag is None else ctypes.c_int32(int(stop_flag))
    _check(self._lib.mcs_ba_optimize_sharded(self._h, ctypes.byref(s), ctypes.byref(o), _p(poses),
                                             _p(points), _p(lvl), _p(chi),
                                             ctypes.byref(sf) if sf is not None else None,
                                             ctypes.byref(rep), ctypes.byref(exchange.shard)))
    return dict(poses=poses, points=points, edge_chi2=chi, report=rep,
                stop_flag=None if sf is None else sf.value, trace=tr[:min(trace, rep.iterations)])


Solver.global_ba = _solver_global_ba
Solver.optimize_sharded = _solver_optimize_sharded


def dense_ldlt_solve(S, b, device=0, tiled=False, path=None):
    """Device LDL^T solve of the reduced camera system (test hook) -> (x, zero_pivot).
    tiled=True forces the pad + per-step panel + backward kernels even for n <= 64 (path 1);
    path=2 forces the pipelined factorisation (one launch); path=3 the per-step panels with the
    one-workgroup backward substitution (every path above 96 tiles); default path 0 = what BA
    uses."""
    from . import lib, _check
    S = np.ascontiguousarray(S, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    n = S.shape[0]
    x = np.zeros(n)
    zp = ctypes.c_int32()
    if path is None:
        path = 1 if tiled else 0
    _check(lib().mcs_dense_ldlt_solve_ex(int(device), _p(S), n, _p(b), _p(x), ctypes.byref(zp),
                                         int(path)))
    return x, zp.value


def set_ldlt_wait_ticks(ticks):
    """Test hook: the pipelined LDL^T's hand-off wait bound (100 MHz ticks; <= 0 = default)."""
    from . import lib, _check
    _check(lib().mcs_ldlt_set_wait_ticks(int(ticks)))


BA_STAGES = ("linearize", "schur", "exchange", "solve", "update")


def _solver_enable_timing(self, on=True):
    from . import _check
    _check(self._lib.mcs_ba_enable_timing(self._h, 1 if on else 0))


def _solver_read_timing(self, reset=True):
    """-> (dict stage -> accumulated ms, iterations, trials, last reduced-system size n)."""
    from . import _check
    ms = np.zeros(len(BA_STAGES))
    it, tr, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    _check(self._lib.mcs_ba_read_timing(self._h, _p(ms), ctypes.byref(it), ctypes.byref(tr),
                                        ctypes.byref(n), 1 if reset else 0))
    return dict(zip(BA_STAGES, ms.tolist())), it.value, tr.value, n.value


BA_HOST_PHASES = ("checks", "structure", "upload", "download", "lba_bookkeeping")


def _solver_read_host_timing(self, reset=True):
    """-> (dict host phase -> accumulated ms, optimize calls) (mcs_ba_read_host_timing)."""
    from . import _check
    ms = np.zeros(len(BA_HOST_PHASES))
    n = ctypes.c_int32()
    _check(self._lib.mcs_ba_read_host_timing(self._h, _p(ms), ctypes.byref(n), 1 if reset else 0))
    return dict(zip(BA_HOST_PHASES, ms.tolist())), n.value


Solver.read_host_timing = _solver_read_host_timing
Solver.enable_timing = _solver_enable_timing
Solver.read_timing = _solver_read_timing
