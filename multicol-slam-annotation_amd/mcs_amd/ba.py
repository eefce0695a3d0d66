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


def as_struct(pr):
    """numpy problem dict -> BAProblem (keeps references alive in the dict)."""
    for k, dt in (("poses", np.float64), ("pose_fixed", np.uint8), ("points", np.float64),
                  ("mc", np.float64), ("cam", np.float64), ("edge_pose", np.int32),
                  ("edge_point", np.int32), ("edge_cam", np.int32), ("edge_meas", np.float64),
                  ("edge_info", np.float64)):
        pr[k] = np.ascontiguousarray(pr[k], dtype=dt)
    s = BAProblem(len(pr["poses"]), len(pr["points"]), len(pr["edge_pose"]), len(pr["mc"]),
                  _p(pr["poses"]), _p(pr["pose_fixed"]), _p(pr["points"]), _p(pr["mc"]),
                  _p(pr["cam"]), _p(pr["edge_pose"]), _p(pr["edge_point"]), _p(pr["edge_cam"]),
                  _p(pr["edge_meas"]), _p(pr["edge_info"]), float(pr["huber_delta"]))
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

    def local_ba(self, pr, stop_flag=0):
        from . import _check
        s = as_struct(pr)
        poses = pr["poses"].copy()
        points = pr["points"].copy()
        inl = np.zeros(len(pr["edge_pose"]), np.uint8)
        wb = ctypes.c_int32()
        sf = ctypes.c_int32(int(stop_flag))
        r1 = BAReport()
        r2 = BAReport()
        _check(self._lib.mcs_local_ba(self._h, ctypes.byref(s), _p(poses), _p(points), _p(inl),
                                      ctypes.byref(wb), ctypes.byref(sf), ctypes.byref(r1),
                                      ctypes.byref(r2)))
        return dict(poses=poses, points=points, edge_inlier=inl, write_back=wb.value,
                    stop_flag=sf.value, report1=r1, report2=r2)

    def linearize(self, pr):
        from . import _check
        s = as_struct(pr)
        n = len(pr["edge_pose"])
        err = np.zeros((n, 2))
        jp = np.zeros((n, 2, 6))
        jl = np.zeros((n, 2, 3))
        _check(self._lib.mcs_ba_linearize(self._h, ctypes.byref(s), _p(err), _p(jp), _p(jl)))
        return err, jp, jl
