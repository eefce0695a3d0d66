"""Projection-guided (windowed) matching on the GPU (include/mcs_matcher.h, window API).

Host mirror of the windowed searches of cORBmatcher (checkOrientation = false,
include/cORBmatcher.h:40):

  RULE_PROJECT_MAPPOINTS  SearchByProjection(F, vpMapPoints, th)   src/cORBmatcher.cpp:67-166
  RULE_PROJECT_LASTFRAME  SearchByProjection(Current, Last, th)    src/cORBmatcher.cpp:1991-2123
  RULE_INITIALIZATION     SearchForInitialization(F1, F2, ...)     src/cORBmatcher.cpp:579-726
  RULE_WINDOW             WindowSearch(F1, F2, windowSize, ...)    src/cORBmatcher.cpp:326-473

The cMultiFrame grid (src/cMultiFrame.cpp:154-184, PosInGrid :342-353) is built on the host
once per frame; GetFeaturesInArea (:272-340) for every query and the Hamming distance of every
candidate run on the GPU (mcs_window_search_device, one wave per query); the sequential
best / second-best rule, which depends on the assignments of earlier queries, runs on the host
(mcs_window_select).  A query is one GetFeaturesInArea call of the reference: (x, y, r),
(cam, minLevel, maxLevel) and the query descriptor (+ its mask with learned mdBRIEF masks).
"""
import ctypes
import math

import numpy as np

from . import MCS_ERR_CAPACITY, McsError, _check, lib

GRID_COLS, GRID_ROWS = 64, 48      # FRAME_GRID_COLS / FRAME_GRID_ROWS (include/cMultiFrame.h:47-48)
RULE_PROJECT_MAPPOINTS, RULE_PROJECT_LASTFRAME, RULE_INITIALIZATION, RULE_WINDOW = 0, 1, 2, 3


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class WindowFrame(ctypes.Structure):
    """Mirror of mcs_window_frame (include/mcs_matcher.h)."""
    _fields_ = [("n_cams", ctypes.c_int32), ("n_kp", ctypes.c_int32), ("bytes", ctypes.c_int32),
                ("grid_params", ctypes.c_void_p), ("kp_xy", ctypes.c_void_p),
                ("kp_cam", ctypes.c_void_p), ("kp_octave", ctypes.c_void_p),
                ("desc", ctypes.c_void_p), ("desc_mask", ctypes.c_void_p)]


def matcher_thresholds(feat_dim, having_masks=False):
    """(TH_HIGH_, TH_LOW_) of the cORBmatcher ctor (src/cORBmatcher.cpp:46-65), feat_dim in bytes."""
    if having_masks:
        return int(math.floor(1.5 * feat_dim)), int(math.floor(feat_dim))
    return 3 * feat_dim, 2 * feat_dim


def grid_params(min_xy, max_xy):
    """[n_cams, 4] = (mnMinX, mnMinY, mfGridElementWidthInv, mfGridElementHeightInv) per camera
    (src/cMultiFrame.cpp:154-157) from the integer image bounds."""
    mn = np.asarray(min_xy, np.int64).reshape(-1, 2)
    mx = np.asarray(max_xy, np.int64).reshape(-1, 2)
    gp = np.zeros((len(mn), 4), np.float64)
    gp[:, :2] = mn
    gp[:, 2] = float(GRID_COLS) / (mx[:, 0] - mn[:, 0]).astype(np.float64)
    gp[:, 3] = float(GRID_ROWS) / (mx[:, 1] - mn[:, 1]).astype(np.float64)
    return gp


def grid_build(kp_xy, kp_cam, gp):
    """mcs_frame_grid_build -> (cell_ptr [n_cams*64*48 + 1], cell_kp [n_in_grid]), host."""
    kp_xy = np.ascontiguousarray(kp_xy, np.float32).reshape(-1, 2)
    kp_cam = np.ascontiguousarray(kp_cam, np.int32).reshape(-1)
    gp = np.ascontiguousarray(gp, np.float64).reshape(-1, 4)
    n = len(kp_xy)
    ptr = np.zeros(len(gp) * GRID_COLS * GRID_ROWS + 1, np.int32)
    cells = np.zeros(max(n, 1), np.int32)
    nin = ctypes.c_int32()
    _check(lib().mcs_frame_grid_build(_p(kp_xy), _p(kp_cam), n, len(gp), _p(gp), _p(ptr),
                                      _p(cells), ctypes.byref(nin)))
    return ptr, cells[:nin.value].copy()


class FrameGrid:
    """Device copy of one cMultiFrame: keypoints (mvKeys pt, octave), descriptors
    (mDescriptors in camera order, + mDescriptorMasks) and the feature grid."""

    def __init__(self, kp_xy, kp_cam, kp_octave, desc, gp, desc_mask=None, device="cuda"):
        import torch
        self.device = torch.device(device)
        self.gp = np.ascontiguousarray(gp, np.float64).reshape(-1, 4)
        self.n_cams = len(self.gp)
        ptr, cells = grid_build(kp_xy, kp_cam, self.gp)

        def up(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        self.cell_ptr = up(ptr)
        self.cell_kp = up(cells if len(cells) else np.zeros(1, np.int32))
        self.d_gp = up(self.gp)
        self.kp_octave = np.ascontiguousarray(kp_octave, np.int32).reshape(-1)
        self.n_kp = len(self.kp_octave)
        self.d_xy = up(np.asarray(kp_xy, np.float32).reshape(-1, 2))
        self.d_oct = up(self.kp_octave)
        desc = np.ascontiguousarray(desc, np.uint8)
        if desc.ndim != 2 or len(desc) != self.n_kp:
            raise ValueError("desc must be [n_kp, bytes]")
        self.bytes = desc.shape[1]
        self.d_desc = up(desc)
        self.d_mask = None if desc_mask is None else up(np.ascontiguousarray(desc_mask, np.uint8))


def window_search(frame, q_xyr, q_cam_lvl, q_desc, q_mask=None, cap=None, retry=True):
    """GetFeaturesInArea + DescriptorDistance64[Masked] of every query on the GPU.
    Returns numpy (cand_ptr [nq+1], cand_kp, cand_dist) in the reference's candidate order."""
    import torch
    dev = frame.device
    q_xyr = np.ascontiguousarray(q_xyr, np.float64).reshape(-1, 3)
    nq = len(q_xyr)
    q_cl = np.ascontiguousarray(q_cam_lvl, np.int32).reshape(nq, 3)
    q_desc = np.ascontiguousarray(q_desc, np.uint8).reshape(nq, frame.bytes)
    if (q_mask is None) != (frame.d_mask is None):
        raise ValueError("query masks and frame masks must both be given (mdBRIEF) or both be None")

    def up(a):
        return torch.from_numpy(a).to(dev)
    d_xyr, d_cl, d_qd = up(q_xyr), up(q_cl), up(q_desc)
    d_qm = None if q_mask is None else up(np.ascontiguousarray(q_mask, np.uint8).reshape(nq, frame.bytes))
    d_ptr = torch.zeros(nq + 1, dtype=torch.int32, device=dev)
    cap = int(cap if cap is not None else max(1024, 32 * nq))
    stream = torch.cuda.current_stream(dev)
    total = ctypes.c_int64()
    while True:
        d_kp = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        d_dist = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        rc = lib().mcs_window_search_device(
            frame.cell_ptr.data_ptr(), frame.cell_kp.data_ptr(), frame.d_gp.data_ptr(), frame.n_cams,
            frame.d_xy.data_ptr(), frame.d_oct.data_ptr(), frame.d_desc.data_ptr(),
            None if frame.d_mask is None else frame.d_mask.data_ptr(), frame.bytes, nq,
            d_xyr.data_ptr(), d_cl.data_ptr(), d_qd.data_ptr(),
            None if d_qm is None else d_qm.data_ptr(), d_ptr.data_ptr(), d_kp.data_ptr(),
            d_dist.data_ptr(), cap, ctypes.byref(total), stream.cuda_stream)
        if rc == MCS_ERR_CAPACITY and retry and total.value > cap:
            cap = int(total.value)
            continue
        _check(rc)
        break
    n = int(total.value)
    return d_ptr.cpu().numpy(), d_kp[:n].cpu().numpy(), d_dist[:n].cpu().numpy()


def window_select(rule, cand_ptr, cand_kp, cand_dist, kp_octave, th, nnratio, kp_assigned=None):
    """The reference's selection loop over the candidate lists (host).
    Returns (match [nq], n_matches, kp_assigned)."""
    cand_ptr = np.ascontiguousarray(cand_ptr, np.int32)
    nq = len(cand_ptr) - 1
    cand_kp = np.ascontiguousarray(cand_kp, np.int32)
    cand_dist = np.ascontiguousarray(cand_dist, np.int32)
    kp_octave = np.ascontiguousarray(kp_octave, np.int32)
    n_kp = len(kp_octave)
    a = np.zeros(max(n_kp, 1), np.uint8)
    if kp_assigned is not None:
        a[:n_kp] = np.asarray(kp_assigned, np.uint8)
    m = np.zeros(max(nq, 1), np.int32)
    n = ctypes.c_int32()
    _check(lib().mcs_window_select(int(rule), nq, _p(cand_ptr), _p(cand_kp), _p(cand_dist),
                                   _p(kp_octave), n_kp, int(th), float(nnratio), _p(a), _p(m),
                                   ctypes.byref(n)))
    return m[:nq], n.value, a[:n_kp]


def window_match(rule, frame, q_xyr, q_cam_lvl, q_desc, th, nnratio, q_mask=None, kp_assigned=None):
    """Device search + host selection on a FrameGrid."""
    ptr, kp, dist = window_search(frame, q_xyr, q_cam_lvl, q_desc, q_mask)
    return window_select(rule, ptr, kp, dist, frame.kp_octave, th, nnratio, kp_assigned)


def window_match_host(rule, gp, kp_xy, kp_cam, kp_octave, desc, q_xyr, q_cam_lvl, q_desc, th,
                      nnratio, desc_mask=None, q_mask=None, kp_assigned=None, device=0):
    """mcs_window_match: host buffers in (the reference call sites' data), one call."""
    gp = np.ascontiguousarray(gp, np.float64).reshape(-1, 4)
    xy = np.ascontiguousarray(kp_xy, np.float32).reshape(-1, 2)
    cam = np.ascontiguousarray(kp_cam, np.int32)
    octv = np.ascontiguousarray(kp_octave, np.int32)
    desc = np.ascontiguousarray(desc, np.uint8)
    dm = None if desc_mask is None else np.ascontiguousarray(desc_mask, np.uint8)
    f = WindowFrame(len(gp), len(xy), desc.shape[1], _p(gp).value, _p(xy).value, _p(cam).value,
                    _p(octv).value, _p(desc).value, None if dm is None else _p(dm).value)
    q_xyr = np.ascontiguousarray(q_xyr, np.float64).reshape(-1, 3)
    nq = len(q_xyr)
    q_cl = np.ascontiguousarray(q_cam_lvl, np.int32).reshape(nq, 3)
    q_desc = np.ascontiguousarray(q_desc, np.uint8).reshape(nq, desc.shape[1])
    qm = None if q_mask is None else np.ascontiguousarray(q_mask, np.uint8)
    a = np.zeros(max(len(xy), 1), np.uint8)
    if kp_assigned is not None:
        a[:len(xy)] = np.asarray(kp_assigned, np.uint8)
    m = np.zeros(max(nq, 1), np.int32)
    n = ctypes.c_int32()
    _check(lib().mcs_window_match(int(device), int(rule), ctypes.byref(f), nq, _p(q_xyr), _p(q_cl),
                                  _p(q_desc), _p(qm), int(th), float(nnratio), _p(a), _p(m),
                                  ctypes.byref(n)))
    return m[:nq], n.value, a[:len(xy)]


__all__ = ["FrameGrid", "WindowFrame", "grid_build", "grid_params", "matcher_thresholds",
           "window_search", "window_select", "window_match", "window_match_host", "McsError",
           "RULE_PROJECT_MAPPOINTS", "RULE_PROJECT_LASTFRAME", "RULE_INITIALIZATION", "RULE_WINDOW"]
