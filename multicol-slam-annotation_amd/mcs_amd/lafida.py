"""Lafida settings / calibration ingest without OpenCV.

Host mirror of the reference's cv::FileStorage reads for the MultiCol-SLAM front-end:

  read_filestorage(path)     ~ cv::FileStorage(path, READ) on the flat `key: value` YAML files
                               of Examples/Lafida (OpenCV 3.x FileNode semantics: an absent key
                               reads as 0, `(int)` of a real node is cvRound, `(double)` of an
                               int node converts)
  load_rig(dir)              ~ cSystem::LoadMCS (src/cSystem.cpp:124-176): CameraSystem.nrCams,
                               M_c as Cayley 6-vectors CameraSystem.cam{c+1}_{1..6}, interior
                               orientation InteriorOrientationFisheye{c}.yaml (nrpol forward
                               coefficients a_i into a 5-vector, nrinvpol inverse coefficients
                               pol_i into a 12-vector, c, d, e, u0, v0, Iw, Ih, mirrorMask)
  extractor_params(settings) ~ cTracking ctor (src/cTracking.cpp:86-158): the tracking
                               extractor (nFeatures, fastTh) and the initialisation extractor
                               (2 * nFeatures, fastTh 5), both with edgeThreshold 25,
                               firstLevel 0, patchSize 32
  tracking_frames(settings)  ~ fps (0 -> 25), mMinFrames = cvRound(fps / 3),
                               mMaxFrames = cvRound(2 * fps / 3)  (src/cTracking.cpp:86-92)
"""
import os
import re

import numpy as np

from . import CamModel, ExtractorParams

_INT_RE = re.compile(r"^[+-]?\d+$")


def _cv_round(x):
    return int(np.rint(x))   # cvRound: round half to even


def parse_filestorage(text):
    """Flat `key: value` FileStorage YAML -> {key: int | float | str}."""
    out = {}
    for line in text.splitlines():
        if line.startswith("%"):
            continue
        line = line.split("#", 1)[0].rstrip()
        if ":" not in line:
            continue
        k, v = line.split(":", 1)
        k, v = k.strip(), v.strip()
        if not k or not v:
            continue
        if _INT_RE.match(v):
            out[k] = int(v)
        else:
            try:
                out[k] = float(v)
            except ValueError:
                out[k] = v.strip('"')
    return out


def read_filestorage(path):
    with open(path, "r") as f:
        return parse_filestorage(f.read())


def as_int(fs, key):
    """(int)fs[key]: absent -> 0, real -> cvRound, string -> INT_MAX (OpenCV 3.x cvReadInt)."""
    v = fs.get(key)
    if v is None:
        return 0
    if isinstance(v, int):
        return v
    if isinstance(v, float):
        return _cv_round(v)
    return 0x7fffffff


def as_real(fs, key):
    """(double)fs[key]: absent -> 0.0, int -> converted, string -> 1e300 (cvReadReal)."""
    v = fs.get(key)
    if v is None:
        return 0.0
    if isinstance(v, (int, float)):
        return float(v)
    return 1e300


def load_rig(calib_dir):
    """cSystem::LoadMCS: per camera M_c (Cayley 6-vector), CamModel, Iw/Ih, mirror-mask flag."""
    mcs = read_filestorage(os.path.join(calib_dir, "MultiCamSys_Calibration.yaml"))
    n = as_int(mcs, "CameraSystem.nrCams")
    mc = np.zeros((n, 6), np.float64)
    cams, sizes, mirror = [], [], []
    for c in range(n):
        for p in range(1, 7):
            mc[c, p - 1] = as_real(mcs, "CameraSystem.cam%d_%d" % (c + 1, p))
        fs = read_filestorage(os.path.join(calib_dir, "InteriorOrientationFisheye%d.yaml" % c))
        nrpol, nrinvpol = as_int(fs, "Camera.nrpol"), as_int(fs, "Camera.nrinvpol")
        poly = np.zeros(5)            # cv::Mat::zeros(5, 1): more than 5 coefficients overflow
        for i in range(nrpol):        # in the reference (Mat::at out of range); rejected here
            if i >= 5:
                raise ValueError("Camera.nrpol > 5 overflows the reference's 5x1 polynomial")
            poly[i] = as_real(fs, "Camera.a%d" % i)
        invpoly = np.zeros(12)
        for i in range(nrinvpol):
            if i >= 12:
                raise ValueError("Camera.nrinvpol > 12 overflows the reference's 12x1 polynomial")
            invpoly[i] = as_real(fs, "Camera.pol%d" % i)
        cam = {"c": as_real(fs, "Camera.c"), "d": as_real(fs, "Camera.d"),
               "e": as_real(fs, "Camera.e"), "u0": as_real(fs, "Camera.u0"),
               "v0": as_real(fs, "Camera.v0"), "a": poly.tolist(), "pol": invpoly.tolist(),
               "Iw": as_int(fs, "Camera.Iw"), "Ih": as_int(fs, "Camera.Ih")}
        cams.append(cam)
        sizes.append((cam["Iw"], cam["Ih"]))
        mirror.append(as_int(fs, "Camera.mirrorMask") == 1)
    return {"n_cams": n, "mc": mc, "cams": cams, "cam_models": [CamModel.from_dict(c) for c in cams],
            "sizes": sizes, "mirror_mask": mirror}


def extractor_params(settings):
    """cTracking ctor (src/cTracking.cpp:107-158) -> (tracking, initialisation) ExtractorParams."""
    fs = settings
    n = as_int(fs, "extractor.nFeatures")
    scale = float(np.float32(as_real(fs, "extractor.scaleFactor")))   # float fScaleFactor
    common = dict(scale_factor=scale, nlevels=as_int(fs, "extractor.nLevels"), edge_threshold=25,
                  first_level=0, score_type=as_int(fs, "extractor.nScoreType"), patch_size=32,
                  use_agast=as_int(fs, "extractor.useAgast"),
                  fast_agast_type=as_int(fs, "extractor.fastAgastType"),
                  do_dbrief=int(bool(as_int(fs, "extractor.usemdBRIEF"))),
                  learn_masks=int(bool(as_int(fs, "extractor.masks"))),
                  desc_size=as_int(fs, "extractor.descSize"))
    if common["score_type"] not in (0, 1):
        raise ValueError("extractor.nScoreType must be 0 or 1 (assert, src/cTracking.cpp:114)")
    if common["desc_size"] not in (16, 32, 64):
        raise ValueError("extractor.descSize must be 16, 32 or 64 (assert, src/cTracking.cpp:133)")
    track = ExtractorParams(nfeatures=n, fast_threshold=as_int(fs, "extractor.fastTh"), **common)
    init = ExtractorParams(nfeatures=2 * n, fast_threshold=5, **common)
    return track, init


def tracking_frames(settings):
    """fps (0 -> 25), mMinFrames, mMaxFrames (src/cTracking.cpp:86-92)."""
    fps = as_real(settings, "Camera.fps")
    if fps == 0:
        fps = 25.0
    return fps, _cv_round(fps / 3), _cv_round(2 * fps / 3)


def load_settings(path):
    return read_filestorage(path)


def mirror_mask_layout(width, height, levels=4):
    """Level sizes/offsets of the packed mirror-mask pyramid (include/mcs_cammodel.h)."""
    from . import _check, lib
    w = np.zeros(levels, np.int32)
    h = np.zeros(levels, np.int32)
    off = np.zeros(levels, np.int64)
    tot = np.zeros(1, np.int64)
    _check(lib().mcs_mirror_mask_layout(int(width), int(height), int(levels),
                                        w.ctypes.data, h.ctypes.data, off.ctypes.data,
                                        tot.ctypes.data))
    return w, h, off, int(tot[0])


def create_mirror_masks(cam, width, height, levels=4, device=0):
    """CreateMirrorMask (src/cam_model_omni.cpp:183-222) on the GPU: list of torch uint8 masks
    (255 inside the mirror circle), one per level, views into one packed device buffer."""
    import torch
    from . import _check, lib
    w, h, off, total = mirror_mask_layout(width, height, levels)
    buf = torch.empty(total, dtype=torch.uint8, device="cuda:%d" % device)
    stream = torch.cuda.current_stream(buf.device).cuda_stream
    _check(lib().mcs_create_mirror_mask_device(float(cam["u0"]), float(cam["v0"]), int(width),
                                               int(height), int(levels), buf.data_ptr(), stream))
    return [buf[int(off[l]):int(off[l]) + int(w[l]) * int(h[l])].view(int(h[l]), int(w[l]))
            for l in range(levels)]


def rig_mirror_masks(rig, device=0):
    """cSystem::LoadMCS mask choice (src/cSystem.cpp:164-172): 4-level mirror masks when
    Camera.mirrorMask == 1, else one all-ones Iw x Ih mask."""
    import torch
    out = []
    for cam, (iw, ih), flag in zip(rig["cams"], rig["sizes"], rig["mirror_mask"]):
        if flag:
            out.append(create_mirror_masks(cam, iw, ih, 4, device))
        else:
            out.append([torch.ones((ih, iw), dtype=torch.uint8, device="cuda:%d" % device)])
    return out


def is_point_in_mirror_mask(mask, u, v):
    """isPointInMirrorMask (src/cam_model_omni.cpp:165-180) on one level's host mask."""
    from . import lib
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    return bool(lib().mcs_is_point_in_mirror_mask(m.ctypes.data, m.shape[1], m.shape[0],
                                                  float(u), float(v)))
