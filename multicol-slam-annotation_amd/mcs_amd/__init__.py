"""mcs_amd -- Python host binding of libmcs_amd.so (MI355X-native MultiCol-SLAM front-end
and local bundle adjustment).

The product is the C-ABI library (include/*.h); this module is a thin ctypes mirror of the
reference operator surface used by tests and bench.py:

  Extractor(params, w, h)       ~ mdBRIEFextractorOct(nfeatures, scaleFactor, ...)
                                   (reference include/mdBRIEFextractorOct.h:339-351)
  Extractor.extract(img, mask)  ~ mdBRIEFextractorOct::operator()(image, mask, kps, cam,
                                   desc, descMasks)  (src/mdBRIEFextractorOct.cpp:1244-1337)
  descriptor_distance64(a, b)   ~ DescriptorDistance64 (src/cORBmatcher.cpp:2443-2455)

There is no CPU fallback: if the shared library is missing or no GPU is visible the calls
raise, so a GPU test can never pass on a silent fallback.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MCS_AMD_LIB: an alternative build of the same library (tools/ ablation runs only)
LIB_PATH = os.environ.get("MCS_AMD_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libmcs_amd.so")
INCLUDE_DIR = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include")

MCS_OK = 0
MCS_ERR_ARG = -1
MCS_ERR_CAPACITY = -2
MCS_ERR_HIP = -3
MCS_ERR_UNSUPPORTED = -4
MCS_ERR_NO_DEVICE = -5


class McsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("mcs error %d: %s" % (code, msg))
        self.code = code


class ExtractorParams(ctypes.Structure):
    """Mirror of mcs_extractor_params (include/mcs_extractor.h) with reference defaults."""
    _fields_ = [("nfeatures", ctypes.c_int32), ("scale_factor", ctypes.c_float),
                ("nlevels", ctypes.c_int32), ("edge_threshold", ctypes.c_int32),
                ("first_level", ctypes.c_int32), ("score_type", ctypes.c_int32),
                ("patch_size", ctypes.c_int32), ("fast_threshold", ctypes.c_int32),
                ("use_agast", ctypes.c_int32), ("fast_agast_type", ctypes.c_int32),
                ("do_dbrief", ctypes.c_int32), ("learn_masks", ctypes.c_int32),
                ("desc_size", ctypes.c_int32)]

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, edge_threshold=25,
                 first_level=0, score_type=0, patch_size=32, fast_threshold=20,
                 use_agast=0, fast_agast_type=2, do_dbrief=0, learn_masks=0, desc_size=32):
        super().__init__(nfeatures, scale_factor, nlevels, edge_threshold, first_level,
                         score_type, patch_size, fast_threshold, use_agast, fast_agast_type,
                         do_dbrief, learn_masks, desc_size)


class CamModel(ctypes.Structure):
    """Mirror of mcs_cam_model (include/mcs_extractor.h): cCamModelGeneral_ parameters."""
    _fields_ = [("c", ctypes.c_double), ("d", ctypes.c_double), ("e", ctypes.c_double),
                ("u0", ctypes.c_double), ("v0", ctypes.c_double),
                ("p_deg", ctypes.c_int32), ("invp_deg", ctypes.c_int32),
                ("p", ctypes.c_double * 16), ("invp", ctypes.c_double * 16)]

    @classmethod
    def from_dict(cls, cam):
        """From a Lafida-style calibration dict (c, d, e, u0, v0, a = p, pol = invP)."""
        m = cls()
        m.c, m.d, m.e, m.u0, m.v0 = (float(cam[k]) for k in ("c", "d", "e", "u0", "v0"))
        a, pol = list(cam["a"]), list(cam["pol"])
        m.p_deg, m.invp_deg = len(a), len(pol)
        for i, v in enumerate(a):
            m.p[i] = float(v)
        for i, v in enumerate(pol):
            m.invp[i] = float(v)
        return m


# numpy view of mcs_keypoint / cv::KeyPoint
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64

# name -> (restype, argtypes); every symbol declared in include/*.h must be here
SIGNATURES = {
    "mcs_version": (ctypes.c_char_p, []),
    "mcs_last_error": (ctypes.c_char_p, []),
    "mcs_device_count": (_I32, []),
    "mcs_extractor_default_params": (None, [_P]),
    "mcs_extractor_create": (ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _P]),
    "mcs_extractor_destroy": (None, [_P]),
    "mcs_extractor_capacity": (_I32, [_P]),
    "mcs_extractor_levels": (ctypes.c_int, [_P, _P, _P, _P]),
    "mcs_extract": (ctypes.c_int, [_P, _P, _I32, _P, _I32, _P, _I32, _P, _P, _P]),
    "mcs_extractor_set_masks_device": (ctypes.c_int, [_P, _P, _I32, _P]),
    "mcs_harris_responses_device": (ctypes.c_int, [_P, _P, _I32, _P, _I32, _I32, ctypes.c_float, _P, _P]),
    "mcs_extract_batch_device": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P]),
    "mcs_extractor_read_stage": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _I64, _P]),
    "mcs_extractor_set_cam_models": (ctypes.c_int, [_P, _P, _I32]),
    "mcs_extract_batch_device_ex": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _P]),
    "mcs_extractor_enable_timing": (ctypes.c_int, [_P, _I32]),
    "mcs_extractor_read_timing": (ctypes.c_int, [_P, _P, _P, _I32]),
    # matcher (include/mcs_matcher.h)
    "mcs_descriptor_distance64": (ctypes.c_int, [_P, _P, _I32]),
    "mcs_descriptor_distance64_masked": (ctypes.c_int, [_P, _P, _P, _P, _I32]),
    "mcs_hamming_top2_device": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, _P, _P, _P, _P, _P]),
    "mcs_hamming_dense_device": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, _P, _P]),
    "mcs_hamming_top2_batch_device": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    # bundle adjustment (include/mcs_ba.h)
    "mcs_ba_default_options": (None, [_P]),
    "mcs_ba_create": (ctypes.c_int, [_I32, _P]),
    "mcs_ba_destroy": (None, [_P]),
    "mcs_ba_optimize": (ctypes.c_int, [_P] * 9),
    "mcs_local_ba": (ctypes.c_int, [_P] * 9),
    "mcs_local_ba_ex": (ctypes.c_int, [_P] * 11),
    "mcs_keypoint_rays_device": (ctypes.c_int, [_P, _P, _I32, _I32, _P, _P, _P, _P]),
    "mcs_multiframe_concat_device": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P, _P, _I32, _P,
                                                    _P, _P, _P, _P, _P, _P, _P, _P]),
    "mcs_is_in_frustum_device": (ctypes.c_int, [_P, _P, _P, _I32, _P, _I32, _I32, _P, _P, _P,
                                                _I32, _P, _I32, _P, _P, _P, _P, _P]),
    "mcs_local_ba_select": (ctypes.c_int, [_P, _I32, _P, _I32, _P]),
    "mcs_global_ba_select": (ctypes.c_int, [_P, _P]),
    "mcs_pose_optimization_select": (ctypes.c_int, [_P, _P]),
    "mcs_ba_linearize": (ctypes.c_int, [_P] * 5),
    "mcs_ba_xchg_doubles": (_I64, [_I32]),
    "mcs_ba_optimize_sharded": (ctypes.c_int, [_P] * 10),
    "mcs_global_ba": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P]),
    "mcs_dense_ldlt_solve": (ctypes.c_int, [_I32, _P, _I32, _P, _P, _P]),
    "mcs_dense_ldlt_solve_ex": (ctypes.c_int, [_I32, _P, _I32, _P, _P, _P, _I32]),
    "mcs_ldlt_set_wait_ticks": (ctypes.c_int, [ctypes.c_int64]),
    "mcs_ba_lm_replay": (ctypes.c_int, [_I32, _P, _P, _P, _I32, _P, _P]),
    "mcs_ba_huber_eval": (ctypes.c_int, [_I32, _P, _I32, ctypes.c_double, _P, _P]),
    "mcs_ba_enable_timing": (ctypes.c_int, [_P, _I32]),
    "mcs_ba_read_timing": (ctypes.c_int, [_P, _P, _P, _P, _P, _I32]),
    "mcs_ba_read_host_timing": (ctypes.c_int, [_P, _P, _P, _I32]),
    "mcs_ba_check_structure": (ctypes.c_int, [_P, _P, _P]),
    "mcs_distinctive_descriptors_device": (ctypes.c_int, [_P, _P, _I32, _P, _P, _I32, _P, _P, _P, _P]),
    "mcs_update_normal_depth_device": (ctypes.c_int, [_P, _I32, _P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P]),
    "mcs_pose_optimization": (ctypes.c_int, [_P] * 8),
    "mcs_search_for_triangulation_raw": (ctypes.c_int, [_P, _P, _P, _P, _I32, _P, _P, _P, _P, _I32, _I32, _P, _I32, _I32, ctypes.c_double, _P, _P]),
    "mcs_search_for_triangulation_raw_masked": (ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _I32, _I32, _P, _I32, _I32, ctypes.c_double, _P, _P]),
    "mcs_compute_e_rig": (ctypes.c_int, [_P, _P, _P, _I32, _P]),
    "mcs_ba_point_block_eval": (ctypes.c_int, [_I32, _P, ctypes.c_double, _P, _P, _I32, _P, _P, _P]),
    "mcs_tri_workspace_create": (ctypes.c_int, [_I32, _I32, _I32, _P]),
    "mcs_tri_workspace_destroy": (None, [_P]),
    "mcs_search_for_triangulation_raw_device": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _I32, _I32, _P, _I32, _I32, ctypes.c_double, _P, _P, _P]),
    "mcs_check_dist_epipolar_line": (ctypes.c_int, [_P, _P, _P, ctypes.c_double]),
    "mcs_frame_grid_build": (ctypes.c_int, [_P, _P, _I32, _I32, _P, _P, _P, _P]),
    "mcs_window_search_device": (ctypes.c_int, [_P, _P, _P, _I32, _P, _P, _P, _P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _P]),
    "mcs_window_select": (ctypes.c_int, [_I32, _I32, _P, _P, _P, _P, _I32, _I32, ctypes.c_double, _P, _P, _P]),
    "mcs_window_match": (ctypes.c_int, [_I32, _I32, _P, _I32, _P, _P, _P, _P, _I32, ctypes.c_double, _P, _P, _P]),
    # DBoW2 vocabulary (include/mcs_vocab.h)
    "mcs_vocab_create": (_I32, [_I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _I32, _P, _I32, _P]),
    "mcs_vocab_destroy": (_I32, [_P]),
    "mcs_vocab_info": (_I32, [_P, _P]),
    "mcs_vocab_transform_words_device": (_I32, [_P, _P, _I32, _I32, _P, _P, _P, _P]),
    "mcs_vocab_transform": (_I32, [_P, _P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]),
    # omni camera mirror masks (include/mcs_cammodel.h)
    "mcs_mirror_mask_layout": (_I32, [_I32, _I32, _I32, _P, _P, _P, _P]),
    "mcs_create_mirror_mask_device": (_I32, [ctypes.c_double, ctypes.c_double, _I32, _I32, _I32, _P, _P]),
    "mcs_is_point_in_mirror_mask": (_I32, [_P, _I32, _I32, ctypes.c_double, ctypes.c_double]),
}

_lib = None


def lib():
    """Load libmcs_amd.so and bind every exported C-ABI symbol (raises if missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise McsError(MCS_ERR_NO_DEVICE, "libmcs_amd.so not built (run __graft_entry__.build())")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7)
    # and loads it by file name, so if our library were loaded first the process would end
    # up with two HIP/HSA runtimes and torch could not see the GPU.  Loading torch first
    # makes our NEEDED libamdhip64.so.7 resolve to torch's copy (device pointers and
    # streams are then shared).  Without torch, /opt/rocm's runtime is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if not hasattr(L, name):
            continue  # symbols of modules not yet built are checked by tests
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _check(rc):
    if rc != MCS_OK:
        raise McsError(rc, lib().mcs_last_error().decode(errors="replace"))


def device_count():
    return int(lib().mcs_device_count())


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class Extractor:
    """Host-side mirror of mdBRIEFextractorOct backed by the HIP pipeline."""

    def __init__(self, params, width, height, max_frames=1, device=0):
        self.params = params
        self.width, self.height = int(width), int(height)
        h = ctypes.c_void_p()
        _check(lib().mcs_extractor_create(ctypes.byref(params), self.width, self.height,
                                          int(max_frames), int(device), ctypes.byref(h)))
        self._h = h
        self.capacity = int(lib().mcs_extractor_capacity(h))
        self.desc_size = int(params.desc_size)

    def close(self):
        if getattr(self, "_h", None):
            lib().mcs_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def levels(self):
        n = ctypes.c_int32()
        wh = np.zeros(2 * 12, np.int32)
        nf = np.zeros(12, np.int32)
        _check(lib().mcs_extractor_levels(self._h, ctypes.byref(n), _ptr(wh), _ptr(nf)))
        k = n.value
        return wh[:2 * k].reshape(k, 2), nf[:k]

    def set_cam_models(self, models):
        """Camera models (list of CamModel or calibration dicts) for dBRIEF / mdBRIEF."""
        arr = (CamModel * len(models))(*[m if isinstance(m, CamModel) else CamModel.from_dict(m)
                                         for m in models])
        _check(lib().mcs_extractor_set_cam_models(self._h, arr, len(models)))

    def extract_with_masks(self, image, mask=None):
        """operator() -> (kps, desc, descMasks) (masks all-zero unless learn_masks)."""
        image = np.ascontiguousarray(image, dtype=np.uint8)
        assert image.shape == (self.height, self.width)
        if mask is not None:
            mask = np.ascontiguousarray(mask, dtype=np.uint8)
            assert mask.shape == image.shape
        kps = np.zeros(self.capacity, KEYPOINT_DTYPE)
        desc = np.zeros((self.capacity, self.desc_size), np.uint8)
        dm = np.zeros((self.capacity, self.desc_size), np.uint8)
        n = ctypes.c_int32()
        _check(lib().mcs_extract(self._h, _ptr(image), self.width, _ptr(mask), self.width,
                                 _ptr(kps), self.capacity, ctypes.byref(n), _ptr(desc), _ptr(dm)))
        k = n.value
        return kps[:k].copy(), desc[:k].copy(), dm[:k].copy()

    def extract_batch_device_ex(self, d_images, n_frames, d_cam_index, d_kps, d_counts, d_desc,
                                d_desc_masks, stream=None):
        _check(lib().mcs_extract_batch_device_ex(self._h, d_images, int(n_frames), d_cam_index,
                                                 d_kps, d_counts, d_desc, d_desc_masks, stream))

    def extract(self, image, mask=None):
        """operator()(image, mask, kps, camModel, desc, descMasks) -> (kps, desc)."""
        image = np.ascontiguousarray(image, dtype=np.uint8)
        assert image.shape == (self.height, self.width)
        if mask is not None:
            mask = np.ascontiguousarray(mask, dtype=np.uint8)
            assert mask.shape == image.shape
        kps = np.zeros(self.capacity, KEYPOINT_DTYPE)
        desc = np.zeros((self.capacity, self.desc_size), np.uint8)
        n = ctypes.c_int32()
        _check(lib().mcs_extract(self._h, _ptr(image), self.width, _ptr(mask), self.width,
                                 _ptr(kps), self.capacity, ctypes.byref(n), _ptr(desc), None))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def set_masks_device(self, d_masks_ptr, n_masks, stream=None):
        _check(lib().mcs_extractor_set_masks_device(self._h, d_masks_ptr, int(n_masks), stream))

    def extract_batch_device(self, d_images, n_frames, d_mask_index, d_kps, d_counts, d_desc,
                             stream=None):
        """Device pointers (ints) in, device pointers out; async on `stream`."""
        _check(lib().mcs_extract_batch_device(self._h, d_images, int(n_frames), d_mask_index,
                                              d_kps, d_counts, d_desc, stream))

    STAGES = ("pyramid", "blur0", "fast", "octree", "orient_desc")

    def enable_timing(self, on=True):
        _check(lib().mcs_extractor_enable_timing(self._h, 1 if on else 0))

    def read_timing(self, reset=True):
        """-> (dict stage -> summed device ms, number of recorded batch calls)."""
        ms = np.zeros(len(self.STAGES), np.float32)
        n = ctypes.c_int32()
        _check(lib().mcs_extractor_read_timing(self._h, _ptr(ms), ctypes.byref(n), 1 if reset else 0))
        return dict(zip(self.STAGES, ms.tolist())), n.value

    def read_stage(self, stage, frame, level):
        wh, _ = self.levels()
        w, h = wh[level]
        if stage in (0, 1):
            buf = np.zeros(w * h, np.uint8)
        else:
            buf = np.zeros(3 * (w * h // 4 + 16), np.int32)
        n = ctypes.c_int64()
        _check(lib().mcs_extractor_read_stage(self._h, stage, frame, level, _ptr(buf),
                                              buf.size, ctypes.byref(n)))
        if stage in (0, 1):
            return buf.reshape(h, w)
        return buf[:3 * n.value].reshape(-1, 3)


def descriptor_distance64(a, b, dim=None):
    """DescriptorDistance64 (src/cORBmatcher.cpp:2443-2455) on two descriptor rows."""
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return int(lib().mcs_descriptor_distance64(_ptr(a), _ptr(b), int(dim or a.size)))
