"""cMultiFrame construction on the device, and the Lafida image-sequence ingest.

Reference:
  * cMultiFrame::cMultiFrame src/cMultiFrame.cpp:92-216 -- per camera: extraction inside the
    level-0 mirror mask (`(*extractor[c])(images[c], camModel.GetMirrorMask(0), ...)`, :138),
    bearing rays by ImgToWorld (:143-152), grid bounds mnMinX = 0 / mnMaxX = width (:131-134);
    then the camera-order concatenation with keypoint_to_cam / cont_idx_to_local_cam_idx and
    PosInGrid (:166-184), and the scale tables (:193-206).
  * LoadImagesAndTimestamps Examples/Lafida/mult_col_slam_lafida.cpp:167-199 and the
    grayscale imread of the main loop (:109-118).

MultiFrameBuilder is the batched drop-in: n_mf multi-frames of C cameras per call, every stage
a HIP kernel (mcs_extract_batch_device_ex, mcs_keypoint_rays_device,
mcs_multiframe_concat_device), all buffers resident in HBM.  No CPU fallback: without the
HIP library or a device the constructor raises McsError.
"""
import ctypes
import os

import numpy as np

from . import KEYPOINT_DTYPE, CamModel, Extractor, _check, lib

FRAME_GRID_COLS = 64
FRAME_GRID_ROWS = 48


# ---------------------------------------------------------------------------------------------
# Lafida sequence ingest (host side of the example driver)
# ---------------------------------------------------------------------------------------------
def load_images_and_timestamps(path2imgs, start_frame, end_frame):
    """LoadImagesAndTimestamps (:167-199): read `images_and_timestamps.txt`, keep lines whose
    1-based number cnt satisfies start_frame <= cnt < end_frame, each `timestamp img1 img2
    img3`; stop at the first kept line that does not parse.  A missing file yields empty lists
    (the reference's ifstream simply reads nothing).  -> ([3][n] paths, [n] timestamps)."""
    names = [[], [], []]
    stamps = []
    path = os.path.join(path2imgs, "images_and_timestamps.txt")
    if not os.path.isfile(path):
        return names, stamps
    with open(path, "r", encoding="latin-1") as f:
        for cnt, line in enumerate(f, start=1):
            if not (start_frame <= cnt < end_frame):
                continue
            tok = line.split()
            try:
                ts = float(tok[0])
                p1, p2, p3 = tok[1], tok[2], tok[3]
            except (IndexError, ValueError):
                break
            stamps.append(ts)
            for c, p in enumerate((p1, p2, p3)):
                names[c].append(path2imgs + "/" + p)
    return names, stamps


def imread_grayscale(path):
    """cv::imread(path, CV_LOAD_IMAGE_GRAYSCALE) -> uint8 [H, W], or None if unreadable (the
    reference then reports "Failed to load image" and stops).  8-bit grayscale files decode
    exactly; colour files are converted with OpenCV's fixed-point BGR2GRAY weights
    ((4899 R + 9617 G + 1868 B + 8192) >> 14) and 16-bit files by >> 8 -- codec-specific
    OpenCV conversions are not reproduced (parity unpinned for non-grayscale inputs)."""
    try:
        from PIL import Image
    except ImportError as e:  # pragma: no cover - PIL ships with this image
        raise RuntimeError("PIL is required to decode images") from e
    try:
        im = Image.open(path)
        im.load()
    except (OSError, ValueError):
        return None
    if im.mode == "L":
        return np.asarray(im, dtype=np.uint8).copy()
    if im.mode in ("I;16", "I;16B", "I;16L", "I"):
        a = np.asarray(im).astype(np.int64)
        return np.clip(a >> 8, 0, 255).astype(np.uint8)
    if im.mode == "1":
        return np.asarray(im.convert("L"), dtype=np.uint8).copy()
    rgb = np.asarray(im.convert("RGB"), dtype=np.int64)
    y = (rgb[..., 0] * 4899 + rgb[..., 1] * 9617 + rgb[..., 2] * 1868 + 8192) >> 14
    return y.astype(np.uint8)


def load_multiframe_images(names, index):
    """The C images of multi-frame `index` (main loop :111-118) -> list of uint8 arrays;
    raises FileNotFoundError naming the first image that fails to load."""
    out = []
    for c in range(len(names)):
        img = imread_grayscale(names[c][index])
        if img is None:
            raise FileNotFoundError("Failed to load image at: " + names[c][index])
        out.append(img)
    return out


# ---------------------------------------------------------------------------------------------
# device cMultiFrame
# ---------------------------------------------------------------------------------------------
def scale_tables(nlevels, scale_factor):
    """mvScaleFactors / mvLevelSigma2 / mvInvLevelSigma2 (:193-206), double recursion on the
    float mfScaleFactor."""
    sf = np.ones(nlevels)
    for i in range(1, nlevels):
        sf[i] = sf[i - 1] * float(np.float32(scale_factor))
    s2 = sf * sf
    return sf, s2, 1.0 / s2


class MultiFrameBuilder:
    """Builds cMultiFrame contents for batches of multi-frames on one GPU.

    rig: mcs_amd.lafida.load_rig(...) (cams, sizes, mirror-mask flags).  params:
    ExtractorParams (lafida.extractor_params).  Images go in as a device uint8 tensor
    [n_mf, C, H, W]; every output stays on the device."""

    def __init__(self, rig, params, max_multiframes=1, device=0, stream=None):
        import torch
        from .lafida import rig_mirror_masks
        self.rig = rig
        self.C = int(rig["n_cams"])
        sizes = set(tuple(s) for s in rig["sizes"])
        if len(sizes) != 1:
            raise ValueError("all cameras of the rig must share one image size")
        self.W, self.H = sizes.pop()
        self.dev = torch.device("cuda", device)
        self.stream = stream
        self.max_mf = int(max_multiframes)
        self.ex = Extractor(params, self.W, self.H, max_frames=self.max_mf * self.C, device=device)
        self.cap = self.ex.capacity
        self.desc_size = int(params.desc_size)
        self.nlevels = int(params.nlevels)
        self.scale_factor = float(params.scale_factor)
        models = [m if isinstance(m, CamModel) else CamModel.from_dict(m) for m in rig["cams"]]
        self.ex.set_cam_models(models)
        self.d_cams = torch.frombuffer(bytearray(b"".join(bytes(m) for m in models)),
                                       dtype=torch.uint8).to(self.dev)
        # GetMirrorMask(0) of every camera: the circle mask, or all ones (mirrorMask == 0)
        lv0 = [m[0] for m in rig_mirror_masks(rig, device)]
        self.d_masks = torch.stack([m.contiguous() for m in lv0]).to(self.dev)
        self.ex.set_masks_device(self.d_masks.data_ptr(), self.C, self._st())
        gp = np.array([[0.0, 0.0, FRAME_GRID_COLS / float(self.W), FRAME_GRID_ROWS / float(self.H)]] *
                      self.C)
        self.grid_params = gp
        self.d_gp = torch.from_numpy(gp).to(self.dev)
        self.scale_factors, self.level_sigma2, self.inv_level_sigma2 = scale_tables(
            self.nlevels, self.scale_factor)

    def _st(self):
        import torch
        s = self.stream if self.stream is not None else torch.cuda.current_stream(self.dev)
        return s.cuda_stream

    def build(self, d_images):
        """d_images: uint8 device tensor [n_mf, C, H, W].  Returns dict of device tensors:
        per camera-frame  counts [n_mf, C], kps [n_mf, C, cap, 7] (int32 words of mcs_keypoint),
                          rays [n_mf, C, cap, 3], desc / desc_masks [n_mf, C, cap, B];
        per multi-frame   keys [n_mf, C*cap, 7], keys_rays [n_mf, C*cap, 3], descs, desc_masks
                          (camera order), kp_to_cam, cont_to_local, grid_pos (x | y << 8 or -1),
                          total [n_mf]."""
        import torch
        n_mf = int(d_images.shape[0])
        if tuple(d_images.shape[1:]) != (self.C, self.H, self.W) or d_images.dtype != torch.uint8:
            raise ValueError("d_images must be uint8 [n_mf, %d, %d, %d]" % (self.C, self.H, self.W))
        if n_mf > self.max_mf:
            raise ValueError("batch of %d multi-frames exceeds max_multiframes=%d" % (n_mf, self.max_mf))
        d_images = d_images.contiguous()
        F, C, cap, B = n_mf * self.C, self.C, self.cap, self.desc_size
        st = self._st()
        dev = self.dev
        cidx = torch.arange(C, dtype=torch.int32, device=dev).repeat(n_mf)
        kps = torch.zeros((F, cap * 7), dtype=torch.int32, device=dev)
        cnt = torch.zeros(F, dtype=torch.int32, device=dev)
        desc = torch.zeros((F, cap, B), dtype=torch.uint8, device=dev)
        dmask = torch.zeros((F, cap, B), dtype=torch.uint8, device=dev)
        self.ex.extract_batch_device_ex(d_images.data_ptr(), F, cidx.data_ptr(), kps.data_ptr(),
                                        cnt.data_ptr(), desc.data_ptr(), dmask.data_ptr(), st)
        rays = torch.zeros((F, cap, 3), dtype=torch.float64, device=dev)
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _check(lib().mcs_keypoint_rays_device(P(kps), P(cnt), F, cap, P(cidx), P(self.d_cams),
                                              P(rays), ctypes.c_void_p(st)))
        keys = torch.zeros((n_mf, C * cap * 7), dtype=torch.int32, device=dev)
        keys_rays = torch.zeros((n_mf, C * cap, 3), dtype=torch.float64, device=dev)
        descs = torch.zeros((n_mf, C * cap, B), dtype=torch.uint8, device=dev)
        k2c = torch.zeros((n_mf, C * cap), dtype=torch.int32, device=dev)
        k2l = torch.zeros_like(k2c)
        grid = torch.zeros_like(k2c)
        tot = torch.zeros(n_mf, dtype=torch.int32, device=dev)
        _check(lib().mcs_multiframe_concat_device(P(cnt), n_mf, C, cap, P(kps), P(rays), P(desc), B,
                                                  P(self.d_gp), P(keys), P(keys_rays), P(descs),
                                                  P(k2c), P(k2l), P(grid), P(tot), ctypes.c_void_p(st)))
        # descriptor masks in camera order: the same concatenation applied to the mask rows
        descm = torch.zeros((n_mf, C * cap, B), dtype=torch.uint8, device=dev)
        _check(lib().mcs_multiframe_concat_device(P(cnt), n_mf, C, cap, P(kps), None, P(dmask), B,
                                                  P(self.d_gp), P(keys), None, P(descm), P(k2c),
                                                  P(k2l), None, P(tot), ctypes.c_void_p(st)))
        return {"counts": cnt.view(n_mf, C), "kps": kps.view(n_mf, C, cap, 7),
                "rays": rays.view(n_mf, C, cap, 3), "desc": desc.view(n_mf, C, cap, B),
                "desc_masks": dmask.view(n_mf, C, cap, B), "keys": keys.view(n_mf, C * cap, 7),
                "keys_rays": keys_rays, "descs": descs, "descs_masks": descm, "kp_to_cam": k2c,
                "cont_to_local": k2l, "grid_pos": grid, "total": tot}

    @staticmethod
    def host_view(out, m):
        """Multi-frame m of a build() result as numpy arrays trimmed to totalN."""
        N = int(out["total"][m])
        keys = out["keys"][m].cpu().numpy().reshape(-1).view(KEYPOINT_DTYPE)[:N]
        return {"mvKeys": keys, "mvKeysRays": out["keys_rays"][m, :N].cpu().numpy(),
                "descriptors": out["descs"][m, :N].cpu().numpy(),
                "descriptor_masks": out["descs_masks"][m, :N].cpu().numpy(),
                "keypoint_to_cam": out["kp_to_cam"][m, :N].cpu().numpy(),
                "cont_idx_to_local_cam_idx": out["cont_to_local"][m, :N].cpu().numpy(),
                "grid_pos": out["grid_pos"][m, :N].cpu().numpy(),
                "N": out["counts"][m].cpu().numpy()}
