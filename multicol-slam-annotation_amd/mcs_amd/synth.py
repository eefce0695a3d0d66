"""Deterministic synthetic fisheye frames and masks (no dataset is available offline).

Frames are rendered by casting each pixel's ray through the Scaramuzza omni model of the
Lafida rig (ImgToWorld, reference src/cam_model_omni.cpp:49-67) into a procedural
panorama (random rectangles + multi-octave noise + checker patches), then adding
Gaussian sensor noise (sigma = 2 DN).  Pixels outside the mirror mask are black.  The
mirror mask follows CreateMirrorMask level 0 (src/cam_model_omni.cpp:183-222): a circle
centred at (row = v0, col = u0) of radius v0 + 22 (float arithmetic, u0/v0 names swapped
as in the reference).

Calibration values are the Lafida fixtures (Examples/Lafida/InteriorOrientationFisheye*.yaml,
MultiCamSys_Calibration.yaml) -- numbers only.
"""
import numpy as np

# Examples/Lafida/InteriorOrientationFisheye{0,1,2}.yaml
LAFIDA_CAMS = [
    dict(Iw=754, Ih=480, c=0.999626131079017, d=-0.0034775192597376, e=0.00385134991673147,
         u0=392.219508388648, v0=243.494438476351,
         a=[-209.200757992065, 0.0, 0.00213741670953883, -4.2203617319086e-06, 1.77146086919594e-08],
         pol=[293.667187375663, 149.982043337335, -10.448650568161, 28.2295300683376,
              7.13365723186292, 0.056303218962532, 10.4144677485333, 0.166354960773665,
              -5.86858687381081, 1.18165998645705, 3.1108311354746, 0.810799620714366]),
    dict(Iw=754, Ih=480, c=1.00025900216253, d=-0.0123492665428806, e=0.012594227848688,
         u0=378.722262294544, v0=253.62515782861,
         a=[-209.071570423477, 0.0, 0.00216428966944475, -4.82076123755912e-06, 1.91902225328321e-08],
         pol=[294.569975726124, 148.608451179358, -12.8584962393538, 28.8889327437629,
              6.33883105861485, -0.89043629163529, 12.3786448516946, 0.165754338732521,
              -7.71927140996498, 0.995360127219927, 3.74959014924028, 1.01240838118284]),
    dict(Iw=754, Ih=480, c=0.99992772614797, d=0.0334716840387143, e=-0.0332451389561491,
         u0=372.796912405235, v0=225.645071214684,
         a=[-208.409533164304, 0.0, 0.00225243935068085, -5.55430532694086e-06, 2.07875001352451e-08],
         pol=[293.775776115273, 147.35852428463, -14.3964307215767, 29.078338589251,
              6.03461468718202, -2.07410652721192, 13.4359111214281, 0.984397095348803,
              -8.64924421339311, 0.491570292475276, 3.92296807229949, 1.10563269391099]),
]

# Examples/Lafida/MultiCamSys_Calibration.yaml: M_c of each camera as Cayley (r1,r2,r3,t1,t2,t3)
LAFIDA_MC = [
    [-0.0238361786473007, -2.05998171167958, 0.695126790868671, -0.140202124607334, 0.0219677971160655, -0.0226322662838432],
    [-0.0103943566650926, 1.12505249943085, -0.402901183146028, 0.108753418890423, 0.0636197216520153, 0.0657911760105832],
    [0.0, 0.0, 0.0, -0.00157612288268783, 0.103615531247527, 0.201416323496156],
]


def load_lafida_cams(ref_dir="/root/reference/Examples/Lafida"):
    """Parse all three Lafida calibrations (when the reference tree is present)."""
    import os
    cams = []
    for c in range(3):
        p = os.path.join(ref_dir, "InteriorOrientationFisheye%d.yaml" % c)
        if not os.path.exists(p):
            return LAFIDA_CAMS
        kv = {}
        for line in open(p):
            line = line.split("#")[0].strip()
            if ":" in line and not line.startswith("%"):
                k, v = line.split(":", 1)
                try:
                    kv[k.strip()] = float(v)
                except ValueError:
                    pass
        cams.append(dict(Iw=int(kv["Camera.Iw"]), Ih=int(kv["Camera.Ih"]), c=kv["Camera.c"],
                         d=kv["Camera.d"], e=kv["Camera.e"], u0=kv["Camera.u0"],
                         v0=kv["Camera.v0"],
                         a=[kv.get("Camera.a%d" % i, 0.0) for i in range(5)],
                         pol=[kv.get("Camera.pol%d" % i, 0.0) for i in range(12)]))
    return cams


def scaled_cam(cam, width, height):
    """Lafida polynomials scaled to a width x height sensor, centred principal point
    (config D: 1024x1024)."""
    s = width / float(cam["Iw"])
    out = dict(cam)
    out.update(Iw=width, Ih=height, u0=width / 2.0, v0=height / 2.0)
    # forward poly f(rho): rho scales by s, z scales by s
    out["a"] = [a * s ** (1 - i) for i, a in enumerate(cam["a"])]
    out["pol"] = [p * s for p in cam["pol"]]
    return out


def mirror_mask(cam):
    """CreateMirrorMask level 0 (src/cam_model_omni.cpp:183-222)."""
    w, h = int(cam["Iw"]), int(cam["Ih"])
    u0 = np.float32(cam["v0"])  # names swapped in the reference (:189-190)
    v0 = np.float32(cam["u0"])
    i = np.arange(h, dtype=np.float64)[:, None]
    j = np.arange(w, dtype=np.float64)[None, :]
    di = ((i - np.float64(u0)) ** 2).astype(np.float32)
    dj = ((j - np.float64(v0)) ** 2).astype(np.float32)
    ans = np.sqrt((di + dj).astype(np.float32)).astype(np.float32)
    return np.where(ans < np.float32(u0 + np.float32(22.0)), 255, 0).astype(np.uint8)


def img_to_world(cam, u, v):
    """ImgToWorld (src/cam_model_omni.cpp:49-67), vectorised."""
    inv_aff = cam["c"] - cam["d"] * cam["e"]
    ut = u - cam["u0"]
    vt = v - cam["v0"]
    x = (ut - cam["d"] * vt) / inv_aff
    y = (-cam["e"] * ut + cam["c"] * vt) / inv_aff
    r = np.sqrt(x * x + y * y)
    z = np.zeros_like(r)
    for a in reversed(cam["a"]):
        z = z * r + a
    z = -z
    n = np.sqrt(x * x + y * y + z * z)
    return x / n, y / n, z / n


def _panorama(rng, W=2048, H=1024):
    img = np.zeros((H, W), np.float32)
    # multi-octave value noise
    for octave, amp in ((8, 60.0), (32, 30.0), (128, 14.0)):
        g = rng.random((octave // 2 + 1, octave + 1)).astype(np.float32)
        yi = np.linspace(0, g.shape[0] - 1, H, dtype=np.float32)
        xi = np.linspace(0, g.shape[1] - 1, W, dtype=np.float32)
        y0 = np.floor(yi).astype(int).clip(0, g.shape[0] - 2)
        x0 = np.floor(xi).astype(int).clip(0, g.shape[1] - 2)
        fy = (yi - y0)[:, None]
        fx = (xi - x0)[None, :]
        a = g[y0][:, x0]
        b = g[y0][:, x0 + 1]
        c = g[y0 + 1][:, x0]
        d = g[y0 + 1][:, x0 + 1]
        img += amp * ((a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy)
    # random rectangles (sharp corners -> FAST corners)
    for _ in range(900):
        w = int(rng.integers(6, 90))
        h = int(rng.integers(6, 70))
        x = int(rng.integers(0, W - w))
        y = int(rng.integers(0, H - h))
        img[y:y + h, x:x + w] = img[y:y + h, x:x + w] * 0.3 + float(rng.uniform(0, 255)) * 0.7
    # checker patches
    for _ in range(40):
        s = int(rng.integers(4, 14))
        n = int(rng.integers(3, 9))
        x = int(rng.integers(0, W - s * n))
        y = int(rng.integers(0, H - s * n))
        lo, hi = sorted(rng.uniform(0, 255, 2))
        yy, xx = np.mgrid[0:s * n, 0:s * n]
        img[y:y + s * n, x:x + s * n] = np.where(((yy // s) + (xx // s)) % 2 == 0, lo, hi)
    return img


_PANO_CACHE = {}


def fisheye_frame(width=754, height=480, seed=0, cam_index=0, yaw=0.0, cam=None, noise=2.0,
                  noise_seed=None):
    """Render one synthetic 8-bit fisheye frame and its mirror mask."""
    cams = LAFIDA_CAMS
    if cam is None:
        cam = cams[cam_index % len(cams)]
        if (width, height) != (cam["Iw"], cam["Ih"]):
            cam = scaled_cam(cam, width, height)
    key = seed % 7
    if key not in _PANO_CACHE:
        _PANO_CACHE[key] = _panorama(np.random.default_rng(1000 + key))
    pano = _PANO_CACHE[key]
    rng = np.random.default_rng(seed)
    yaw = yaw + float(rng.uniform(0, 2 * np.pi))
    pitch = float(rng.uniform(-0.3, 0.3))
    v, u = np.mgrid[0:height, 0:width].astype(np.float64)
    x, y, z = img_to_world(cam, u, v)
    # rotate: pitch about x, then yaw about the (camera) optical axis
    cy, sy = np.cos(pitch), np.sin(pitch)
    y, z = cy * y - sy * z, sy * y + cy * z
    az = np.arctan2(y, x) + yaw
    el = np.arctan2(-z, np.sqrt(x * x + y * y))
    H, W = pano.shape
    px = ((az / (2 * np.pi)) % 1.0) * (W - 1)
    py = np.clip((el / np.pi + 0.5), 0, 1) * (H - 1)
    x0 = np.floor(px).astype(int)
    y0 = np.floor(py).astype(int)
    x1 = np.minimum(x0 + 1, W - 1)
    y1 = np.minimum(y0 + 1, H - 1)
    fx = px - x0
    fy = py - y0
    val = (pano[y0, x0] * (1 - fx) + pano[y0, x1] * fx) * (1 - fy) + \
          (pano[y1, x0] * (1 - fx) + pano[y1, x1] * fx) * fy
    nrng = rng if noise_seed is None else np.random.default_rng(noise_seed)
    val = val + nrng.normal(0, noise, val.shape)
    img = np.clip(np.rint(val), 0, 255).astype(np.uint8)
    mask = mirror_mask(cam)
    img[mask == 0] = 0
    return img, mask


def rig_sequence(n_multiframes, width=754, height=480, ncams=3, seed=0, yaw_step=0.015):
    """A moving multi-camera rig: frame (t, c) rotates camera c's view by t*yaw_step.
    Returns images [n_multiframes*ncams, H, W] (t-major, camera-minor, like the
    cMultiFrame camera concatenation) and masks [ncams, H, W]."""
    imgs = np.zeros((n_multiframes * ncams, height, width), np.uint8)
    masks = np.zeros((ncams, height, width), np.uint8)
    for t in range(n_multiframes):
        for c in range(ncams):
            img, m = fisheye_frame(width, height, seed=seed * 100 + c, cam_index=c,
                                   yaw=t * yaw_step, noise_seed=seed * 100000 + t * 16 + c)
            imgs[t * ncams + c] = img
            masks[c] = m
    return imgs, masks


def config_b_batch(n_multiframes=171, n_unique=12, rank=0, width=754, height=480, ncams=3):
    """The headline workload's input (bench.py config B), built the same way for the bench and
    for its parity test: `n_unique` rendered multi-frames of the moving Lafida rig, repeated to
    `n_multiframes` (t-major, camera-minor camera-frames), the per-camera mirror masks, the
    camera index of every frame, and the match pairs (camera c of multi-frame t against camera
    c of t+1, SearchForTriangulationRaw's same-camera rule, src/cORBmatcher.cpp:1040-1041).
    Returns (unique_imgs, imgs, masks, mask_index, pairs)."""
    U = min(n_unique, n_multiframes)
    uimgs, masks = rig_sequence(U, width, height, ncams, seed=1 + rank)
    idx = np.arange(n_multiframes) % U
    imgs = uimgs.reshape(U, ncams, height, width)[idx].reshape(n_multiframes * ncams, height, width)
    midx = np.tile(np.arange(ncams, dtype=np.int32), n_multiframes)
    pairs = np.array([[t * ncams + c, (t + 1) * ncams + c]
                      for t in range(n_multiframes - 1) for c in range(ncams)], np.int32)
    return uimgs, imgs, masks, midx, pairs


def random_frame(width, height, seed):
    """Unstructured uniform-noise frame (edge-case tests: many weak corners)."""
    return np.random.default_rng(seed).integers(0, 256, (height, width), dtype=np.uint8)
