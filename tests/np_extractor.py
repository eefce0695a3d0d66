"""Independent numpy / Python restatements of the extractor's OpenCV-defined pieces.

TEST INFRASTRUCTURE ONLY.  These are written from the spec and the
reference's own loops, vectorised over whole images, not from oracle/extractor_oracle.cpp, so
that a mistake in one restatement shows up as a disagreement with the other
(tests/test_oracle_crosscheck.py):

  resize_linear   A.1  INTER_LINEAR 8U fixed point, SSE2-split or scalar vertical pass
                       (src/mdBRIEFextractorOct.cpp:1179)
  resize_nearest  A.3  legacy INTER_NEAREST mask pyramid (:1182)
  fast_level      A.4 + A.5  FAST-9/16 + cornerScore<16> + cell-local strict NMS + mask after
                       NMS over the 30 px cell grid (ComputeKeyPointsOctTree :863-949)
  distribute_octree    DistributeOctTree (:569-861) on Python lists, heap-pointer tie-break
                       modelled as node creation order
"""
import math

import numpy as np

COEF = 2048  # INTER_RESIZE_COEF_SCALE (11 bits)


def _linear_taps(sw, dw):
    scale = 1.0 / (dw / sw)
    d = np.arange(dw, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo] = 0
    s[lo] = 0
    hi = s >= sw - 1
    f[hi] = 0
    s[hi] = sw - 1
    a0 = np.rint((np.float32(1) - f).astype(np.float32) * np.float32(COEF)).astype(np.int64)
    a1 = np.rint(f * np.float32(COEF)).astype(np.int64)
    return s, a0, a1


def resize_linear(src, dw, dh, mode=1):
    """mode 1: vertical pass in the SSE2 form on x < 16*floor(w/16) and then 4-wide while
    x < w - 4 (OpenCV 3.1 split), scalar tail; mode 0: scalar everywhere."""
    src = np.asarray(src, np.int64)
    sh, sw = src.shape
    xs, a0, a1 = _linear_taps(sw, dw)
    ys, b0, b1 = _linear_taps(sh, dh)
    x1 = np.minimum(xs + 1, sw - 1)
    H = src[:, xs] * a0 + src[:, x1] * a1          # horizontal pass, int32 range
    S0 = H[ys]
    S1 = H[np.minimum(ys + 1, sh - 1)]
    B0 = b0[:, None]
    B1 = b1[:, None]
    scalar = np.clip((S0 * B0 + S1 * B1 + (1 << 21)) >> 22, 0, 255)
    if mode == 0:
        return scalar.astype(np.uint8)
    sat16 = lambda v: np.clip(v, -32768, 32767)
    p0 = sat16(S0 >> 4)
    p1 = sat16(S1 >> 4)
    m = sat16(((p0 * B0) >> 16) + ((p1 * B1) >> 16))
    simd = np.clip(sat16(m + 2) >> 2, 0, 255)
    nsimd = (dw // 16) * 16
    x = nsimd
    while x < dw - 4:
        x += 4
    out = scalar.copy()
    out[:, :x] = simd[:, :x]
    return out.astype(np.uint8)


def resize_nearest(src, dw, dh):
    src = np.asarray(src)
    sh, sw = src.shape
    fx = 1.0 / (dw / sw)
    fy = 1.0 / (dh / sh)
    xo = np.minimum(np.floor(np.arange(dw) * fx).astype(np.int64), sw - 1)
    yo = np.minimum(np.floor(np.arange(dh) * fy).astype(np.int64), sh - 1)
    return src[yo][:, xo]


# ---- FAST -----------------------------------------------------------------------------------
CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3),
          (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def fast_score_map(img, t):
    """FAST-9/16 corner test and cornerScore<16> at every pixel with a full circle inside the
    image; 0 where not a corner.  t is clamped to [0, 255]."""
    t = int(min(max(t, 0), 255))
    I = np.asarray(img, np.int64)
    h, w = I.shape
    v = I[3:h - 3, 3:w - 3]
    ring = np.stack([I[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in CIRCLE])
    d = v[None] - ring                              # d[k] = v - I[k]
    d = np.concatenate([d, d[:9]])                  # 25 entries, wrapped
    bright = d < -t
    dark = d > t
    corner = np.zeros(v.shape, bool)
    for k in range(16):
        corner |= bright[k:k + 9].all(0) | dark[k:k + 9].all(0)
    a0 = np.full(v.shape, t)
    for k in range(0, 16, 2):
        a = d[k + 1:k + 9].min(0)
        a0 = np.maximum(a0, np.maximum(np.minimum(a, d[k]), np.minimum(a, d[k + 9])))
    b0 = -a0
    for k in range(0, 16, 2):
        b = d[k + 1:k + 9].max(0)
        b0 = np.minimum(b0, np.minimum(np.maximum(b, d[k]), np.maximum(b, d[k + 9])))
    score = np.zeros((h, w), np.int64)
    score[3:h - 3, 3:w - 3] = np.where(corner, -b0 - 1, 0)
    return score


def _roi_fast(img, mask, x0, y0, x1, y1, t):
    """FastFeatureDetector::detect on the ROI [x0,x1) x [y0,y1) with the mask ROI: detection in
    [3, dim-3), strict NMS against neighbours inside the ROI's detection window (others 0),
    then runByPixelsMask.  -> list of (x_roi, y_roi, score) in row-major order."""
    roi = img[y0:y1, x0:x1]
    h, w = roi.shape
    if h < 7 or w < 7:
        return []
    s = fast_score_map(roi, t)                      # zero outside [3, dim-3)
    c = s[3:h - 3, 3:w - 3]
    keep = c > 0
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx or dy:
                keep &= c > s[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx]
    ys, xs = np.nonzero(keep)                       # row-major emission
    out = []
    for y, x in zip(ys + 3, xs + 3):
        if mask is not None and mask[y0 + int(y + 0.5), x0 + int(x + 0.5)] == 0:
            continue
        out.append((int(x), int(y), int(s[y, x])))
    return out


def fast_level(img, mask, t, edge=25):
    """ComputeKeyPointsOctTree cell loop (:863-949) for one level -> int array [n, 3] of
    (x, y, score) relative to minBorder, in the reference's push order."""
    H, W = img.shape
    minB = edge - 3
    maxBX, maxBY = W - edge + 3, H - edge + 3
    width, height = float(maxBX - minB), float(maxBY - minB)
    ncols, nrows = int(width / 30.0), int(height / 30.0)
    wc, hc = int(math.ceil(width / ncols)), int(math.ceil(height / nrows))
    out = []
    for i in range(nrows):
        iniY = minB + i * hc
        maxY = iniY + hc + 6
        if iniY >= maxBY - 3:
            continue
        maxY = min(maxY, maxBY)
        for j in range(ncols):
            iniX = minB + j * wc
            maxX = iniX + wc + 6
            if iniX >= maxBX - 6:
                continue
            maxX = min(maxX, maxBX)
            for x, y, sc in _roi_fast(img, mask, iniX, iniY, maxX, maxY, t):
                out.append((x + j * wc, y + i * hc, sc))
    return np.array(out, np.int64).reshape(-1, 3)


# ---- DistributeOctTree ----------------------------------------------------------------------
class _Node:
    __slots__ = ("UL", "UR", "BL", "BR", "keys", "no_more", "uid")

    def __init__(self, uid):
        self.uid = uid
        self.keys = []
        self.no_more = False


def distribute_octree(cands, minX, maxX, minY, maxY, N):
    """cands: [n, 3] (x, y, response) relative to minBorder, in push order.  Returns the
    indices of the retained keypoints in output order."""
    uid = [0]

    def new():
        uid[0] += 1
        return _Node(uid[0])

    def divide(nd):
        halfX = int(math.ceil((nd.UR[0] - nd.UL[0]) / 2.0))
        halfY = int(math.ceil((nd.BR[1] - nd.UL[1]) / 2.0))
        n1, n2, n3, n4 = new(), new(), new(), new()
        n1.UL = nd.UL
        n1.UR = (nd.UL[0] + halfX, nd.UL[1])
        n1.BL = (nd.UL[0], nd.UL[1] + halfY)
        n1.BR = (nd.UL[0] + halfX, nd.UL[1] + halfY)
        n2.UL, n2.UR, n2.BL, n2.BR = n1.UR, nd.UR, n1.BR, (nd.UR[0], nd.UL[1] + halfY)
        n3.UL, n3.UR, n3.BL, n3.BR = n1.BL, n1.BR, nd.BL, (n1.BR[0], nd.BL[1])
        n4.UL, n4.UR, n4.BL, n4.BR = n3.UR, n2.BR, n3.BR, nd.BR
        for k in nd.keys:
            x, y = xs[k], ys[k]
            if x < n1.UR[0]:
                (n1 if y < n1.BR[1] else n3).keys.append(k)
            elif y < n1.BR[1]:
                n2.keys.append(k)
            else:
                n4.keys.append(k)
        for c in (n1, n2, n3, n4):
            if len(c.keys) == 1:
                c.no_more = True
        return n1, n2, n3, n4

    cands = np.asarray(cands)
    xs = [float(np.float32(v)) for v in cands[:, 0]]
    ys = [float(np.float32(v)) for v in cands[:, 1]]
    resp = [float(np.float32(v)) for v in cands[:, 2]]
    nIni = int(np.rint((maxX - minX) / (maxY - minY)))
    hX = (maxX - minX) / nIni
    nodes = []
    ini = []
    for i in range(nIni):
        nd = new()
        nd.UL = (int(hX * i), 0)
        nd.UR = (int(hX * (i + 1)), 0)
        nd.BL = (nd.UL[0], maxY - minY)
        nd.BR = (nd.UR[0], maxY - minY)
        nodes.append(nd)
        ini.append(nd)
    for k in range(len(cands)):
        ini[int(xs[k] / hX)].keys.append(k)
    kept = []
    for nd in nodes:
        if len(nd.keys) == 1:
            nd.no_more = True
            kept.append(nd)
        elif nd.keys:
            kept.append(nd)
    nodes = kept

    def push_children(children, expand):
        """push_front each non-empty child (n1..n4 order); record the >1 ones."""
        n = 0
        for c in children:
            if c.keys:
                nodes.insert(0, c)
                if len(c.keys) > 1:
                    expand.append(c)
                    n += 1
        return n

    finish = False
    expand = []
    while not finish:
        prev = len(nodes)
        expand = []
        n_to_expand = 0
        for nd in list(nodes):
            if nd.no_more:
                continue
            n_to_expand += push_children(divide(nd), expand)
            nodes.remove(nd)
        if len(nodes) >= N or len(nodes) == prev:
            finish = True
        elif len(nodes) + n_to_expand * 3 > N:
            while not finish:
                prev = len(nodes)
                prev_expand = sorted(expand, key=lambda c: (len(c.keys), c.uid))
                expand = []
                for nd in reversed(prev_expand):
                    push_children(divide(nd), expand)
                    nodes.remove(nd)
                    if len(nodes) >= N:
                        break
                if len(nodes) >= N or len(nodes) == prev:
                    finish = True
    out = []
    for nd in nodes:
        best = nd.keys[0]
        for k in nd.keys[1:]:
            if resp[k] > resp[best]:
                best = k
        out.append(best)
    return np.array(out, np.int64)
