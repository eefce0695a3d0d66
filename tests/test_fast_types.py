"""FAST TYPE_7_12 and TYPE_5_8 (FastFeatureDetector types 1 and 0), selected by the
extractor's fastAgastType (src/mdBRIEFextractorOct.cpp:871-872, 916-917).

The reference delegates to OpenCV 3.x FAST_t<12> / FAST_t<8> + cornerScore<12> / <8>
(fast.cpp, fast_score.cpp).  OpenCV is not in this image, so these two types are
**parity unpinned**: the oracle (oracle/extractor_oracle.cpp fast_small) and the Python
restatement below both follow the published OpenCV algorithm -- notably its quick test,
which uses the pixel pairs (0,8) (2,10) ... (7,15) of the 16-point pattern on the wrapped
offset table (pixel[k] = pixel[k mod P]) and is therefore stricter than the arc test for 12
and 8 points.  The HIP path must equal the oracle bit for bit (candidates per level, the
selected keypoints and the descriptors).
"""
import numpy as np
import pytest

from tests import oracle_bind as ob

OFFS = {
    12: [(0, 2), (1, 2), (2, 1), (2, 0), (2, -1), (1, -2), (0, -2), (-1, -2), (-2, -1), (-2, 0),
         (-2, 1), (-1, 2)],
    8: [(0, 1), (1, 1), (1, 0), (1, -1), (0, -1), (-1, -1), (-1, 0), (-1, 1)],
}


def _fast_t(img, y, x, t, P):
    """OpenCV FAST_t<P> for one pixel, literally: quick test, arc count, cornerScore<P>
    with its early-continue loops.  -> score or None."""
    K, N = P // 2, P + P // 2 + 1
    pix = [int(img[y + OFFS[P][k % P][1], x + OFFS[P][k % P][0]]) for k in range(25)]
    v = int(img[y, x])

    def tab(p):
        return 1 if p - v < -t else (2 if p - v > t else 0)

    d = tab(pix[0]) | tab(pix[8])
    if d == 0:
        return None
    for a, b in ((2, 10), (4, 12), (6, 14)):
        d &= tab(pix[a]) | tab(pix[b])
    if d == 0:
        return None
    for a, b in ((1, 9), (3, 11), (5, 13), (7, 15)):
        d &= tab(pix[a]) | tab(pix[b])
    corner = False
    for bit, cmp in ((1, lambda p: p < v - t), (2, lambda p: p > v + t)):
        if corner or not (d & bit):
            continue
        cnt = 0
        for k in range(N):
            if cmp(pix[k]):
                cnt += 1
                if cnt > K:
                    corner = True
                    break
            else:
                cnt = 0
    if not corner:
        return None
    dd = [v - pix[k] for k in range(K * 3 + 1)]
    a0 = t
    for k in range(0, P, 2):           # cornerScore<P>: a loop
        a = min(dd[k + 1], dd[k + 2])
        if a <= a0:
            continue
        for j in range(3, K + 1):
            a = min(a, dd[k + j])
        a0 = max(a0, min(a, dd[k]))
        a0 = max(a0, min(a, dd[k + K + 1]))
    b0 = -a0
    for k in range(0, P, 2):           # b loop
        b = max(dd[k + 1], dd[k + 2])
        for j in range(3, K):
            b = max(b, dd[k + j])
        if b >= b0:
            continue
        b = max(b, dd[k + K])
        b0 = min(b0, max(b, dd[k]))
        b0 = min(b0, max(b, dd[k + K + 1]))
    return -b0 - 1


def _level_candidates_py(img, mask, t, P):
    """ComputeKeyPointsOctTree's cell sweep (:874-949) with FAST_t<P> + NMS + mask."""
    h, w = img.shape
    minB, maxBX, maxBY = 22, w - 25 + 3, h - 25 + 3
    width, height = maxBX - minB, maxBY - minB
    ncols, nrows = int(width / 30.0), int(height / 30.0)
    wc, hc = int(np.ceil(width / ncols)), int(np.ceil(height / nrows))
    out = []
    for i in range(nrows):
        iy = minB + i * hc
        my = min(iy + hc + 6, maxBY)
        if iy >= maxBY - 3:
            continue
        for j in range(ncols):
            ix = minB + j * wc
            mx = min(ix + wc + 6, maxBX)
            if ix >= maxBX - 6:
                continue
            rows, cols = my - iy, mx - ix
            sc = np.zeros((rows, cols), np.int32)
            cor = np.zeros((rows, cols), bool)
            for yy in range(3, rows - 3):
                for xx in range(3, cols - 3):
                    s = _fast_t(img, iy + yy, ix + xx, t, P)
                    if s is not None:
                        cor[yy, xx] = True
                        sc[yy, xx] = s
            for yy in range(3, rows - 3):
                for xx in range(3, cols - 3):
                    if not cor[yy, xx]:
                        continue
                    s = sc[yy, xx]
                    nb = sc[yy - 1:yy + 2, xx - 1:xx + 2].copy()
                    nb[1, 1] = -1
                    if s <= nb.max():
                        continue
                    if mask is not None and mask[iy + yy, ix + xx] == 0:
                        continue
                    out.append((xx + j * wc, yy + i * hc, s))
    return np.array(out, np.int32).reshape(-1, 3)


def _smooth_image(w, h, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (h // 4 + 2, w // 4 + 2)).astype(np.float64)
    img = np.kron(base, np.ones((4, 4)))[:h, :w]
    img += rng.normal(0, 6, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("fast_type,P", [(1, 12), (0, 8)])
@pytest.mark.parametrize("th", [8, 20])
def test_oracle_matches_literal_restatement(fast_type, P, th):
    img = _smooth_image(110, 96, 3 + P + th)
    mask = (np.random.default_rng(9).random(img.shape) > 0.15).astype(np.uint8) * 255
    for m in (None, mask):
        ref = _level_candidates_py(img, m, th, P)
        got = ob.level_candidates(img, m, th, fast_type=fast_type)
        assert len(ref) > 0
        assert np.array_equal(got, ref), (fast_type, th, len(got), len(ref))


def test_oracle_5_8_corner_needs_all_neighbours_on_one_side():
    """The wrapped quick test makes TYPE_5_8 demand all 8 neighbours darker (or brighter)."""
    img = _smooth_image(120, 100, 5)
    t = 10
    got = ob.level_candidates(img, None, t, fast_type=0)
    assert len(got) > 0
    for x, y, _ in got:
        X, Y = x + 22, y + 22
        v = int(img[Y, X])
        nb = img[Y - 1:Y + 2, X - 1:X + 2].astype(int).ravel()
        nb = np.delete(nb, 4)
        assert (nb < v - t).all() or (nb > v + t).all()


def test_oracle_types_differ_and_default_unchanged():
    img = _smooth_image(160, 120, 8)
    c16 = ob.level_candidates(img, None, 20)
    assert np.array_equal(ob.level_candidates(img, None, 20, fast_type=2), c16)
    c12 = ob.level_candidates(img, None, 20, fast_type=1)
    c8 = ob.level_candidates(img, None, 20, fast_type=0)
    assert not np.array_equal(c12, c16) and not np.array_equal(c8, c16)


# ---------------------------------------------------------------------------- GPU parity
def _frame(w=754, h=480, seed=3):
    from mcs_amd import synth
    return synth.fisheye_frame(w, h, seed=seed)


@pytest.mark.gpu
@pytest.mark.parametrize("fast_type", [1, 0])
def test_gpu_fast_type_candidates_per_level(gpu, fast_type):
    import mcs_amd
    img, mask = _frame(seed=60 + fast_type)
    ex = mcs_amd.Extractor(mcs_amd.ExtractorParams(nfeatures=2000, fast_agast_type=fast_type), 754, 480)
    ex.extract(img, mask)
    lv = ob.pyramid(img)
    mk = ob.mask_pyramid(mask)
    for l in range(8):
        ref = ob.level_candidates(lv[l], mk[l], 20, fast_type=fast_type)
        got = ex.read_stage(2, 0, l)
        assert np.array_equal(got, ref), "level %d: %d vs %d candidates" % (l, len(got), len(ref))


@pytest.mark.gpu
@pytest.mark.parametrize("fast_type,th,masked", [(1, 20, True), (1, 7, False), (0, 12, True),
                                                 (0, 5, False)])
def test_gpu_fast_type_end_to_end(gpu, fast_type, th, masked):
    import mcs_amd
    img, mask = _frame(seed=70 + th)
    if not masked:
        mask = None
    ex = mcs_amd.Extractor(mcs_amd.ExtractorParams(nfeatures=2000, fast_threshold=th,
                                                   fast_agast_type=fast_type), 754, 480)
    kps, desc = ex.extract(img, mask)
    okps, odesc = ob.extract(img, mask, nfeatures=2000, fast_th=th, fast_type=fast_type)
    assert len(kps) == len(okps) > 0
    assert np.array_equal(kps, okps) and np.array_equal(desc, odesc)


@pytest.mark.gpu
def test_gpu_agast_and_bad_type_rejected(gpu):
    import mcs_amd
    for kw in (dict(use_agast=1), dict(fast_agast_type=3), dict(fast_agast_type=-1)):
        with pytest.raises(Exception):
            mcs_amd.Extractor(mcs_amd.ExtractorParams(**kw), 754, 480)
