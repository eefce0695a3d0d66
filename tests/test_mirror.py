"""Omni camera mirror masks (CreateMirrorMask / isPointInMirrorMask).

Reference: src/cam_model_omni.cpp:165-222, called from cSystem::LoadMCS
(src/cSystem.cpp:164-172) with 4 levels when Camera.mirrorMask == 1. The oracle
(oracle/mirror_oracle.cpp) is the reference's literal pixel loop; it is pinned here against an
independent numpy restatement and run on the reference's own Lafida calibration
(tests/golden/lafida_settings.json). OpenCV is absent, so cv::buildPyramid's level sizes are
the documented ((w+1)/2, (h+1)/2) rule (parity of that rule with OpenCV itself is unpinned).
"""
import json
import os

import numpy as np
import pytest

from tests import oracle_bind as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "lafida_settings.json")


def _lafida_cams():
    fx = json.load(open(FIXTURE))
    return [(fx["InteriorOrientationFisheye%d.yaml" % c]["Camera.u0"],
             fx["InteriorOrientationFisheye%d.yaml" % c]["Camera.v0"],
             fx["InteriorOrientationFisheye%d.yaml" % c]["Camera.Iw"],
             fx["InteriorOrientationFisheye%d.yaml" % c]["Camera.Ih"]) for c in range(3)]


def oracle_masks(u0, v0, w, h, levels=4):
    sizes = []
    for l in range(levels):
        if l:
            w, h = (w + 1) // 2, (h + 1) // 2
        sizes.append((w, h))
    out = np.zeros(sum(a * b for a, b in sizes), np.uint8)
    assert ob.lib().oracle_create_mirror_mask(u0, v0, sizes[0][0], sizes[0][1], levels,
                                              ob._p(out)) == 0
    res, off = [], 0
    for w_, h_ in sizes:
        res.append(out[off:off + w_ * h_].reshape(h_, w_))
        off += w_ * h_
    return res


def numpy_masks(u0, v0, w, h, levels=4):
    """Independent vectorised restatement (float32 differences squared in float64)."""
    offs = np.float32([22.0, 10.0, 5.0, 1.0])
    r, c = np.float32(v0), np.float32(u0)
    res = []
    for l in range(levels):
        if l:
            w, h = (w + 1) // 2, (h + 1) // 2
            r = np.float32(np.ceil(r / np.float32(2.0)))
            c = np.float32(np.ceil(c / np.float32(2.0)))
        di = (np.arange(h, dtype=np.float32) - r).astype(np.float64)
        dj = (np.arange(w, dtype=np.float32) - c).astype(np.float64)
        a = (di * di).astype(np.float32)[:, None]
        b = (dj * dj).astype(np.float32)[None, :]
        ans = np.sqrt((a + b).astype(np.float32))
        res.append(np.where(ans < np.float32(r + offs[l]), 255, 0).astype(np.uint8))
    return res


CASES = [(30.3, 20.7, 61, 41), (376.5, 240.5, 754, 480), (10.0, 10.0, 7, 5)] + \
        [tuple(c) for c in _lafida_cams()]


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_numpy_restatement(case):
    for a, b in zip(oracle_masks(*case), numpy_masks(*case)):
        np.testing.assert_array_equal(a, b)


def test_oracle_mask_properties_lafida():
    for u0, v0, w, h in _lafida_cams():
        m = oracle_masks(u0, v0, w, h)
        assert [x.shape for x in m] == [(480, 754), (240, 377), (120, 189), (60, 95)]
        c = m[0]
        assert c[int(round(v0)), int(round(u0))] == 255       # centre inside
        assert c[0, 0] == 0 and c[-1, -1] == 0                 # image corners outside
        assert set(np.unique(c)) <= {0, 255}
        _check_disc(c, row=v0, col=u0, radius=v0 + 22.0)


def _check_disc(m, row, col, radius):
    """255 strictly inside the disc (1 px margin), 0 strictly outside, and the mask is mirror-
    symmetric about the centre row / column wherever both sides are in the image."""
    h, w = m.shape
    i = np.arange(h)[:, None]
    j = np.arange(w)[None, :]
    dist = np.sqrt((i - row) ** 2 + (j - col) ** 2)
    assert (m[dist < radius - 1] == 255).all()
    assert (m[dist > radius + 1] == 0).all()
    r0, c0 = int(round(row)), int(round(col))
    if abs(row - r0) < 1e-6 and abs(col - c0) < 1e-6:
        k = min(r0, h - 1 - r0)
        assert np.array_equal(m[r0 - k:r0], m[r0 + 1:r0 + k + 1][::-1])
        k = min(c0, w - 1 - c0)
        assert np.array_equal(m[:, c0 - k:c0], m[:, c0 + 1:c0 + k + 1][:, ::-1])


def test_mirror_mask_centre_is_row_v0_col_u0():
    """The reference swaps the names (src/cam_model_omni.cpp:189-190): the disc is centred at
    row = Camera.v0, column = Camera.u0 with radius Camera.v0 + 22 at level 0.  With u0 != v0 the
    swapped reading would give a different disc: pin the real one."""
    u0, v0, w, h = 300.0, 200.0, 754, 480
    m = oracle_masks(u0, v0, w, h)
    _check_disc(m[0], row=200.0, col=300.0, radius=222.0)
    assert m[0][200, 517] == 255     # 217 px right of the centre, inside r = 222
    assert m[0][479, 300] == 0       # 279 px below: outside (the swapped disc would hold it)
    # level 1: centre ceil(200/2), ceil(300/2); radius 100 + 10
    _check_disc(m[1], row=100.0, col=150.0, radius=110.0)
    for a, b in zip(m, numpy_masks(u0, v0, w, h)):
        np.testing.assert_array_equal(a, b)


def test_layout_and_point_lookup_host():
    from mcs_amd import lafida
    w, h, off, total = lafida.mirror_mask_layout(754, 480, 4)
    assert list(w) == [754, 377, 189, 95] and list(h) == [480, 240, 120, 60]
    assert list(off) == [0, 754 * 480, 754 * 480 + 377 * 240, 754 * 480 + 377 * 240 + 189 * 120]
    assert total == off[-1] + 95 * 60
    m = oracle_masks(*_lafida_cams()[0])[0]
    rng = np.random.default_rng(3)
    pts = np.concatenate([rng.uniform(-5, 760, (400, 2)),
                          np.array([[0.5, 10], [1.5, 10], [753.4, 5], [753.6, 5], [2.5, 479.5],
                                    [300, 0.49], [300, 0.51]])])
    for u, v in pts:
        assert lafida.is_point_in_mirror_mask(m, u, v) == bool(
            ob.lib().oracle_is_point_in_mirror_mask(ob._p(m), m.shape[1], m.shape[0], u, v))


def test_layout_rejects_bad_levels():
    from mcs_amd import McsError, lafida
    with pytest.raises(McsError):
        lafida.mirror_mask_layout(754, 480, 5)
    with pytest.raises(McsError):
        lafida.mirror_mask_layout(0, 480, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("levels", [1, 4])
def test_gpu_mirror_masks_match_oracle(case, levels):
    from mcs_amd import lafida
    u0, v0, w, h = case
    got = lafida.create_mirror_masks({"u0": u0, "v0": v0}, w, h, levels)
    for g, e in zip(got, oracle_masks(u0, v0, w, h, levels)):
        np.testing.assert_array_equal(g.cpu().numpy(), e)


@pytest.mark.gpu
def test_gpu_rig_mirror_masks_lafida():
    from mcs_amd import lafida
    fx = json.load(open(FIXTURE))
    rig = {"cams": [], "sizes": [], "mirror_mask": []}
    for c, (u0, v0, w, h) in enumerate(_lafida_cams()):
        rig["cams"].append({"u0": u0, "v0": v0})
        rig["sizes"].append((w, h))
        rig["mirror_mask"].append(fx["InteriorOrientationFisheye%d.yaml" % c]["Camera.mirrorMask"] == 1)
    rig["mirror_mask"][2] = False          # exercise the all-ones branch (src/cSystem.cpp:170)
    masks = lafida.rig_mirror_masks(rig)
    for c, (u0, v0, w, h) in enumerate(_lafida_cams()):
        if rig["mirror_mask"][c]:
            for g, e in zip(masks[c], oracle_masks(u0, v0, w, h)):
                np.testing.assert_array_equal(g.cpu().numpy(), e)
        else:
            assert len(masks[c]) == 1 and bool((masks[c][0] == 1).all())
