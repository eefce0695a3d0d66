"""Cross-check the extractor oracle (oracle/extractor_oracle.cpp) against independent
restatements (tests/np_extractor.py) on Lafida-calibrated frames.

Both sides restate the same written spec (OpenCV is absent, so the
OpenCV-defined pieces stay unpinned against a real OpenCV build -- DESIGN.md §6), but they
are written independently: C++ scalar loops vs whole-image numpy / Python lists.  Frames are
the synthetic fisheye renders with the Lafida camera models and their mirror masks
(mcs_amd.synth), run through all 8 pyramid levels.  Exact equality everywhere.
"""
import numpy as np
import pytest

from tests import np_extractor as npx
from tests import oracle_bind as ob


@pytest.fixture(scope="module")
def frames():
    from mcs_amd import synth
    out = []
    for cam in range(3):
        img, mask = synth.fisheye_frame(754, 480, seed=40 + cam, cam_index=cam)
        out.append((img, mask))
    return out


def test_resize_linear_both_forms(built, frames):
    for img, _ in frames:
        sizes = ob.level_sizes(754, 480)
        for mode in (1, 0):
            src = img
            for l in range(1, 8):
                w, h = sizes[l]
                a = ob.resize_linear(src, w, h, mode=mode)
                b = npx.resize_linear(src, w, h, mode=mode)
                assert np.array_equal(a, b), (mode, l)
                src = a


def test_resize_linear_odd_sizes(built):
    rng = np.random.default_rng(2)
    for sw, sh, dw, dh in ((97, 61, 81, 51), (40, 33, 33, 28), (1024, 1024, 853, 853),
                           (19, 17, 16, 14), (64, 64, 21, 64)):
        img = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
        for mode in (1, 0):
            assert np.array_equal(ob.resize_linear(img, dw, dh, mode), npx.resize_linear(img, dw, dh, mode))


def test_resize_nearest_mask_pyramid(built, frames):
    for _, mask in frames:
        a = ob.mask_pyramid(mask)
        src = mask
        for l, (w, h) in enumerate(ob.level_sizes(754, 480)):
            if l == 0:
                continue
            src = npx.resize_nearest(src, w, h)
            assert np.array_equal(a[l], src), l


def test_fast_score_map_matches_per_pixel_definition():
    """numpy FAST vs a literal per-pixel loop: segment test (>= 9 contiguous of 16 all brighter
    than v+t or all darker than v-t) and the cornerScore<16> max-min definition: the largest
    threshold t' for which the pixel is still a corner, minus nothing (score = max t' - 1 + 1)."""
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (24, 26), dtype=np.uint8)
    img[8:12, 8:12] = 250          # a bright blob creates dark-ring corners
    s = npx.fast_score_map(img, 20)
    I = img.astype(int)
    n_corners = 0
    for y in range(3, 21):
        for x in range(3, 23):
            v = I[y, x]
            ring = [I[y + dy, x + dx] for dx, dy in npx.CIRCLE]

            def is_corner(t):
                for sign in (1, -1):
                    ok = [sign * (p - v) > t for p in ring]
                    ok2 = ok + ok
                    if any(all(ok2[k:k + 9]) for k in range(16)):
                        return True
                return False
            if is_corner(20):
                n_corners += 1
                # cornerScore = the largest t with is_corner(t) (t < score+1 fails)
                best = max(t for t in range(20, 255) if is_corner(t))
                assert s[y, x] == best, (y, x)
            else:
                assert s[y, x] == 0
    assert n_corners > 10


@pytest.mark.parametrize("th", [20, 7])
def test_fast_cells_with_mask(built, frames, th):
    for img, mask in frames:
        lv = ob.pyramid(img)
        mk = ob.mask_pyramid(mask)
        for l in (0, 1, 3, 7):
            a = ob.level_candidates(lv[l], mk[l], th)
            b = npx.fast_level(lv[l], mk[l], th)
            assert len(a) > 0
            assert np.array_equal(a, b), l


def test_fast_cells_mask_after_nms(built):
    """A masked-out corner still suppresses its neighbour (runByPixelsMask after NMS)."""
    from mcs_amd import synth
    img, _ = synth.fisheye_frame(754, 480, seed=9)
    full = npx.fast_level(img, None, 20)
    # mask exactly the strongest corner: its weaker 8-neighbours must not reappear
    k = int(np.argmax(full[:, 2]))
    x, y = full[k, 0] + 22, full[k, 1] + 22
    mask = np.full(img.shape, 255, np.uint8)
    mask[y, x] = 0
    a = ob.level_candidates(img, mask, 20)
    b = npx.fast_level(img, mask, 20)
    assert np.array_equal(a, b)
    assert len(a) == len(full) - 1


def test_octree_matches_python_restatement(built, frames):
    for img, mask in frames[:2]:
        lv = ob.pyramid(img)
        mk = ob.mask_pyramid(mask)
        budgets = ob.features_per_level(2000)
        for l in (0, 2, 5, 7):
            h, w = lv[l].shape
            c = ob.level_candidates(lv[l], mk[l], 20)
            a = ob.octree(c, w, h, int(budgets[l]))
            b = npx.distribute_octree(c, 22, w - 22, 22, h - 22, int(budgets[l]))
            assert np.array_equal(a, b), l


@pytest.mark.parametrize("N", [1, 5, 60, 434, 5000])
def test_octree_budgets(built, frames, N):
    img, mask = frames[2]
    c = ob.level_candidates(img, mask, 20)
    a = ob.octree(c, 754, 480, N)
    b = npx.distribute_octree(c, 22, 754 - 22, 22, 480 - 22, N)
    assert np.array_equal(a, b)
