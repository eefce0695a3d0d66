"""GPU parity of the row-streaming FAST kernel (k_fast_rows) at its capacity limits.

k_fast_rows tests a run of up to 8 cells per wave in bands of 4 rows: survivors of the
compass pre-test and the corners of a band's last row share one LDS list sized to the worst
case (every pixel of 4 rows of a 246 px run, plus one carried row), and the NMS excludes
neighbours across cell borders.  These cases drive those limits and compare the per-level
candidate lists (cell order, raster order inside a cell, score) bit-exactly with the oracle's
per-cell FAST (ComputeKeyPointsOctTree, src/mdBRIEFextractorOct.cpp:874-949):
  * uniform noise at threshold 0 / 1: nearly every pixel survives the pre-test and is a corner
    (full lists, 246 carried corners per band);
  * odd frame sizes: level-0 rows at odd pitch (unaligned row starts), clamped last cells,
    other run splits;
  * 2x2 bright blocks on a dark field every 7 px: four equal-score corners per block (strict
    NMS keeps none of them), blocks straddling cell borders (where the NMS must not look
    across).
"""
import numpy as np
import pytest

from tests import oracle_bind as ob

pytestmark = pytest.mark.gpu


def _extractor(w, h, fast_th, nfeatures=2000):
    import mcs_amd
    p = mcs_amd.ExtractorParams(nfeatures=nfeatures, fast_threshold=fast_th, desc_size=32)
    return mcs_amd.Extractor(p, w, h, max_frames=1)


def _check_levels(img, mask, th, nfeatures=2000):
    h, w = img.shape
    ex = _extractor(w, h, th, nfeatures)
    ex.extract(img, mask)
    lv = ob.pyramid(img)
    mk = ob.mask_pyramid(mask) if mask is not None else [None] * len(lv)
    total = 0
    for l in range(len(lv)):
        ref = ob.level_candidates(lv[l], mk[l], th)
        got = ex.read_stage(2, 0, l)
        assert got.shape == ref.shape, (l, got.shape, ref.shape)
        assert np.array_equal(got, ref), "FAST candidates differ at level %d" % l
        total += len(ref)
    return total


@pytest.mark.parametrize("th", [0, 1])
def test_noise_full_lists(gpu, th):
    rng = np.random.default_rng(7 + th)
    img = rng.integers(0, 256, size=(480, 754), dtype=np.uint8)
    n = _check_levels(img, None, th)
    assert n > 10000   # the lists really are full


@pytest.mark.parametrize("w,h", [(641, 363), (901, 517), (401, 300)])
def test_odd_sizes_with_mask(gpu, w, h):
    from mcs_amd import synth
    img, mask = synth.fisheye_frame(w, h, seed=w + h)
    _check_levels(img, mask, 20)


def test_block_ties_across_cell_borders(gpu):
    y, x = np.mgrid[0:480, 0:754]
    img = np.where(((x % 7) < 2) & ((y % 7) < 2), 200, 40).astype(np.uint8)
    _check_levels(img, None, 10)
