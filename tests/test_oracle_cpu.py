"""CPU tests: pin the oracle (the CPU restatement of the reference extractor) against
everything the reference itself fixes for this path, and check the C-ABI library loads
and exports every symbol declared in include/*.h (no compute without a GPU).

Pins available in the reference: the learned pattern table
(include/mdBRIEFextractorOct.h:44-47), umax (ctor :187-202), the per-level budget formula
(:167-179) and level sizes (:1164-1165).  OpenCV semantics are our written spec
 -> parity unpinned against the real reference binary.
"""
import os
import re

import numpy as np
import pytest

from tests import oracle_bind as ob

REF = "/root/reference"


def test_level_sizes_match_survey():
    # 754x480 and 1024^2 level geometry
    assert ob.level_sizes(754, 480).tolist() == [[754, 480], [628, 400], [524, 333], [436, 278],
                                                  [364, 231], [303, 193], [253, 161], [210, 134]]
    assert [w for w, h in ob.level_sizes(1024, 1024)] == [1024, 853, 711, 593, 494, 412, 343, 286]


def test_features_per_level_match_survey():
    assert ob.features_per_level(1000).tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    assert ob.features_per_level(2000).tolist() == [434, 362, 302, 251, 209, 175, 145, 122]
    assert ob.features_per_level(4000).tolist() == [869, 724, 603, 503, 419, 349, 291, 242]
    assert ob.features_per_level(400).tolist() == [87, 72, 60, 50, 42, 35, 29, 25]


def test_umax():
    assert ob.umax().tolist() == [16, 16, 16, 16, 15, 15, 15, 14, 14, 13, 12, 12, 11, 9, 8, 6, 3]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not mounted")
def test_pattern_table_matches_reference_header():
    src = open(os.path.join(REF, "include/mdBRIEFextractorOct.h"), encoding="latin-1").read()
    m = re.search(r"\n\s*static int learned_pattern_64_ORB\[4 \* 512\] =\s*\{([^}]*)\}", src)
    vals = [int(v) for v in m.group(1).replace("\n", " ").split(",") if v.strip()]
    assert ob.pattern().tolist() == vals


def test_fast_atan2_quadrants():
    # fastAtan2 is a 4th-order polynomial in degrees; error < 0.01 deg, range [0, 360)
    rng = np.random.default_rng(0)
    for _ in range(2000):
        y, x = rng.normal(size=2) * 1000
        a = ob.lib().oracle_fast_atan2(float(y), float(x))
        ref = np.degrees(np.arctan2(y, x)) % 360
        d = abs(a - ref)
        assert min(d, 360 - d) < 0.02
    assert ob.lib().oracle_fast_atan2(0.0, 1.0) == 0.0


def test_resize_modes_agree_on_smooth_and_differ_rarely():
    from mcs_amd import synth
    img, _ = synth.fisheye_frame(754, 480, seed=3)
    a = ob.resize_linear(img, 628, 400, mode=1)
    b = ob.resize_linear(img, 628, 400, mode=0)
    diff = np.abs(a.astype(int) - b.astype(int))
    assert diff.max() <= 1          # SSE2 vs scalar vertical rounding differ by <= 1 DN
    assert (diff > 0).mean() < 0.2


def test_blur_is_rounded_mean():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (40, 50), dtype=np.uint8)
    b = ob.box_blur5(img)
    pad = np.pad(img.astype(np.int64), 2, mode="reflect")  # numpy reflect == REFLECT_101
    s = sum(pad[dy:dy + 40, dx:dx + 50] for dy in range(5) for dx in range(5))
    assert np.array_equal(b, np.floor(s / 25 + 0.5).astype(np.uint8))


def test_octree_returns_budget_and_best_responses():
    from mcs_amd import synth
    img, mask = synth.fisheye_frame(754, 480, seed=9)
    lv = ob.pyramid(img)
    c = ob.level_candidates(lv[0], mask, 20)
    sel = ob.octree(c, 754, 480, 434)
    assert 434 <= len(sel) <= 437 or len(sel) == len(c)
    assert len(set(sel.tolist())) == len(sel)


def test_fast_matches_bruteforce_definition():
    """FAST candidates == per-pixel segment test + cornerScore + cell-local NMS, restated
    independently in tests/np_extractor.py (itself checked against a literal per-pixel loop in
    tests/test_oracle_crosscheck.py), on a small random image with one masked-out block."""
    from tests import np_extractor as npx
    rng = np.random.default_rng(4)
    img = (rng.random((120, 140)) * 255).astype(np.uint8)
    mask = np.full(img.shape, 255, np.uint8)
    mask[40:70, 50:90] = 0
    for m in (None, mask):
        c = ob.level_candidates(img, m, 20)
        assert len(c) > 20
        assert np.array_equal(c, npx.fast_level(img, m, 20))
        assert (c[:, 2] >= 20).all()


def test_extract_deterministic_and_ordered():
    from mcs_amd import synth
    img, mask = synth.fisheye_frame(754, 480, seed=5)
    k1, d1 = ob.extract(img, mask, nfeatures=1000)
    k2, d2 = ob.extract(img, mask, nfeatures=1000)
    assert np.array_equal(k1, k2) and np.array_equal(d1, d2)
    assert (np.diff(k1["octave"]) >= 0).all()
    assert (k1["class_id"] == -1).all()
    # level-0 keypoints lie inside the mirror mask
    k0 = k1[k1["octave"] == 0]
    assert (mask[k0["y"].astype(int), k0["x"].astype(int)] > 0).all()


def test_library_exports_every_declared_symbol(built):
    import ctypes
    import mcs_amd
    L = ctypes.CDLL(mcs_amd.LIB_PATH)
    declared = set()
    for h in os.listdir(mcs_amd.INCLUDE_DIR):
        if h.endswith(".h"):
            txt = open(os.path.join(mcs_amd.INCLUDE_DIR, h)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)  # drop comments
            declared |= set(re.findall(r"\b(mcs_[a-z0-9_]+)\s*\(", txt))
    assert declared, "no declarations found"
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    assert set(mcs_amd.SIGNATURES) >= declared - {"mcs_status"}


def test_library_reports_no_device_on_cpu_host(built):
    import mcs_amd
    if mcs_amd.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(mcs_amd.McsError):
        mcs_amd.Extractor(mcs_amd.ExtractorParams(), 754, 480)


def test_pyramid_fixed_point_forms_are_exact():
    """The integer rewrites k_pyr_rows relies on, checked over their whole operand ranges
    (csrc/pyr_math.hpp, csrc/k_pyramid.hip):
      * box blur: (2s + 25) // 50 == (s * 671090 + 8388625) >> 24 for every 5x5 sum s of u8,
        with no 32-bit overflow (the quotient is the top byte);
      * SSE2 vertical resize: (x0 * b) >> 16 == ((x0 << 8) * (b << 8)) >> 32 with both
        operands < 2^24 (v_mul_hi_u32_u24), x0 = s >> 4 for s = p0 a0 + p1 a1, p <= 255,
        a0 + a1 = 2048, b in [0, 2048]; and x0 << 8 == (s << 4) & ~0xFF."""
    s = np.arange(0, 25 * 255 + 1, dtype=np.int64)
    q = s * 671090 + 8388625
    assert q.max() < 2 ** 32
    assert np.array_equal(q >> 24, (2 * s + 25) // 50)
    rng = np.random.default_rng(0)
    p = rng.integers(0, 256, size=(2, 200000), dtype=np.int64)
    a0 = rng.integers(0, 2049, size=200000, dtype=np.int64)
    sv = p[0] * a0 + p[1] * (2048 - a0)
    sv = np.concatenate([sv, [0, 255 * 2048]])
    x0 = sv >> 4
    X = (sv << 4) & ~0xFF
    assert np.array_equal(X, x0 << 8) and X.max() < 2 ** 24
    for b in (0, 1, 2, 511, 1024, 1707, 2047, 2048):
        assert np.array_equal((X * (b << 8)) >> 32, (x0 * b) >> 16)
    # and the sum of the two taps never needs the u8 clamp
    assert ((x0.max() * 2048) >> 16) <= 1020


def test_descriptor_integer_and_rounding_forms_are_exact():
    """k_orient_desc (csrc/k_desc.hip): the raw-patch row of dword q is (57 q) >> 9 == q // 9
    for every lane's q < 320; and rint_magic(v) = low word of v + 1.5 * 2^52 equals rint(v)
    (round half to even) for the rotated pattern coordinates, |v| <= 15 * sqrt(2)."""
    q = np.arange(320)
    assert np.array_equal((q * 57) >> 9, q // 9)
    v = np.concatenate([np.arange(-25, 25.01, 0.25), np.random.default_rng(1).uniform(-22, 22, 100000)])
    m = (v + 6755399441055744.0).view(np.int64) & 0xFFFFFFFF
    m = np.where(m >= 2 ** 31, m - 2 ** 32, m)
    assert np.array_equal(m, np.rint(v).astype(np.int64))
