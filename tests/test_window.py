"""Projection-guided (windowed) matching: the cMultiFrame grid (src/cMultiFrame.cpp:154-184,
PosInGrid :342-353), GetFeaturesInArea (:272-340) and the windowed selection rules of
cORBmatcher (checkOrientation = false, include/cORBmatcher.h:40):
  rule 0 SearchByProjection(F, vpMapPoints, th)   src/cORBmatcher.cpp:67-166
  rule 1 SearchByProjection(Current, Last, th)    src/cORBmatcher.cpp:1991-2123
  rule 2 SearchForInitialization                  src/cORBmatcher.cpp:579-726
  rule 3 WindowSearch                             src/cORBmatcher.cpp:326-473
against the oracle restatement (oracle/matcher_oracle.cpp).  Index / distance outputs: exact.

CPU (not gpu): grid build and the host selection rule (mcs_window_select) on oracle candidate
lists.  GPU: device candidate lists (order, keypoints, distances), the device pipeline, the
host-buffer entry point mcs_window_match and the capacity / empty / out-of-range cases.
Parity unpinned against a reference binary (it needs OpenCV); the rules are restated from the
reference lines cited above.
"""
import ctypes

import numpy as np
import pytest

from tests import oracle_bind as ob

NC, W, H = 3, 754, 480
LEVEL_P = np.array([434, 362, 302, 251, 209, 175, 145, 122], np.float64)
RATIO = {0: 0.8, 1: 0.8, 2: 0.9, 3: 0.7}


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _flip(d, nbits, rng):
    bits = np.unpackbits(d.copy())
    bits[rng.choice(bits.size, nbits, replace=False)] ^= 1
    return np.packbits(bits)


def _frame(seed, n_kp=8000, nbytes=32, masks=False):
    from mcs_amd import window as mw
    rng = np.random.default_rng(seed)
    gp = mw.grid_params([(0, 0), (3, 5), (0, 0)], [(W, H), (W - 4, H - 10), (W, H)])
    xy = np.stack([rng.uniform(-4, W + 4, n_kp), rng.uniform(-4, H + 4, n_kp)], 1).astype(np.float32)
    xy[:64, 0] = (np.arange(64) + 0.5) * (W / 64.0)          # on cell boundaries (cvRound ties)
    xy[64:112, 1] = (np.arange(48) + 0.5) * (H / 48.0)
    xy[112:400] = np.round(xy[112:400])                      # integer pixel positions
    cam = rng.integers(0, NC, n_kp).astype(np.int32)
    octave = rng.choice(8, n_kp, p=LEVEL_P / LEVEL_P.sum()).astype(np.int32)
    desc = rng.integers(0, 256, (n_kp, nbytes), dtype=np.uint8)
    dm = None
    if masks:
        dm = np.packbits((rng.random((n_kp, nbytes * 8)) < 0.85).astype(np.uint8), axis=1)
    return dict(gp=gp, xy=xy, cam=cam, oct=octave, desc=desc, mask=dm, bytes=nbytes)


def _queries(fr, rule, seed, nq=2500):
    """One query per GetFeaturesInArea call, shaped like the rule's caller."""
    rng = np.random.default_rng(seed)
    n, nb = len(fr["xy"]), fr["bytes"]
    xyr = np.zeros((nq, 3))
    cl = np.zeros((nq, 3), np.int32)
    qd = np.zeros((nq, nb), np.uint8)
    for i in range(nq):
        k = int(rng.integers(n))
        if rng.random() < 0.8:
            xyr[i, :2] = fr["xy"][k] + rng.normal(0, 2.5, 2)
            cl[i, 0] = fr["cam"][k]
            qd[i] = _flip(fr["desc"][k], int(rng.integers(0, 60)), rng)
        else:
            xyr[i, :2] = rng.uniform([-60, -60], [W + 60, H + 60])
            cl[i, 0] = rng.integers(NC)
            qd[i] = rng.integers(0, 256, nb, dtype=np.uint8)
        o = int(fr["oct"][k])
        if rule == 0:    # r = RadiusByViewingCos * th * scale(level), levels (level-1, level)
            xyr[i, 2] = rng.choice([2.5, 4.0]) * rng.choice([1.0, 3.0]) * 1.2 ** o
            cl[i, 1:] = (o - 1, o)
        elif rule == 1:  # radius = th * scale(octave), levels (octave-1, octave+1)
            xyr[i, 2] = rng.choice([7.0, 15.0, 30.0]) * 1.2 ** o
            cl[i, 1:] = (o - 1, o + 1)
        elif rule == 2:  # windowSize, the query's level only
            xyr[i, 2] = rng.choice([10.0, 50.0, 100.0])
            cl[i, 1:] = (o, o)
        else:            # windowSize, any level
            xyr[i, 2] = float(rng.choice([5, 15, 40]))
            cl[i, 1:] = (-1, -1)
    qm = None
    if fr["mask"] is not None:
        qm = np.packbits((rng.random((nq, nb * 8)) < 0.85).astype(np.uint8), axis=1)
    return xyr, cl, qd, qm


def _frame_args(fr):
    return (len(fr["gp"]), _p(fr["gp"]), _p(fr["xy"]), _p(fr["cam"]), _p(fr["oct"]),
            _p(fr["desc"]), _p(fr["mask"]), len(fr["xy"]), fr["bytes"])


def _oracle_candidates(fr, xyr, cl, qd, qm):
    nq = len(xyr)
    cap = 400 * nq + 16
    ptr = np.zeros(nq + 1, np.int32)
    kp = np.zeros(cap, np.int32)
    dist = np.zeros(cap, np.int32)
    tot = ob.lib().oracle_window_candidates(*_frame_args(fr), nq, _p(xyr), _p(cl), _p(qd), _p(qm),
                                            _p(ptr), _p(kp), _p(dist), cap)
    assert 0 <= tot <= cap
    return ptr, kp[:tot], dist[:tot]


def _th(fr, rule):
    from mcs_amd import window as mw
    hi, lo = mw.matcher_thresholds(fr["bytes"], fr["mask"] is not None)
    return lo if rule == 2 else hi


def _assigned0(fr, rule, seed):
    a = np.zeros(len(fr["xy"]), np.uint8)
    if rule in (0, 1):   # keypoints that already hold a map point
        a[np.random.default_rng(seed).random(len(a)) < 0.1] = 1
    return a


def _oracle_match(fr, rule, xyr, cl, qd, qm, assigned):
    a = assigned.copy()
    m = np.full(len(xyr), -7, np.int32)
    n = ob.lib().oracle_window_match(rule, *_frame_args(fr), len(xyr), _p(xyr), _p(cl), _p(qd),
                                     _p(qm), _th(fr, rule), RATIO[rule], _p(a), _p(m))
    return n, m, a


def test_grid_build_matches_oracle(built):
    from mcs_amd import window as mw
    fr = _frame(1)
    ptr, cells = mw.grid_build(fr["xy"], fr["cam"], fr["gp"])
    optr = np.zeros_like(ptr)
    ocell = np.zeros(len(fr["xy"]), np.int32)
    n = ob.lib().oracle_frame_grid(len(fr["gp"]), _p(fr["gp"]), _p(fr["xy"]), _p(fr["cam"]),
                                   len(fr["xy"]), _p(optr), _p(ocell))
    assert np.array_equal(ptr, optr) and np.array_equal(cells, ocell[:n])
    # keypoints outside their camera's bounds are dropped, every other one appears once
    assert len(np.unique(cells)) == len(cells) and 0 < n < len(fr["xy"])


@pytest.mark.parametrize("masks", [False, True])
@pytest.mark.parametrize("rule", [0, 1, 2, 3])
def test_window_select_matches_oracle(built, rule, masks):
    from mcs_amd import window as mw
    fr = _frame(2 + rule, masks=masks)
    xyr, cl, qd, qm = _queries(fr, rule, 10 + rule)
    ptr, kp, dist = _oracle_candidates(fr, xyr, cl, qd, qm)
    assert len(kp) > 1000
    a0 = _assigned0(fr, rule, 3)
    n_o, m_o, a_o = _oracle_match(fr, rule, xyr, cl, qd, qm, a0)
    m, n, a = mw.window_select(rule, ptr, kp, dist, fr["oct"], _th(fr, rule), RATIO[rule], a0)
    assert n_o > 50
    assert n == n_o and np.array_equal(m, m_o)
    if rule != 2:
        assert np.array_equal(a, a_o)


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes,masks", [(32, False), (32, True), (16, False), (64, True)])
def test_window_candidates_device(gpu, nbytes, masks):
    from mcs_amd import window as mw
    fr = _frame(7, nbytes=nbytes, masks=masks)
    frame = mw.FrameGrid(fr["xy"], fr["cam"], fr["oct"], fr["desc"], fr["gp"], fr["mask"])
    for rule in (0, 2, 3):
        xyr, cl, qd, qm = _queries(fr, rule, 20 + rule)
        ptr, kp, dist = mw.window_search(frame, xyr, cl, qd, qm)
        optr, okp, odist = _oracle_candidates(fr, xyr, cl, qd, qm)
        assert np.array_equal(ptr, optr)
        assert np.array_equal(kp, okp) and np.array_equal(dist, odist)


@pytest.mark.gpu
@pytest.mark.parametrize("rule", [0, 1, 2, 3])
def test_window_match_device_and_host_entry(gpu, rule):
    from mcs_amd import window as mw
    fr = _frame(30 + rule, masks=(rule == 1))
    xyr, cl, qd, qm = _queries(fr, rule, 40 + rule)
    a0 = _assigned0(fr, rule, 5)
    n_o, m_o, a_o = _oracle_match(fr, rule, xyr, cl, qd, qm, a0)
    assert n_o > 50
    frame = mw.FrameGrid(fr["xy"], fr["cam"], fr["oct"], fr["desc"], fr["gp"], fr["mask"])
    m, n, a = mw.window_match(rule, frame, xyr, cl, qd, _th(fr, rule), RATIO[rule], q_mask=qm,
                              kp_assigned=a0)
    assert n == n_o and np.array_equal(m, m_o)
    m2, n2, a2 = mw.window_match_host(rule, fr["gp"], fr["xy"], fr["cam"], fr["oct"], fr["desc"],
                                      xyr, cl, qd, _th(fr, rule), RATIO[rule], desc_mask=fr["mask"],
                                      q_mask=qm, kp_assigned=a0)
    assert n2 == n_o and np.array_equal(m2, m_o)
    if rule != 2:
        assert np.array_equal(a, a_o) and np.array_equal(a2, a_o)


@pytest.mark.gpu
def test_window_search_edge_cases(gpu):
    import mcs_amd
    from mcs_amd import window as mw
    fr = _frame(50, n_kp=3000)
    frame = mw.FrameGrid(fr["xy"], fr["cam"], fr["oct"], fr["desc"], fr["gp"])
    xyr, cl, qd, _ = _queries(fr, 3, 51, nq=300)
    optr, okp, odist = _oracle_candidates(fr, xyr, cl, qd, None)
    assert len(okp) > 7
    # capacity too small: MCS_ERR_CAPACITY (required size reported), then the retry succeeds
    with pytest.raises(mcs_amd.McsError) as ei:
        mw.window_search(frame, xyr, cl, qd, cap=7, retry=False)
    assert ei.value.code == mcs_amd.MCS_ERR_CAPACITY
    ptr, kp, dist = mw.window_search(frame, xyr, cl, qd, cap=7)
    assert np.array_equal(ptr, optr) and np.array_equal(kp, okp) and np.array_equal(dist, odist)
    # no queries
    ptr, kp, dist = mw.window_search(frame, np.zeros((0, 3)), np.zeros((0, 3), np.int32),
                                     np.zeros((0, 32), np.uint8))
    assert ptr.tolist() == [0] and len(kp) == 0
    # camera index outside the rig, windows far outside the image: empty lists
    cl2 = cl.copy()
    cl2[:100, 0] = NC
    cl2[100:150, 0] = -1
    xyr2 = xyr.copy()
    xyr2[150:200, :2] = (-500.0, -500.0)
    xyr2[200:250, :2] = (5000.0, 5000.0)
    ptr, kp, dist = mw.window_search(frame, xyr2, cl2, qd)
    assert (np.diff(ptr)[:250] == 0).all()
    assert np.array_equal(np.diff(ptr)[250:], np.diff(optr)[250:])
    # a frame without keypoints
    empty = mw.FrameGrid(np.zeros((0, 2), np.float32), np.zeros(0, np.int32), np.zeros(0, np.int32),
                         np.zeros((0, 32), np.uint8), fr["gp"])
    ptr, kp, dist = mw.window_search(empty, xyr, cl, qd)
    assert ptr[-1] == 0 and len(kp) == 0
    # masks on one side only are rejected
    with pytest.raises(ValueError):
        mw.window_search(frame, xyr, cl, qd, q_mask=qd)
