"""Matcher parity: DescriptorDistance64 (host, CPU test), Hamming top-2 / dense / batched
top-2 and SearchForTriangulationRaw on the GPU vs the oracle -- exact integer equality.

Reference: src/cORBmatcher.cpp:2443-2477 (distances), :968-1156 (triangulation search),
:67-163 (best / second-best rule).
"""
import ctypes

import numpy as np
import pytest

from tests import oracle_bind as ob


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _descs(n, bytes_=32, seed=0):
    return np.random.default_rng(seed).integers(0, 256, (n, bytes_), dtype=np.uint8)


def _noisy_copy(d, nflip, seed):
    rng = np.random.default_rng(seed)
    out = d.copy()
    bits = np.unpackbits(out, axis=1)
    for i in range(len(bits)):
        idx = rng.choice(bits.shape[1], nflip[i], replace=False)
        bits[i, idx] ^= 1
    return np.packbits(bits, axis=1)


@pytest.mark.parametrize("nbytes", [16, 32, 64])
def test_descriptor_distance64_host(built, nbytes):
    import mcs_amd
    L = mcs_amd.lib()
    a = _descs(200, nbytes, 1)
    b = _descs(200, nbytes, 2)
    for i in range(200):
        ref = ob.lib().oracle_descriptor_distance64(_p(a[i]), _p(b[i]), nbytes)
        assert ref == int(np.unpackbits(a[i] ^ b[i]).sum())
        assert L.mcs_descriptor_distance64(_p(a[i]), _p(b[i]), nbytes) == ref
    ma = _descs(200, nbytes, 3)
    mb = _descs(200, nbytes, 4)
    for i in range(50):
        ref = ob.lib().oracle_descriptor_distance64_masked(_p(a[i]), _p(b[i]), _p(ma[i]), _p(mb[i]), nbytes)
        got = L.mcs_descriptor_distance64_masked(_p(a[i]), _p(b[i]), _p(ma[i]), _p(mb[i]), nbytes)
        assert got == ref


def _oracle_top2(q, t):
    n = len(q)
    bi = np.zeros(n, np.int32)
    bd = np.zeros(n, np.int32)
    sd = np.zeros(n, np.int32)
    ob.lib().oracle_hamming_top2(_p(np.ascontiguousarray(q)), len(q), _p(np.ascontiguousarray(t)),
                                 len(t), q.shape[1], _p(bi), _p(bd), _p(sd))
    return bi, bd, sd


@pytest.mark.gpu
@pytest.mark.parametrize("nq,nt,nbytes", [(1000, 1300, 32), (257, 5, 16), (600, 700, 64), (1, 1, 32),
                                          (400, 8193, 32), (300, 20000, 32)])
def test_top2_device(gpu, nq, nt, nbytes):
    """nt > 8192 takes k_top2_mfma32<false> (train index beyond the 13-bit packed key)."""
    import torch
    import mcs_amd
    L = mcs_amd.lib()
    q = _descs(nq, nbytes, 5)
    t = np.concatenate([_noisy_copy(q[:min(nq, nt) // 2], [3] * (min(nq, nt) // 2), 6),
                        _descs(nt - min(nq, nt) // 2, nbytes, 7)])
    t[-1] = t[0]  # duplicate -> exercises the tie rule
    dq = torch.from_numpy(q).cuda()
    dt = torch.from_numpy(t).cuda()
    out = [torch.zeros(nq, dtype=torch.int32, device="cuda") for _ in range(4)]
    rc = L.mcs_hamming_top2_device(dq.data_ptr(), nq, dt.data_ptr(), nt, nbytes,
                                   *[o.data_ptr() for o in out],
                                   torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    bi, bd, sd = _oracle_top2(q, t)
    assert np.array_equal(out[0].cpu().numpy(), bi)
    assert np.array_equal(out[1].cpu().numpy(), bd)
    assert np.array_equal(out[3].cpu().numpy(), sd)


@pytest.mark.gpu
def test_dense_device(gpu):
    import torch
    import mcs_amd
    a = _descs(300, 32, 8)
    b = _descs(517, 32, 9)
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    dd = torch.zeros((300, 517), dtype=torch.int16, device="cuda")
    assert mcs_amd.lib().mcs_hamming_dense_device(da.data_ptr(), 300, db.data_ptr(), 517, 32,
                                                  dd.data_ptr(), None) == 0
    torch.cuda.synchronize()
    ref = np.unpackbits(a[:, None, :] ^ b[None, :, :], axis=2).sum(2)
    assert np.array_equal(dd.cpu().numpy().astype(np.int64), ref)


@pytest.mark.gpu
def test_top2_batch_ragged(gpu):
    import torch
    import mcs_amd
    cap, nb = 700, 32
    counts = np.array([700, 5, 0, 333], np.int32)
    sets = np.zeros((4, cap, nb), np.uint8)
    for s in range(4):
        sets[s, :counts[s]] = _descs(counts[s], nb, 20 + s)
    pairs = np.array([[0, 3], [3, 0], [1, 0], [2, 3], [3, 2]], np.int32)
    d = torch.from_numpy(sets).cuda()
    dc = torch.from_numpy(counts).cuda()
    dp = torch.from_numpy(pairs).cuda()
    out = [torch.full((len(pairs), cap), -7, dtype=torch.int32, device="cuda") for _ in range(4)]
    rc = mcs_amd.lib().mcs_hamming_top2_batch_device(d.data_ptr(), dc.data_ptr(), dp.data_ptr(),
                                                     len(pairs), cap, nb,
                                                     *[o.data_ptr() for o in out], None)
    assert rc == 0
    torch.cuda.synchronize()
    for p, (qs, ts) in enumerate(pairs):
        nq = counts[qs]
        bi, bd, sd = _oracle_top2(sets[qs, :nq], sets[ts, :counts[ts]])
        assert np.array_equal(out[0][p, :nq].cpu().numpy(), bi)
        assert np.array_equal(out[1][p, :nq].cpu().numpy(), bd)
        assert np.array_equal(out[3][p, :nq].cpu().numpy(), sd)


def _tri_problem(seed, n1=1500, n2=1400, ncams=3, nbytes=32):
    rng = np.random.default_rng(seed)
    d1 = _descs(n1, nbytes, seed)
    nm = min(n1, n2) // 2
    perm = rng.permutation(n2)
    d2 = _descs(n2, nbytes, seed + 1)
    d2[perm[:nm]] = _noisy_copy(d1[:nm], rng.integers(0, 40, nm), seed + 2)
    cam1 = rng.integers(0, ncams, n1).astype(np.int32)
    cam2 = rng.integers(0, ncams, n2).astype(np.int32)
    cam2[perm[:nm]] = cam1[:nm]
    has1 = (rng.random(n1) < 0.1).astype(np.uint8)
    has2 = (rng.random(n2) < 0.1).astype(np.uint8)
    r1 = rng.normal(size=(n1, 3))
    r1 /= np.linalg.norm(r1, axis=1, keepdims=True)
    r2 = rng.normal(size=(n2, 3))
    r2 /= np.linalg.norm(r2, axis=1, keepdims=True)
    E = rng.normal(size=(ncams, ncams, 3, 3))
    return d1, d2, cam1, cam2, has1, has2, r1, r2, E


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_search_for_triangulation_raw(gpu, seed):
    import mcs_amd
    d1, d2, cam1, cam2, has1, has2, r1, r2, E = _tri_problem(seed)
    thresh = 0.3
    ref = np.zeros(len(d1), np.int32)
    nref = ob.lib().oracle_search_for_triangulation_raw(
        _p(d1), len(d1), _p(d2), len(d2), 32, _p(cam1), _p(cam2), _p(has1), _p(has2),
        _p(np.ascontiguousarray(r1)), _p(np.ascontiguousarray(r2)),
        _p(np.ascontiguousarray(E)), thresh, 3, _p(ref))
    got = np.zeros(len(d1), np.int32)
    nm = ctypes.c_int32()
    rc = mcs_amd.lib().mcs_search_for_triangulation_raw(
        _p(d1), _p(cam1), _p(has1), _p(np.ascontiguousarray(r1)), len(d1),
        _p(d2), _p(cam2), _p(has2), _p(np.ascontiguousarray(r2)), len(d2), 3,
        _p(np.ascontiguousarray(E)), 32, 64, thresh, _p(got), ctypes.byref(nm))
    assert rc == 0
    assert nref > 50
    assert nm.value == nref
    assert np.array_equal(got, ref)


def _oracle_tri(d1, d2, cam1, cam2, has1, has2, r1, r2, E, thresh, m1=None, m2=None):
    ref = np.zeros(len(d1), np.int32)
    nb = d1.shape[1]
    n = ob.lib().oracle_search_for_triangulation_raw_ex(
        _p(d1), None if m1 is None else _p(m1), len(d1), _p(d2), None if m2 is None else _p(m2),
        len(d2), nb, _p(cam1), _p(cam2), _p(has1), _p(has2), _p(np.ascontiguousarray(r1)),
        _p(np.ascontiguousarray(r2)), _p(np.ascontiguousarray(E)), thresh, E.shape[0], _p(ref))
    return n, ref


def _masks(n, nbytes, seed, keep=0.8):
    bits = (np.random.default_rng(seed).random((n, nbytes * 8)) < keep).astype(np.uint8)
    return np.packbits(bits, axis=1)


def test_triangulation_rejects_oversized_train(built):
    """KF2 must hold fewer than 2^19 keypoints (LDS vbMatched2 bitmap of the device search); the check
    runs before any buffer is touched or a device is needed."""
    import mcs_amd
    got = np.zeros(4, np.int32)
    nm = ctypes.c_int32()
    rc = mcs_amd.lib().mcs_search_for_triangulation_raw(
        None, None, None, None, 4, None, None, None, None, 1 << 19, 3, None, 32, 64, 0.3, _p(got),
        ctypes.byref(nm))
    assert rc == -1 and np.all(got == -1) and nm.value == 0
    rc = mcs_amd.lib().mcs_search_for_triangulation_raw_masked(
        None, None, None, None, None, 4, None, None, None, None, None, 1 << 19, 3, None, 32, 32,
        0.3, _p(got), ctypes.byref(nm))
    assert rc == -1


def test_oracle_triangulation_unmasked_entry_agrees(built):
    """The _ex oracle with no masks is the original restatement (TH_LOW = 2 * featDim)."""
    d1, d2, cam1, cam2, has1, has2, r1, r2, E = _tri_problem(3, n1=300, n2=280)
    n_ex, ref_ex = _oracle_tri(d1, d2, cam1, cam2, has1, has2, r1, r2, E, 0.3)
    ref = np.zeros(len(d1), np.int32)
    n = ob.lib().oracle_search_for_triangulation_raw(
        _p(d1), len(d1), _p(d2), len(d2), 32, _p(cam1), _p(cam2), _p(has1), _p(has2),
        _p(np.ascontiguousarray(r1)), _p(np.ascontiguousarray(r2)), _p(np.ascontiguousarray(E)),
        0.3, 3, _p(ref))
    assert n == n_ex and np.array_equal(ref, ref_ex) and n > 5


@pytest.mark.gpu
@pytest.mark.parametrize("seed,nbytes", [(0, 32), (4, 16), (5, 64)])
def test_search_for_triangulation_raw_masked(gpu, seed, nbytes):
    """havingMasks (mdBRIEF): DescriptorDistance64Masked and TH_LOW = floor(featDim)."""
    import mcs_amd
    d1, d2, cam1, cam2, has1, has2, r1, r2, E = _tri_problem(seed, n1=1200, n2=1100, nbytes=nbytes)
    m1 = _masks(len(d1), nbytes, seed + 10)
    m2 = _masks(len(d2), nbytes, seed + 11)
    thresh = 0.3
    nref, ref = _oracle_tri(d1, d2, cam1, cam2, has1, has2, r1, r2, E, thresh, m1, m2)
    got = np.zeros(len(d1), np.int32)
    nm = ctypes.c_int32()
    rc = mcs_amd.lib().mcs_search_for_triangulation_raw_masked(
        _p(d1), _p(m1), _p(cam1), _p(has1), _p(np.ascontiguousarray(r1)), len(d1),
        _p(d2), _p(m2), _p(cam2), _p(has2), _p(np.ascontiguousarray(r2)), len(d2), 3,
        _p(np.ascontiguousarray(E)), nbytes, nbytes, thresh, _p(got), ctypes.byref(nm))
    assert rc == 0
    assert nref > 30
    assert nm.value == nref
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_config_b_size_matching(gpu):
    """Config-B scale (2000 keypoints per frame, BASELINE configs[1]): batched top-2 between two
    2000-keypoint sets and SearchForTriangulationRaw over 2000 x 2000, both vs the oracle."""
    import torch
    import mcs_amd
    n = 2000
    rng = np.random.default_rng(77)
    a = _descs(n, 32, 70)
    b = _descs(n, 32, 71)
    perm = rng.permutation(n)
    b[perm[:n // 2]] = _noisy_copy(a[:n // 2], rng.integers(0, 30, n // 2), 72)
    sets = np.stack([a, b])
    counts = np.array([n, n], np.int32)
    pairs = np.array([[0, 1], [1, 0]], np.int32)
    d = torch.from_numpy(sets).cuda()
    dc = torch.from_numpy(counts).cuda()
    dp = torch.from_numpy(pairs).cuda()
    out = [torch.zeros((2, n), dtype=torch.int32, device="cuda") for _ in range(4)]
    rc = mcs_amd.lib().mcs_hamming_top2_batch_device(d.data_ptr(), dc.data_ptr(), dp.data_ptr(),
                                                     2, n, 32, *[o.data_ptr() for o in out], None)
    assert rc == 0
    torch.cuda.synchronize()
    for p, (qs, ts) in enumerate(pairs):
        bi, bd, sd = _oracle_top2(sets[qs], sets[ts])
        assert np.array_equal(out[0][p].cpu().numpy(), bi)
        assert np.array_equal(out[1][p].cpu().numpy(), bd)
        assert np.array_equal(out[3][p].cpu().numpy(), sd)
    d1, d2, cam1, cam2, has1, has2, r1, r2, E = _tri_problem(78, n1=n, n2=n, ncams=3)
    nref, ref = _oracle_tri(d1, d2, cam1, cam2, has1, has2, r1, r2, E, 0.3)
    got = np.zeros(n, np.int32)
    nm = ctypes.c_int32()
    rc = mcs_amd.lib().mcs_search_for_triangulation_raw(
        _p(d1), _p(cam1), _p(has1), _p(np.ascontiguousarray(r1)), n,
        _p(d2), _p(cam2), _p(has2), _p(np.ascontiguousarray(r2)), n, 3,
        _p(np.ascontiguousarray(E)), 32, 64, 0.3, _p(got), ctypes.byref(nm))
    assert rc == 0 and nm.value == nref and np.array_equal(got, ref) and nref > 100


def _tri_problem_shared(seed, n1=900, n2=1000, ncams=2, nbytes=32):
    """Queries that compete for the same KF2 keypoints (the order-dependent vbMatched2 greedy):
    KF1 and KF2 hold noisy copies of a few base descriptors, and queries 0..3 have more
    candidates than the device keeps per query (the rescan path)."""
    rng = np.random.default_rng(seed)
    bases = _descs(12, nbytes, seed + 100)
    d1 = _descs(n1, nbytes, seed)
    d2 = _descs(n2, nbytes, seed + 1)
    pick1 = rng.integers(0, 12, 400)
    d1[:400] = _noisy_copy(bases[pick1], rng.integers(0, 14, 400), seed + 2)
    pick2 = rng.integers(0, 12, 500)
    d2[:500] = _noisy_copy(bases[pick2], rng.integers(0, 14, 500), seed + 3)
    d1[:4] = bases[0]
    d2[500:650] = _noisy_copy(np.repeat(bases[:1], 150, 0), rng.integers(0, 10, 150), seed + 4)
    cam1 = rng.integers(0, ncams, n1).astype(np.int32)
    cam2 = rng.integers(0, ncams, n2).astype(np.int32)
    cam1[:4] = 0
    cam2[500:650] = 0
    has1 = (rng.random(n1) < 0.05).astype(np.uint8)
    has1[:4] = 0
    has2 = (rng.random(n2) < 0.05).astype(np.uint8)
    r1 = rng.normal(size=(n1, 3))
    r1 /= np.linalg.norm(r1, axis=1, keepdims=True)
    r2 = rng.normal(size=(n2, 3))
    r2 /= np.linalg.norm(r2, axis=1, keepdims=True)
    E = rng.normal(size=(ncams, ncams, 3, 3))
    return d1, d2, cam1, cam2, has1, has2, r1, r2, E


def _run_tri_device(ws, d1, d2, cam1, cam2, has1, has2, r1, r2, E, nbytes, th, thresh, m1=None, m2=None):
    import torch
    import mcs_amd
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    bufs = [dev(x) for x in (d1, cam1, has1, r1, d2, cam2, has2, r2, E)]
    mb = [dev(m) for m in (m1, m2)] if m1 is not None else [None, None]
    out = torch.full((len(d1),), -9, dtype=torch.int32, device="cuda")
    n = torch.full((1,), -9, dtype=torch.int32, device="cuda")
    ptr = lambda t: None if t is None else t.data_ptr()
    rc = mcs_amd.lib().mcs_search_for_triangulation_raw_device(
        ws, ptr(bufs[0]), ptr(mb[0]), ptr(bufs[1]), ptr(bufs[2]), ptr(bufs[3]), len(d1),
        ptr(bufs[4]), ptr(mb[1]), ptr(bufs[5]), ptr(bufs[6]), ptr(bufs[7]), len(d2), E.shape[0],
        ptr(bufs[8]), nbytes, th, thresh, out.data_ptr(), n.data_ptr(),
        torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    return int(n.item()), out.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,masked", [(0, False), (1, False), (2, True)])
def test_triangulation_device_shared_candidates(gpu, seed, masked):
    """The device-resident entry on queries that compete for KF2 keypoints (the vbMatched2
    greedy order matters) and on queries with more candidates than a slot holds, vs the oracle;
    the host entry on the same input agrees too."""
    import mcs_amd
    nbytes = 32
    d1, d2, cam1, cam2, has1, has2, r1, r2, E = _tri_problem_shared(seed)
    m1 = _masks(len(d1), nbytes, seed + 10, keep=0.9) if masked else None
    m2 = _masks(len(d2), nbytes, seed + 11, keep=0.9) if masked else None
    th = nbytes if masked else 2 * nbytes
    thresh = 0.3
    nref, ref = _oracle_tri(d1, d2, cam1, cam2, has1, has2, r1, r2, E, thresh, m1, m2)
    assert nref > 50
    # the problem really exercises both device paths: shared candidates and slot overflow
    dist = np.unpackbits(d1[:4, None, :] ^ d2[None, :, :], axis=2).sum(2)
    assert int(((dist <= th) & (cam2[None, :] == 0) & (has2[None, :] == 0)).sum(1).max()) > 64
    L = mcs_amd.lib()
    ws = ctypes.c_void_p()
    assert L.mcs_tri_workspace_create(0, len(d1), len(d2), ctypes.byref(ws)) == 0
    try:
        n, got = _run_tri_device(ws, d1, d2, cam1, cam2, has1, has2, r1, r2, E, nbytes, th, thresh, m1, m2)
        assert n == nref and np.array_equal(got, ref)
        # a second call on the same workspace (state fully reset per call)
        n, got = _run_tri_device(ws, d1, d2, cam1, cam2, has1, has2, r1, r2, E, nbytes, th, thresh, m1, m2)
        assert n == nref and np.array_equal(got, ref)
    finally:
        L.mcs_tri_workspace_destroy(ws)
    got = np.zeros(len(d1), np.int32)
    nm = ctypes.c_int32()
    if masked:
        rc = L.mcs_search_for_triangulation_raw_masked(
            _p(d1), _p(m1), _p(cam1), _p(has1), _p(np.ascontiguousarray(r1)), len(d1),
            _p(d2), _p(m2), _p(cam2), _p(has2), _p(np.ascontiguousarray(r2)), len(d2), E.shape[0],
            _p(np.ascontiguousarray(E)), nbytes, th, thresh, _p(got), ctypes.byref(nm))
    else:
        rc = L.mcs_search_for_triangulation_raw(
            _p(d1), _p(cam1), _p(has1), _p(np.ascontiguousarray(r1)), len(d1),
            _p(d2), _p(cam2), _p(has2), _p(np.ascontiguousarray(r2)), len(d2), E.shape[0],
            _p(np.ascontiguousarray(E)), nbytes, th, thresh, _p(got), ctypes.byref(nm))
    assert rc == 0 and nm.value == nref and np.array_equal(got, ref)


@pytest.mark.gpu
def test_triangulation_device_capacity_errors(gpu):
    import mcs_amd
    L = mcs_amd.lib()
    ws = ctypes.c_void_p()
    assert L.mcs_tri_workspace_create(0, 10, 1 << 19, ctypes.byref(ws)) == -1
    assert L.mcs_tri_workspace_create(0, 10, 20, ctypes.byref(ws)) == 0
    try:
        n = np.zeros(1, np.int32)
        rc = L.mcs_search_for_triangulation_raw_device(ws, None, None, None, None, None, 11, None, None, None,
                                                       None, None, 5, 1, None, 32, 64, 0.3, None, _p(n), None)
        assert rc == -2 and b"capacity" in L.mcs_last_error()
    finally:
        L.mcs_tri_workspace_destroy(ws)
