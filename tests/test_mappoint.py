"""Map-point refresh after the LocalBA write-back (src/cOptimizer.cpp:885-902), batched on the
device (include/mcs_mappoint.h), against the oracle's literal restatements:

  ComputeDistinctiveDescriptors  src/cMapPoint.cpp:297-390 -- exact (integer distances, the
      upper-triangle-row median quirk: row i only sees j > i, row N-1 never counts, N <= 2 -> 0)
  UpdateNormalAndDepth           src/cMapPoint.cpp:453-496 -- bitwise (the same correctly
      rounded + - * / sqrt in the reference's order)
"""
import ctypes

import numpy as np
import pytest

from tests import oracle_bind as ob


def _descs(n, nb, seed):
    return np.random.default_rng(seed).integers(0, 256, (n, nb), dtype=np.uint8)


def _observations(counts, nrows, seed):
    rng = np.random.default_rng(seed)
    ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    rows = rng.integers(0, nrows, int(ptr[-1])).astype(np.int32)
    return ptr, rows


def _oracle_distinctive(desc, masks, nb, ptr, rows):
    best = np.zeros(len(ptr) - 1, np.int32)
    ob.lib().oracle_distinctive_descriptors(ob._p(desc), ob._p(masks), nb, ob._p(ptr), ob._p(rows),
                                            len(ptr) - 1, ob._p(best))
    return best


def test_oracle_median_quirk_by_hand(built):
    """N = 4 descriptors 0, A, B, C: row 0 sees {d01, d02, d03} (median = 2nd smallest), row 1
    {d12, d13} (median = the larger), row 2 {d23}; row 3 is never a candidate."""
    nb = 32
    base = np.zeros((4, nb), np.uint8)
    base[1, :2] = 0xFF     # d01 = 16
    base[2, :1] = 0xFF     # d02 = 8, d12 = 8
    base[3, 2:5] = 0xFF    # d03 = 24, d13 = 40, d23 = 32
    ptr = np.array([0, 4], np.int32)
    rows = np.arange(4, dtype=np.int32)
    # medians: row 0 -> sorted (8, 16, 24)[1] = 16; row 1 -> (8, 40)[1] = 40; row 2 -> 32
    assert _oracle_distinctive(base, None, nb, ptr, rows)[0] == 0
    base[3] = base[2]      # now d23 = 0: row 2's median 0 wins
    assert _oracle_distinctive(base, None, nb, ptr, rows)[0] == 2
    for n in (0, 1, 2):    # N <= 2 -> index 0, N = 0 -> nothing (-1)
        assert _oracle_distinctive(base, None, nb, np.array([0, n], np.int32), rows[:n])[0] == \
            (-1 if n == 0 else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("nb,masked", [(32, False), (16, False), (64, False), (32, True)])
def test_gpu_distinctive_descriptors(gpu, nb, masked):
    import torch
    import mcs_amd
    # clustered descriptors (a few prototypes + noise) so medians differ and ties occur
    rng = np.random.default_rng(nb + 7 * masked)
    proto = _descs(40, nb, 11)
    nrows = 4000
    pick = rng.integers(0, 40, nrows)
    flips = rng.random((nrows, nb * 8)) < rng.choice([0.02, 0.1, 0.3], nrows)[:, None]
    desc = proto[pick] ^ np.packbits(flips, axis=1)
    masks = (_descs(nrows, nb, 5) | _descs(nrows, nb, 6)) if masked else None
    counts = np.concatenate([[0, 1, 2, 3, 4, 5, 63, 64, 65, 130, 200],
                             rng.integers(2, 30, 500)])
    ptr, rows = _observations(counts, nrows, 3)
    ref = _oracle_distinctive(desc, masks, nb, ptr, rows)
    dev = torch.device("cuda", 0)
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    d_desc = torch.from_numpy(desc).to(dev)
    d_mask = torch.from_numpy(masks).to(dev) if masked else None
    d_ptr, d_rows = torch.from_numpy(ptr).to(dev), torch.from_numpy(rows).to(dev)
    n = len(counts)
    d_best = torch.full((n,), -7, dtype=torch.int32, device=dev)
    d_od = torch.zeros((n, nb), dtype=torch.uint8, device=dev)
    d_om = torch.zeros((n, nb), dtype=torch.uint8, device=dev)
    rc = mcs_amd.lib().mcs_distinctive_descriptors_device(P(d_desc), P(d_mask), nb, P(d_ptr), P(d_rows),
                                                          n, P(d_best), P(d_od), P(d_om), None)
    assert rc == 0
    torch.cuda.synchronize()
    best = d_best.cpu().numpy()
    assert np.array_equal(best, ref)
    od = d_od.cpu().numpy()
    for p in range(n):
        if ref[p] >= 0:
            assert np.array_equal(od[p], desc[rows[ptr[p] + ref[p]]]), p
            if masked:
                assert np.array_equal(d_om[p].cpu().numpy(), masks[rows[ptr[p] + ref[p]]]), p
        else:
            assert not od[p].any()


@pytest.mark.gpu
def test_gpu_update_normal_depth(gpu):
    import torch
    import mcs_amd
    rng = np.random.default_rng(21)
    n, nkf, nlev = 3000, 40, 8
    pts = rng.normal(0, 3, (n, 3))
    kfc = rng.normal(0, 1, (nkf, 3))
    counts = rng.integers(0, 9, n)
    counts[:3] = [0, 1, 2]
    ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    obs = rng.integers(0, nkf, int(ptr[-1])).astype(np.int32)
    ref = rng.integers(0, nkf, n).astype(np.int32)
    lvl = rng.integers(-1, nlev, n).astype(np.int32)
    sf = float(np.float32(1.2))
    scale = np.cumprod([1.0] + [sf] * (nlev - 1))          # mvScaleFactors
    on, omin, omax = np.zeros((n, 3)), np.zeros(n), np.zeros(n)
    ob.lib().oracle_update_normal_depth(ob._p(pts), n, ob._p(ptr), ob._p(obs), ob._p(kfc), ob._p(ref),
                                        ob._p(lvl), ob._p(scale), nlev, ob._p(on), ob._p(omin), ob._p(omax))
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    d = [T(pts), T(ptr), T(obs), T(kfc), T(ref), T(lvl), T(scale)]
    dn = torch.zeros((n, 3), dtype=torch.float64, device=dev)
    dmin = torch.zeros(n, dtype=torch.float64, device=dev)
    dmax = torch.zeros(n, dtype=torch.float64, device=dev)
    rc = mcs_amd.lib().mcs_update_normal_depth_device(P(d[0]), n, P(d[1]), P(d[2]), P(d[3]), P(d[4]),
                                                      P(d[5]), P(d[6]), nlev, P(dn), P(dmin), P(dmax), None)
    assert rc == 0
    torch.cuda.synchronize()
    assert np.array_equal(dn.cpu().numpy(), on)
    assert np.array_equal(dmin.cpu().numpy(), omin)
    assert np.array_equal(dmax.cpu().numpy(), omax)
    assert not dn[0].any().item()   # no observation: untouched
