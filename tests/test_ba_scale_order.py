"""computeScale's summation order (the product sums the poses' and the points' parts
of the model decrease separately, g2o sums the whole update vector in one index-order loop).

g2o: OptimizationAlgorithmLevenberg::computeScale
(/root/reference/ThirdParty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:182-189),
scale = sum_j x_j (lambda x_j + b_j), then rho = (currentChi - tempChi) / (scale + 1e-3)
(:128-131).  The product (csrc/ba.hip lm_control) adds a poses' partial sum and a points'
partial sum, each reduced in parallel.

The bound (stated in DESIGN.md §3.5): every summation order of n terms t_j lands within
gamma_{n-1} * sum|t_j| of the exact sum (gamma_k = k u / (1 - k u), u = 2^-53), so two orders
differ by at most 2 gamma * sum|t_j|.  If scale + 1e-3 exceeds that, the denominator is positive
in EVERY order, so sign(rho) = sign(currentChi - tempChi) in every order and the three branches
of :134 (rho > 0), :151 (rho < 0) and :160 (rho == 0) are order-independent; only the VALUE of
rho moves, by a relative amount <= 2 gamma sum|t| / (scale + 1e-3), which enters lambda through
alpha = 1 - (2 rho - 1)^3 (:135) and nothing else.

The test records every LM trial of the oracle (which sums in g2o's index order) on config C
(LocalBA, three seeds) and a small config E (GlobalBA) and checks, per trial:
  * the margin: scale + 1e-3 > 2 gamma sum|t|  (branches identical in every order);
  * the split order the product uses is inside the bound;
  * the relative rho perturbation is <= 1e-9.
"""
import ctypes

import numpy as np
import pytest

from tests import oracle_bind as ob

U = 2.0 ** -53


def _gamma(n):
    return n * U / (1 - n * U)


def _trials(run):
    ob.scale_trace(True)
    try:
        run()
        return ob.scale_trace_read()
    finally:
        ob.scale_trace(False)


def _check(tr, what):
    assert len(tr) > 0, what
    d, s, split, sabs, n, lam = tr.T
    g = np.array([_gamma(int(k)) for k in n])
    bound = 2 * g * sabs
    # mathematically scale = 2 lambda |x|^2 + x^T H x >= 0 (g2o adds lambda to H's diagonal)
    assert np.all(s + 1e-3 > bound), "%s: a trial where the summation order could flip rho's sign" % what
    assert np.all(np.abs(split - s) <= bound), "%s: split order outside the bound" % what
    rel = bound / (s + 1e-3)
    assert rel.max() <= 1e-9, "%s: rho perturbation %.3g" % (what, rel.max())
    # the branch inputs: sign(rho) is sign(currentChi - tempChi) in both orders
    assert np.array_equal(np.sign(d / (s + 1e-3)), np.sign(d / (split + 1e-3))), what
    return rel.max(), int(len(tr))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_localba_scale_order_bound(seed):
    from mcs_amd import ba
    pr = ba.make_problem(seed=seed)
    tr = _trials(lambda: ob.local_ba(pr))
    rel, n = _check(tr, "config C seed %d" % seed)
    assert n >= 5


def test_globalba_scale_order_bound():
    from mcs_amd import ba
    pr = ba.make_global_problem(n_kf=24, n_points=3000, target_edges=24000, ncams=8, seed=1)
    L = ob.lib()
    f = L.oracle_global_ba
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32] + [ctypes.c_void_p] * 4
    s = ba.as_struct(pr)
    poses, points = pr["poses"].copy(), pr["points"].copy()
    rep = ba.BAReport()
    sf = ctypes.c_int32(0)
    tr = _trials(lambda: f(ctypes.byref(s), 0, ob._p(poses), ob._p(points), ctypes.byref(sf),
                           ctypes.byref(rep)))
    _check(tr, "config E small")


def test_bound_detects_a_fragile_trial():
    """The check is not vacuous: terms that cancel to below 1e-3 of their magnitude sum fail."""
    t = np.array([1e12, -1e12, 1e-4])
    tr = np.array([[1.0, t.sum(), t.sum(), np.abs(t).sum(), 3, 1.0]])
    with pytest.raises(AssertionError):
        _check(tr, "synthetic")
