"""g2o's solver control and robust kernel, pinned to the reference TEXT.

tests/golden/g2o_solver.npz holds literal evaluations of the reference's
SparseOptimizer::optimize, OptimizationAlgorithmLevenberg (ctor, solve, computeLambdaInit,
computeScale), SparseOptimizerTerminateAction and RobustKernelHuber, translated statement by
statement from ThirdParty/g2o/g2o/core/*.cpp by tests/golden/gen_g2o_solver.py and run on 60
scripted scenarios (446 LM trials: accepted and rejected steps, failed solves, rho == 0, ten
failures in a row, stalls that trip Raul's nBad stop and the terminate action's gain test).

The product's device code is replayed on the same scripted inputs through test hooks that call
the production device functions (mcs_ba_lm_replay -> lm_start_body / lm_lambda0_body /
lm_control, mcs_ba_huber_eval -> huber, csrc/ba.hip) and must reproduce every lambda, nu and
accept / reject decision bit for bit, the number of trials and iterations each optimize() call
runs, the terminate action's stop flag, and the Huber rho / rho' values.
"""
import ctypes
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "g2o_solver.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_golden_structure(gold):
    """The reference keeps Huber's delta^2 in a float member (robust_kernel_impl.h), and its
    Huber values reflect that: at e = (double)delta^2 just above the float threshold the
    kernel already robustifies (or not) as the float comparison says."""
    assert int(gold["huber_dsqr_is_float"]) == 1
    e, d, r0, r1 = gold["huber_e"], gold["huber_delta"], gold["huber_rho0"], gold["huber_rho1"]
    f2 = (d * d).astype(np.float32).astype(np.float64)
    inl = e <= f2
    assert np.array_equal(r0[inl], e[inl]) and np.all(r1[inl] == 1.0)
    out = ~inl
    assert np.array_equal(r1[out], d[out] / np.sqrt(e[out]))
    assert np.array_equal(r0[out], 2 * np.sqrt(e[out]) * d[out] - f2[out])
    # computeScale = sum_j x_j (lambda x_j + b_j) in index order
    x, b, lam = gold["scale_x"], gold["scale_b"], float(gold["scale_lambda"])
    s = 0.0
    for j in range(len(x)):
        s += x[j] * (lam * x[j] + b[j])
    assert s == float(gold["scale_value"])
    meta = gold["lm_meta"]
    assert int(meta[:, 0].sum()) == 446 and np.any(meta[:, 2] == 1) and np.any(meta[:, 2] == 0)


@pytest.mark.gpu
def test_gpu_lm_control_replays_reference(gpu, gold):
    import mcs_amd
    from mcs_amd import ba
    L = mcs_amd.lib()
    ins, trials, outs, meta = gold["lm_in"], gold["lm_trials"], gold["lm_out"], gold["lm_meta"]
    for s in range(len(ins)):
        n_ref, it_ref, stop_ref, max_it = (int(v) for v in meta[s])
        o = ba.BAOptions(max_iterations=max_it, gain_threshold=1e-6, terminate_max_iter=15,
                         max_trials=10, tau=1e-5)
        tr = np.ascontiguousarray(trials[s])
        out = np.zeros((len(tr), 10))
        n = ctypes.c_int32()
        rc = L.mcs_ba_lm_replay(0, ctypes.byref(o), ba._p(np.ascontiguousarray(ins[s])), ba._p(tr), len(tr),
                                ba._p(out), ctypes.byref(n))
        assert rc == 0
        assert n.value == n_ref, s
        ref = outs[s][:n_ref]
        got = out[:n_ref]
        assert np.array_equal(got[:, 0], ref[:, 0]), (s, "lambda used")
        assert np.array_equal(got[:, 1], ref[:, 1]), (s, "lambda after")
        assert np.array_equal(got[:, 2], ref[:, 2]), (s, "nu")
        assert np.array_equal(got[:, 3], ref[:, 3]), (s, "accept / reject")
        assert int(got[-1, 6]) == it_ref, (s, "iterations")
        assert int(got[-1, 7]) == 1, (s, "done")
        assert int(got[-1, 8]) == stop_ref, (s, "terminate action stop flag")


@pytest.mark.gpu
def test_gpu_huber_matches_reference(gpu, gold):
    import mcs_amd
    from mcs_amd import ba
    L = mcs_amd.lib()
    e, d = gold["huber_e"], gold["huber_delta"]
    for delta in np.unique(d):
        sel = d == delta
        ee = np.ascontiguousarray(e[sel])
        r0, r1 = np.zeros(len(ee)), np.zeros(len(ee))
        assert L.mcs_ba_huber_eval(0, ba._p(ee), len(ee), float(delta), ba._p(r0), ba._p(r1)) == 0
        assert np.array_equal(r0, gold["huber_rho0"][sel]), delta
        assert np.array_equal(r1, gold["huber_rho1"][sel]), delta


SCHUR = os.path.join(HERE, "golden", "g2o_schur.npz")


def test_schur_golden_structure():
    """g2o_schur.npz: the per-landmark block of BlockSolver::solve (block_solver.hpp:381-403)
    in Eigen 3.2.10's order (tests/golden/gen_g2o_schur.py).  The cofactor table parsed from
    Eigen's Inverse.h: row 0 holds the column-0 cofactors, entry (r, c) otherwise cofactor(c, r);
    and the determinant's c0 + (c1 + c2) differs from (c0 + c1) + c2 in some blocks, so the
    fixture does tell the two orders apart."""
    g = np.load(SCHUR)
    assert sorted(map(tuple, g["table"].tolist())) == [(r, c, c, r) for r in range(3) for c in range(3)]
    H, lam = g["H"].reshape(-1, 3, 3), float(g["lam"])
    differ = 0
    for t in range(len(H)):
        m = H[t].tolist()
        for i in range(3):
            m[i][i] += lam
        cof = lambda i, j: (m[(i + 1) % 3][(j + 1) % 3] * m[(i + 2) % 3][(j + 2) % 3]
                            - m[(i + 1) % 3][(j + 2) % 3] * m[(i + 2) % 3][(j + 1) % 3])
        p = [cof(k, 0) * m[k][0] for k in range(3)]
        differ += (p[0] + (p[1] + p[2])) != ((p[0] + p[1]) + p[2])
        assert g["Dinv"][t, 0] == cof(0, 0) * (1.0 / (p[0] + (p[1] + p[2])))
    assert differ > 10


@pytest.mark.gpu
def test_gpu_point_block_matches_reference_order(gpu):
    """The product's device Dinv / db / Y helpers (the ones k_build_trial and k_point_trial run)
    reproduce the per-landmark block of the reference's BlockSolver::solve bit for bit."""
    import mcs_amd
    from mcs_amd import ba
    g = np.load(SCHUR)
    n = len(g["H"])
    Dinv, db, Y = np.zeros((n, 9)), np.zeros((n, 3)), np.zeros((n, 18))
    rc = mcs_amd.lib().mcs_ba_point_block_eval(0, ba._p(np.ascontiguousarray(g["H"])), float(g["lam"]),
                                               ba._p(np.ascontiguousarray(g["b"])),
                                               ba._p(np.ascontiguousarray(g["hpl"])), n, ba._p(Dinv),
                                               ba._p(db), ba._p(Y))
    assert rc == 0
    assert np.array_equal(Dinv, g["Dinv"])
    assert np.array_equal(db, g["db"])
    assert np.array_equal(Y, g["Y"])
