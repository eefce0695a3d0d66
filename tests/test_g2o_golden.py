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
