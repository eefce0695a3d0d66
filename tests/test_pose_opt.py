"""cOptimizer::PoseOptimization (src/cOptimizer.cpp:264-486): one MultiFrame pose vertex, map
points fixed (:382), Mc / IO fixed, Huber delta 1.345 * huberMultiplier (:344), information
invSigma2(octave) (:405-406), two optimize(10) rounds with outlier classification
(chi2 > delta^2) after each (:432-474).

g2o detail reproduced: no force-stop flag is set, so SparseOptimizerTerminateAction keeps its
own auxiliary flag installed (sparse_optimizer_terminate_action.cpp:64-72) -- once it stops
round 1, round 2 runs zero iterations.  The same persistence applies to LocalBundleAdjustment
called with pbStopFlag == NULL (src/cOptimizer.cpp:773-826).

Tolerances as tests/test_ba.py: identical iteration counts, outlier sets and inlier counts;
per-iteration robust chi2 rel 1e-6; pose abs 1e-8 (one 6x6 system per trial).
Parity unpinned against a reference binary (g2o + OpenCV not buildable here).
"""
import numpy as np
import pytest

from tests import oracle_bind as ob


@pytest.fixture(scope="module", params=[0, 1, 2])
def pproblem(request):
    from mcs_amd import ba
    return ba.make_pose_problem(seed=request.param)


def _converged_problem():
    from mcs_amd import ba
    return ba.make_pose_problem(seed=5, outlier_frac=0.0, noise_scale=0.05,
                                pose_noise=(1e-4, 1e-4))


def test_pose_problem_shape(pproblem):
    assert len(pproblem["poses"]) == 1 and pproblem["pose_fixed"][0] == 0
    assert np.all(pproblem["edge_pose"] == 0) and len(pproblem["edge_pose"]) > 200
    assert pproblem["edge_point"].max() == len(pproblem["points"]) - 1


def test_oracle_pose_optimization_improves_pose(pproblem):
    o = ob.pose_optimization(pproblem)
    gt = pproblem["gt_pose"]
    assert np.abs(o["pose"] - gt).max() < 0.5 * np.abs(pproblem["poses"][0] - gt).max()
    n = len(pproblem["edge_pose"])
    assert o["n_good"] + int(o["outlier"].sum()) == n
    assert abs(o["bad_ratio"] - o["outlier"].mean()) < 1e-12
    assert o["report1"].iterations >= 1


def test_oracle_aux_terminate_flag_persists():
    o = ob.pose_optimization(_converged_problem())
    # the terminate action stopped round 1 through its own flag; round 2 does nothing
    assert o["report1"].stop_flag == 1 and o["report2"].iterations == 0


def test_oracle_local_ba_null_stop_flag():
    from mcs_amd import ba
    pr = ba.make_problem(n_local=3, n_fixed=1, n_points=300, target_edges=2000, seed=5,
                         outlier_frac=0.02, noise_scale=0.05, pose_noise=(1e-3, 1e-3),
                         point_noise=1e-3)
    o = ob.local_ba(pr, stop_flag=None)
    assert o["write_back"] == 1
    if o["report1"].stop_flag:
        assert o["report2"].iterations == 0
    # with a caller flag the same convergence ends the call after round 1 (bDoMore = false)
    o2 = ob.local_ba(pr, stop_flag=0)
    if o2["stop_flag"]:
        assert o2["write_back"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("mult", [1.0, 2.0])
def test_gpu_pose_optimization_matches_oracle(gpu, pproblem, mult):
    from mcs_amd import ba
    pr = dict(pproblem)
    pr["huber_delta"] = 1.345 * mult
    g = ba.Solver().pose_optimization(pr, trace=20)
    o = ob.pose_optimization(pr, trace=20)
    assert g["report1"].iterations == o["report1"].iterations
    assert g["report2"].iterations == o["report2"].iterations
    assert np.allclose(g["trace1"], o["trace1"], rtol=1e-6)
    assert np.array_equal(g["outlier"], o["outlier"])
    assert g["n_good"] == o["n_good"] and abs(g["bad_ratio"] - o["bad_ratio"]) < 1e-15
    assert np.abs(g["pose"] - o["pose"]).max() < 1e-8


@pytest.mark.gpu
def test_gpu_pose_optimization_aux_flag(gpu):
    from mcs_amd import ba
    pr = _converged_problem()
    g = ba.Solver().pose_optimization(pr)
    o = ob.pose_optimization(pr)
    assert g["report1"].stop_flag == o["report1"].stop_flag == 1
    assert g["report2"].iterations == o["report2"].iterations == 0
    assert np.abs(g["pose"] - o["pose"]).max() < 1e-8


@pytest.mark.gpu
def test_gpu_local_ba_null_stop_flag_matches_oracle(gpu):
    from mcs_amd import ba
    pr = ba.make_problem(n_local=3, n_fixed=1, n_points=300, target_edges=2000, seed=5,
                         outlier_frac=0.02, noise_scale=0.05, pose_noise=(1e-3, 1e-3),
                         point_noise=1e-3)
    g = ba.Solver().local_ba(pr, stop_flag=None)
    o = ob.local_ba(pr, stop_flag=None)
    assert g["write_back"] == o["write_back"]
    assert g["report1"].iterations == o["report1"].iterations
    assert g["report2"].iterations == o["report2"].iterations
    assert np.array_equal(g["edge_inlier"], o["edge_inlier"])
    assert np.abs(g["poses"] - o["poses"]).max() < 1e-6
