"""Global BA (cOptimizer::BundleAdjustment, src/cOptimizer.cpp:73-261), the dense reduced-camera
LDL^T (LinearSolverEigen::solve, ThirdParty/g2o/g2o/solvers/linear_solver_eigen.h:94-126) and
point-sharded BA.

Tolerances: dense solve relative residual <= 1e-10 (well-conditioned SPD); GPU vs oracle robust
chi2 per iteration rel 1e-6, poses abs 1e-6, well-constrained points abs 1e-5, identical
iteration counts (same as tests/test_ba.py).  Sharded vs unsharded: the Schur sum is
re-associated across ranks, so the same tolerances apply; every rank must hold bit-identical
poses (lock-step).
"""
import ctypes
import threading

import numpy as np
import pytest

from tests import oracle_bind as ob


@pytest.fixture(scope="module")
def gproblem():
    from mcs_amd import ba
    return ba.make_global_problem(n_kf=24, n_points=3000, target_edges=24000, ncams=8, seed=1)


def _oracle_global(pr, pose_only=False, trace=20):
    from mcs_amd import ba
    L = ob.lib()
    f = L.oracle_global_ba
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32] + [ctypes.c_void_p] * 4
    s = ba.as_struct(pr)
    poses = pr["poses"].copy()
    points = pr["points"].copy()
    tr = np.zeros(trace)
    rep = ba.BAReport(0, 0, 0, 0, 0, 0, 0, 0, ob._p(tr), trace)
    sf = ctypes.c_int32(0)
    f(ctypes.byref(s), 1 if pose_only else 0, ob._p(poses), ob._p(points), ctypes.byref(sf),
      ctypes.byref(rep))
    return dict(poses=poses, points=points, report=rep, trace=tr[:min(trace, rep.iterations)],
                stop_flag=sf.value)


def _partial_schur(pr, pose_cnt, lam, lam_diag):
    from mcs_amd import ba
    L = ob.lib()
    f = L.oracle_ba_partial_schur
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_double,
                  ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    s = ba.as_struct(pr)
    cap = 6 * len(pr["poses"])
    S = np.zeros(cap * cap)
    bs = np.zeros(cap)
    pc = None if pose_cnt is None else np.ascontiguousarray(pose_cnt, np.float64)
    n = f(ctypes.byref(s), None if pc is None else ob._p(pc), lam, lam_diag, ob._p(S), cap,
          ob._p(bs))
    assert n >= 0
    return S[:n * n].reshape(n, n), bs[:n]


def test_global_problem_shape(gproblem):
    pr = gproblem
    assert pr["pose_fixed"][0] == 1 and pr["pose_fixed"][1:].sum() == 0
    assert np.all(pr["edge_info"] == 1.0)
    assert abs(pr["huber_delta"] - np.sqrt(5.991)) < 1e-15
    cnt = np.bincount(pr["edge_point"], minlength=len(pr["points"]))
    assert cnt.min() >= 2


def test_shard_points_partition(gproblem):
    from mcs_amd import ba
    for world in (1, 2, 3, 8):
        rng = ba.shard_points(gproblem, world)
        assert rng[0][0] == 0 and rng[-1][1] == len(gproblem["points"])
        assert all(rng[i][1] == rng[i + 1][0] for i in range(world - 1))
        eids = np.concatenate([ba.shard_problem(gproblem, r, world)[2] for r in range(world)])
        assert np.array_equal(np.sort(eids), np.arange(len(gproblem["edge_pose"])))


def test_oracle_global_ba_converges(gproblem):
    o = _oracle_global(gproblem)
    assert o["report"].chi2_final < o["report"].chi2_initial and o["report"].iterations >= 2
    assert o["report"].n_active_poses == len(gproblem["poses"]) - 1
    po = _oracle_global(gproblem, pose_only=True)
    assert po["report"].n_active_points == 0
    assert np.array_equal(po["points"], gproblem["points"])
    # edges whose every vertex is fixed (keyframe 0 + fixed points) are not active
    n0 = int((gproblem["edge_pose"] == 0).sum())
    assert po["report"].n_active_edges == len(gproblem["edge_pose"]) - n0


def _gloo_partial_schur(rank, world, port, pr, ret):
    import torch
    import torch.distributed as dist
    from mcs_amd import ba
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    try:
        sub, _, _ = ba.shard_problem(pr, rank, world)
        cnt = torch.tensor(np.bincount(sub["edge_pose"], minlength=len(pr["poses"])).astype(np.float64))
        dist.all_reduce(cnt)   # global pose activity (as the library's structure exchange)
        S, bs = _partial_schur(sub, cnt.numpy(), 1e-3, 1e-3 if rank == 0 else 0.0)
        t = torch.tensor(np.concatenate([S.ravel(), bs]))
        dist.all_reduce(t)
        ret[rank] = t.numpy()
    finally:
        dist.destroy_process_group()


def test_sharded_schur_sum_equals_full_gloo(gproblem):
    """world_size 2 over gloo: the sum of the per-rank partial Schur complements (points
    sharded with all their edges, lambda on rank 0 only) equals the unsharded system."""
    import torch.multiprocessing as mp
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    world = 2
    mgr = mp.get_context("spawn").Manager()
    ret = mgr.dict()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_gloo_partial_schur, args=(r, world, port, gproblem, ret))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    S, bs = _partial_schur(gproblem, None, 1e-3, 1e-3)
    full = np.concatenate([S.ravel(), bs])
    for r in range(world):
        got = ret[r]
        assert np.allclose(got, full, rtol=1e-10, atol=1e-9 * np.abs(full).max())
    assert np.array_equal(ret[0], ret[1])


# ------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 6, 60, 64, 65, 130, 600, 1194])
def test_gpu_dense_ldlt_solve(gpu, n):
    from mcs_amd import ba
    rng = np.random.default_rng(n)
    A = rng.normal(size=(n, n))
    S = A @ A.T + n * np.eye(n)
    b = rng.normal(size=n)
    x, zp = ba.dense_ldlt_solve(S, b)
    assert zp == 0
    ref = np.linalg.solve(S, b)
    assert np.linalg.norm(S @ x - b) <= 1e-10 * np.linalg.norm(b) * max(1.0, np.linalg.norm(S, 2))
    assert np.allclose(x, ref, rtol=1e-9, atol=1e-12 * np.abs(ref).max())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 7, 36, 60, 63, 64])
def test_gpu_one_tile_solve_matches_tiled(gpu, n):
    """The fused one-tile solve (LocalBA systems) is bitwise the pad + panel + backward path,
    including a zero pivot and a right-hand side with signed zeros."""
    from mcs_amd import ba
    rng = np.random.default_rng(100 + n)
    A = rng.normal(size=(n, n))
    S = A @ A.T + n * np.eye(n)
    b = rng.normal(size=n)
    b[::5] = -0.0
    x0, z0 = ba.dense_ldlt_solve(S, b)
    x1, z1 = ba.dense_ldlt_solve(S, b, tiled=True)
    assert z0 == z1 == 0
    assert x0.tobytes() == x1.tobytes()
    if n > 3:
        S2 = S.copy()
        S2[2, :] = 0.0
        S2[:, 2] = 0.0
        x0, z0 = ba.dense_ldlt_solve(S2, b)
        x1, z1 = ba.dense_ldlt_solve(S2, b, tiled=True)
        assert z0 == z1 == 1
        assert np.array_equal(x0, x1, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [65, 128, 129, 300, 700, 1194])
def test_gpu_pipelined_solve_matches_per_step(gpu, n):
    """The pipelined factorisation (one launch: a diagonal workgroup factoring each A_kk once
    with look-ahead, TRSM / UPDATE tasks from a device queue) is bitwise the one-launch-per-step
    path (same operations in the same order), including a zero pivot in a later tile."""
    from mcs_amd import ba
    rng = np.random.default_rng(500 + n)
    A = rng.normal(size=(n, n))
    S = A @ A.T + n * np.eye(n)
    b = rng.normal(size=n)
    x1, z1 = ba.dense_ldlt_solve(S, b, path=1)
    x2, z2 = ba.dense_ldlt_solve(S, b, path=2)
    assert z1 == z2 == 0
    assert x1.tobytes() == x2.tobytes()
    ref = np.linalg.solve(S, b)
    assert np.allclose(x2, ref, rtol=1e-9, atol=1e-12 * np.abs(ref).max())
    S2 = S.copy()
    k = n - 3
    S2[k, :] = 0.0
    S2[:, k] = 0.0
    x1, z1 = ba.dense_ldlt_solve(S2, b, path=1)
    x2, z2 = ba.dense_ldlt_solve(S2, b, path=2)
    assert z1 == z2 == 1
    assert np.array_equal(x1, x2, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [65, 300])
def test_gpu_legacy_solve_path(gpu, n):
    """Path 3 (one k_panel launch per step + the one-workgroup k_backward, what every path runs
    above 96 tiles) solves like the others (it sums the backward substitution in another order,
    so the comparison is to the solution, not bitwise); a zero pivot is reported the same way."""
    from mcs_amd import ba
    rng = np.random.default_rng(900 + n)
    A = rng.normal(size=(n, n))
    S = A @ A.T + n * np.eye(n)
    b = rng.normal(size=n)
    x3, z3 = ba.dense_ldlt_solve(S, b, path=3)
    assert z3 == 0
    ref = np.linalg.solve(S, b)
    assert np.allclose(x3, ref, rtol=1e-9, atol=1e-12 * np.abs(ref).max())
    S2 = S.copy()
    S2[n - 2, :] = 0.0
    S2[:, n - 2] = 0.0
    _, z3 = ba.dense_ldlt_solve(S2, b, path=3)
    assert z3 == 1


def _banded_spd(n, band, seed):
    """A symmetric diagonally dominant matrix whose entries vanish beyond `band` diagonals."""
    rng = np.random.default_rng(seed)
    S = np.zeros((n, n))
    for d in range(1, band + 1):
        v = rng.uniform(-1, 1, n - d) * (rng.random(n - d) < 0.7)
        S[np.arange(d, n), np.arange(n - d)] = v
        S[np.arange(n - d), np.arange(d, n)] = v
    S[np.arange(n), np.arange(n)] = 2.0 * band + 1.0
    return S


@pytest.mark.gpu
@pytest.mark.parametrize("n,band", [(300, 70), (1194, 150), (1194, 300), (3000, 64)])
def test_gpu_banded_solve_matches_dense(gpu, n, band):
    """The banded pipelined factorisation (path 0: tiles below the widest non-zero tile diagonal
    are skipped, as the BA skips pose pairs no point connects) gives the dense pipelined path's
    solution bit for bit: the skipped products are exact zeros."""
    from mcs_amd import ba
    S = _banded_spd(n, band, 7 * n + band)
    b = np.random.default_rng(n).normal(size=n)
    x0, z0 = ba.dense_ldlt_solve(S, b, path=0)
    x2, z2 = ba.dense_ldlt_solve(S, b, path=2)
    assert z0 == z2 == 0
    assert np.array_equal(x0, x2)
    ref = np.linalg.solve(S, b)
    assert np.allclose(x0, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())
    S2 = S.copy()
    k = n - 70
    S2[k, :] = 0.0
    S2[:, k] = 0.0
    _, z0 = ba.dense_ldlt_solve(S2, b, path=0)
    assert z0 == 1


@pytest.mark.gpu
def test_gpu_banded_solve_beyond_dense_cap(gpu):
    """n = 13000 (204 tiles, above the 192 the one-workgroup backward substitution holds):
    the banded pipelined path solves it (the dense paths report MCS_ERR_UNSUPPORTED);
    checked against LAPACK's banded Cholesky (scipy.linalg.solveh_banded)."""
    import scipy.linalg
    from mcs_amd import ba, McsError
    n, band = 13000, 200
    S = _banded_spd(n, band, 13)
    b = np.random.default_rng(13).normal(size=n)
    x, zp = ba.dense_ldlt_solve(S, b, path=0)
    assert zp == 0
    ab = np.zeros((band + 1, n))
    for d in range(band + 1):
        ab[d, :n - d] = np.diagonal(S, -d)
    ref = scipy.linalg.solveh_banded(ab, b, lower=True)
    assert np.allclose(x, ref, rtol=1e-9, atol=1e-12 * np.abs(ref).max())
    with pytest.raises(McsError):
        ba.dense_ldlt_solve(S, b, path=3)


@pytest.mark.gpu
def test_gpu_global_ba_beyond_2048_poses(gpu):
    """GlobalBA of 2100 MultiKeyframes (n = 12594, 197 tiles: above the dense solve's 2048-pose
    bound, which used to return MCS_ERR_UNSUPPORTED) through mcs_global_ba_select: the banded
    reduced camera system (tile band 11 of 197) is solved, the LM converges and every pose moves
    towards the ground truth.  Size-independent properties (the oracle's dense LDL^T would take
    minutes here); the banded solve itself is checked against LAPACK above."""
    from mcs_amd import ba
    pr = ba.config_e_problem(n_kf=2100, n_points=60000, target_edges=500000, seed=3)
    r = ba.Solver().global_ba(pr, trace=20)
    rep = r["report"]
    assert rep.iterations >= 3 and rep.n_active_poses == 2099
    assert rep.chi2_final < 0.9 * rep.chi2_initial        # 2 % outliers set the floor
    assert np.all(np.diff(r["trace"]) <= 1e-9 * rep.chi2_initial)   # accepted steps only lower chi2
    gt = pr["gt_poses"]
    e0 = np.abs(pr["poses"][1:, 3:] - gt[1:, 3:]).max(axis=1)
    e1 = np.abs(r["poses"][1:, 3:] - gt[1:, 3:]).max(axis=1)
    assert np.median(e1) < 0.5 * np.median(e0)


@pytest.mark.gpu
def test_gpu_solve_above_pipeline_tiles(gpu):
    """T = 97 tiles (n = 6150 > 96 * 64): paths 1 and 2 run the per-step kernels without the
    pipeline's sync words (no dense pipeline above kPipeMaxT tiles); path 0 runs the banded
    pipeline (the matrix's band is 70 entries, two tile diagonals)."""
    from mcs_amd import ba
    n = 6150
    rng = np.random.default_rng(6150)
    S = np.zeros((n, n))
    for d in range(0, 70, 7):            # a symmetric band, diagonally dominant
        v = rng.uniform(-1, 1, n - d)
        S[np.arange(d, n), np.arange(n - d)] = v
        S[np.arange(n - d), np.arange(d, n)] = v
    S[np.arange(n), np.arange(n)] = 20.0
    b = rng.normal(size=n)
    for path in (0, 1, 2):
        x, zp = ba.dense_ldlt_solve(S, b, path=path)
        assert zp == 0
        assert np.linalg.norm(S @ x - b) <= 1e-10 * np.linalg.norm(b) * 30.0


@pytest.mark.gpu
def test_gpu_ldlt_timeout_is_an_error(gpu, gproblem):
    """A hand-off wait that gives up (forced with a 1-tick bound) is an error of the solve
    (MCS_ERR_HIP), never a zero pivot that the LM would take as a rejected trial; the BA
    entries return it too, and a normal bound afterwards solves again."""
    from mcs_amd import ba, McsError
    n = 1194
    rng = np.random.default_rng(77)
    A = rng.normal(size=(n, n))
    S = A @ A.T + n * np.eye(n)
    b = rng.normal(size=n)
    try:
        ba.set_ldlt_wait_ticks(1)
        with pytest.raises(McsError) as ei:
            ba.dense_ldlt_solve(S, b, path=2)
        assert "timed out" in str(ei.value)
        with pytest.raises(McsError) as ei:
            ba.Solver().global_ba(gproblem, trace=20)
        assert "timed out" in str(ei.value)
    finally:
        ba.set_ldlt_wait_ticks(0)
    x, zp = ba.dense_ldlt_solve(S, b, path=2)
    assert zp == 0
    assert np.allclose(x, np.linalg.solve(S, b), rtol=1e-9)


@pytest.mark.gpu
def test_gpu_dense_ldlt_zero_pivot(gpu):
    from mcs_amd import ba
    S = np.eye(70)
    S[3, 3] = 0.0
    _, zp = ba.dense_ldlt_solve(S, np.ones(70))
    assert zp == 1


@pytest.mark.gpu
@pytest.mark.parametrize("pose_only", [False, True])
def test_gpu_global_ba_matches_oracle(gpu, gproblem, pose_only):
    from mcs_amd import ba
    S = ba.Solver()
    g = S.global_ba(gproblem, pose_only=pose_only, trace=20)
    o = _oracle_global(gproblem, pose_only=pose_only, trace=20)
    assert g["report"].iterations == o["report"].iterations
    assert g["report"].n_active_edges == o["report"].n_active_edges
    assert g["report"].n_active_poses == o["report"].n_active_poses
    assert g["report"].n_active_points == o["report"].n_active_points
    assert np.allclose(g["trace"], o["trace"], rtol=1e-6)
    assert np.abs(g["poses"] - o["poses"]).max() < 1e-6
    cnt = np.bincount(gproblem["edge_point"], minlength=len(gproblem["points"]))
    wc = cnt >= 3
    assert np.abs(g["points"][wc] - o["points"][wc]).max() < 1e-5
    if pose_only:
        assert np.array_equal(g["points"], gproblem["points"])


class ThreadExchange:
    """In-process stand-in for the collective: `world` ranks run on threads of one process,
    each with its own solver context / stream and exchange buffer on the same GPU.

    ordered=False: the library drains its stream before each call; rank 0 sums the slices and
    every rank returns once the sum is on the device.  ordered=True (stream_ordered shards, as
    TorchExchange on a GPU): nobody waits on the host -- every rank records an event on its
    stream, rank 0's stream waits for all of them and sums, and every rank's stream waits for
    rank 0's; the callback returns as soon as that is enqueued."""

    def __init__(self, world, n_poses, ordered=False):
        import torch
        from mcs_amd import ba, lib
        self.world, self.ordered = world, ordered
        cap = int(lib().mcs_ba_xchg_doubles(int(n_poses)))
        self.bufs = [torch.zeros(cap, dtype=torch.float64, device="cuda") for _ in range(world)]
        self.bar = threading.Barrier(world)
        self.calls = [[] for _ in range(world)]
        self.ev = [None] * world
        self.done = None
        self.streams = {}
        self.fns, self.shards = [], []
        for r in range(world):
            fn = ba.ALLREDUCE_FN(lambda u, op, off, cnt, st, r=r: self._cb(r, op, off, cnt, st))
            self.fns.append(fn)
            self.shards.append(ba.BAShard(r, world, self.bufs[r].data_ptr(), cap, fn, None,
                                          1 if ordered else 0))

    def _reduce(self, op, off, cnt):
        import torch
        sl = [b[off:off + cnt] for b in self.bufs]
        for t in sl[1:]:                # in place: no allocation on a foreign stream
            if op == 0:
                sl[0].add_(t)
            else:
                torch.maximum(sl[0], t, out=sl[0])
        for t in sl[1:]:
            t.copy_(sl[0])

    def _cb(self, r, op, off, cnt, stream):
        import torch
        try:
            self.calls[r].append((op, off, cnt))
            if not self.ordered:
                self.bar.wait(60)
                if r == 0:
                    self._reduce(op, off, cnt)
                    torch.cuda.synchronize()
                self.bar.wait(60)
                return 0
            s = self.streams.get(stream)
            if s is None:
                s = self.streams[stream] = torch.cuda.ExternalStream(stream)
            ev = torch.cuda.Event()
            ev.record(s)
            self.ev[r] = ev
            self.bar.wait(60)
            if r == 0:
                with torch.cuda.stream(s):
                    for e in self.ev[1:]:
                        s.wait_event(e)
                    self._reduce(op, off, cnt)
                    done = torch.cuda.Event()
                    done.record(s)
                self.done = done
            self.bar.wait(60)
            if r != 0:
                s.wait_event(self.done)
            return 0
        except Exception:
            return 1

    class _One:
        def __init__(self, shard):
            self.shard = shard

    def member(self, r):
        return ThreadExchange._One(self.shards[r])


@pytest.mark.gpu
@pytest.mark.parametrize("world,ordered", [(2, False), (3, False), (2, True), (3, True)])
def test_gpu_sharded_global_ba_lockstep(gpu, gproblem, world, ordered):
    from mcs_amd import ba
    X = ThreadExchange(world, len(gproblem["poses"]), ordered=ordered)
    out = [None] * world
    err = [None] * world
    stages = [None] * world

    def run(r):
        try:
            sub, rng, _ = ba.shard_problem(gproblem, r, world)
            S = ba.Solver()
            S.enable_timing(ordered)   # the stage clock must not change the call sequence
            out[r] = (S.global_ba(sub, exchange=X.member(r), trace=20), rng)
            stages[r] = S.read_timing()
        except Exception as e:   # surfaced below
            err[r] = e

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert all(e is None for e in err), err
    # every rank took the same collectives and ended with bit-identical poses
    assert all(X.calls[r] == X.calls[0] for r in range(world))
    # the per-trial reduced-system exchange covers bs + the leading (non-zero) tile diagonals
    # only: strictly less than the whole tile triangle once the system has 3+ tiles
    n = 6 * int(out[0][0]["report"].n_active_poses)
    T = (n + 63) // 64
    big = [c for c in X.calls[0] if c[0] == 0 and c[1] == 0 and c[2] >= 64 * T]
    assert big and all(c[2] <= 64 * T + T * (T + 1) // 2 * 4096 for c in big)
    if ordered:   # exchange stage = stream time of the all-reduce
        assert all(st[0]["exchange"] > 0 for st in stages), stages
    for r in range(1, world):
        assert np.array_equal(out[r][0]["poses"], out[0][0]["poses"])
        assert out[r][0]["report"].iterations == out[0][0]["report"].iterations
    pts = np.zeros_like(gproblem["points"])
    for g, (lo, hi) in out:
        pts[lo:hi] = g["points"]
    full = ba.Solver().global_ba(gproblem, trace=20)
    g0 = out[0][0]
    assert g0["report"].iterations == full["report"].iterations
    assert g0["report"].n_active_edges == full["report"].n_active_edges
    assert g0["report"].n_active_points == full["report"].n_active_points
    assert np.allclose(g0["trace"], full["trace"], rtol=1e-6)
    assert np.abs(g0["poses"] - full["poses"]).max() < 1e-6
    cnt = np.bincount(gproblem["edge_point"], minlength=len(gproblem["points"]))
    wc = cnt >= 3
    assert np.abs(pts[wc] - full["points"][wc]).max() < 1e-5
