"""Host structure of a BA call (ba_structure.hpp: scan_edges + build_structure, two branch-free
passes) against a plain restatement of g2o's initializeOptimization(0) + buildIndexMapping +
BlockSolver::buildStructure (sparse_optimizer.cpp:166-267, block_solver.hpp:143-295): active
edges (level 0, not all vertices fixed) in edge order, non-fixed poses with an active edge and
points with an active edge numbered in vertex order, CSR lists point -> edges and pose -> edges
in edge order, lower pose blocks.  Random graphs with level masks, fixed poses, pose-only BA
(points fixed), duplicate (pose, point) observations and out-of-range indices.  CPU only."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("bs") / "structure_dump")
    subprocess.check_call(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "structure_dump.cpp"),
                           "-pthread", "-o", out])
    return out


def _run(exe, npose, npt, ep, el, ec, fixed, level, points_fixed, ncam=3, threads=1):
    lines = ["%d %d %d %d %d %d" % (npose, npt, len(ep), ncam, int(points_fixed), int(level is not None)),
             " ".join(str(int(x)) for x in fixed)]
    lv = level if level is not None else np.zeros(len(ep), np.uint8)
    lines += ["%d %d %d %d" % (a, b, c, d) for a, b, c, d in zip(ep, el, ec, lv)]
    out = subprocess.run([exe, str(threads)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         timeout=60, check=True).stdout.split("\n")
    if out[0].strip() == "bad":
        return None
    r = {}
    a = out[0].split()
    r["np"], r["nl"] = int(a[1]), int(a[3])
    for ln in out[1:]:
        f = ln.split()
        if f:
            r[f[0]] = [int(x) for x in f[2:]]
    return r


def _restated(npose, npt, ep, el, fixed, level, points_fixed):
    act = [e for e in range(len(ep)) if not (level is not None and level[e])
           and not (points_fixed and fixed[ep[e]])]
    pose_cnt = np.bincount([ep[e] for e in act], minlength=npose)
    pose_h, hpose = [-1] * npose, []
    for i in range(npose):
        if pose_cnt[i] > 0 and not fixed[i]:
            pose_h[i] = len(hpose)
            hpose.append(i)
    point_h, hpt = [-1] * npt, []
    if not points_fixed:
        seen = set(el[e] for e in act)
        for i in range(npt):
            if i in seen:
                point_h[i] = len(hpt)
                hpt.append(i)
    pt_lists = [[] for _ in hpt]
    ps_lists = [[] for _ in hpose]
    for e in act:
        if point_h[el[e]] >= 0:
            pt_lists[point_h[el[e]]].append(e)
        if pose_h[ep[e]] >= 0:
            ps_lists[pose_h[ep[e]]].append(e)
    pt_ptr = np.concatenate([[0], np.cumsum([len(x) for x in pt_lists])]).astype(int).tolist()
    ps_ptr = np.concatenate([[0], np.cumsum([len(x) for x in ps_lists])]).astype(int).tolist()
    pt_edges = [e for x in pt_lists for e in x]
    ps_edges = [e for x in ps_lists for e in x]
    nl_count = len(set(el[e] for e in act)) if not points_fixed else 0
    cnt = list(pose_cnt) + [nl_count, len(act)]
    blk_i = [i for i in range(len(hpose)) for j in range(i + 1)]
    blk_j = [j for i in range(len(hpose)) for j in range(i + 1)]
    return dict(np=len(hpose), nl=len(hpt), cnt=[int(x) for x in cnt], aedge=act, pose_h=pose_h,
                point_h=point_h, hpose_vtx=hpose, hpt_vtx=hpt, pt_ptr=pt_ptr, pt_edges=pt_edges,
                pt_h=[pose_h[ep[e]] for e in pt_edges], ps_ptr=ps_ptr, ps_edges=ps_edges,
                blk_i=blk_i, blk_j=blk_j)


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("seed", range(8))
def test_host_structure_matches_restatement(exe, seed, threads):
    rng = np.random.default_rng(seed)
    npose, npt = int(rng.integers(1, 12)), int(rng.integers(1, 60))
    ne = int(rng.integers(0, 300))
    ep = rng.integers(0, npose, ne)
    el = rng.integers(0, npt, ne)
    if seed % 2 == 0:   # edges grouped by point, as LocalBA builds them
        o = np.argsort(el, kind="stable")
        ep, el = ep[o], el[o]
    ec = rng.integers(0, 3, ne)
    fixed = (rng.random(npose) < 0.3).astype(np.uint8)
    level = (rng.random(ne) < 0.2).astype(np.uint8) if seed % 3 else None
    points_fixed = seed in (5, 7)
    got = _run(exe, npose, npt, ep, el, ec, fixed, level, points_fixed, threads=threads)
    want = _restated(npose, npt, ep.tolist(), el.tolist(), fixed.tolist(),
                     None if level is None else level.tolist(), points_fixed)
    for k, v in want.items():
        assert got[k] == v, k


def test_host_structure_rejects_out_of_range(exe):
    ep, el, ec = np.array([0, 1, 2]), np.array([0, 1, 0]), np.array([0, 0, 0])
    fixed = np.zeros(2, np.uint8)
    assert _run(exe, 2, 2, ep, el, ec, fixed, None, False) is None            # pose 2 of 2
    assert _run(exe, 2, 2, ep, el, ec, fixed, None, False, threads=2) is None
    assert _run(exe, 3, 2, ep, np.array([0, 1, 2]), ec, np.zeros(3, np.uint8), None, False) is None
    assert _run(exe, 3, 2, ep, el, np.array([0, 3, 0]), np.zeros(3, np.uint8), None, False) is None


@pytest.mark.parametrize("sorted_points", [True, False])
@pytest.mark.parametrize("points_fixed", [False, True])
def test_host_structure_threaded_equals_one_thread(exe, points_fixed, sorted_points):
    """The threaded path (HostPool chunks) on a larger graph: identical output to one thread,
    with the edges in point order (the point lists are the edge list) and in random order."""
    rng = np.random.default_rng(11)
    npose, npt, ne = 40, 3000, 20000
    el = rng.integers(0, npt, ne)
    if sorted_points:
        el = np.sort(el)
    ep = rng.integers(0, npose, ne)
    ec = rng.integers(0, 3, ne)
    fixed = (rng.random(npose) < 0.2).astype(np.uint8)
    level = (rng.random(ne) < 0.1).astype(np.uint8)
    one = _run(exe, npose, npt, ep, el, ec, fixed, level, points_fixed)
    want = _restated(npose, npt, ep.tolist(), el.tolist(), fixed.tolist(), level.tolist(), points_fixed)
    for k, v in want.items():
        assert one[k] == v, k
    for t in (2, 5, 8):
        assert _run(exe, npose, npt, ep, el, ec, fixed, level, points_fixed, threads=t) == one


def test_host_pool_runs_every_index_once(tmp_path):
    """csrc/host_pool.hpp: each run(f) calls f(0..n-1) once and waits for all of them."""
    out = str(tmp_path / "host_pool_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-pthread",
                           os.path.join(ROOT, "tests", "cpp", "host_pool_check.cpp"), "-o", out])
    r = subprocess.run([out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
