"""C++ host mirror (multicol-slam-annotation_amd/host/mcs_multicol.hpp): a small C++ program
written against the reference call shapes links libmcs_amd.so directly (no Python, no torch)
and must reproduce the oracle's keypoints for the same frame."""
import os
import subprocess

import numpy as np
import pytest

from tests import oracle_bind as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    lib = os.path.join(ROOT, "multicol-slam-annotation_amd", "lib")
    exe = str(tmp_path / "host_api_demo")
    subprocess.check_call(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "host_api_demo.cpp"),
                           "-I", os.path.join(ROOT, "include"), "-L", lib, "-lmcs_amd",
                           "-Wl,-rpath," + lib, "-o", exe])
    return exe


def test_host_header_compiles(built, tmp_path):
    assert os.path.exists(_build(tmp_path))


def _fnv64(b):
    h = 1469598103934665603
    for x in bytes(b):
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_host_cpp_extract_matches_oracle(gpu, tmp_path, mode):
    """ORB, dBRIEF and mdBRIEF through the C++ mirror's operator()(image, mask, kps, camModel,
    desc, descMasks) vs the oracle (keypoints, descriptors and descriptor masks)."""
    from mcs_amd import CamModel, synth
    exe = _build(tmp_path)
    img, mask = synth.fisheye_frame(754, 480, seed=77)
    cam = CamModel.from_dict(synth.LAFIDA_CAMS[0])
    fi, fm, fc = tmp_path / "img.raw", tmp_path / "mask.raw", tmp_path / "cam.bin"
    img.tofile(fi)
    mask.tofile(fm)
    fc.write_bytes(bytes(cam))
    out = subprocess.check_output([exe, str(fi), str(fm), str(mode), str(fc)], timeout=120).decode()
    tok = out.split()
    n = int(tok[1])
    if mode == 0:
        okps, odesc = ob.extract(img, mask, nfeatures=1000)
        omask = np.zeros_like(odesc)
    else:
        okps, odesc, omask = ob.extract_ex(img, cam, mask, nfeatures=1000, do_dbrief=1,
                                           learn_masks=int(mode == 2))
    assert n == len(okps)
    d01 = int(np.unpackbits(odesc[0] ^ odesc[1]).sum())
    assert int(tok[3]) == d01
    assert float(tok[5]) == okps[0]["x"] and float(tok[7]) == okps[0]["y"]
    assert int(tok[9]) == _fnv64(odesc.tobytes())
    assert int(tok[11]) == _fnv64(omask.tobytes())
    assert int(tok[13]) == int(mode == 2)


def _build_refresh(tmp_path):
    lib = os.path.join(ROOT, "multicol-slam-annotation_amd", "lib")
    exe = str(tmp_path / "host_refresh_demo")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__",
                           os.path.join(ROOT, "tests", "cpp", "host_refresh_demo.cpp"),
                           "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                           "-L", lib, "-lmcs_amd", "-L", "/opt/rocm/lib", "-lamdhip64",
                           "-Wl,-rpath," + lib, "-Wl,-rpath,/opt/rocm/lib", "-o", exe])
    return exe


def test_host_refresh_demo_compiles(built, tmp_path):
    assert os.path.exists(_build_refresh(tmp_path))


@pytest.mark.gpu
def test_host_cpp_round3_abi(gpu, tmp_path):
    """mcs_compute_e_rig (SearchForTriangulationRaw's Es, src/cORBmatcher.cpp:985-998) and the
    post-BA map-point refresh (mcs_distinctive_descriptors_device / mcs_update_normal_depth_device,
    src/cOptimizer.cpp:899-901 -> src/cMapPoint.cpp:297-390, 453-496) called from C++ through
    the C-ABI: E equals the reference-text evaluation in tests/golden/refmath.npz bit for bit,
    the refresh equals the oracle, and a bad argument returns a status with its message."""
    exe = _build_refresh(tmp_path)
    gold = np.load(os.path.join(ROOT, "tests", "golden", "refmath.npz"))
    mt1, mt2, mc = gold["rig_mt1"], gold["rig_mt2"], gold["rig_mc"]
    rng = np.random.default_rng(31)
    nb, nrows = 32, 3000
    proto = rng.integers(0, 256, (30, nb), dtype=np.uint8)
    flips = rng.random((nrows, nb * 8)) < 0.08
    desc = proto[rng.integers(0, 30, nrows)] ^ np.packbits(flips, axis=1)
    cnt = np.concatenate([[0, 1, 2, 3, 64, 65], rng.integers(2, 20, 300)])
    ptr = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
    rows = rng.integers(0, nrows, int(ptr[-1])).astype(np.int32)
    npd = len(cnt)
    n, nkf, nlev = 1000, 25, 8
    pts = rng.normal(0, 3, (n, 3))
    ocnt = rng.integers(0, 8, n)
    ocnt[:2] = [0, 1]
    optr = np.concatenate([[0], np.cumsum(ocnt)]).astype(np.int32)
    okf = rng.integers(0, nkf, int(optr[-1])).astype(np.int32)
    kfc = rng.normal(0, 1, (nkf, 3))
    ref = rng.integers(0, nkf, n).astype(np.int32)
    lvl = rng.integers(-1, nlev, n).astype(np.int32)
    scale = np.cumprod([1.0] + [float(np.float32(1.2))] * (nlev - 1))
    i32 = lambda *v: np.array(v, np.int32).tobytes()  # noqa: E731
    blob = b"".join([i32(len(mt1), len(mc)), mt1.tobytes(), mt2.tobytes(), np.ascontiguousarray(mc).tobytes(),
                     i32(nb, nrows, npd), desc.tobytes(), ptr.tobytes(), rows.tobytes(),
                     i32(n, nkf, nlev), pts.tobytes(), optr.tobytes(), okf.tobytes(), kfc.tobytes(),
                     ref.tobytes(), lvl.tobytes(), scale.tobytes()])
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    fin.write_bytes(blob)
    out = subprocess.check_output([exe, str(fin), str(fout)], timeout=120).decode()
    assert "ok" in out
    assert "bad_bytes_status -" in out and "bytes must be 16, 32 or 64" in out
    raw = fout.read_bytes()
    nc = len(mc)
    o = 0
    E = np.frombuffer(raw, np.float64, len(mt1) * nc * nc * 9, o).reshape(len(mt1), nc, nc, 3, 3)
    o += E.nbytes
    best = np.frombuffer(raw, np.int32, npd, o)
    o += best.nbytes
    od = np.frombuffer(raw, np.uint8, npd * nb, o).reshape(npd, nb)
    o += od.nbytes
    nrm = np.frombuffer(raw, np.float64, 3 * n, o).reshape(n, 3)
    o += nrm.nbytes
    dmin = np.frombuffer(raw, np.float64, n, o)
    o += dmin.nbytes
    dmax = np.frombuffer(raw, np.float64, n, o)
    assert np.array_equal(E, gold["rig_E"])               # reference text, bit for bit
    ref_best = np.zeros(npd, np.int32)
    ob.lib().oracle_distinctive_descriptors(ob._p(desc), None, nb, ob._p(ptr), ob._p(rows), npd,
                                            ob._p(ref_best))
    assert np.array_equal(best, ref_best)
    for p in range(npd):
        if ref_best[p] >= 0:
            assert np.array_equal(od[p], desc[rows[ptr[p] + ref_best[p]]])
    on, omin, omax = np.zeros((n, 3)), np.zeros(n), np.zeros(n)
    ob.lib().oracle_update_normal_depth(ob._p(pts), n, ob._p(optr), ob._p(okf), ob._p(kfc), ob._p(ref),
                                        ob._p(lvl), ob._p(scale), nlev, ob._p(on), ob._p(omin), ob._p(omax))
    assert np.array_equal(nrm, on) and np.array_equal(dmin, omin) and np.array_equal(dmax, omax)


# ---------------------------------------------------------------- GlobalBA / PoseOptimization
GBA_FIX = os.path.join(ROOT, "tests", "golden", "globalba_ref.npz")


def _build_ba_demo(tmp_path):
    lib = os.path.join(ROOT, "multicol-slam-annotation_amd", "lib")
    exe = str(tmp_path / "ba_graph_demo")
    subprocess.check_call(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "ba_graph_demo.cpp"),
                           "-I", os.path.join(ROOT, "include"), "-L", lib, "-lmcs_amd",
                           "-Wl,-rpath," + lib, "-o", exe])
    return exe


def _ba_blob(z, g, p, pose_only, stop):
    """The map of globalba_ref case g and the frame of case p as ba_graph_demo reads them."""
    i32 = lambda *v: np.array(v, np.int32).tobytes()  # noqa: E731
    a = lambda k, dt: np.ascontiguousarray(z[k], dt).tobytes()  # noqa: E731
    q = g + "_map_"
    nk, npt, nobs, nc = len(z[q + "kf_id"]), len(z[q + "pt_id"]), len(z[q + "obs_kf"]), len(z[q + "mc"])
    parts = [i32(nk, npt, nobs, nc), a(q + "kf_id", np.int64), a(q + "kf_bad", np.uint8),
             a(q + "kf_pose", np.float64), a(q + "pt_id", np.int64), a(q + "pt_bad", np.uint8),
             a(q + "pt_pos", np.float64), a(q + "pt_obs_off", np.int32), a(q + "obs_kf", np.int32),
             a(q + "obs_cam", np.int32), a(q + "obs_meas", np.float64), a(q + "mc", np.float64),
             a(q + "cam", np.float64), i32(pose_only, stop)]
    r = p + "_"
    parts += [i32(len(z[r + "key_mp"]), len(z[r + "pt_id"]), len(z[r + "mc"]), len(z[r + "inv_sigma2"])),
              a(r + "key_mp", np.int32), a(r + "key_cam", np.int32), a(r + "key_pt", np.float64),
              a(r + "key_oct", np.int32), a(r + "inv_sigma2", np.float64), a(r + "pt_id", np.int64),
              a(r + "pt_pos", np.float64), a(r + "pose", np.float64), a(r + "mc", np.float64),
              a(r + "cam", np.float64), np.float64(z[r + "huber_mult"]).tobytes()]
    return b"".join(parts)


@pytest.mark.parametrize("g,p", [("g1", "p0"), ("g4", "p1"), ("c0", "p2")])
def test_host_cpp_graph_select(built, tmp_path, g, p):
    """The BundleAdjustment / PoseOptimization graph assembly called from C++ through the C-ABI
    (host code, no GPU) equals the reference-text fixture: vertex ids, the maxKF rule, bad-keyframe
    / bad-point skips, the id collision, edges, write-back slots, PoseOptimization's point vertices
    and edges."""
    z = np.load(GBA_FIX)
    exe = _build_ba_demo(tmp_path)
    meta = z[g + "_meta"]
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    fin.write_bytes(_ba_blob(z, g, p, int(meta[0]), int(meta[1])))
    out = subprocess.check_output([exe, str(fin), str(fout), "0"], timeout=120).decode()
    assert "select ok" in out
    raw = fout.read_bytes()
    o = [0]

    def take(dt, n):
        v = np.frombuffer(raw, dt, n, o[0])
        o[0] += v.nbytes
        return v
    st = int(take(np.int32, 1)[0])
    coll = int(take(np.int64, 1)[0])
    npo, npp, ne = [int(x) for x in take(np.int32, 3)]
    q = g + "_"
    verts = z[q + "vertices"]
    if int(meta[2]) >= 0:
        assert st < 0 and coll == int(meta[2])
    else:
        assert st == 0 and coll == -1
        pose_kf, pose_fixed = take(np.int32, npo), take(np.uint8, npo)
        points, pvid = take(np.int32, npp), take(np.int64, npp)
        mc0, io0 = [int(x) for x in take(np.int64, 2)]
        nk, npt = len(z[q + "map_kf_id"]), len(z[q + "map_pt_id"])
        kf_slot, pt_slot = take(np.int32, nk), take(np.int32, npt)
        eo, ep, eq = take(np.int32, ne), take(np.int32, ne), take(np.int32, ne)
        mt = verts[verts[:, 1] == 0]
        assert np.array_equal(z[q + "map_kf_id"][pose_kf], mt[:, 0]) and np.array_equal(pose_fixed, mt[:, 2])
        assert mc0 == verts[verts[:, 1] == 1, 0][0] and io0 == verts[verts[:, 1] == 2, 0][0]
        pv = z[q + "point_vertices"]
        assert np.array_equal(pvid, pv[:, 0]) and np.array_equal(points, pv[:, 1])
        e = z[q + "edges"]
        assert np.array_equal(pose_kf[ep], e[:, 0]) and np.array_equal(pvid[eq], e[:, 1])
        assert np.array_equal(z[q + "map_obs_cam"][eo], e[:, 2])
        assert np.array_equal(np.nonzero(kf_slot < 0)[0], z[q + "pose_ub"])
        assert np.array_equal(np.nonzero(pt_slot < 0)[0], z[q + "point_ub"])
    # the PoseOptimization part follows the BundleAdjustment part (whose arrays a collision
    # leaves unread above)
    o[0] = _po_offset(raw, st, npo, npp, ne, z, q)
    pn, pe = [int(x) for x in take(np.int32, 2)]
    pp, pv2 = take(np.int32, pn), take(np.int64, pn)
    po, pq = take(np.int32, pe), take(np.int32, pe)
    r = p + "_"
    pvz = z[r + "point_vertices"]
    assert np.array_equal(pv2, pvz[:, 0]) and np.array_equal(pp, pvz[:, 1])
    assert np.array_equal(pp[pq], z[r + "edges"][:, 0])
    assert np.array_equal(z[r + "key_cam"][po], z[r + "edges"][:, 1])
    assert o[0] == len(raw)


def _po_offset(raw, st, npo, npp, ne, z, q):
    """Byte offset of the PoseOptimization part in ba_graph_demo's mode-0 output."""
    nk, npt = len(z[q + "map_kf_id"]), len(z[q + "map_pt_id"])
    head = 4 + 8 + 12
    return head + npo * 4 + npo + npp * 4 + npp * 8 + 16 + nk * 4 + npt * 4 + 3 * ne * 4


@pytest.mark.gpu
@pytest.mark.parametrize("g,p", [("g1", "p0"), ("g3", "p3")])
def test_host_cpp_global_ba_pose_opt(gpu, tmp_path, g, p):
    """cTracking's GlobalBundleAdjustment / PoseOptimization call shapes through the C++ adapter
    (mcs::GlobalBA::run, mcs::PoseOptimizer::run) on the GPU against the reference-text fixture:
    iterations, written-back poses 1e-6 / points 1e-5 of their scale, the list entries written,
    outlier flags and counts."""
    z = np.load(GBA_FIX)
    exe = _build_ba_demo(tmp_path)
    meta = z[g + "_meta"]
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    fin.write_bytes(_ba_blob(z, g, p, int(meta[0]), int(meta[1])))
    out = subprocess.check_output([exe, str(fin), str(fout), "1"], timeout=300).decode()
    assert "run ok" in out
    raw = fout.read_bytes()
    q = g + "_"
    nk, npt = len(z[q + "map_kf_id"]), len(z[q + "map_pt_id"])
    o = 0
    kp = np.frombuffer(raw, np.float64, 6 * nk, o).reshape(nk, 6)
    o += kp.nbytes
    pp = np.frombuffer(raw, np.float64, 3 * npt, o).reshape(npt, 3)
    o += pp.nbytes
    kw = np.frombuffer(raw, np.uint8, nk, o)
    o += nk
    pw = np.frombuffer(raw, np.uint8, npt, o)
    o += npt
    it = int(np.frombuffer(raw, np.int32, 1, o)[0])
    o += 4
    assert it == int(z[q + "optimize_log"][0, 1])
    pwz, qwz = z[q + "pose_write"], z[q + "point_write"]
    assert np.array_equal(np.nonzero(kw)[0], pwz[:, 0].astype(int))
    assert np.array_equal(np.nonzero(pw)[0], qwz[:, 0].astype(int))
    assert np.abs(kp[pwz[:, 0].astype(int)] - pwz[:, 1:]).max() < 1e-6
    scale = np.maximum(1.0, np.linalg.norm(qwz[:, 1:], axis=1))
    assert (np.abs(pp[qwz[:, 0].astype(int)] - qwz[:, 1:]).max(axis=1) / scale).max() < 1e-5
    r = p + "_"
    N = len(z[r + "key_mp"])
    ngood = int(np.frombuffer(raw, np.int32, 1, o)[0])
    o += 4
    ratio = float(np.frombuffer(raw, np.float64, 1, o)[0])
    o += 8
    outl = np.frombuffer(raw, np.uint8, N, o)
    o += N
    pose = np.frombuffer(raw, np.float64, 6, o)
    assert ngood == int(z[r + "ret"]) and ratio == float(z[r + "inliers"])
    assert np.array_equal(outl, z[r + "outlier"])
    assert np.abs(pose - z[r + "pose_out"]).max() < 1e-6
