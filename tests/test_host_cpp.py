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
