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
