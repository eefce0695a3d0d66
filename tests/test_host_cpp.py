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


@pytest.mark.gpu
def test_host_cpp_extract_matches_oracle(gpu, tmp_path):
    from mcs_amd import synth
    exe = _build(tmp_path)
    img, mask = synth.fisheye_frame(754, 480, seed=77)
    fi, fm = tmp_path / "img.raw", tmp_path / "mask.raw"
    img.tofile(fi)
    mask.tofile(fm)
    out = subprocess.check_output([exe, str(fi), str(fm)], timeout=120).decode()
    tok = out.split()
    n = int(tok[1])
    okps, odesc = ob.extract(img, mask, nfeatures=1000)
    assert n == len(okps)
    d01 = int(np.unpackbits(odesc[0] ^ odesc[1]).sum())
    assert int(tok[3]) == d01
    assert float(tok[5]) == okps[0]["x"] and float(tok[7]) == okps[0]["y"]
