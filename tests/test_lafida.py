"""Lafida settings / calibration ingest.

Reference: cSystem::LoadMCS (src/cSystem.cpp:124-176), cTracking ctor settings reads
(src/cTracking.cpp:86-158), Examples/Lafida/*.yaml.  The key/value data of the reference's own
YAML files is the fixture tests/golden/lafida_settings.json (tools/make_lafida_fixture.py); the
files are rebuilt from it in a temporary directory so the loaders run on real files everywhere.
"""
import json
import os

import numpy as np
import pytest

from tests import oracle_bind as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "lafida_settings.json")
REF_DIR = "/root/reference/Examples/Lafida"


def _fixture():
    with open(FIXTURE) as f:
        return json.load(f)


@pytest.fixture
def lafida_dir(tmp_path):
    for name, kv in _fixture().items():
        with open(tmp_path / name, "w") as f:
            f.write("%YAML:1.0\n# rebuilt from tests/golden/lafida_settings.json\n")
            for k, v in kv.items():
                f.write("%s: %s   # comment\n" % (k, repr(v)))
    return str(tmp_path)


def test_fixture_matches_reference_files():
    from mcs_amd import lafida
    fx = _fixture()
    assert len(fx) == 8
    if os.path.isdir(REF_DIR):                    # build container only
        for name, kv in fx.items():
            assert lafida.read_filestorage(os.path.join(REF_DIR, name)) == kv, name


def test_load_rig_matches_lafida_constants(lafida_dir):
    from mcs_amd import lafida, synth
    rig = lafida.load_rig(lafida_dir)
    assert rig["n_cams"] == 3 and rig["sizes"] == [(754, 480)] * 3
    assert rig["mirror_mask"] == [True, True, True]
    assert np.array_equal(rig["mc"], np.array(synth.LAFIDA_MC))
    for cam, ref in zip(rig["cams"], synth.LAFIDA_CAMS):
        for k in ("c", "d", "e", "u0", "v0"):
            assert cam[k] == ref[k], k
        assert cam["a"] == list(ref["a"]) and cam["pol"] == list(ref["pol"])
    m = rig["cam_models"][0]
    assert (m.p_deg, m.invp_deg) == (5, 12) and m.p[2] == rig["cams"][0]["a"][2]


def test_extractor_params_from_settings(lafida_dir):
    from mcs_amd import lafida
    s = lafida.load_settings(os.path.join(lafida_dir, "Slam_Settings_indoor1.yaml"))
    track, init = lafida.extractor_params(s)
    assert (track.nfeatures, track.fast_threshold, init.nfeatures, init.fast_threshold) == (400, 20, 800, 5)
    for p in (track, init):
        assert p.scale_factor == np.float32(1.2) and p.nlevels == 8 and p.desc_size == 32
        assert (p.edge_threshold, p.first_level, p.patch_size) == (25, 0, 32)
        assert (p.use_agast, p.fast_agast_type, p.do_dbrief, p.learn_masks) == (0, 2, 0, 0)
    assert lafida.tracking_frames(s) == (25.0, 8, 17)


def test_filestorage_semantics():
    from mcs_amd import lafida
    fs = lafida.parse_filestorage("%YAML:1.0\na: 2.5\nb: 3.5\nc: 7   # x\nd: \"txt\"\ne:\n")
    assert lafida.as_int(fs, "a") == 2 and lafida.as_int(fs, "b") == 4    # cvRound half-even
    assert lafida.as_int(fs, "c") == 7 and lafida.as_real(fs, "c") == 7.0
    assert lafida.as_int(fs, "missing") == 0 and lafida.as_real(fs, "missing") == 0.0
    assert lafida.as_int(fs, "d") == 0x7fffffff
    assert lafida.tracking_frames({}) == (25.0, 8, 17)                   # fps 0 -> 25
    with pytest.raises(ValueError):
        lafida.extractor_params({"extractor.descSize": 24, "extractor.nScoreType": 1})


@pytest.mark.gpu
def test_gpu_extractor_from_lafida_settings(gpu, lafida_dir):
    """The tracking extractor configured from Slam_Settings_indoor1 + camera 1's calibration
    extracts exactly what the oracle extracts with the same settings."""
    import mcs_amd
    from mcs_amd import lafida, synth
    s = lafida.load_settings(os.path.join(lafida_dir, "Slam_Settings_indoor1.yaml"))
    rig = lafida.load_rig(lafida_dir)
    track, _ = lafida.extractor_params(s)
    W, H = rig["sizes"][1]
    img, mask = synth.fisheye_frame(W, H, seed=31, cam_index=1, cam=rig["cams"][1])
    ex = mcs_amd.Extractor(track, W, H)
    kps, desc = ex.extract(img, mask)
    okps, odesc = ob.extract(img, mask, nfeatures=track.nfeatures, fast_th=track.fast_threshold)
    assert len(kps) == len(okps) > 0
    for f in okps.dtype.names:
        assert np.array_equal(kps[f], okps[f]), f
    assert np.array_equal(desc, odesc)
