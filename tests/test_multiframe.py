"""Device cMultiFrame construction and the Lafida sequence ingest.

Reference: cMultiFrame::cMultiFrame src/cMultiFrame.cpp:92-216 (extraction inside
GetMirrorMask(0), ImgToWorld rays, concatenation, PosInGrid, scale tables) and
Examples/Lafida/mult_col_slam_lafida.cpp:109-118, 167-199 (LoadImagesAndTimestamps, grayscale
imread).  CPU: the loader's line-window / parse-stop rules and the grayscale decode on files
written here.  GPU: MultiFrameBuilder on the reference's Lafida rig (calibration rebuilt from
tests/golden/lafida_settings.json) equals, per camera, the oracle extractor run with the
oracle's level-0 mirror mask; every keypoint lies inside the mirror circle; rays and the
concatenation equal the oracle / host restatement exactly.
"""
import os

import numpy as np
import pytest

from tests import oracle_bind as ob
from tests.test_lafida import lafida_dir  # noqa: F401  (fixture)


def _write_list(d, lines):
    with open(os.path.join(d, "images_and_timestamps.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")


def test_load_images_and_timestamps_window(tmp_path):
    from mcs_amd import multiframe as mf
    lines = ["%.3f c0/%03d.png c1/%03d.png c2/%03d.png" % (0.04 * i, i, i, i) for i in range(1, 11)]
    _write_list(str(tmp_path), lines)
    names, ts = mf.load_images_and_timestamps(str(tmp_path), 3, 7)   # lines 3..6 (1-based)
    assert ts == [0.12, 0.16, 0.2, 0.24]
    assert names[0][0] == str(tmp_path) + "/c0/003.png" and names[2][-1] == str(tmp_path) + "/c2/006.png"
    assert all(len(n) == 4 for n in names)
    names, ts = mf.load_images_and_timestamps(str(tmp_path), 0, 100)
    assert len(ts) == 10


def test_load_images_and_timestamps_stops_at_bad_line(tmp_path):
    from mcs_amd import multiframe as mf
    _write_list(str(tmp_path), ["1.0 a b c", "2.0 a b c", "3.0 a b", "4.0 a b c"])
    names, ts = mf.load_images_and_timestamps(str(tmp_path), 1, 10)
    assert ts == [1.0, 2.0] and len(names[1]) == 2          # the 3-token line ends the read
    # lines before start_frame are skipped without being parsed
    _write_list(str(tmp_path), ["garbage", "5.0 a b c"])
    assert mf.load_images_and_timestamps(str(tmp_path), 2, 3)[1] == [5.0]
    assert mf.load_images_and_timestamps(str(tmp_path / "missing"), 1, 5) == ([[], [], []], [])


def test_imread_grayscale(tmp_path):
    from PIL import Image
    from mcs_amd import multiframe as mf
    rng = np.random.default_rng(1)
    g = rng.integers(0, 256, (48, 64), dtype=np.uint8)
    Image.fromarray(g, "L").save(tmp_path / "g.png")
    assert np.array_equal(mf.imread_grayscale(str(tmp_path / "g.png")), g)
    rgb = rng.integers(0, 256, (20, 30, 3), dtype=np.uint8)
    Image.fromarray(rgb, "RGB").save(tmp_path / "c.png")
    r, gg, b = (rgb[..., i].astype(np.int64) for i in range(3))
    want = ((r * 4899 + gg * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)
    assert np.array_equal(mf.imread_grayscale(str(tmp_path / "c.png")), want)
    w16 = rng.integers(0, 65536, (10, 12), dtype=np.uint16)
    Image.fromarray(w16).save(tmp_path / "w.png")
    assert np.array_equal(mf.imread_grayscale(str(tmp_path / "w.png")), (w16 >> 8).astype(np.uint8))
    (tmp_path / "bad.png").write_bytes(b"not an image")
    assert mf.imread_grayscale(str(tmp_path / "bad.png")) is None
    assert mf.imread_grayscale(str(tmp_path / "none.png")) is None
    with pytest.raises(FileNotFoundError, match="bad.png"):
        mf.load_multiframe_images([[str(tmp_path / "g.png")], [str(tmp_path / "bad.png")]], 0)


def test_scale_tables():
    from mcs_amd import multiframe as mf
    sf, s2, inv = mf.scale_tables(8, 1.2)
    f = float(np.float32(1.2))
    assert sf[0] == 1.0 and sf[3] == f * f * f and np.allclose(s2, sf ** 2) and inv[7] == 1 / s2[7]


@pytest.mark.gpu
def test_gpu_multiframe_builder_lafida(gpu, lafida_dir):  # noqa: F811
    import torch
    from mcs_amd import lafida, multiframe as mf, rig as rigmod, synth
    from tests.test_mirror import oracle_masks
    rig = lafida.load_rig(lafida_dir)
    s = lafida.load_settings(os.path.join(lafida_dir, "Slam_Settings_indoor1.yaml"))
    track, _ = lafida.extractor_params(s)
    n_mf, C, W, H = 2, rig["n_cams"], 754, 480
    imgs = np.zeros((n_mf, C, H, W), np.uint8)
    for m in range(n_mf):
        for c in range(C):
            imgs[m, c], _ = synth.fisheye_frame(W, H, seed=60 + 3 * m + c, cam_index=c, cam=rig["cams"][c])
    b = mf.MultiFrameBuilder(rig, track, max_multiframes=n_mf)
    out = b.build(torch.from_numpy(imgs).cuda())
    torch.cuda.synchronize()
    masks0 = [oracle_masks(cam["u0"], cam["v0"], W, H, 1)[0] for cam in rig["cams"]]
    for c in range(C):
        assert np.array_equal(b.d_masks[c].cpu().numpy(), masks0[c])
    for m in range(n_mf):
        hv = mf.MultiFrameBuilder.host_view(out, m)
        per_cam_k, per_cam_d = [], []
        for c in range(C):
            okps, odesc = ob.extract(imgs[m, c], masks0[c], nfeatures=track.nfeatures,
                                     fast_th=track.fast_threshold)
            n = int(hv["N"][c])
            assert n == len(okps) > 50
            k = out["kps"][m, c, :n].cpu().numpy().reshape(-1).view(ob.KEYPOINT_DTYPE)
            for f in okps.dtype.names:
                assert np.array_equal(k[f], okps[f]), (m, c, f)
            assert np.array_equal(out["desc"][m, c, :n].cpu().numpy(), odesc)
            # GetMirrorMask(0): every keypoint is inside the circle
            assert (masks0[c][np.rint(k["y"]).astype(int), np.rint(k["x"]).astype(int)] > 0).all()
            rays = out["rays"][m, c, :n].cpu().numpy()
            for i in range(0, n, 11):
                ref = ob.cam_img_to_world(rig["cam_models"][c], float(k["x"][i]), float(k["y"][i]))
                assert np.array_equal(rays[i], np.asarray(ref))
            per_cam_k.append(k)
            per_cam_d.append(odesc)
        cnt = hv["N"]
        kp_blocks = np.zeros((C, max(cnt)), ob.KEYPOINT_DTYPE)
        d_blocks = np.zeros((C, max(cnt), 32), np.uint8)
        for c in range(C):
            kp_blocks[c, :cnt[c]] = per_cam_k[c]
            d_blocks[c, :cnt[c]] = per_cam_d[c]
        ref = rigmod.concat_multiframe(cnt, kp_blocks, d_blocks)
        assert hv["mvKeys"].tobytes() == ref["mvKeys"].tobytes()
        assert np.array_equal(hv["keypoint_to_cam"], ref["keypoint_to_cam"])
        assert np.array_equal(hv["cont_idx_to_local_cam_idx"], ref["cont_idx_to_local_cam_idx"])
        assert np.array_equal(hv["descriptors"], np.concatenate(ref["descriptors"]))
        assert not hv["descriptor_masks"].any()            # ORB settings: Mat::zeros masks
        px, py, inside = rigmod.grid_positions(ref["mvKeys"]["x"], ref["mvKeys"]["y"], W, H)
        assert np.array_equal(hv["grid_pos"], np.where(inside, px | (py << 8), -1))


@pytest.mark.gpu
def test_gpu_multiframe_builder_rejects_bad_batches(gpu, lafida_dir):  # noqa: F811
    import torch
    from mcs_amd import lafida, multiframe as mf
    rig = lafida.load_rig(lafida_dir)
    track, _ = lafida.extractor_params(lafida.load_settings(os.path.join(lafida_dir, "Slam_Settings_indoor1.yaml")))
    b = mf.MultiFrameBuilder(rig, track, max_multiframes=1)
    with pytest.raises(ValueError):
        b.build(torch.zeros((2, 3, 480, 754), dtype=torch.uint8, device="cuda"))
    with pytest.raises(ValueError):
        b.build(torch.zeros((1, 2, 480, 754), dtype=torch.uint8, device="cuda"))
