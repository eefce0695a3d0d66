"""Camera, rig and epipolar math pinned to the reference's own text.

tests/golden/refmath.npz holds evaluations of the reference functions themselves, produced by
tests/golden/gen_refmath.py from the reference sources read as text (statement by statement):
  ImgToWorld     src/cam_model_omni.cpp:49-67       -> bearing rays (row a10)
  WorldToImg     src/cam_model_omni.cpp:147-163     -> projections (rows a15, f2)
  cayley2rot     include/misc.h:134-162             -> rotations (row a14)
  computeError   src/g2o_MultiCol_vertices_edges.cpp:32-63 -> residuals (row a15)
  ComputeE       src/misc.cpp:72-86 per camera pair (src/cORBmatcher.cpp:985-998)
  CheckDistEpipolarLine  src/misc.cpp:54-70         -> epipolar decisions (row a12)

Checked against it: the oracle (CPU tests) and the product (GPU tests, through the C-ABI).
Tolerances: rays, ComputeE, epipolar dsqr / decisions and cayley2rot EXACT (the same correctly
rounded + - * / sqrt in the same order); projections and residuals rel 1e-12 of the pixel
value (they go through atan: device atan vs glibc atan may differ in the last ulp).
"""
import ctypes
import os

import numpy as np
import pytest

from tests import oracle_bind as ob

GOLD = os.path.join(os.path.dirname(__file__), "golden", "refmath.npz")


@pytest.fixture(scope="module")
def gold():
    g = np.load(GOLD)
    return {k: g[k] for k in g.files}


def _cam_model(g, i):
    from mcs_amd import CamModel
    c = g["cam"][i]
    return CamModel.from_dict(dict(Iw=754, Ih=480, c=c[0], d=c[1], e=c[2], u0=c[3], v0=c[4],
                                   a=list(g["cam_p"][i]), pol=list(g["cam_invp"][i])))


def test_fixture_shape(gold):
    assert int(gold["n_statements"]) >= 70
    assert len(gold["rays"]) == 600 and len(gold["uv"]) == 402
    assert gold["ep_ok"].sum() > 50 and (1 - gold["ep_ok"]).sum() > 50
    near = (gold["ep_dsqr"] > 5e-3) & (gold["ep_dsqr"] < 2e-2)
    assert near.sum() > 30          # decisions close to the 1e-2 threshold are covered
    assert np.isnan(gold["ep_dsqr"][-1]) and gold["ep_ok"][-1] == 0   # den == 0


# ------------------------------------------------------------------ oracle vs reference text
def test_oracle_img_to_world(built, gold):
    for i in range(len(gold["px"])):
        cam = _cam_model(gold, gold["px_cam"][i])
        got = ob.cam_img_to_world(cam, *gold["px"][i])
        assert np.array_equal(got, gold["rays"][i]), i


def test_oracle_world_to_img(built, gold):
    for i in range(len(gold["pts"])):
        cam = _cam_model(gold, gold["pt_cam"][i])
        got = ob.cam_world_to_img(cam, *gold["pts"][i])
        ref = gold["uv"][i]
        assert np.all(np.abs(got - ref) <= 1e-12 * np.maximum(1.0, np.abs(ref))), i


def test_oracle_compute_error(built, gold):
    for i in range(len(gold["e_err"])):
        err, _, _ = ob.ba_edge(gold["e_pose"][i], gold["e_pt"][i], gold["e_mc"][i],
                               gold["e_cam"][i], gold["e_meas"][i])
        proj = gold["e_meas"][i] - err
        ref = gold["e_proj"][i]
        assert np.all(np.abs(proj - ref) <= 1e-12 * np.abs(ref)), i
        assert np.all(np.abs(err - gold["e_err"][i]) <= 1e-12 * np.abs(ref)), i


def test_oracle_compute_e_and_epipolar(built, gold):
    for k in range(len(gold["rig_mt1"])):
        E = ob.compute_e_rig(gold["rig_mt1"][k], gold["rig_mt2"][k], gold["rig_mc"])
        assert np.array_equal(E, gold["rig_E"][k]), k
    for i in range(len(gold["ep_ok"])):
        E = gold["rig_E"][gold["ep_rig"][i], gold["ep_cam"][i], gold["ep_cam"][i]]
        ok, d = ob.check_dist_epipolar_line(gold["ep_ray1"][i], gold["ep_ray2"][i], E, 1e-2)
        assert ok == bool(gold["ep_ok"][i]), i
        assert np.array_equal(d, gold["ep_dsqr"][i], equal_nan=True), i


# ------------------------------------------------------------------ product vs reference text
@pytest.mark.gpu
def test_product_compute_e_and_epipolar(gpu, gold):
    import mcs_amd
    L = mcs_amd.lib()
    P = ob._p
    for k in range(len(gold["rig_mt1"])):
        E = np.zeros((3, 3, 3, 3))
        mc = np.ascontiguousarray(gold["rig_mc"])
        assert L.mcs_compute_e_rig(P(np.ascontiguousarray(gold["rig_mt1"][k])),
                                   P(np.ascontiguousarray(gold["rig_mt2"][k])), P(mc), 3, P(E)) == 0
        assert np.array_equal(E, gold["rig_E"][k]), k
    for i in range(len(gold["ep_ok"])):
        E = np.ascontiguousarray(gold["rig_E"][gold["ep_rig"][i], gold["ep_cam"][i], gold["ep_cam"][i]])
        r = L.mcs_check_dist_epipolar_line(P(np.ascontiguousarray(gold["ep_ray1"][i])),
                                           P(np.ascontiguousarray(gold["ep_ray2"][i])), P(E), 1e-2)
        assert r == int(gold["ep_ok"][i]), i


@pytest.mark.gpu
def test_gpu_keypoint_rays(gpu, gold):
    import torch
    import mcs_amd
    from mcs_amd import KEYPOINT_DTYPE
    cams = [_cam_model(gold, c) for c in range(3)]
    cap = 640
    kps = np.zeros((3, cap), KEYPOINT_DTYPE)
    cnt = np.zeros(3, np.int32)
    slot = []
    for i in range(len(gold["px"])):
        c = gold["px_cam"][i]
        kps[c, cnt[c]]["x"], kps[c, cnt[c]]["y"] = gold["px"][i]
        slot.append((c, cnt[c]))
        cnt[c] += 1
    dev = torch.device("cuda", 0)
    d_kps = torch.from_numpy(kps.view(np.int32).reshape(3, cap * 7).copy()).to(dev)
    d_cnt = torch.from_numpy(cnt).to(dev)
    cidx = torch.arange(3, dtype=torch.int32, device=dev)
    d_cams = torch.frombuffer(bytearray(b"".join(bytes(c) for c in cams)), dtype=torch.uint8).to(dev)
    d_rays = torch.zeros((3, cap, 3), dtype=torch.float64, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = torch.cuda.current_stream().cuda_stream
    assert mcs_amd.lib().mcs_keypoint_rays_device(P(d_kps), P(d_cnt), 3, cap, P(cidx), P(d_cams),
                                                  P(d_rays), ctypes.c_void_p(st)) == 0
    torch.cuda.synchronize()
    rays = d_rays.cpu().numpy()
    for i, (c, s) in enumerate(slot):
        assert np.array_equal(rays[c, s], gold["rays"][i]), i


def _edge_problem(poses, pts, mc, cam, meas):
    n = len(pts)
    return dict(poses=np.ascontiguousarray(poses), pose_fixed=np.zeros(n, np.uint8),
                points=np.ascontiguousarray(pts), mc=np.ascontiguousarray(mc),
                cam=np.ascontiguousarray(cam), edge_pose=np.arange(n, dtype=np.int32),
                edge_point=np.arange(n, dtype=np.int32), edge_cam=np.arange(n, dtype=np.int32),
                edge_meas=np.ascontiguousarray(meas), edge_info=np.tile(np.eye(2), (n, 1, 1)),
                huber_delta=1.345 * 2)


@pytest.mark.gpu
def test_gpu_compute_error(gpu, gold):
    from mcs_amd import ba
    pr = _edge_problem(gold["e_pose"], gold["e_pt"], gold["e_mc"], gold["e_cam"], gold["e_meas"])
    err, _, _ = ba.Solver().linearize(pr)
    proj = gold["e_meas"] - err
    ref = gold["e_proj"]
    assert np.all(np.abs(proj - ref) <= 1e-12 * np.abs(ref))
    assert np.all(np.abs(err - gold["e_err"]) <= 1e-12 * np.abs(ref))


@pytest.mark.gpu
def test_gpu_world_to_img_through_identity_rig(gpu, gold):
    """WorldToImg on the device: an edge whose rig poses are the identity Cayley vector maps the
    point through I (cayley2hom(0) = I exactly, invMat(I) = I), so the residual is meas - uv."""
    from mcs_amd import ba
    n = len(gold["pts"])
    cam = np.concatenate([gold["cam"], gold["cam_invp"]], 1)[gold["pt_cam"]]
    pr = _edge_problem(np.zeros((n, 6)), gold["pts"], np.zeros((n, 6)), cam, np.zeros((n, 2)))
    err, _, _ = ba.Solver().linearize(pr)
    ref = gold["uv"]
    assert np.all(np.abs(-err - ref) <= 1e-12 * np.maximum(1.0, np.abs(ref)))
