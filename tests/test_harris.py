"""HarrisResponses opt-in: src/mdBRIEFextractorOct.cpp:86-132.

The reference defines it but its octree extractor never calls it, so it is a separate device
entry point (mcs_harris_responses_device).  CPU: the oracle (padded-level pointer walk, as the
reference) equals an independent numpy restatement (reflect-101 padding + vectorised Sobel
sums, float32 expression in the same order).  GPU: the kernel equals the oracle bit-exactly on
all 8 levels of a Lafida frame, keypoints near the borders included.
"""
import ctypes

import numpy as np
import pytest

from tests import oracle_bind as ob


def _oracle(img, xy, bs=7, k=0.04):
    img = np.ascontiguousarray(img, np.uint8)
    xy = np.ascontiguousarray(xy, np.float32)
    out = np.zeros(len(xy), np.float32)
    ob.lib().oracle_harris_responses(ob._p(img), img.shape[1], img.shape[0], ob._p(xy), len(xy),
                                     bs, k, ob._p(out))
    return out


def _numpy(img, xy, bs=7, k=np.float32(0.04)):
    P = np.pad(img.astype(np.int64), 25, mode="reflect")      # numpy reflect == REFLECT_101
    Ix = 2 * (P[1:-1, 2:] - P[1:-1, :-2]) + (P[:-2, 2:] - P[:-2, :-2]) + (P[2:, 2:] - P[2:, :-2])
    Iy = 2 * (P[2:, 1:-1] - P[:-2, 1:-1]) + (P[2:, :-2] - P[:-2, :-2]) + (P[2:, 2:] - P[:-2, 2:])
    r = bs // 2
    out = np.zeros(len(xy), np.float32)
    for i, (x, y) in enumerate(xy):
        x0, y0 = int(np.rint(np.float32(x))), int(np.rint(np.float32(y)))
        # Ix/Iy index (py-1, px-1) of the padded image = level pixel (py-26, px-26)
        ys = slice(y0 - r + 24, y0 - r + 24 + bs)
        xs = slice(x0 - r + 24, x0 - r + 24 + bs)
        gx, gy = Ix[ys, xs], Iy[ys, xs]
        a, b, c = (gx * gx).sum(), (gy * gy).sum(), (gx * gy).sum()
        fa, fb, fc = np.float32(a), np.float32(b), np.float32(c)
        scale = np.float32(1) / (np.float32(4 * bs) * np.float32(255))
        s4 = scale * scale * scale * scale
        out[i] = (fa * fb - fc * fc - k * (fa + fb) * (fa + fb)) * s4
    return out


def _points(w, h, n, seed):
    rng = np.random.default_rng(seed)
    xy = np.stack([rng.integers(0, w, n), rng.integers(0, h, n)], 1).astype(np.float32)
    xy[: n // 4] += 0.5          # cvRound ties (half to even)
    xy[0] = (0, 0)
    xy[1] = (w - 1, h - 1)
    xy[2] = (2, h - 3)
    return xy


def test_oracle_matches_numpy_restatement(built):
    from mcs_amd import synth
    img, _ = synth.fisheye_frame(754, 480, seed=21)
    for bs in (7, 3, 9):
        xy = _points(754, 480, 300, bs)
        assert np.array_equal(_oracle(img, xy, bs), _numpy(img, xy, bs))
    xy = _points(754, 480, 50, 1)
    assert not np.array_equal(_oracle(img, xy, 7), _oracle(img, xy + 1.0, 7))


@pytest.mark.gpu
def test_gpu_harris_matches_oracle(gpu):
    import torch
    from mcs_amd import KEYPOINT_DTYPE, lib, synth
    img, _ = synth.fisheye_frame(754, 480, seed=22)
    lv = ob.pyramid(img)
    dev_levels = [torch.from_numpy(np.ascontiguousarray(L)).cuda() for L in lv]
    ptrs = torch.tensor([t.data_ptr() for t in dev_levels], dtype=torch.int64).cuda()
    geom = torch.tensor([[L.shape[1], L.shape[0], L.shape[1]] for L in lv], dtype=torch.int32).cuda()
    kps, want = [], []
    for l, L in enumerate(lv):
        xy = _points(L.shape[1], L.shape[0], 200, 100 + l)
        k = np.zeros(len(xy), KEYPOINT_DTYPE)
        k["x"], k["y"], k["octave"], k["class_id"] = xy[:, 0], xy[:, 1], l, -1
        kps.append(k)
        want.append(_oracle(L, xy))
    kps = np.concatenate(kps)
    want = np.concatenate(want)
    d_kps = torch.from_numpy(kps.view(np.int32).reshape(-1)).cuda()
    out = torch.zeros(len(kps), dtype=torch.float32, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert lib().mcs_harris_responses_device(P(ptrs), P(geom), len(lv), P(d_kps), len(kps), 7,
                                             0.04, P(out), None) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    assert (got != 0).mean() > 0.4      # points on the black outside of the mirror give 0
    assert lib().mcs_harris_responses_device(P(ptrs), P(geom), len(lv), P(d_kps), len(kps), 46,
                                             0.04, P(out), None) == -1
