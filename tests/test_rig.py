"""Camera-per-rank sharding of a MultiFrame on CPU with gloo.

The N>1 exchange step of the front-end is one all-gather per per-camera buffer
(mcs_amd/rig.py).  These tests run it with world_size 2 (and 3) on the gloo backend over
127.0.0.1, with per-camera keypoints/descriptors produced by the CPU oracle, and check the
gathered MultiFrame against the single-process concatenation of cMultiFrame
(src/cMultiFrame.cpp:166-184).
"""
import os
import socket

import numpy as np
import pytest

from mcs_amd import rig


def test_owned_cameras_partition_every_rig():
    for world in range(1, 9):
        for ncams in range(1, 9):
            owned = [rig.owned_cameras(ncams, world, r) for r in range(world)]
            flat = sorted(c for o in owned for c in o)
            assert flat == list(range(ncams))
            S = rig.slots_per_rank(ncams, world)
            assert all(len(o) <= S for o in owned)
            idx = rig.camera_order_index(ncams, world)
            # row of camera c = its rank's block + its slot on that rank
            for c in range(ncams):
                r = c % world
                assert idx[c] == r * S + owned[r].index(c)


def test_concat_multiframe_maps():
    from mcs_amd import KEYPOINT_DTYPE
    counts = [3, 0, 2]
    cap = 4
    kps = np.zeros((3, cap), KEYPOINT_DTYPE)
    for c in range(3):
        kps[c]["x"] = np.arange(cap) + 100 * c
        kps[c]["octave"] = c
    desc = np.arange(3 * cap * 32, dtype=np.uint32).astype(np.uint8).reshape(3, cap, 32)
    mf = rig.concat_multiframe(counts, kps, desc)
    assert list(mf["keypoint_to_cam"]) == [0, 0, 0, 2, 2]
    assert list(mf["cont_idx_to_local_cam_idx"]) == [0, 1, 2, 0, 1]
    assert list(mf["mvKeys"]["x"]) == [0, 1, 2, 200, 201]
    assert [d.shape[0] for d in mf["descriptors"]] == counts
    np.testing.assert_array_equal(mf["descriptors"][2], desc[2, :2])


def test_grid_positions_round_half_even():
    # 754 px wide / 64 cols: x = 5.890625 * k maps exactly to k; halfway points go to even
    w, h = 754, 480
    px, py, inside = rig.grid_positions([0.0, 753.0, 754.0], [0.0, 479.0, 480.0], w, h)
    assert list(px) == [0, 64, 64] and list(py) == [0, 48, 48]
    assert list(inside) == [True, False, False]
    half = (0.5 * w / 64.0)
    px, _, _ = rig.grid_positions([half, 3 * half], [0.0, 0.0], w, h)
    assert list(px) == [0, 2]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _camera_blocks(ncams, cap, nfeat):
    """Per-camera (count, kps words, desc) from the oracle on a rendered rig frame."""
    from mcs_amd import synth
    from tests import oracle_bind as ob
    imgs, masks = synth.rig_sequence(1, 754, 480, ncams, seed=5)
    cnt = np.zeros(ncams, np.int32)
    kw = np.zeros((ncams, cap, 7), np.int32)
    de = np.zeros((ncams, cap, 32), np.uint8)
    for c in range(ncams):
        k, d = ob.extract(imgs[c], masks[c], nfeatures=nfeat)
        n = min(len(k), cap)
        cnt[c] = n
        kw[c, :n] = np.ascontiguousarray(k[:n]).view(np.int32).reshape(n, 7)
        de[c, :n] = d[:n]
    return cnt, kw, de


def _worker(rank, world, port, ncams, cap, nfeat, out_dir):
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    try:
        cnt, kw, de = _camera_blocks(ncams, cap, nfeat)
        S = rig.slots_per_rank(ncams, world)
        mine = rig.owned_cameras(ncams, world, rank)
        lc = torch.zeros(S, dtype=torch.int32)
        lk = torch.zeros((S, cap, 7), dtype=torch.int32)
        ld = torch.zeros((S, cap, 32), dtype=torch.uint8)
        for s, c in enumerate(mine):   # "extract" only the cameras this rank owns
            lc[s] = int(cnt[c])
            lk[s] = torch.from_numpy(kw[c])
            ld[s] = torch.from_numpy(de[c])
        gc = rig.gather_camera_blocks(lc, ncams)
        gk = rig.gather_camera_blocks(lk, ncams)
        gd = rig.gather_camera_blocks(ld, ncams)
        mf = rig.concat_multiframe(gc.numpy(), gk.numpy(), gd.numpy())
        ref = rig.concat_multiframe(cnt, kw, de)
        assert np.array_equal(mf["N"], ref["N"])
        assert mf["mvKeys"].tobytes() == ref["mvKeys"].tobytes()
        assert np.array_equal(mf["keypoint_to_cam"], ref["keypoint_to_cam"])
        assert np.array_equal(mf["cont_idx_to_local_cam_idx"], ref["cont_idx_to_local_cam_idx"])
        for a, b in zip(mf["descriptors"], ref["descriptors"]):
            assert np.array_equal(a, b)
        open(os.path.join(out_dir, "ok%d" % rank), "w").write("%d" % len(mf["mvKeys"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,ncams", [(2, 3), (3, 3), (2, 8)])
def test_gather_multiframe_gloo(built, tmp_path, world, ncams):
    import torch.multiprocessing as mp
    cap, nfeat = 400, 300
    mp.spawn(_worker, args=(world, _free_port(), ncams, cap, nfeat, str(tmp_path)),
             nprocs=world, join=True)
    counts = [open(tmp_path / ("ok%d" % r)).read() for r in range(world)]
    assert len(set(counts)) == 1 and int(counts[0]) > 0
