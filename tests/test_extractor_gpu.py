"""GPU parity: the HIP extractor vs the CPU restatement (oracle/), stage by stage and
end to end, bit-exact (integer/byte/index work -> no tolerance).

Reference path: mdBRIEFextractorOct::operator() (src/mdBRIEFextractorOct.cpp:1244-1337).
"""
import numpy as np
import pytest

from tests import oracle_bind as ob

pytestmark = pytest.mark.gpu


def _extractor(w, h, nfeatures=1000, fast_th=20, max_frames=1, desc_size=32):
    import mcs_amd
    p = mcs_amd.ExtractorParams(nfeatures=nfeatures, fast_threshold=fast_th, desc_size=desc_size)
    return mcs_amd.Extractor(p, w, h, max_frames=max_frames)


def _frame(w=754, h=480, seed=3):
    from mcs_amd import synth
    return synth.fisheye_frame(w, h, seed=seed)


def test_pyramid_and_blur_stages(gpu):
    img, mask = _frame(seed=11)
    ex = _extractor(754, 480)
    ex.extract(img, mask)
    ref = ob.pyramid(img)
    for l in range(8):
        got = ex.read_stage(0, 0, l)
        assert np.array_equal(got, ref[l]), "pyramid level %d differs (%d px)" % (
            l, int((got != ref[l]).sum()))
        gb = ex.read_stage(1, 0, l)
        assert np.array_equal(gb, ob.box_blur5(ref[l])), "blur level %d differs" % l


def test_fast_candidates_and_octree_stages(gpu):
    img, mask = _frame(seed=12)
    ex = _extractor(754, 480, nfeatures=2000)
    ex.extract(img, mask)
    lv = ob.pyramid(img)
    mk = ob.mask_pyramid(mask)
    nfl = ob.features_per_level(2000)
    for l in range(8):
        ref = ob.level_candidates(lv[l], mk[l], 20)
        got = ex.read_stage(2, 0, l)
        assert got.shape == ref.shape, (l, got.shape, ref.shape)
        assert np.array_equal(got, ref), "FAST candidates differ at level %d" % l
        h, w = lv[l].shape
        sel_ref = ref[ob.octree(ref, w, h, int(nfl[l]))]
        sel = ex.read_stage(3, 0, l)
        assert np.array_equal(sel, sel_ref), "octree selection differs at level %d" % l


@pytest.mark.parametrize("seed,nfeat,th", [(1, 1000, 20), (2, 2000, 20), (3, 2000, 5), (4, 400, 20)])
def test_extract_end_to_end(gpu, seed, nfeat, th):
    img, mask = _frame(seed=seed)
    ex = _extractor(754, 480, nfeatures=nfeat, fast_th=th)
    kps, desc = ex.extract(img, mask)
    okps, odesc = ob.extract(img, mask, nfeatures=nfeat, fast_th=th)
    assert len(kps) == len(okps)
    for f in okps.dtype.names:
        assert np.array_equal(kps[f], okps[f]), "field %s differs" % f
    assert np.array_equal(desc, odesc)


def test_extract_no_mask_and_noise_image(gpu):
    from mcs_amd import synth
    img = synth.random_frame(754, 480, seed=5)
    ex = _extractor(754, 480, nfeatures=1000)
    kps, desc = ex.extract(img, None)
    okps, odesc = ob.extract(img, None, nfeatures=1000)
    assert np.array_equal(kps, okps) and np.array_equal(desc, odesc)


def test_extract_empty_and_flat_image(gpu):
    ex = _extractor(754, 480)
    flat = np.full((480, 754), 128, np.uint8)
    kps, desc = ex.extract(flat)
    assert len(kps) == 0 and desc.shape[0] == 0


@pytest.mark.parametrize("desc_size", [16, 64])
def test_descriptor_sizes(gpu, desc_size):
    img, mask = _frame(seed=21)
    ex = _extractor(754, 480, nfeatures=1000, desc_size=desc_size)
    kps, desc = ex.extract(img, mask)
    okps, odesc = ob.extract(img, mask, nfeatures=1000, desc_size=desc_size)
    assert np.array_equal(kps, okps) and np.array_equal(desc, odesc)


def test_config_d_frame_1024(gpu):
    img, mask = _frame(1024, 1024, seed=31)
    ex = _extractor(1024, 1024, nfeatures=4000)
    kps, desc = ex.extract(img, mask)
    okps, odesc = ob.extract(img, mask, nfeatures=4000)
    assert np.array_equal(kps, okps) and np.array_equal(desc, odesc)


def test_batch_device_matches_single(gpu):
    import torch
    import mcs_amd
    frames, masks = [], []
    for s in range(6):
        img, mask = _frame(seed=40 + s)
        frames.append(img)
        masks.append(mask)
    ex = _extractor(754, 480, nfeatures=2000, max_frames=6)
    dev = torch.device("cuda:0")
    d_img = torch.from_numpy(np.stack(frames)).to(dev)
    d_mask = torch.from_numpy(np.stack(masks[:3])).to(dev)
    d_midx = torch.tensor([0, 1, 2, 0, 1, 2], dtype=torch.int32, device=dev)
    ex.set_masks_device(d_mask.data_ptr(), 3)
    cap = ex.capacity
    d_kps = torch.zeros((6, cap * 7), dtype=torch.int32, device=dev)
    d_cnt = torch.zeros(6, dtype=torch.int32, device=dev)
    d_desc = torch.zeros((6, cap, 32), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ex.extract_batch_device(d_img.data_ptr(), 6, d_midx.data_ptr(), d_kps.data_ptr(),
                            d_cnt.data_ptr(), d_desc.data_ptr(), s)
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy()
    kp_all = d_kps.cpu().numpy().view(mcs_amd.KEYPOINT_DTYPE).reshape(6, cap)
    de_all = d_desc.cpu().numpy()
    for f in range(6):
        okps, odesc = ob.extract(frames[f], masks[f % 3], nfeatures=2000)
        assert cnt[f] == len(okps)
        assert np.array_equal(kp_all[f, :cnt[f]], okps)
        assert np.array_equal(de_all[f, :cnt[f]], odesc)
