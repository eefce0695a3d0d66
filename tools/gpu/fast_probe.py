"""Phase split of k_fast_rows on the config-B batch, from a variant build with -DMCS_FAST_PROBE
(tools/build_variants.sh probe "-DMCS_FAST_PROBE"): shader cycles summed over all waves per
phase, survivors / corners per band.  Usage: MCS_AMD_LIB=<variant lib> python fast_probe.py"""
import ctypes
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "multicol-slam-annotation_amd"))
import numpy as np
import torch
import mcs_amd
from mcs_amd import synth

M, NC = 171, 3
uimgs, imgs, masks, midx, pairs = synth.config_b_batch(M)
F = M * NC
ex = mcs_amd.Extractor(mcs_amd.ExtractorParams(nfeatures=2000, fast_threshold=20), 754, 480, max_frames=F)
dev = torch.device("cuda:0")
s = torch.cuda.current_stream().cuda_stream
d_img = torch.from_numpy(imgs).to(dev)
d_mask = torch.from_numpy(masks).to(dev)
ex.set_masks_device(d_mask.data_ptr(), NC, s)
d_midx = torch.from_numpy(midx).to(dev)
cap = ex.capacity
d_kps = torch.zeros((F, cap * 7), dtype=torch.int32, device=dev)
d_cnt = torch.zeros(F, dtype=torch.int32, device=dev)
d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
L = mcs_amd.lib()
f = L.mcs_debug_fast_probe
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = np.zeros(8, np.uint64)
for rep in range(3):
    f(out.ctypes.data_as(ctypes.c_void_p), 1)
    ex.extract_batch_device(d_img.data_ptr(), F, d_midx.data_ptr(), d_kps.data_ptr(), d_cnt.data_ptr(),
                            d_desc.data_ptr(), s)
    torch.cuda.synchronize()
f(out.ctypes.data_as(ctypes.c_void_p), 0)
tot = float(out[4])
names = ["load+ring", "compass+list", "exact+score", "nms+mask+append"]
print("k_fast_rows phase split (cycles summed over waves, one batch of %d frames):" % F)
for k in range(4):
    print("  %-16s %6.1f %%" % (names[k], 100.0 * float(out[k]) / tot))
print("  skipped bands    %6.1f %%" % (100.0 * float(out[6]) / tot))
print("  setup            %6.1f %%" % (100.0 * float(out[7]) / tot))
print("  other            %6.1f %%" % (100.0 * (tot - sum(float(out[k]) for k in (0, 1, 2, 3, 6, 7))) / tot))
print("  bands %d  cycles/band %.0f" % (out[5], tot / max(1, out[5])))
