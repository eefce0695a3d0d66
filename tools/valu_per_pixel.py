#!/usr/bin/env python3
"""VALU instructions per pixel of the headline kernels from an SQ pass-A counter file
(tools/gpu/final_profile.sh: SQ_WAVES, SQ_INSTS_VALU per dispatch).

  lane-ops per pixel = SQ_INSTS_VALU (wave instructions) * 64 lanes / pixels processed
  k_pyr_rows<true, 2>: output pixels of levels 1..L-1 (one dispatch per level per call)
  k_fast_rows<16>    : level pixels of levels 0..L-1 (one dispatch per call)
Level sizes follow the extractor plan (cvRound(W / 1.2^l), the scale factor as float).
Usage: valu_per_pixel.py counter_collection.csv frames_per_call [W H nlevels] > out.json"""
import csv
import json
import sys
from collections import defaultdict

import numpy as np


def level_px(W, H, n, scale=1.2):
    sf, out = 1.0, []
    s = float(np.float32(scale))
    for l in range(n):
        if l:
            sf *= s
        isf = 1.0 / sf
        out.append(int(np.rint(W * isf)) * int(np.rint(H * isf)))
    return out


def main():
    path, frames = sys.argv[1], float(sys.argv[2])   # per dispatch group (a split step: 513 / 2)
    W, H, nl = (int(v) for v in sys.argv[3:6]) if len(sys.argv) >= 6 else (754, 480, 8)
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("mcs::", "")
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add(row.get("Dispatch_Id", ""))
    px = level_px(W, H, nl)
    out = {"source": path, "frames_per_call": frames, "level_pixels": px,
           "method": "SQ_INSTS_VALU * 64 / pixels (wave instructions x lanes)"}
    for name, per_call_launches, pixels in (("k_pyr_rows<true, 2>", nl - 1, sum(px[1:]) * frames),
                                            ("k_fast_rows<16>", 1, sum(px) * frames)):
        if name not in acc:
            continue
        calls = len(disp[name]) / per_call_launches
        valu = acc[name]["SQ_INSTS_VALU"] / calls
        out[name] = {"calls": calls, "valu_wave_instr_per_call": valu,
                     "valu_lane_ops_per_pixel": round(valu * 64 / pixels, 2),
                     "waves_per_call": acc[name]["SQ_WAVES"] / calls}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
