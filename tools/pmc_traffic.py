#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; collected in SEPARATE runs as
MI355X_MICROARCH.md prescribes) into HBM bytes per kernel launch.

Units/corrections (MI355X_MICROARCH.md "HBM"): both counters are in KiB.  On gfx950
FETCH_SIZE reads half the bytes of a wide (16 B/lane) coalesced stream, so the corrected
read bytes are 2 * FETCH_SIZE * 1024; for other access widths the factor is uncalibrated,
so both the raw and the x2-corrected figures are recorded.  WRITE_SIZE * 1024 is exact for
16 B/lane stores.

usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json> [extractor calls per step]
(bench.py runs a step as two extractor calls, one per half of its multi-frames: pass 2)
"""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            per[name].append(float(row["Counter_Value"]))
    return per


def short(name):
    return name.split("(")[0].replace("void ", "").replace("mcs::", "")


def main(fetch_csv, write_csv, out_json, per_step="1"):
    per_step = int(per_step)
    fe = load(fetch_csv, "FETCH_SIZE")
    wr = load(write_csv, "WRITE_SIZE")
    out = {"note": "bytes per launch; fetch_raw = FETCH_SIZE*1024, fetch_x2 = gfx950 wide-read "
                   "correction (exact only for 16B/lane streams); write = WRITE_SIZE*1024",
           "kernels": {}}
    for name in sorted(set(fe) | set(wr)):
        f = fe.get(name, [])
        w = wr.get(name, [])
        out["kernels"][short(name)] = {
            "launches": max(len(f), len(w)),
            "fetch_raw": (sum(f) / len(f) * 1024) if f else None,
            "fetch_x2": (2 * sum(f) / len(f) * 1024) if f else None,
            "write": (sum(w) / len(w) * 1024) if w else None,
        }
    k = out["kernels"]
    # per extractor call (= one k_fast_rows launch): every k_pyr_rows<true> launch of the call
    # (one per level 1..L-1: resize + fused blur) + the FAST launch
    fa = next((v for n, v in k.items() if n.startswith("k_fast_rows") or n.startswith("k_fast_cells")), None)
    rs = [v for n, v in k.items() if n.startswith("k_pyr_rows<true")]
    if rs and fa and fa["launches"]:
        calls = fa["launches"] / per_step   # bench steps (a "call" below is one step)
        out["extractor_calls_per_step"] = per_step
        rd = sum(v["fetch_raw"] * v["launches"] for v in rs) / calls + fa["fetch_raw"] * per_step
        rd2 = sum(v["fetch_x2"] * v["launches"] for v in rs) / calls + fa["fetch_x2"] * per_step
        wt = sum((v["write"] or 0) * v["launches"] for v in rs) / calls + (fa["write"] or 0) * per_step
        out["pyr_launches_per_call"] = sum(v["launches"] for v in rs) / calls
        out["pyramid+fast_raw_bytes_per_call"] = rd + wt
        out["pyramid+fast_fetch_raw_per_call"] = rd
        out["pyramid+fast_write_per_call"] = wt
        # gfx950 x2 read correction (MI355X_MICROARCH.md "HBM"; exact for 16 B/lane only)
        out["pyramid+fast_bytes_per_call"] = rd2 + wt
    out["source"] = {"fetch": fetch_csv, "write": write_csv}
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
