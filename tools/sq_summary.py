#!/usr/bin/env python3
"""Per-kernel SQ counter summary from a rocprofv3 --pmc counter_collection.csv.

Default: instructions per wave and the wave-cycle split active / issue-stall / parked.
--all: additionally every collected counter per kernel (sum over dispatches) and per wave."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(set)
args = [a for a in sys.argv[1:] if not a.startswith("--")]
path = args[0]
for row in csv.DictReader(open(path)):
    k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("mcs::", "")
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    cnt[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
print("# " + path)
if "SQ_ACTIVE_INST_ANY" in next(iter(acc.values()), {}):
    print("%-28s %6s %9s %8s %8s %8s %7s %7s %7s" % ("kernel", "disp", "waves", "valu/w", "lds/w",
                                                     "salu/w", "act%", "stall%", "park%"))
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        w = c.get("SQ_WAVES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print("%-28s %6d %9d %8.0f %8.0f %8.0f %7.1f %7.1f %7.1f" % (
            k[:28], len(cnt[k]), w, c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_LDS", 0) / w,
            c.get("SQ_INSTS_SALU", 0) / w, 100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            100 * c.get("SQ_WAIT_INST_ANY", 0) / wc, 100 * c.get("SQ_WAIT_ANY", 0) / wc))
if "SQ_LDS_IDX_ACTIVE" in next(iter(acc.values()), {}):
    # pass B: VALU-issue share of wave time, LDS bank-conflict cycles per LDS-array cycle,
    # and SQ_LEVEL_WAVES / SQ_BUSY_CYCLES (mean resident waves per sampled SQ while busy)
    print("%-28s %9s %8s %10s %10s %9s" % ("kernel", "waves", "valu%", "ldsconf/acc", "lvl/busy", "salu_cyc/w"))
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        w = c.get("SQ_WAVES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        idx = c.get("SQ_LDS_IDX_ACTIVE", 0)
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0)
        busy = c.get("SQ_BUSY_CYCLES", 0) or 1
        print("%-28s %9d %8.1f %10.3f %10.2f %9.0f" % (
            k[:28], w, 100 * c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            bc / (idx - bc) if idx > bc else 0.0, c.get("SQ_LEVEL_WAVES", 0) / busy,
            c.get("SQ_INST_CYCLES_SALU", 0) / w))
# Issue utilisation per SIMD (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* count
# quad-cycles; SQ_BUSY_CYCLES is summed over the 32 SQs (8 XCDs x 4 SEs) in cycles): a VALU
# instruction occupies its SIMD for one quad-cycle, so
#   valu_util = 4 * SQ_ACTIVE_INST_VALU / 1024 SIMDs / (SQ_BUSY_CYCLES / 32)
# is the fraction of the kernel's busy time each SIMD spent issuing VALU (MFMA included).
NSQ, NSIMD = 32, 1024
if "SQ_BUSY_CYCLES" in next(iter(acc.values()), {}):
    util = {}
    print("%-28s %9s %10s" % ("kernel", "valu_util", "waves/SIMD"))
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        busy = c.get("SQ_BUSY_CYCLES", 0) / NSQ
        if busy <= 0 or "SQ_ACTIVE_INST_VALU" not in c:
            continue
        u = 4 * c["SQ_ACTIVE_INST_VALU"] / NSIMD / busy
        occ = 4 * c.get("SQ_WAVE_CYCLES", 0) / NSIMD / busy
        util[k] = {"valu_util": round(u, 3), "waves_per_simd": round(occ, 2), "dispatches": len(cnt[k])}
        print("%-28s %9.3f %10.2f" % (k[:28], u, occ))
    for a in sys.argv:
        if a.startswith("--json="):
            import json
            json.dump({"source": path, "method": "4*SQ_ACTIVE_INST_VALU/1024/(SQ_BUSY_CYCLES/32)",
                       "kernels": util}, open(a[7:], "w"), indent=1)
if "--all" in sys.argv:
    for k, c in sorted(acc.items()):
        if not k.startswith(("k_", "pyr", "fast", "ldlt", "ba::", "voc")) and "k_" not in k:
            continue
        print("%s  dispatches=%d" % (k[:60], len(cnt[k])))
        for n, v in sorted(c.items()):
            print("    %-26s %16.0f" % (n, v))
