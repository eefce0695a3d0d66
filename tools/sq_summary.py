#!/usr/bin/env python3
"""Per-kernel SQ counter summary from a rocprofv3 --pmc counter_collection.csv.

Default: instructions per wave and the wave-cycle split active / issue-stall / parked.
--all: additionally every collected counter per kernel (sum over dispatches) and per wave."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(set)
for row in csv.DictReader(open(sys.argv[1])):
    k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("mcs::", "")
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    cnt[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
print("# " + sys.argv[1])
if "SQ_WAVE_CYCLES" in next(iter(acc.values()), {}):
    print("%-28s %6s %9s %8s %8s %8s %7s %7s %7s" % ("kernel", "disp", "waves", "valu/w", "lds/w",
                                                     "salu/w", "act%", "stall%", "park%"))
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        w = c.get("SQ_WAVES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print("%-28s %6d %9d %8.0f %8.0f %8.0f %7.1f %7.1f %7.1f" % (
            k[:28], len(cnt[k]), w, c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_LDS", 0) / w,
            c.get("SQ_INSTS_SALU", 0) / w, 100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            100 * c.get("SQ_WAIT_INST_ANY", 0) / wc, 100 * c.get("SQ_WAIT_ANY", 0) / wc))
if "--all" in sys.argv:
    for k, c in sorted(acc.items()):
        if not k.startswith(("k_", "pyr", "fast", "ldlt", "ba::", "voc")) and "k_" not in k:
            continue
        print("%s  dispatches=%d" % (k[:60], len(cnt[k])))
        for n, v in sorted(c.items()):
            print("    %-26s %16.0f" % (n, v))
