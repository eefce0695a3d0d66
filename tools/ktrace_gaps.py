"""Split the last `calls` LocalBA calls of a rocprofv3 kernel trace (calls are separated by the
first k_edges launch after a gap > 150 us... simpler: the trace's tail, 1/N of the rows per
call) into per-kernel device time and the idle gaps between consecutive kernels, listing the
largest gaps with the kernels on either side."""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
# the script runs 3 warm-up calls + ncalls traced calls: keep the last ncalls / (ncalls + 3)
rows = rows[len(rows) * 3 // (ncalls + 3):]
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "")[:44]  # noqa: E731
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print("calls %d kernels %d: busy %.1f us, span %.1f us per call (busy %.0f%%)" % (
    ncalls, len(rows), busy / 1e3 / ncalls, span / 1e3 / ncalls, 100.0 * busy / span))
d = defaultdict(list)
for r in rows:
    d[name(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print("  %-46s n/call %5.1f mean %6.2f us  total/call %7.1f" % (k, len(v) / ncalls, sum(v) / len(v), sum(v) / ncalls))
gaps = []
for i in range(len(rows) - 1):
    g = (int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3
    gaps.append((g, name(rows[i]), name(rows[i + 1])))
tot = sum(g for g, _, _ in gaps)
print("gaps: total %.1f us per call" % (tot / ncalls))
agg = defaultdict(lambda: [0, 0.0])
for g, a, b in gaps:
    agg[(a, b)][0] += 1
    agg[(a, b)][1] += g
for (a, b), (n, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:14]:
    print("  %7.1f us/call  n/call %5.1f  %s -> %s" % (s / ncalls, n / ncalls, a, b))
