"""Per-launch kernel durations grouped by (kernel, grid size) from a rocprofv3 kernel trace.

    python tools/ktrace_by_grid.py <run_kernel_trace.csv> [name-substring ...]
"""
import csv
import sys
from collections import defaultdict


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    g = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if pats and not any(p in name for p in pats):
                continue
            grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
            wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or "1"
            try:
                nwg = int(grid) // max(1, int(wg))
            except ValueError:
                nwg = grid
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            g[(name.split("(")[0][:48], nwg)].append(dur)
    for (n, nwg), v in sorted(g.items(), key=lambda kv: (kv[0][0], -1 if not isinstance(kv[0][1], int) else kv[0][1])):
        v.sort()
        print("%-48s wg=%-6s n=%-5d med=%9.2f us  min=%9.2f  max=%9.2f" % (n, nwg, len(v), v[len(v) // 2], v[0], v[-1]))


if __name__ == "__main__":
    main()
