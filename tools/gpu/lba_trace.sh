# Kernel trace of LocalBA calls (config C): per-kernel durations and the idle gaps between them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lbatr -o run -- python3 tools/gpu/lba_time.py > gpurun_out/lbatr.log 2>&1 || { tail -5 gpurun_out/lbatr.log; exit 1; }
T=$(find gpurun_out/lbatr -name '*kernel_trace.csv' | head -1)
python3 - "$T" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# last ~400 kernels (the max_iterations=10 optimize calls at the end)
rows = rows[-400:]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print("kernels", len(rows), "busy us %.1f span us %.1f busy%% %.1f" % (busy / 1e3, span / 1e3, 100 * busy / span))
from collections import defaultdict
d = defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0][:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print("%-42s n=%4d mean %.2f us total %.1f" % (k, len(v), sum(v) / len(v), sum(v)))
gaps = [(int(rows[i + 1]["Start_Timestamp"]) - int(rows[i]["End_Timestamp"])) / 1e3 for i in range(len(rows) - 1)]
gaps.sort()
print("gap us: median %.2f p90 %.2f max %.1f" % (gaps[len(gaps) // 2], gaps[int(len(gaps) * 0.9)], gaps[-1]))
PY
