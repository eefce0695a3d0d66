# Kernel trace of the extract+match leg (5 steps): per-kernel stats + per-launch durations of
# the kernels named in $2 (regex).  Usage: ktrace_extract.sh TAG [REGEX]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-kt}; RX=${2:-k_octree}
OUT=gpurun_out/kt_$TAG; mkdir -p $OUT
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "prof failed"; tail -5 $OUT/bench.err; exit 1; }
S=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$S" $OUT/kernel_stats.csv
T=$(find $OUT/prof -name '*kernel_trace.csv' | head -1); cp "$T" $OUT/kernel_trace.csv
cut -d, -f1-4 $OUT/kernel_stats.csv | head -14 | cut -c1-150
python3 - $OUT/kernel_trace.csv "$RX" <<'PY'
import csv, sys, re
from collections import defaultdict
d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if re.search(sys.argv[2], n):
        d[n.split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print(k, len(v), "us:", [round(x, 1) for x in v[:12]])
PY
