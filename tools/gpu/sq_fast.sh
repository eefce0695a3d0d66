# SQ counter passes of the extract+match leg alone (issue / wait breakdown per kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sqf}
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --stage-timing 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/prof_$TAG/a -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_a.log 2>&1 || { echo "pass a failed"; tail -20 gpurun_out/prof_${TAG}_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LEVEL_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof_$TAG/b -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_b.log 2>&1 || { echo "pass b failed"; tail -20 gpurun_out/prof_${TAG}_b.log; exit 1; }
python3 - gpurun_out/prof_$TAG <<'PY' | tee gpurun_out/prof_$TAG/summary.txt
import csv, sys, glob
from collections import defaultdict
root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
for f in glob.glob(root + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    w = max(c.get("SQ_WAVES", 1), 1) / 2  # SQ_WAVES collected in both passes (WAVE_CYCLES too)
    print(k)
    for n in sorted(c):
        print("   %-24s %16.0f  per-wave %10.1f" % (n, c[n], c[n] / w))
PY
