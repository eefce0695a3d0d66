# MFMA counters of the GlobalBA (config E) dense LDL^T: one rocprofv3 --pmc pass per counter
# group on the bench's GlobalBA leg alone.  Usage: mfma_counters.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-mf}
O=gpurun_out/mf_$TAG; mkdir -p $O
ARGS="--steps 1 --warmup 0 --multiframes 8 --no-cpu-baseline --ba-calls 0 --gba-calls 1 --d-multiframes 0 --bow-reps 0 --latency-reps 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/a -o run -- python3 bench.py $ARGS > $O/bench_a.json 2> $O/a.err || { echo "pass a failed"; tail -5 $O/a.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 --output-format csv -d $O/b -o run -- python3 bench.py $ARGS > $O/bench_b.json 2> $O/b.err || { echo "pass b failed"; tail -5 $O/b.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 bench.py $ARGS > $O/bench_t.json 2> $O/t.err || { echo "trace failed"; tail -5 $O/t.err; exit 1; }
A=$(find $O/a -name '*counter_collection.csv' | head -1)
B=$(find $O/b -name '*counter_collection.csv' | head -1)
S=$(find $O/t -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
python3 - "$A" "$B" $O/kernel_stats.csv $O/mfma_summary.json <<'PY'
import csv, json, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); disp = defaultdict(set)
for path in sys.argv[1:3]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", ""))
dur = {}
for r in csv.DictReader(open(sys.argv[3])):
    dur[r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")] = (int(r["Calls"]), float(r["TotalDurationNs"]))
out = {"note": "SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs? (see MI355X_MICROARCH.md); "
               "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (SQ_BUSY_CYCLES / 32 SQs); "
               "F64 MOPS: 256 flops per unit of SQ_INSTS_VALU_MFMA_MOPS_F64 is NOT assumed: raw value reported",
       "kernels": {}}
for k, c in acc.items():
    if "ldlt" not in k and "ba::" not in k:
        continue
    busy = c.get("SQ_BUSY_CYCLES", 0) / 32
    d = {n: v for n, v in c.items()}
    if busy > 0:
        d["mfma_busy_frac"] = round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / busy, 4)
    d["dispatches"] = len(disp[k])
    if k in dur:
        d["calls_traced"], d["total_ns_traced"] = dur[k]
    out["kernels"][k] = d
json.dump(out, open(sys.argv[4], "w"), indent=1)
for k, d in sorted(out["kernels"].items()):
    print(k[:50], {x: (round(y, 4) if isinstance(y, float) else y) for x, y in d.items() if x.startswith(("mfma", "SQ_INSTS", "SQ_VALU", "dispatch"))})
PY
