# rocprofv3 kernel trace of the LocalBA leg alone (config C), for launch/latency analysis.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-c}
OUT=gpurun_out/cfgc_$TAG; mkdir -p $OUT
ARGS="--multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 5 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "prof failed"; tail -5 $OUT/bench.err; exit 1; }
S=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$S" $OUT/kernel_stats.csv
T=$(find $OUT/prof -name '*kernel_trace.csv' | head -1); cp "$T" $OUT/kernel_trace.csv
M=$(find $OUT/prof -name '*memory_copy_trace.csv' | head -1); [ -n "$M" ] && cp "$M" $OUT/memcpy_trace.csv
head -16 $OUT/kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['localba'])"
