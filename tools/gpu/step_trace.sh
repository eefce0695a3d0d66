# Kernel trace of the production extract+match step (no stage events): the timeline of one timed
# step (tools/step_timeline.py), split into SPLIT parts.  Usage: step_trace.sh TAG [SPLIT]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-st}; K=${2:-2}
OUT=gpurun_out/st_$TAG; mkdir -p $OUT
ARGS="--steps 4 --warmup 1 --split $K --pipeline ${PL:-1} --stage-timing 0 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --tri-reps 0 --latency-reps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "prof failed"; tail -5 $OUT/bench.err; exit 1; }
T=$(find $OUT/prof -name '*kernel_trace.csv' | head -1); cp "$T" $OUT/kernel_trace.csv
python3 tools/step_timeline.py $OUT/kernel_trace.csv 3 $K > $OUT/timeline.txt
tail -1 $OUT/timeline.txt
