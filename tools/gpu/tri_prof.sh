# Kernel stats of the SearchForTriangulationRaw bench leg alone (extraction shrunk to the 6
# multi-frames the leg needs).  Usage: tri_prof.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-tp}
OUT=gpurun_out/triprof_$TAG; mkdir -p $OUT
ARGS="--multiframes 6 --unique 6 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0 --tri-reps 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "prof failed"; tail -5 $OUT/bench.err; exit 1; }
S=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$S" $OUT/kernel_stats.csv
cut -d, -f1-4 $OUT/kernel_stats.csv | head -14 | cut -c1-160
