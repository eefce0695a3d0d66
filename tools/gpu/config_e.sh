# Config E: full-size parity tests (unsharded + sharded world 2/8 on one GPU) and a rocprofv3
# kernel-trace/stats pass of the GlobalBA leg alone (the extractor leg shrunk to 2 frames, no
# other BA leg), so ldlt/ba kernel stats come from config E only.  Usage: config_e.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-e}
OUT=gpurun_out/cfge_$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_config_e.py -x -v -m gpu --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -8 $OUT/tests.log
[ $rc -eq 0 ] || exit 1
ARGS="--multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --d-multiframes 0 --bow-reps 0 --gba-calls 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "prof failed"; tail -5 $OUT/bench.err; exit 1; }
S=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp "$S" $OUT/kernel_stats.csv
head -12 $OUT/kernel_stats.csv | cut -c1-200
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(json.dumps(d['globalba']))"
T=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
[ -n "$T" ] && python3 tools/ktrace_by_grid.py "$T" k_panel k_backward k_schur k_point_trial k_edges > $OUT/by_grid.txt && cat $OUT/by_grid.txt
true
