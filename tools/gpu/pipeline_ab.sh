# Extract+match leg with and without step pipelining (bench.py --pipeline), split 1 and 2.
# Usage: pipeline_ab.sh [steps]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
STEPS=${1:-20}
ARGS="--steps $STEPS --warmup 3 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --tri-reps 0 --latency-reps 0"
for PL in ${PLS:-0 1}; do for K in ${KS:-2 1 3}; do
  timeout -k 10 200 python3 bench.py $ARGS --pipeline $PL --split $K > gpurun_out/pl.json 2> gpurun_out/pl.err || { echo "pipeline $PL split $K failed"; tail -3 gpurun_out/pl.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/pl.json')); print('pipeline $PL split $K', d['value'], d['ms_per_step'], d['parity_check'] if 'parity_check' in d else '')"
done; done
