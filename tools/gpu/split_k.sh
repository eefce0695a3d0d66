# Headline step with the batch in K parts on K streams (bench.py --split K), K = 1..4, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2; do for K in 2 3 4 1; do
timeout -k 10 200 python3 bench.py --split $K --steps 20 --warmup 3 --no-cpu-baseline --stage-timing 0 --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0 --tri-reps 0 > gpurun_out/splitk.json 2> gpurun_out/splitk.err || { tail -5 gpurun_out/splitk.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/splitk.json')); print('split $K', d['value'], d['ms_per_step'])"
done; done
