# The kernel-trace pass of final_profile.sh alone: TAG -> gpurun_out/fp_TAG/{kernel_stats.csv,
# kernel_trace.csv, stage_kernel_trace.json, bench_stats.json}
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06}
O=gpurun_out/fp_$TAG; mkdir -p $O
SARGS="--steps 5 --warmup 2 --split 1 --pipeline 0 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0 --tri-reps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py $SARGS > $O/bench_stats.json 2> $O/stats.err || { echo "stats pass failed"; tail -5 $O/stats.err; exit 1; }
S=$(find $O/stats -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
T=$(find $O/stats -name '*kernel_trace.csv' | head -1); cp "$T" $O/kernel_trace.csv
ALG=$(python3 -c "import json; print(json.load(open('$O/bench_stats.json'))['roofline']['alg_bytes_per_call'])")
python3 tools/stage_trace_summary.py $O/kernel_trace.csv 5 8 $ALG "stats_pass.sh $TAG: the 5 stage-timed extractor calls (stages back to back on one stream)" > $O/stage_kernel_trace.json || { echo "stage trace summary failed"; exit 1; }
head -8 $O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
python3 -c "import json; d=json.load(open('$O/stage_kernel_trace.json')); print(d['k_pyr_rows<true,2>_ms_per_call'], d['k_fast_rows<16>_ms_per_call'], d['frac_of_8000']); b=json.load(open('$O/bench_stats.json')); print(b['stage_ms_per_step'])"
