# The kernel-trace pass of final_profile.sh alone: TAG -> gpurun_out/fp_TAG/{kernel_stats.csv, bench_stats.json}
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06}
O=gpurun_out/fp_$TAG; mkdir -p $O
SARGS="--steps 1 --warmup 0 --split 1 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0 --tri-reps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py $SARGS > $O/bench_stats.json 2> $O/stats.err || { echo "stats pass failed"; tail -5 $O/stats.err; exit 1; }
S=$(find $O/stats -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
head -8 $O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
