# rocprofv3 passes for the bench workload (kernel trace + stats, then separate PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --ba-calls 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/stats -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_stats.log 2>&1 || { echo "stats pass failed"; tail -20 gpurun_out/prof_${TAG}_stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_$TAG/fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 gpurun_out/prof_${TAG}_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_$TAG/write -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_write.log 2>&1 || { echo "write pass failed"; tail -20 gpurun_out/prof_${TAG}_write.log; exit 1; }
find gpurun_out/prof_$TAG -name '*.csv' | head -20
F=$(find gpurun_out/prof_$TAG/fetch -name '*counter_collection.csv' | head -1)
W=$(find gpurun_out/prof_$TAG/write -name '*counter_collection.csv' | head -1)
python3 tools/pmc_traffic.py "$F" "$W" gpurun_out/prof_$TAG/pmc_traffic.json > /dev/null && echo "traffic ok"
S=$(find gpurun_out/prof_$TAG/stats -name '*kernel_stats.csv' | head -1)
cp "$S" gpurun_out/prof_$TAG/kernel_stats.csv && head -30 gpurun_out/prof_$TAG/kernel_stats.csv
