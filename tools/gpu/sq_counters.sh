# SQ counter pass (issue / wait breakdown per kernel) for the extractor + matcher workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sq}
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --ba-calls 0 --stage-timing 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/prof_$TAG/sq -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_sq.log 2>&1 || { echo "sq pass failed"; tail -20 gpurun_out/prof_${TAG}_sq.log; exit 1; }
F=$(find gpurun_out/prof_$TAG/sq -name '*counter_collection.csv' | head -1)
python3 tools/sq_summary.py "$F" | tee gpurun_out/prof_$TAG/sq_summary.txt
