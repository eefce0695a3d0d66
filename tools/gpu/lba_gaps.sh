# LocalBA kernel timeline: per-kernel device time and the idle gaps of the last 3 calls.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 120 python3 tools/gpu/lba_gaps.py 200 > gpurun_out/lba_wall_$TAG.log 2>&1 || { tail -5 gpurun_out/lba_wall_$TAG.log; exit 1; }
cat gpurun_out/lba_wall_$TAG.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lbag_$TAG -o run -- python3 tools/gpu/lba_gaps.py 3 > gpurun_out/lbag_$TAG.log 2>&1 || { tail -5 gpurun_out/lbag_$TAG.log; exit 1; }
T=$(find gpurun_out/lbag_$TAG -name '*kernel_trace.csv' | head -1)
python3 tools/ktrace_gaps.py "$T" 3 | tee gpurun_out/lba_gaps_$TAG.txt
