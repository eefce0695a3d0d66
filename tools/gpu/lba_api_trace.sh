# LocalBA (config C): kernel + memory-copy + HIP runtime API trace of a few calls, to place the
# device idle gaps of a call against the host API calls that precede them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d gpurun_out/lbaapi -o run -- python3 tools/gpu/lba_gaps.py 5 > gpurun_out/lbaapi.log 2>&1 || { tail -5 gpurun_out/lbaapi.log; exit 1; }
find gpurun_out/lbaapi -name '*.csv' | head
