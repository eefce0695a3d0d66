# Run a subset of the GPU tests: bash tools/gpu/tests_subset.sh TAG test_a.py test_b.py ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=$1; shift
F=""; for t in "$@"; do F="$F tests/$t"; done
timeout -k 10 900 python -u -m pytest $F -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/sub_$TAG.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/sub_$TAG.log | tail -40
exit $rc
