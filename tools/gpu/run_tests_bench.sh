set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1; rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/tests_$TAG.log
tail -15 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?; echo "BENCH EXIT $rc"
cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit 1
if [ -n "$PROFILE" ]; then bash tools/gpu/profile.sh $TAG; fi
