set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu2_tests.log 2>&1; echo "TESTS EXIT $?" >> gpurun_out/gpu2_tests.log
tail -5 gpurun_out/gpu2_tests.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench2.json 2> gpurun_out/bench2.err; echo "BENCH EXIT $?"
cat gpurun_out/bench2.json; tail -5 gpurun_out/bench2.err
