# Round-6 checkpoint: the whole GPU suite (no -x: every failure listed), then the default bench.
# Usage: bash tools/gpu/r06_check.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 900 python3 -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/tests_$TAG.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['localba']['ms_per_call'], d['globalba']['ms_per_call'], d['globalba'].get('host_ms_per_call'), d['globalba'].get('stage_ms_per_trial'))"
