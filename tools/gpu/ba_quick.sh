# BA parity tests + the LocalBA timeline (wall ms per call, per-kernel device time) and the
# GlobalBA stage times, for BA kernel iteration.  Usage: ba_quick.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-b}
timeout -k 10 400 python -u -m pytest tests/test_ba.py tests/test_global_ba.py tests/test_config_e.py tests/test_g2o_golden.py tests/test_local_ba_select.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/baq_$TAG.log 2>&1 || { tail -30 gpurun_out/baq_$TAG.log; exit 1; }
tail -1 gpurun_out/baq_$TAG.log
bash tools/gpu/lba_gaps.sh $TAG > gpurun_out/baq_gaps_$TAG.txt || exit 1; sed -n 1,14p gpurun_out/baq_gaps_$TAG.txt
timeout -k 10 200 python bench.py --multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 40 --d-multiframes 0 --bow-reps 0 --gba-calls 3 --latency-reps 0 --tri-reps 0 > gpurun_out/baq_$TAG.json 2> gpurun_out/baq_$TAG.err || { tail -5 gpurun_out/baq_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/baq_$TAG.json')); print(d['localba']['ms_per_call'], d['globalba']['stage_ms_per_trial'])"
