# Checkpoint + GlobalBA upload A/B.  (1) pytest -m gpu (whole suite) on the default library;
# (2) the default bench (N = 1) as the driver runs it; (3) the config E / GlobalBA parity tests
# with MCS_SPLIT_UPLOAD=1; (4) the bench's GlobalBA leg: default, MCS_SPLIT_UPLOAD=1 and
# MCS_HOST_THREADS=1, alternating twice.  Usage: bash tools/gpu/split_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 600 python3 -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['localba']['ms_per_call'], d['globalba']['ms_per_call'], d['globalba'].get('host_ms_per_call'))"
MCS_SPLIT_UPLOAD=1 timeout -k 10 600 python3 -u -m pytest tests/test_config_e.py tests/test_global_ba.py -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/split_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/split_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/split_tests_$TAG.log
ARGS="--multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --d-multiframes 0 --bow-reps 0 --tri-reps 0 --gba-calls 5"
for rep in 1 2; do
  for v in main split t1; do
    sp=0; th=8
    [ $v = split ] && sp=1
    [ $v = t1 ] && th=1
    MCS_SPLIT_UPLOAD=$sp MCS_HOST_THREADS=$th timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/sp_$v.json 2> gpurun_out/sp_$v.err || { tail -5 gpurun_out/sp_$v.err; exit 1; }
    python3 -c "import json; g=json.load(open('gpurun_out/sp_$v.json'))['globalba']; print('$v', g.get('ms_per_call'), g.get('stage_ms_per_trial'), g.get('host_ms_per_call'))"
  done
done
