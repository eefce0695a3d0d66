# GlobalBA (config E) host threads: parity tests of the threaded host path, then the bench's
# GlobalBA leg with MCS_HOST_THREADS=8 (default) against 1, alternating twice.
# Usage: bash tools/gpu/host_threads_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_config_e.py tests/test_global_ba.py -x -v -m gpu \
  --timeout 400 --timeout-method thread > gpurun_out/ht_tests.txt 2>&1 || { tail -30 gpurun_out/ht_tests.txt; exit 1; }
tail -3 gpurun_out/ht_tests.txt
ARGS="--multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --d-multiframes 0 --bow-reps 0 --tri-reps 0 --gba-calls 5"
for rep in 1 2; do
  for th in 8 1; do
    MCS_HOST_THREADS=$th timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ht_$th.json 2> gpurun_out/ht_$th.err || { tail -5 gpurun_out/ht_$th.err; exit 1; }
    python3 -c "import json; g=json.load(open('gpurun_out/ht_$th.json'))['globalba']; print('threads $th', g.get('ms_per_call'), g.get('host_ms_per_call'))"
  done
done
