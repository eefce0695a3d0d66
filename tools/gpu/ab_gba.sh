# A/B of the GlobalBA (config E) leg under an environment toggle: ab_gba.sh VAR TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VAR=$1; TAG=${2:-ab}
ARGS="--multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --d-multiframes 0 --bow-reps 0 --tri-reps 0 --gba-calls 3"
for v in 0 1; do
  env $VAR=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/gba_${TAG}_$v.json 2> gpurun_out/gba_${TAG}_$v.err || { tail -5 gpurun_out/gba_${TAG}_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/gba_${TAG}_$v.json')); g=d['globalba']; print('$VAR=$v', g.get('ms_per_call'), g.get('stage_ms_per_trial'))"
done
