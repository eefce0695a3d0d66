# GlobalBA (config E) leg: the main library against variant builds (lib/var_NAME), alternating
# twice.  Usage: bash tools/gpu/gba_ab.sh NAME [NAME ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=multicol-slam-annotation_amd/lib
ARGS="--multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --d-multiframes 0 --bow-reps 0 --tri-reps 0 --gba-calls 3"
for rep in 1 2; do
  for v in main "$@"; do
    if [ "$v" = main ]; then lib=$L/libmcs_amd.so; else lib=$L/var_$v/libmcs_amd.so; fi
    MCS_AMD_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/gab_$v.json 2> gpurun_out/gab_$v.err || { tail -5 gpurun_out/gab_$v.err; exit 1; }
    python3 -c "import json; g=json.load(open('gpurun_out/gab_$v.json'))['globalba']; print('$v', g.get('ms_per_call'), g.get('stage_ms_per_trial'))"
  done
done
