# Headline step and per-stage times of the main library against variant builds (lib/var_NAME),
# alternating twice.  Usage: bash tools/gpu/desc_ab.sh NAME [NAME ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=multicol-slam-annotation_amd/lib
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --bow-reps 0 --d-multiframes 0 --latency-reps 0 --tri-reps 0"
for rep in 1 2; do
  for v in main "$@"; do
    if [ "$v" = main ]; then lib=$L/libmcs_amd.so; else lib=$L/var_$v/libmcs_amd.so; fi
    MCS_AMD_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/dab_$v.json 2> gpurun_out/dab_$v.err || { tail -5 gpurun_out/dab_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/dab_$v.json')); print('$v', d['ms_per_step'], d['stage_ms_per_step'])"
  done
done
