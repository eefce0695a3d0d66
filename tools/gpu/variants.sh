# Time the extract+match leg for the default build and every lib/var_*/ variant
# (tools/build_variants.sh).  Usage: variants.sh [steps]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
STEPS=${1:-10}
for L in lib $(cd multicol-slam-annotation_amd && ls -d lib/var_* 2>/dev/null); do
  MCS_AMD_LIB=$PWD/multicol-slam-annotation_amd/$L/libmcs_amd.so timeout -k 10 200 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0 > gpurun_out/var.json 2>gpurun_out/var.err || { echo "$L failed"; tail -3 gpurun_out/var.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/var.json')); print('$L', d['value'], d['roofline']['frac'], {k: round(v, 3) for k, v in d['stage_ms_per_step'].items()})"
done
