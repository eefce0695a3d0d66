# Time the extractor leg with ablated builds of k_pyr_fast (MCS_ABLATE=1: no exact tests,
# 2: no compass survivors) next to the real build.  Libraries are built beforehand in
# multicol-slam-annotation_amd/lib/abl*/ (tools/build_ablations.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for L in lib lib/abl1 lib/abl2; do
  MCS_AMD_LIB=$PWD/multicol-slam-annotation_amd/$L/libmcs_amd.so timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 > gpurun_out/abl.json 2>/dev/null || { echo "$L failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abl.json')); print('$L', d['value'], d['stage_ms_per_step'])"
done
