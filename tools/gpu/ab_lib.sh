# A/B of the BA legs (LocalBA ms per call, GlobalBA stage times) between the default library and
# a variant (tools/build_variants.sh NAME ...), after the BA parity tests on the variant.
# Usage: ab_lib.sh NAME
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$PWD/multicol-slam-annotation_amd/lib/var_${1:?variant name}/libmcs_amd.so
MCS_AMD_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_ba.py tests/test_global_ba.py tests/test_config_e.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -20 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for i in 1 2; do for L in multicol-slam-annotation_amd/lib/libmcs_amd.so $V; do
MCS_AMD_LIB=$PWD/${L#$PWD/} timeout -k 10 200 python bench.py --multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 40 --d-multiframes 0 --bow-reps 0 --gba-calls 3 --latency-reps 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$L'[-30:], d['localba']['ms_per_call'], d['globalba']['stage_ms_per_trial'])"
done; done
