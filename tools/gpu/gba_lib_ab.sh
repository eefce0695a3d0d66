# GlobalBA (config E) A/B of the default library against a variant (tools/build_variants.sh NAME),
# after the config-E / GlobalBA parity tests on the default library.  Usage: gba_lib_ab.sh NAME
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$PWD/multicol-slam-annotation_amd/lib/var_${1:?variant name}/libmcs_amd.so
timeout -k 10 400 python3 -u -m pytest tests/test_config_e.py tests/test_global_ba.py tests/test_ba_structure_host.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gba_ab_tests.log 2>&1 || { tail -20 gpurun_out/gba_ab_tests.log; exit 1; }
tail -1 gpurun_out/gba_ab_tests.log
for i in 1 2 3; do for L in multicol-slam-annotation_amd/lib/libmcs_amd.so $V; do
MCS_AMD_LIB=$PWD/${L#$PWD/} timeout -k 10 300 python3 bench.py --multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --gba-calls 6 --d-multiframes 0 --bow-reps 0 --latency-reps 0 --tri-reps 0 > gpurun_out/gba_ab.json 2> gpurun_out/gba_ab.err || { tail -5 gpurun_out/gba_ab.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/gba_ab.json'))['globalba']; print('${L: -30}', d['ms_per_call'], {k: round(v, 3) for k, v in d['host_ms_per_call'].items()}, round(sum(d['host_ms_per_call'].values()), 3))"
done; done
