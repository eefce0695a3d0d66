# GlobalBA (config E): parity tests of the default library (threaded host path) and of the
# sc1-consumer k_pipe variant (EXTR=ldlt.hip tools/build_variants.sh sc1 -DMCS_PIPE_SC1), then
# the bench's GlobalBA leg for the default library, the variant and the default with
# MCS_HOST_THREADS=1, alternating twice.  Usage: bash tools/gpu/host_threads_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$PWD/multicol-slam-annotation_amd/lib
timeout -k 10 900 python3 -u -m pytest tests/test_config_e.py tests/test_global_ba.py -x -v -m gpu \
  --timeout 400 --timeout-method thread > gpurun_out/ht_tests.txt 2>&1 || { tail -30 gpurun_out/ht_tests.txt; exit 1; }
tail -3 gpurun_out/ht_tests.txt
MCS_AMD_LIB=$L/var_sc1/libmcs_amd.so timeout -k 10 900 python3 -u -m pytest tests/test_config_e.py tests/test_global_ba.py -x -v -m gpu \
  --timeout 400 --timeout-method thread > gpurun_out/ht_tests_sc1.txt 2>&1 || { tail -30 gpurun_out/ht_tests_sc1.txt; exit 1; }
tail -3 gpurun_out/ht_tests_sc1.txt
ARGS="--multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --d-multiframes 0 --bow-reps 0 --tri-reps 0 --gba-calls 5"
for rep in 1 2; do
  for v in main sc1 t1; do
    lib=$L/libmcs_amd.so; th=8
    [ $v = sc1 ] && lib=$L/var_sc1/libmcs_amd.so
    [ $v = t1 ] && th=1
    MCS_AMD_LIB=$lib MCS_HOST_THREADS=$th timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ht_$v.json 2> gpurun_out/ht_$v.err || { tail -5 gpurun_out/ht_$v.err; exit 1; }
    python3 -c "import json; g=json.load(open('gpurun_out/ht_$v.json'))['globalba']; print('$v', g.get('ms_per_call'), g.get('stage_ms_per_trial'), g.get('host_ms_per_call'))"
  done
done
