# Extractor parity tests (GPU) against a variant library (tools/build_variants.sh NAME ...).
# Usage: var_check.sh NAME
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$PWD/multicol-slam-annotation_amd/lib/var_${1:?variant name}/libmcs_amd.so
MCS_AMD_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_extractor_gpu.py tests/test_extractor_ref.py tests/test_config_b.py tests/test_lafida.py tests/test_dbrief.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/var_check_$1.log 2>&1
rc=$?
tail -2 gpurun_out/var_check_$1.log
exit $rc
