# LocalBA wall time per call for the main library and variant builds (lib/var_NAME); with
# TRACE=1 also each one's kernel timeline (per-kernel time and the idle gaps of 3 calls).
# Usage: [TRACE=1] bash tools/gpu/lba_ab.sh NAME [NAME ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=multicol-slam-annotation_amd/lib
for v in main "$@" main; do
  if [ "$v" = main ]; then lib=$L/libmcs_amd.so; else lib=$L/var_$v/libmcs_amd.so; fi
  echo "== $v"
  MCS_AMD_LIB=$lib timeout -k 10 120 python3 tools/gpu/lba_gaps.py 200 2>&1 | grep -E "LBA wall|host ms" || exit 1
  if [ "${TRACE:-0}" = 1 ]; then
    MCS_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lbav_$v -o run -- python3 tools/gpu/lba_gaps.py 3 > gpurun_out/lbav_$v.log 2>&1 || { tail -5 gpurun_out/lbav_$v.log; exit 1; }
    T=$(find gpurun_out/lbav_$v -name '*kernel_trace.csv' | head -1)
    python3 tools/ktrace_gaps.py "$T" 3 | grep -A6 "gaps:"
  fi
done
