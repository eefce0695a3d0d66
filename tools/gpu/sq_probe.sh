set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sqp; export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/sqp/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" gpurun_out/sqp/avail.txt | sort -u > gpurun_out/sqp/sq_names.txt || true
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/sqp/p1 -o run -- ./tools/bench/ldlt_probe > gpurun_out/sqp/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_BUSY_CYCLES --output-format csv -d gpurun_out/sqp/p2 -o run -- ./tools/bench/ldlt_probe > gpurun_out/sqp/p2.log 2>&1
for f in $(find gpurun_out/sqp -name '*counter_collection.csv'); do python3 - "$f" <<'PY'
import csv,sys
from collections import defaultdict
acc=defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_probe' in r['Kernel_Name']: acc[r['Counter_Name']]+=float(r['Counter_Value'])
print({k: v for k,v in sorted(acc.items())})
PY
done
