# SQ counter passes (issue / wait / LDS breakdown per kernel) on the extract+match workload,
# plus the measured FP64 MFMA peak.  Usage: bash tools/gpu/sq_extract.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-sq}
OUT=gpurun_out/sq_$TAG; mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --stage-timing 0"
hipcc --offload-arch=gfx950 -O3 tools/bench/mfma_f64_peak.hip -o tools/bench/mfma_f64_peak && \
  timeout -k 10 60 ./tools/bench/mfma_f64_peak > $OUT/mfma_f64_peak.json || { echo "peak probe failed"; exit 1; }
cat $OUT/mfma_f64_peak.json
timeout -k 5 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"
P3="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
for f in $(find $OUT -name '*counter_collection.csv'); do python3 tools/sq_summary.py "$f" --all >> $OUT/summary.txt 2>&1; done
cat $OUT/summary.txt | head -80
