# Round-end profile set for the headline workload (config B extract + match), each pass its
# own rocprofv3 run (MI355X_MICROARCH.md: separate --pmc passes, counter-slot limits):
#   1. kernel trace + stats          -> kernel_stats.csv (durations the bench roofline must match)
#   2. FETCH_SIZE, 3. WRITE_SIZE     -> pmc_traffic.json (HBM bytes per launch, raw and x2)
#   4. SQ issue/wait split, 5. SQ VALU-busy / LDS bank conflicts / wave level
# Usage: final_profile.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r02}
O=gpurun_out/fp_$TAG; mkdir -p $O
# --split 1: every launch covers the whole 513-frame batch on one stream (the bench's stage-timed
# roofline launches), so per-launch durations, bytes and VALU counts are per step
ARGS="--steps 5 --warmup 1 --split 1 --pipeline 0 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0 --tri-reps 0"
# kernel-trace pass: 2 warmup + 5 timed steps (the clocks settle: a pass of one step measured
# every kernel 7-13 % slower), then the bench's 5 stage-timed steps (stages back to back, the
# level-0 blur not beside the resize chain), which stage_trace_summary.py picks out
SARGS=$(echo "$ARGS" | sed "s/--warmup 1/--warmup 2/")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py $SARGS > $O/bench_stats.json 2> $O/stats.err || { echo "stats pass failed"; tail -5 $O/stats.err; exit 1; }
S=$(find $O/stats -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
T=$(find $O/stats -name '*kernel_trace.csv' | head -1); cp "$T" $O/kernel_trace.csv
ALG=$(python3 -c "import json; print(json.load(open('$O/bench_stats.json'))['roofline']['alg_bytes_per_call'])")
python3 tools/stage_trace_summary.py $O/kernel_trace.csv 5 8 $ALG "final_profile.sh $TAG stats pass: the 5 stage-timed extractor calls (stages back to back on one stream)" > $O/stage_kernel_trace.json || { echo "stage trace summary failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py $ARGS > /dev/null 2> $O/fetch.err || { echo "fetch pass failed"; tail -5 $O/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py $ARGS > /dev/null 2> $O/write.err || { echo "write pass failed"; tail -5 $O/write.err; exit 1; }
F=$(find $O/fetch -name '*counter_collection.csv' | head -1)
W=$(find $O/write -name '*counter_collection.csv' | head -1)
python3 tools/pmc_traffic.py "$F" "$W" $O/pmc_traffic.json 1 > /dev/null || { echo "traffic summary failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/sqa -o run -- python3 bench.py $ARGS --stage-timing 0 > /dev/null 2> $O/sqa.err || { echo "sq pass A failed"; tail -5 $O/sqa.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LEVEL_WAVES SQ_INST_CYCLES_SALU --output-format csv -d $O/sqb -o run -- python3 bench.py $ARGS --stage-timing 0 > /dev/null 2> $O/sqb.err || { echo "sq pass B failed"; tail -5 $O/sqb.err; exit 1; }
A=$(find $O/sqa -name '*counter_collection.csv' | head -1)
B=$(find $O/sqb -name '*counter_collection.csv' | head -1)
python3 tools/sq_summary.py "$A" > $O/sq_summary.txt
python3 tools/valu_per_pixel.py "$A" 513 > $O/valu_per_pixel.json
python3 tools/sq_summary.py --all --json=$O/sq_issue.json "$B" > $O/sq_summary_b.txt
head -14 $O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
python3 -c "import json; d=json.load(open('$O/pmc_traffic.json')); print({k: v for k, v in d.items() if k != 'kernels'})"
head -12 $O/sq_summary.txt
