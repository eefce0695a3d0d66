# LocalBA leg only (config C), three back-to-back bench runs: ms per call and host phases.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 200 python bench.py --multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 40 --gba-calls 0 --d-multiframes 0 --bow-reps 0 --latency-reps 0 --tri-reps 0 > gpurun_out/lba_b.json 2> gpurun_out/lba_b.err || { tail -5 gpurun_out/lba_b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/lba_b.json'))['localba']; print(d['ms_per_call'], d['host_ms_per_call'])"
done
