# GlobalBA (config E) host-thread A/B: MCS_HOST_THREADS 8 / 16 alternating, GlobalBA leg only.
# Usage: gba_threads_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2; do for T in 8 16 4; do
MCS_HOST_THREADS=$T timeout -k 10 300 python3 bench.py --multiframes 2 --unique 2 --steps 1 --warmup 1 --no-cpu-baseline --ba-calls 0 --gba-calls 6 --d-multiframes 0 --bow-reps 0 --latency-reps 0 --tri-reps 0 > gpurun_out/gba_t.json 2> gpurun_out/gba_t.err || { tail -5 gpurun_out/gba_t.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/gba_t.json'))['globalba']; print('threads $T', d['ms_per_call'], d['host_ms_per_call'], round(sum(d['host_ms_per_call'].values()), 3))"
done; done
