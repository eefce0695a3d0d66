# Extractor parity tests + a short extract-only bench (stage timings), for kernel iteration.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 400 python -u -m pytest tests/test_extractor_gpu.py tests/test_dbrief.py tests/test_lafida.py tests/test_host_cpp.py tests/test_rig.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/quick_$TAG.log 2>&1 || { tail -40 gpurun_out/quick_$TAG.log; exit 1; }
tail -2 gpurun_out/quick_$TAG.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --gba-calls 0 --d-multiframes 0 --bow-reps 0 > gpurun_out/quick_$TAG.json 2> gpurun_out/quick_$TAG.err || { tail -5 gpurun_out/quick_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/quick_$TAG.json')); print(d['value'], d['roofline']['frac'], d['stage_ms_per_step'], d['match_ms_per_step'])"
