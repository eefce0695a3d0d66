"""GPU: the bench's production schedule (two parts on two streams, pipelined steps with
double-buffered outputs) end to end.  bench.py raises when its post-run spot check of the last
pipelined step's output set (keypoints, descriptors, top-2 matches) differs from the oracle;
with --stage-timing 0 that check reads the pipelined set, not the one-stream stage-timed run.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("steps", [3, 4])   # last step in output set 0 / set 1
def test_bench_pipelined_parity(gpu, steps):
    args = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup", "1",
            "--multiframes", "12", "--unique", "4", "--split", "2", "--pipeline", "1",
            "--stage-timing", "0", "--cpu-sample", "4", "--ba-calls", "0", "--gba-calls", "0",
            "--d-multiframes", "0", "--bow-reps", "0", "--tri-reps", "0", "--latency-reps", "0"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    pc = d["parity_check"]
    assert pc["of_step"] == "last timed step"
    assert pc["camera_frames_bitexact"] == 12 and pc["match_pairs_bitexact"] == 9
    assert "pipelined" in d["config"]["schedule"]
