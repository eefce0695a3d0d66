"""The profile summarisers the bench's roofline fields come from (tools/pmc_traffic.py,
tools/valu_per_pixel.py) on small synthetic rocprofv3 counter files: per-launch averages, the
per-step sums of the pyramid's level launches and FAST, the extractor-calls-per-step scaling
(a bench step split into two halves is two extractor calls) and the pixel normalisation.
CPU only."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PYR = "void mcs::k_pyr_rows<true, 2>(mcs::PyrArgs)"
FAST = "void mcs::k_fast_rows<16>(mcs::FastRowArgs)"


def _write(path, counter, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for i, (k, v) in enumerate(rows):
            w.writerow([i, k, counter, v])


def _rows(calls, pyr_kib, fast_kib):
    """`calls` extractor calls: 7 pyramid level launches + 1 FAST launch each."""
    out = []
    for _ in range(calls):
        out += [(PYR, v) for v in pyr_kib] + [(FAST, fast_kib)]
    return out


def test_pmc_traffic_per_step(tmp_path):
    pyr = [70, 50, 35, 25, 17, 12, 8]            # KiB per level launch
    fe, wr = str(tmp_path / "f.csv"), str(tmp_path / "w.csv")
    _write(fe, "FETCH_SIZE", _rows(4, pyr, 100))
    _write(wr, "WRITE_SIZE", _rows(4, [2 * v for v in pyr], 10))
    for per_step in (1, 2):
        out = str(tmp_path / ("t%d.json" % per_step))
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), fe, wr, out,
                        str(per_step)], check=True, capture_output=True, timeout=60)
        d = json.load(open(out))
        # per step: per_step extractor calls, each 7 level launches + FAST
        fetch = per_step * (sum(pyr) + 100) * 1024
        write = per_step * (2 * sum(pyr) + 10) * 1024
        assert d["extractor_calls_per_step"] == per_step
        assert d["pyr_launches_per_call"] == 7 * per_step
        assert abs(d["pyramid+fast_fetch_raw_per_call"] - fetch) < 1e-6
        assert abs(d["pyramid+fast_write_per_call"] - write) < 1e-6
        assert abs(d["pyramid+fast_raw_bytes_per_call"] - (fetch + write)) < 1e-6
        assert abs(d["pyramid+fast_bytes_per_call"] - (2 * fetch + write)) < 1e-6
        assert d["kernels"]["k_fast_rows<16>"]["launches"] == 4


def test_valu_per_pixel(tmp_path):
    path = str(tmp_path / "a.csv")
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        n = 0
        for _ in range(2):                         # two calls of a 3-level pyramid
            for _ in range(2):                     # levels 1, 2
                w.writerow([n, PYR, "SQ_INSTS_VALU", 1000]); w.writerow([n, PYR, "SQ_WAVES", 10]); n += 1
            w.writerow([n, FAST, "SQ_INSTS_VALU", 5000]); w.writerow([n, FAST, "SQ_WAVES", 20]); n += 1
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "valu_per_pixel.py"), path, "2.5",
                        "100", "50", "3"], check=True, capture_output=True, text=True, timeout=60)
    d = json.loads(r.stdout)
    px = d["level_pixels"]
    assert px[0] == 100 * 50 and len(px) == 3
    assert d["k_pyr_rows<true, 2>"]["calls"] == 2.0   # (levels - 1) = 2 launches per call
    assert abs(d["k_pyr_rows<true, 2>"]["valu_lane_ops_per_pixel"]
               - round(2000 * 64 / (sum(px[1:]) * 2.5), 2)) < 1e-9
    assert d["k_fast_rows<16>"]["calls"] == 2.0
    assert abs(d["k_fast_rows<16>"]["valu_lane_ops_per_pixel"]
               - round(5000 * 64 / (sum(px) * 2.5), 2)) < 1e-9


def test_stage_trace_summary(tmp_path):
    """tools/stage_trace_summary.py: the last CALLS extractor calls of a kernel trace, the
    median per level (one stretched dispatch does not move it) and the roofline fraction."""
    path = str(tmp_path / "trace.csv")
    lv = [170, 140, 90, 77, 68, 61, 35]                      # us per level launch
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        t, n = 1000, 0
        for call in range(4):                                # call 0 is a timed step: dropped
            for l, us in enumerate(lv):
                d = us * 1000 * (3 if (call == 0 or (call == 2 and l == 1)) else 1)
                w.writerow([n, PYR, t, t + d]); t += d + 500; n += 1
            w.writerow([n, FAST, t, t + 650000]); t += 650500; n += 1
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "stage_trace_summary.py"), path,
                        "3", "8", "1523973204", "synthetic"], check=True, capture_output=True,
                       text=True, timeout=60)
    d = json.loads(r.stdout)
    assert d["k_pyr_rows_per_level_us"] == [float(v) for v in lv]
    assert d["k_pyr_rows_per_level_us_mean"][1] == round((140 * 3 + 140 * 2) / 3, 1)
    assert abs(d["k_pyr_rows<true,2>_ms_per_call"] - sum(lv) / 1e3) < 1e-9
    assert abs(d["k_fast_rows<16>_ms_per_call"] - 0.65) < 1e-9
    frac = 1523973204 / ((sum(lv) / 1e3 + 0.65) / 1e3) / 1e9 / 8000.0
    assert abs(d["frac_of_8000"] - round(frac, 4)) < 1e-12
