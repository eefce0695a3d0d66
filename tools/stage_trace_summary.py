"""Per-call pyramid + FAST durations from the kernel trace of tools/gpu/final_profile.sh's stats
pass (kernel_trace.csv): the last CALLS extractor calls are the bench's stage-timed steps
(stages back to back on one stream), so their k_pyr_rows<true> launches (LEVELS - 1 per call)
and k_fast_rows launch give the kernel time the bench's roofline line divides by.

Usage: stage_trace_summary.py kernel_trace.csv CALLS LEVELS ALG_BYTES_PER_CALL SOURCE_NOTE
(host-only; prints JSON)"""
import csv
import json
import sys


def main():
    path, calls, levels, alg = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    note = sys.argv[5] if len(sys.argv) > 5 else path
    pyr, fast = [], []
    for r in sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"])):
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "k_pyr_rows<true" in n:
            pyr.append(d)
        elif "k_fast_rows<" in n:
            fast.append(d)
    per = levels - 1
    if len(pyr) < calls * per or len(fast) < calls:
        raise SystemExit("trace holds %d pyramid / %d FAST launches, fewer than %d calls" % (len(pyr), len(fast), calls))
    pyr_c, fast_c = pyr[-calls * per:], fast[-calls:]
    # per level (and for FAST) the median over the calls: a profiled run now and then stretches
    # one dispatch many times over (one level-2 launch of 1594 against ~150 us seen)
    med = lambda v: sorted(v)[len(v) // 2] if len(v) % 2 else 0.5 * (sorted(v)[len(v) // 2 - 1] + sorted(v)[len(v) // 2])
    lv = [round(med([pyr_c[c * per + l] for c in range(calls)]), 1) for l in range(per)]
    lv_mean = [round(sum(pyr_c[c * per + l] for c in range(calls)) / calls, 1) for l in range(per)]
    pyr_ms = sum(lv) / 1e3
    fast_ms = med(fast_c) / 1e3
    gbs = alg / ((pyr_ms + fast_ms) / 1e3) / 1e9
    print(json.dumps({"source": note, "stage_timed_calls": calls,
                      "statistic": "median over the calls, per level",
                      "k_pyr_rows<true,2>_ms_per_call": round(pyr_ms, 4),
                      "k_pyr_rows_per_level_us": lv,
                      "k_pyr_rows_per_level_us_mean": lv_mean,
                      "k_fast_rows<16>_ms_per_call": round(fast_ms, 4),
                      "k_fast_rows<16>_ms_per_call_mean": round(sum(fast_c) / calls / 1e3, 4),
                      "alg_bytes_per_call": alg, "achieved_GBs": round(gbs, 1),
                      "frac_of_8000": round(gbs / 8000.0, 4),
                      "all_dispatch_means_ms": {"k_pyr_rows<true,2>": round(sum(pyr) / len(pyr) * per / 1e3, 4),
                                                "k_fast_rows<16>": round(sum(fast) / len(fast) / 1e3, 4)}},
                     indent=1))


if __name__ == "__main__":
    main()
