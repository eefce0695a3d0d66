"""Timeline of one bench step from a rocprofv3 kernel trace (kernel_trace.csv): every dispatch of
the step with its start offset and duration, the busy union (time with at least one kernel
running), the time with two or more running, and the sum of the dispatch durations.  Steps are
cut at the level-0 blur launch that starts each extractor call (`k_pyr_rows<false`); with
--split K a step holds K such calls, so pass K as the third argument.

Usage: step_timeline.py kernel_trace.csv STEP_INDEX [CALLS_PER_STEP]   (host-only)"""
import csv
import json
import sys


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mcs::", "")))
    rows.sort()
    return rows


def steps(rows, calls):
    starts = [i for i, r in enumerate(rows) if r[2].startswith("k_pyr_rows<false")]
    starts = starts[::calls]
    # the level-0 blur runs on a side stream: level 1 of the same call may start just before it
    for j, i in enumerate(starts):
        while i > 0 and rows[i - 1][2].startswith("k_pyr_rows") and rows[i][0] - rows[i - 1][0] < 50000:
            i -= 1
        starts[j] = i
    out = []
    for j, i in enumerate(starts):
        end = starts[j + 1] if j + 1 < len(starts) else len(rows)
        out.append(rows[i:end])
    return out


def union(ivs):
    ev = sorted([(s, 1) for s, e, _ in ivs] + [(e, -1) for s, e, _ in ivs])
    busy = two = 0
    depth, last = 0, None
    for t, d in ev:
        if last is not None:
            if depth >= 1:
                busy += t - last
            if depth >= 2:
                two += t - last
        depth += d
        last = t
    return busy, two


def main():
    rows = load(sys.argv[1])
    k = int(sys.argv[2])
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    st = steps(rows, calls)
    s = st[k]
    t0 = s[0][0]
    span = max(e for _, e, _ in s) - t0
    busy, two = union(s)
    for a, e, n in s:
        print("%9.1f %8.1f  %s" % ((a - t0) / 1e3, (e - a) / 1e3, n))
    print(json.dumps({"steps_found": len(st), "dispatches": len(s), "span_us": round(span / 1e3, 1),
                      "busy_us": round(busy / 1e3, 1), "two_or_more_us": round(two / 1e3, 1),
                      "sum_durations_us": round(sum(e - a for a, e, _ in s) / 1e3, 1)}))


if __name__ == "__main__":
    main()
