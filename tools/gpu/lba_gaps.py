"""LocalBA (config C) wall time per call, then (under rocprofv3 --kernel-trace) a few calls
whose kernel timeline tools/gpu/lba_gaps.sh splits into device-busy time and idle gaps."""
import sys, time
sys.path.insert(0, "multicol-slam-annotation_amd")
import numpy as np
from mcs_amd import ba as mba

pr = mba.make_problem(seed=1)
s = mba.Solver(device=0)
for _ in range(3):
    s.local_ba(pr)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
s.read_host_timing(reset=True)
ts = []
for _ in range(n):
    t0 = time.perf_counter()
    r = s.local_ba(pr)
    ts.append((time.perf_counter() - t0) * 1e3)
its = r["report1"].iterations + r["report2"].iterations
print("LBA wall ms/call median %.3f min %.3f mean %.3f  iterations %d+%d" % (
    float(np.median(ts)), min(ts), float(np.mean(ts)), r["report1"].iterations, r["report2"].iterations))
ht, nc = s.read_host_timing(reset=True)
print("host ms per LocalBA call: " + ", ".join("%s %.3f" % (k, v / n) for k, v in ht.items()))
