"""LocalBA (config C) time split: wall per call vs device stage time (HIP events) and the host
phases, to see where a call's time goes.  Run on the GPU box."""
import os, sys, time
sys.path.insert(0, "multicol-slam-annotation_amd")
import numpy as np
from mcs_amd import ba as mba

pr = mba.make_problem(seed=1)
s = mba.Solver(device=0)
s.local_ba(pr)
N = 20
ts = []
for _ in range(100):
    t0 = time.perf_counter()
    r = s.local_ba(pr)
    ts.append((time.perf_counter() - t0) * 1e3)
wall = float(np.median(ts))
its = r["report1"].iterations + r["report2"].iterations
print("wall ms/call median %.3f  min %.3f  mean %.3f  iterations/call %d  ms/iter %.4f" % (
    wall, min(ts), np.mean(ts), its, wall / its))
s.enable_timing(True)
for _ in range(N):
    r = s.local_ba(pr)
tm = s.read_timing()
print("timed (events on, no graph):", tm)
s.enable_timing(False)
# an optimize() with max_iterations=1: the per-call fixed cost
for mi in (0, 1, 2, 5, 10):
    o1 = mba.BAOptions(max_iterations=mi)
    s.optimize(pr, o1)
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        r = s.optimize(pr, o1)
        ts.append((time.perf_counter() - t0) * 1e3)
    print("optimize(max_iterations=%d) ms/call median %.3f  min %.3f  iterations %d" % (
        mi, float(np.median(ts)), min(ts), r["report"].iterations))
