#!/usr/bin/env python3
"""Headline benchmark: kfeatures/sec (+ LocalBA iters/sec) for the MultiCol-SLAM
front-end on MI355X.

Workload (BASELINE.json configs[1], "config B"): 3-camera Lafida rig, 754x480 fisheye
frames, 2000 features per camera, extract + match on one MI355X.  One step = one batch of
M multi-frames (3*M camera-frames, default M=171 -> 513 camera-frames, inputs resident in
HBM): pyramid -> FAST -> octree -> orientation -> ORB descriptor for every camera-frame,
then brute-force Hamming best/second-best matching of every camera's descriptors against
the same camera of the previous multi-frame (the O(N1*N2) part of
SearchForTriangulationRaw, src/cORBmatcher.cpp:968-1156).

Multi-GPU (torchrun, one process per GPU): every rank runs the same step on its own
segment of multi-frames (independent units -> weak scaling, no data-path collective);
the timed region is bracketed by barrier + synchronize and the max over ranks is taken.
Side legs in the same JSON line: LocalBA (config C, replicas), GlobalBA (config E, points
sharded, RCCL all-reduce per LM trial) and config D (8 cams 1024^2, camera per GPU, RCCL
all-gather of the per-camera blocks).

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "multicol-slam-annotation_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

METRIC = "kfeatures/sec + LocalBA iters/sec, 3×754×480 fisheye, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# FP64 dense matrix peak of MI355X: the AMD spec figure is `peak`; the rate this repo's probe
# reached (tools/bench/mfma_f64_peak.hip: back-to-back v_mfma_f64_16x16x4_f64 on every CU,
# profiles/r02_mfma_f64_peak.json) is reported beside it, with the fraction against each
FP64_MFMA_PEAK_TFLOPS = 78.6
FP64_MFMA_PEAK_SRC = "AMD MI355X spec (FP64 matrix)"
FP64_MFMA_MEASURED_TFLOPS = 45.14
FP64_MFMA_MEASURED_SRC = "profiles/r02_mfma_f64_peak.json (probe, one event-timed launch)"
# algorithmic bytes of pyramid + FAST per 754x480 camera-frame
PYR_FAST_BYTES_754x480 = 2_970_708


def pmc_traffic(alg_bytes):
    """HBM traffic of the pyramid+FAST launches from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py output named in profiles/pmc_traffic.json): FETCH_SIZE + WRITE_SIZE
    per bench step, raw and with the guide's x2 correction of FETCH_SIZE for wide streaming
    reads.  The kernels read dwords, for which the correction is uncalibrated, so both are
    reported; `traffic` is the raw figure."""
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(tf):
        return {}
    try:
        d = json.load(open(tf))
        raw = d["pyramid+fast_raw_bytes_per_call"]
        return {"traffic": raw, "traffic_raw": raw,
                "traffic_fetch_x2": d.get("pyramid+fast_bytes_per_call"),
                "traffic_source": d.get("source", tf),
                "traffic_over_alg": round(raw / alg_bytes, 3) if raw else None}
    except (KeyError, ValueError):
        return {}


def sq_issue():
    """VALU issue utilisation per SIMD of the pyramid + FAST kernels from the committed SQ pass
    (tools/sq_summary.py --json: 4 * SQ_ACTIVE_INST_VALU / 1024 SIMDs / (SQ_BUSY_CYCLES / 32
    SQs), MI355X_MICROARCH.md counter units).  These kernels are issue-bound, not HBM-bound:
    this is the roofline that actually binds them."""
    tf = os.path.join(ROOT, "profiles", "sq_issue.json")
    if not os.path.exists(tf):
        return {}
    try:
        d = json.load(open(tf))
        k = d["kernels"]
        out = {"method": d.get("method"), "source": d.get("source", tf)}
        for name, key in (("k_pyr_rows<true, 2>", "pyramid"), ("k_fast_rows<16>", "fast"),
                          ("k_orient_desc", "orient_desc"), ("k_top2_mfma32<true>", "match_mfma")):
            if name in k:
                out[key + "_valu_util"] = k[name]["valu_util"]
        # VALU lane-operations per pixel (tools/valu_per_pixel.py on the SQ pass A counters)
        vp = os.path.join(ROOT, "profiles", "valu_per_pixel.json")
        if os.path.exists(vp):
            v = json.load(open(vp))
            for name, key in (("k_pyr_rows<true, 2>", "pyramid"), ("k_fast_rows<16>", "fast")):
                if name in v:
                    out[key + "_valu_lane_ops_per_pixel"] = v[name]["valu_lane_ops_per_pixel"]
            out["valu_per_pixel_source"] = v.get("source")
        return {"issue": out}
    except (KeyError, ValueError):
        return {}


def alg_bytes_pyr_fast(level_wh):
    """B = sum_{l>=1}(|L_{l-1}| + |L_l|) + sum_l |L_l|  (SURVEY.md §8(d))."""
    px = [int(w) * int(h) for w, h in level_wh]
    return sum(px[l - 1] + px[l] for l in range(1, len(px))) + sum(px)


# HALF_PATCH_SIZE = 16 disc of IC_Angle (src/mdBRIEFextractorOct.cpp:85, :153-170 umax)
def ic_disc_pixels(half=16):
    import math
    vmax = int(math.floor(half * math.sqrt(2.0) / 2 + 1))
    vmin = int(math.ceil(half * math.sqrt(2.0) / 2))
    umax = [0] * (half + 1)
    for v in range(vmax + 1):
        umax[v] = int(round(math.sqrt(half * half - v * v)))
    v0 = 0
    for v in range(half, vmin - 1, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    return sum(2 * umax[abs(v)] + 1 for v in range(-half, half + 1))


def stage_rooflines(ex, F, stage_ms, n_kp, desc_size):
    """Roofline lines of the two extractor kernels after pyramid + FAST.

    k_orient_desc, per keypoint: the selection record in (4 B), the IC_Angle disc of the raw
    level image (845 px, :221-248), the 2 x 8 x desc_size blurred samples of the rotated
    pattern (:285-354), the keypoint out (28 B) and the descriptor out (desc_size B).  These are
    the bytes the kernel must touch; neighbouring patches overlap and are served from L2/MALL,
    so this is a touched-bytes rate against the HBM peak, and the binding limit is VALU issue
    (committed SQ pass: issue share).
    k_octree: 4 B per FAST candidate in (packed x|y|score) and 4 B per selection out
    (:569-861); the per-cell counts (a few hundred words per level) are left out.  Latency /
    barrier bound."""
    import mcs_amd
    L = mcs_amd.lib()
    nlev = len(ex.levels()[0])
    n_cand = 0
    n_out = ctypes.c_int64()
    for f in range(F):   # cap 0: the call reports the level's candidate count (MCS_ERR_CAPACITY)
        for lv in range(nlev):
            L.mcs_extractor_read_stage(ex._h, 2, f, lv, None, 0, ctypes.byref(n_out))
            n_cand += int(n_out.value)
    iss = sq_issue().get("issue", {})
    disc = ic_disc_pixels()
    b_kp = 4 + disc + 2 * 8 * desc_size + 28 + desc_size
    od, oc = None, None
    t_od = stage_ms.get("orient_desc", 0.0) / 1e3
    if t_od > 0:
        a = b_kp * n_kp / t_od / 1e9
        od = {"kernel": "k_orient_desc (IC_Angle + rotated-pattern ORB, one wave per keypoint pair)",
              "bound": "hbm", "binding": "VALU issue", "achieved": round(a, 1),
              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(a / HBM_PEAK_GBS, 4),
              "traffic": None, "ms_per_call": round(t_od * 1e3, 4), "keypoints_per_call": n_kp,
              "alg_bytes_per_keypoint": b_kp,
              "alg_bytes_note": "4 sel + %d IC disc + %d pattern samples + 28 kp + %d desc; "
                                "touched bytes (patch overlap is cache-served)" % (
                                    disc, 16 * desc_size, desc_size),
              "valu_issue_share": iss.get("orient_desc_valu_util")}
    t_oc = stage_ms.get("octree", 0.0) / 1e3
    if t_oc > 0:
        b = 4 * n_cand + 4 * n_kp
        a = b / t_oc / 1e9
        oc = {"kernel": "k_octree (DistributeOctTree, one workgroup per (frame, level))",
              "bound": "hbm", "binding": "barrier / LDS latency", "achieved": round(a, 1),
              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(a / HBM_PEAK_GBS, 5),
              "traffic": None, "ms_per_call": round(t_oc * 1e3, 4),
              "candidates_per_call": n_cand, "selected_per_call": n_kp,
              "alg_bytes_per_call": b,
              "valu_issue_share": None}
    return od, oc


def baseline_cpus(k):
    """The first k CPUs of this process's allowed set: the CPU baseline legs pin their threads
    to them (taskset-style, one thread per CPU) so the timing does not migrate across cores."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        return []
    return cpus[:k]


class pinned_thread:
    """Pin the calling thread to one CPU while a single-threaded baseline leg runs; the
    thread's previous CPU set is restored afterwards."""

    def __init__(self, cpu):
        self.cpu = cpu

    def __enter__(self):
        self.old = None
        if self.cpu is not None and hasattr(os, "sched_setaffinity"):
            self.old = os.sched_getaffinity(0)
            os.sched_setaffinity(0, {self.cpu})
        return self

    def __exit__(self, *exc):
        if self.old is not None:
            os.sched_setaffinity(0, self.old)
        return False


def pin_note(cpus):
    return "threads pinned one per CPU to %s (sched_setaffinity)" % (cpus,) if cpus else "unpinned"


def cpu_baseline(imgs, masks, ncams, nfeatures, n_multiframes):
    """Oracle (CPU restatement) on a bounded sample: one thread per camera, like the
    reference's `#pragma omp parallel for num_threads(nrCams)` (src/cMultiFrame.cpp:128);
    matching single-threaded per camera pair.  Returns (kfeatures/s, sample text, threads)."""
    from tests import oracle_bind as ob
    ob.lib()
    nkp = 0
    kpss = [[None] * ncams for _ in range(n_multiframes)]
    descs = [[None] * ncams for _ in range(n_multiframes)]
    top2 = [[None] * ncams for _ in range(n_multiframes - 1)]
    lock = threading.Lock()
    cpus = baseline_cpus(ncams)

    match_s = [0.0] * ncams

    def work(c):
        nonlocal nkp
        if len(cpus) == ncams:   # fresh thread: pinned for its whole life
            os.sched_setaffinity(0, {cpus[c]})
        for t in range(n_multiframes):
            k, d = ob.extract(imgs[t * ncams + c], masks[c], nfeatures=nfeatures)
            kpss[t][c] = k
            descs[t][c] = d
            with lock:
                nkp += len(k)
        tm = time.perf_counter()
        for t in range(1, n_multiframes):
            q, tr = descs[t - 1][c], descs[t][c]
            top2[t - 1][c] = ob.hamming_top2(q, tr)
        match_s[c] = time.perf_counter() - tm

    ob.stage_ns(reset=True)
    t0 = time.perf_counter()
    ths = [threading.Thread(target=work, args=(c,)) for c in range(ncams)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    sample = "%d multi-frames x %d cams (extract+match), oracle restatement; %s" % (
        n_multiframes, ncams, pin_note(cpus if len(cpus) == ncams else []))
    ns = ob.stage_ns(reset=True)
    nf = n_multiframes * ncams
    stages = {k: round(float(v) / 1e6 / nf, 3) for k, v in
              zip(("pyramid", "fast", "octree", "ic_angle", "blur_desc"), ns)}
    stages["match_per_pair"] = round(1e3 * sum(match_s) / max(1, (n_multiframes - 1) * ncams), 3)
    return nkp / dt / 1e3, sample, ncams, (kpss, descs, top2), stages


def check_against_cpu_baseline(ref, d_kps, d_cnt, d_desc, d_m, ncams, of_step="last timed step"):
    """Untimed post-run parity check of the timed batch: the camera-frames and match pairs the
    CPU baseline leg computed (the first multi-frames of the batch) against the GPU's outputs of
    the LAST timed step, bit-exact: keypoint fields, descriptors, (best idx, best dist, second
    dist).  Returns a summary dict; raises if anything differs."""
    import mcs_amd
    kpss, descs, top2 = ref
    cap = d_kps.shape[1] // 7
    nmf = len(kpss)
    frames = [t * ncams + c for t in range(nmf) for c in range(ncams)]
    cnt = d_cnt.cpu().numpy()
    kp = d_kps[:len(frames)].cpu().numpy().view(mcs_amd.KEYPOINT_DTYPE).reshape(len(frames), cap)
    de = d_desc[:len(frames)].cpu().numpy()
    for f in frames:
        t, c = divmod(f, ncams)
        n = len(kpss[t][c])
        if cnt[f] != n or not np.array_equal(kp[f, :n], kpss[t][c]) or \
                not np.array_equal(de[f, :n], descs[t][c]):
            raise RuntimeError("bench parity: camera-frame %d differs from the oracle" % f)
    npairs = (nmf - 1) * ncams
    m = [x[:npairs].cpu().numpy() for x in d_m]
    for t in range(nmf - 1):
        for c in range(ncams):
            p = t * ncams + c
            n = len(kpss[t][c])
            bi, bd, sd = top2[t][c]
            if not (np.array_equal(m[0][p, :n], bi) and np.array_equal(m[1][p, :n], bd)
                    and np.array_equal(m[3][p, :n], sd)):
                raise RuntimeError("bench parity: match pair %d differs from the oracle" % p)
    return {"camera_frames_bitexact": len(frames), "match_pairs_bitexact": npairs,
            "keypoints_checked": int(sum(len(k) for row in kpss for k in row)),
            "of_step": of_step}


def single_multiframe_latency(ex, d_img, d_midx, d_kps, d_cnt, d_desc, ncams, stream, reps):
    """Latency of one cMultiFrame extraction (the NC cameras of one multi-frame, one batched
    call, inputs resident in HBM), wall clock around launch + stream synchronise; median and
    p90 over `reps` calls.  Complements the batched throughput."""
    import torch
    ex.enable_timing(False)
    ts = []
    for r in range(reps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ex.extract_batch_device(d_img.data_ptr(), ncams, d_midx.data_ptr(), d_kps.data_ptr(),
                                d_cnt.data_ptr(), d_desc.data_ptr(), stream.cuda_stream)
        stream.synchronize()
        if r >= 2:
            ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return {"multiframe_extract_ms_median": round(ts[len(ts) // 2], 4),
            "multiframe_extract_ms_p90": round(ts[int(0.9 * (len(ts) - 1))], 4),
            "reps": reps, "cameras": ncams, "keypoints": int(d_cnt[:ncams].sum().item())}


def host_cpu_info():
    """CPU model and thread count of the host the CPU baseline ran on."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"cpu_model": model, "host_threads_visible": avail,
            "oracle_build": "g++ -O3 -ffp-contract=off -fno-fast-math (portable x86-64, no -march)"}


def run_global_ba(args, rank, world, local_rank, dev):
    """Config E: GlobalBA (cOptimizer::BundleAdjustment) over 200 MultiKeyFrames / ~50k points /
    ~400k edges of an 8-camera 1024^2 ring rig.  N GPUs: points sharded with all their edges,
    poses replicated, one RCCL all-reduce of the reduced camera system per LM trial
    (strong scaling: the same problem on every N).  Returns (result dict, cpu baseline)."""
    if args.gba_calls <= 0:
        return None, None
    import torch
    import torch.distributed as dist
    from mcs_amd import ba as mba
    # the map -> graph assembly of BundleAdjustment (mcs_global_ba_select), as a caller would
    pr = mba.config_e_problem(n_kf=args.gba_kf, n_points=args.gba_points,
                              target_edges=args.gba_edges, seed=7)
    xch = None
    sub = pr
    if world > 1:
        sub, _, _ = mba.shard_problem(pr, rank, world)
        xch = mba.TorchExchange(len(pr["poses"]), dev)
    solver = mba.Solver(device=local_rank)
    solver.global_ba(sub, exchange=xch)       # warm-up (allocations, code objects)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    solver.read_host_timing(reset=True)
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.gba_calls):
        r = solver.global_ba(sub, exchange=xch)
        iters += r["report"].iterations
    tg = time.perf_counter() - t0
    host_ms, _ = solver.read_host_timing(reset=True)
    # stage breakdown from one more call with per-stage HIP events (that call synchronises per
    # trial, so it is not part of the timed calls above)
    solver.enable_timing(True)
    solver.read_timing(reset=True)
    solver.global_ba(sub, exchange=xch)
    st, n_it, n_tr, n = solver.read_timing(reset=True)
    solver.enable_timing(False)
    tt = torch.tensor([tg], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    tg = float(tt.item())
    # dense LDL^T of the n x n reduced camera system per trial, counted exactly as SURVEY.md
    # section 8(d) defines it: n^3/3 for the factorisation + 2 n^2 for the two triangular
    # solves (the same count the MFMA-utilisation target is stated against)
    flops = n ** 3 / 3.0 + 2.0 * n * n
    t_solve = st["solve"] / max(1, n_tr) / 1e3
    achieved = flops / t_solve / 1e12 if t_solve > 0 else None
    out = {"iters_per_s": round(iters / tg, 2), "ms_per_call": round(tg / args.gba_calls * 1e3, 2),
           "iterations_per_call": r["report"].iterations,
           "chi2": [r["report"].chi2_initial, r["report"].chi2_final],
           "scaling": "strong", "parallelism": "points sharded over %d rank(s)" % world,
           "problem": "config E: %d MKF (1 fixed), %d points, %d edges, 8 cams 1024^2" % (
               len(pr["poses"]), len(pr["points"]), len(pr["edge_pose"])),
           "stage_ms_per_trial": {k: round(v / max(1, n_tr), 4) for k, v in st.items()},
           "host_ms_per_call": {k: round(v / args.gba_calls, 4) for k, v in host_ms.items()},
           "trials": n_tr,
           "roofline_solve": {"kernel": "ldlt k_pipe (pipelined factorisation, one launch) + k_bwd (n=%d)" % n, "bound": "mfma",
                              "achieved": None if achieved is None else round(achieved, 4),
                              "peak": FP64_MFMA_PEAK_TFLOPS, "peak_source": FP64_MFMA_PEAK_SRC,
                              "unit": "TFLOP/s",
                              "frac": None if achieved is None else round(achieved / FP64_MFMA_PEAK_TFLOPS, 5),
                              "peak_measured": FP64_MFMA_MEASURED_TFLOPS,
                              "peak_measured_source": FP64_MFMA_MEASURED_SRC,
                              "frac_vs_measured": None if achieved is None else round(
                                  achieved / FP64_MFMA_MEASURED_TFLOPS, 5),
                              "flops_per_trial": flops,
                              "flops_definition": "n^3/3 + 2 n^2 (SURVEY.md 8(d))"}}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from tests import oracle_bind as ob
        o = mba.BAOptions(max_iterations=1, terminate_max_iter=15)
        cpus = baseline_cpus(1)
        with pinned_thread(cpus[0] if cpus else None):
            t0 = time.perf_counter()
            rr = ob.ba_optimize(pr, options=o)
            tc = time.perf_counter() - t0
        cpu = {"value": round(rr["report"].iterations / tc, 4), "unit": "GlobalBA iters/s",
               "cores": 1, "kind": "port",
               "sample": "1 LM iteration of config E (oracle restatement, dense LDL^T, single "
                         "thread); " + pin_note(cpus)}
    return out, cpu


def run_config_d(args, rank, world, local_rank, dev, stream):
    """Config D: 8 synthetic fisheye cameras 1024^2, 4000 features/camera, camera c extracted
    on rank c % N (cMultiFrame's per-camera OpenMP loop, src/cMultiFrame.cpp:128, becomes one
    camera per GPU); per step every rank extracts its cameras for `d_multiframes` multi-frames
    and one all-gather per per-camera buffer (RCCL over xGMI) hands every rank the whole
    MultiFrame (the host concatenation :166-184).  Strong scaling: the same 8 x MD
    camera-frames on every N."""
    if args.d_multiframes <= 0:
        return None
    import torch
    import torch.distributed as dist
    import mcs_amd
    from mcs_amd import synth, rig
    NC, W, H, MD = 8, 1024, 1024, args.d_multiframes
    S = rig.slots_per_rank(NC, world)
    owned = rig.owned_cameras(NC, world, rank)
    slot_cam = [owned[min(s, len(owned) - 1)] if owned else 0 for s in range(S)]
    U = max(1, min(args.d_unique, MD))
    imgs = np.zeros((S, U, H, W), np.uint8)
    masks = np.zeros((S, H, W), np.uint8)
    for s, c in enumerate(slot_cam):
        for t in range(U):
            img, m = synth.fisheye_frame(W, H, seed=500 + c, cam_index=c, yaw=0.015 * t,
                                         noise_seed=900000 + 16 * t + c)
            imgs[s, t] = img
            masks[s] = m
    # slot-major frame order f = s * MD + t, so each slot's block is contiguous for the gather
    frames = imgs[:, np.arange(MD) % U].reshape(S * MD, H, W)
    F = S * MD
    params = mcs_amd.ExtractorParams(nfeatures=4000, fast_threshold=20)
    ex = mcs_amd.Extractor(params, W, H, max_frames=F, device=local_rank)
    cap = ex.capacity
    d_img = torch.from_numpy(frames).to(dev)
    d_mask = torch.from_numpy(masks).to(dev)
    ex.set_masks_device(d_mask.data_ptr(), S, stream.cuda_stream)
    d_midx = torch.from_numpy(np.repeat(np.arange(S, dtype=np.int32), MD)).to(dev)
    d_kps = torch.zeros((F, cap * 7), dtype=torch.int32, device=dev)
    d_cnt = torch.zeros(F, dtype=torch.int32, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gathered = {}

    def step(timed):
        ex.extract_batch_device(d_img.data_ptr(), F, d_midx.data_ptr(), d_kps.data_ptr(),
                                d_cnt.data_ptr(), d_desc.data_ptr(), stream.cuda_stream)
        if timed:
            ev0.record(stream)
        gathered["cnt"] = rig.gather_camera_blocks(d_cnt.view(S, MD), NC)
        gathered["kps"] = rig.gather_camera_blocks(d_kps.view(S, MD * cap * 7), NC)
        gathered["desc"] = rig.gather_camera_blocks(d_desc.view(S, MD * cap * 32), NC)
        if timed:
            ev1.record(stream)

    for _ in range(max(1, args.warmup)):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    cnt = gathered["cnt"]                       # [8, MD] in camera order, on every rank
    kp_per_step = int(cnt.sum().item())
    # the gathered MultiFrame must hold every camera's own extraction (rank-local check)
    mine = d_cnt.view(S, MD)
    for s, c in enumerate(owned):
        if not torch.equal(cnt[c], mine[s]):
            raise RuntimeError("config D all-gather mismatch for camera %d" % c)
    gb = (d_kps.numel() * 4 + d_desc.numel() + d_cnt.numel() * 4) * world / 1e9
    return {"kfeatures_per_s": round(kp_per_step * args.steps / dt / 1e3, 2),
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "allgather_ms_last_step": round(ev0.elapsed_time(ev1), 4),
            "allgather_gb_per_step": round(gb, 4),
            "keypoints_per_step": kp_per_step,
            "scaling": "strong", "parallelism": "camera-per-GPU (%d camera slot(s) per rank)" % S,
            "problem": "config D: 8 cams 1024x1024, 4000 feat/cam, %d multi-frames per step" % MD}


def run_triangulation(args, rank, world, dev, stream, d_kps, d_cnt, d_desc, cap, ncams, U):
    """SearchForTriangulationRaw as CreateNewMapPoints drives it (src/cLocalMapping.cpp:223-266
    -> src/cORBmatcher.cpp:968-1156): the current keyframe against its 5 best covisible
    neighbours, one device call per neighbour, on the keyframes the timed extraction produced
    (multi-frame 5 against multi-frames 0..4: 3 cameras x up to 2000 keypoints each), with
    keypoint rays from the Lafida omni model (ImgToWorld) and E from mcs_compute_e_rig.  Timed
    with events on the launch stream over `tri_reps` keyframes; untimed afterwards, every
    neighbour's match list is checked against the oracle.  Reported beside the headline."""
    if args.tri_reps <= 0 or U < 6:
        return None, None
    import torch
    import mcs_amd
    from mcs_amd import synth
    L = mcs_amd.lib()
    cams = [synth.LAFIDA_CAMS[c % len(synth.LAFIDA_CAMS)] for c in range(ncams)]
    cnt = d_cnt.cpu().numpy()
    kps = d_kps.view(-1, cap, 7)
    rng = np.random.default_rng(31 + rank)
    kf = []
    for t in range(6):
        fr = [t * ncams + c for c in range(ncams)]
        desc = torch.cat([d_desc[f, :cnt[f]] for f in fr]).contiguous()
        xy = torch.cat([kps[f, :cnt[f], :2] for f in fr]).cpu().numpy().view(np.float32).astype(np.float64)
        cam = np.concatenate([np.full(cnt[f], c, np.int32) for c, f in enumerate(fr)])
        rays = np.zeros((len(cam), 3))
        for c in range(ncams):
            sel = cam == c
            x, y, z = synth.img_to_world(cams[c], xy[sel, 0], xy[sel, 1])
            rays[sel] = np.stack([x, y, z], 1)
        has = (rng.random(len(cam)) < 0.3).astype(np.uint8)   # keypoints already tracked
        kf.append(dict(desc=desc, cam=cam, rays=rays, has=has, n=len(cam),
                       d_cam=torch.from_numpy(cam).to(dev), d_rays=torch.from_numpy(rays).to(dev),
                       d_has=torch.from_numpy(has).to(dev)))
    mc = np.array(synth.LAFIDA_MC[:ncams], np.float64)
    Es = []
    for j in range(5):
        mt1 = np.array([0.0, 0.0, 0.0, 0.0, 0.0, 0.0])
        mt2 = np.array([0.01 * (j + 1), -0.005 * j, 0.002, 0.05 * (j + 1), 0.01, -0.02 * j])
        E = np.zeros((ncams, ncams, 9))
        assert L.mcs_compute_e_rig(mt1.ctypes.data, mt2.ctypes.data, mc.ctypes.data, ncams,
                                   E.ctypes.data) == 0
        Es.append(E)
    d_E = [torch.from_numpy(E).to(dev) for E in Es]
    th_low, thresh = 64, 1e-2   # TH_LOW (32 B, unmasked) and CheckDistEpipolarLine's 1e-2
    n1 = kf[5]["n"]
    n2max = max(k["n"] for k in kf[:5])
    ws = ctypes.c_void_p()
    if L.mcs_tri_workspace_create(dev.index, n1, n2max, ctypes.byref(ws)) != 0:
        raise RuntimeError("tri workspace: " + L.mcs_last_error().decode())
    out = [torch.empty(n1, dtype=torch.int32, device=dev) for _ in range(5)]
    nm = torch.empty(5, dtype=torch.int32, device=dev)
    k1 = kf[5]

    def one_kf():
        for j in range(5):
            k2 = kf[j]
            rc = L.mcs_search_for_triangulation_raw_device(
                ws, k1["desc"].data_ptr(), None, k1["d_cam"].data_ptr(), k1["d_has"].data_ptr(),
                k1["d_rays"].data_ptr(), n1, k2["desc"].data_ptr(), None, k2["d_cam"].data_ptr(),
                k2["d_has"].data_ptr(), k2["d_rays"].data_ptr(), k2["n"], ncams, d_E[j].data_ptr(),
                32, th_low, thresh, out[j].data_ptr(), nm[j:].data_ptr(), stream.cuda_stream)
            if rc != 0:
                raise RuntimeError("triangulation: " + L.mcs_last_error().decode())

    for _ in range(3):
        one_kf()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(args.tri_reps):
        one_kf()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.tri_reps
    # host entry (host buffers in and out, one synchronisation per neighbour), for comparison
    hd1 = k1["desc"].cpu().numpy()
    hd2 = [k["desc"].cpu().numpy() for k in kf[:5]]
    t0 = time.perf_counter()
    reps_h = max(1, min(5, args.tri_reps))
    for _ in range(reps_h):
        for j in range(5):
            got = np.zeros(n1, np.int32)
            n = ctypes.c_int32()
            rc = L.mcs_search_for_triangulation_raw(
                hd1.ctypes.data, k1["cam"].ctypes.data, k1["has"].ctypes.data, k1["rays"].ctypes.data,
                n1, hd2[j].ctypes.data, kf[j]["cam"].ctypes.data, kf[j]["has"].ctypes.data,
                kf[j]["rays"].ctypes.data, kf[j]["n"], ncams, Es[j].ctypes.data, 32, th_low, thresh,
                got.ctypes.data, ctypes.byref(n))
            if rc != 0:
                raise RuntimeError("triangulation host entry failed")
    ms_host = (time.perf_counter() - t0) / reps_h * 1e3
    L.mcs_tri_workspace_destroy(ws)
    same_cam = sum(int(sum(int((k1["cam"] == c).sum()) * int((kf[j]["cam"] == c).sum())
                           for c in range(ncams))) for j in range(5))
    res = {"ms_per_keyframe": round(ms, 4), "neighbours": 5,
           "host_entry_ms_per_keyframe": round(ms_host, 3),
           "distances_per_s": round(same_cam / (ms / 1e3), 1),
           "matches_per_neighbour": [int(v) for v in nm.cpu().numpy()],
           "keypoints": {"kf1": n1, "neighbours": [k["n"] for k in kf[:5]]},
           "th_low": th_low, "epi_thresh": thresh,
           "path": "mcs_search_for_triangulation_raw_device: k_tri_radius + k_tri_pass + k_tri_private + "
                   "k_tri_gather + k_tri_seq (ordered pass, one wave per camera)"}
    cpu = None
    if rank == 0 and world == 1:
        from tests import oracle_bind as ob
        t0 = time.perf_counter()
        refs = []
        for j in range(5):
            ref = np.zeros(n1, np.int32)
            ob.lib().oracle_search_for_triangulation_raw_ex(
                hd1.ctypes.data, None, n1, hd2[j].ctypes.data, None, kf[j]["n"], 32,
                k1["cam"].ctypes.data, kf[j]["cam"].ctypes.data, k1["has"].ctypes.data,
                kf[j]["has"].ctypes.data, np.ascontiguousarray(k1["rays"]).ctypes.data,
                np.ascontiguousarray(kf[j]["rays"]).ctypes.data, Es[j].ctypes.data, thresh, ncams,
                ref.ctypes.data)
            refs.append(ref)
        tc = time.perf_counter() - t0
        for j in range(5):
            if not np.array_equal(out[j].cpu().numpy(), refs[j]):
                raise RuntimeError("bench parity: triangulation neighbour %d differs from the oracle" % j)
        res["oracle_check"] = "5 of 5 neighbour match lists bit-exact"
        if not args.no_cpu_baseline:
            cpu = {"value": round(1e3 * tc, 2), "unit": "ms per keyframe (5 neighbours)", "cores": 1,
                   "kind": "port", "sample": "the same 5 neighbour searches, oracle restatement, "
                   "single thread (unpinned)"}
    return res, cpu


def run_bow(args, rank, world, dev, stream, d_desc, n_valid):
    """DBoW2 transform: every descriptor slot of one step's extraction
    output through the reference's own vocabulary (small_orb_omni_voc_9_6, k=9, L=6),
    levelsup = 4 as cMultiFrame::ComputeBoW.  Reported beside the headline, not in `value`."""
    if args.bow_reps <= 0:
        return None, None
    import torch
    from mcs_amd import vocab
    v = vocab.load_npz(os.path.join(ROOT, "tests", "golden", "small_orb_omni_voc_9_6.npz"))
    V = vocab.Vocabulary(v, device=dev.index)
    flat = d_desc.view(-1, 32)
    n = flat.shape[0]
    word = torch.empty(n, dtype=torch.int32, device=dev)
    weight = torch.empty(n, dtype=torch.float64, device=dev)
    node = torch.empty(n, dtype=torch.int32, device=dev)
    ptrs = (flat.data_ptr(), n, 4, word.data_ptr(), weight.data_ptr(), node.data_ptr(),
            stream.cuda_stream)
    V.transform_words_device(*ptrs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.bow_reps):
        V.transform_words_device(*ptrs)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.bow_reps
    V.close()
    bpd = 48   # 32 B descriptor in, word (4) + weight (8) + node (4) out
    gbs = n * bpd / (ms / 1e3) / 1e9
    out = {"descriptors_per_s": round(n / (ms / 1e3), 1), "ms_per_call": round(ms, 4),
           "descriptor_slots": n, "valid_descriptors": n_valid,
           "vocabulary": "small_orb_omni_voc_9_6 (k=9, L=6, 8822 nodes, 6999 words), levelsup=4",
           "roofline": {"kernel": "k_descend", "bound": "hbm", "achieved": round(gbs, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_descriptor": bpd}}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from tests import oracle_bind as ob
        sample = flat[: min(n, 200000)].cpu().numpy()
        cpus = baseline_cpus(1)
        with pinned_thread(cpus[0] if cpus else None):
            t0 = time.perf_counter()
            ob.vocab_words(v, sample, 4)
            tc = time.perf_counter() - t0
        cpu = {"value": round(len(sample) / tc, 1), "unit": "descriptors/s", "cores": 1,
               "kind": "port", "sample": "%d descriptor slots of the step, oracle restatement "
                                         "(vocabulary build included); %s" % (
                                             len(sample), pin_note(cpus))}
    return out, cpu


def launch_ranks(n):
    """One process per GPU via torch.distributed.run (rendezvous on 127.0.0.1); the children
    re-enter main() with RANK/LOCAL_RANK/WORLD_SIZE set.  Returns the launcher's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def reduce_over_ranks(dt, kp_total, dev, world):
    """Timed-region reduction of every leg: MAX of the wall time, SUM of the work."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    k = torch.tensor([kp_total], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(k, op=dist.ReduceOp.SUM)
    return float(t.item()), float(k.item())


def selftest_dist(rank, world):
    """`--selftest-dist`: the N-rank launch and the collective code of the legs on CPU (gloo):
    the timed-region reduction, the config-D camera all-gather (mcs_amd/rig.py) and the
    GlobalBA exchange callback (mcs_amd/ba.py TorchExchange).  No GPU is touched."""
    import torch
    import torch.distributed as dist
    from mcs_amd import rig
    from mcs_amd import ba as mba
    dist.init_process_group("gloo")
    dev = torch.device("cpu")
    dt, kp = reduce_over_ranks(0.01 * (rank + 1), 1000.0 * (rank + 1), dev, world)
    assert dt == 0.01 * world and kp == 1000.0 * world * (world + 1) / 2
    NC, MD = 8, 3
    S = rig.slots_per_rank(NC, world)
    own = rig.owned_cameras(NC, world, rank)
    local = torch.full((S, MD), -1, dtype=torch.int32)
    for s, c in enumerate(own):
        local[s] = torch.arange(MD, dtype=torch.int32) + 100 * c
    g = rig.gather_camera_blocks(local, NC)
    want = torch.stack([torch.arange(MD, dtype=torch.int32) + 100 * c for c in range(NC)])
    assert torch.equal(g, want), g
    xch = mba.TorchExchange(10, dev)
    xch.buf.fill_(float(rank + 1))
    assert xch.shard.stream_ordered == 0     # CPU buffer: synchronous reduction
    assert xch._allreduce(None, 0, 0, 60, None) == 0
    assert float(xch.buf[0]) == world * (world + 1) / 2
    if rank == 0:
        print(json.dumps({"selftest": "ok", "n_gpus": world, "ms_per_step": dt * 1e3,
                          "value": kp, "allgather_cameras": NC}))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--multiframes", type=int, default=171, help="multi-frames per rank per step")
    ap.add_argument("--split", type=int, default=2,
                    help="K: extract the step's multi-frames as K parts on K streams, each "
                         "part's pairs matched beside the other parts' extraction (1: one launch "
                         "chain over the whole batch)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="1: consecutive steps overlap (step s+1's extraction beside step s's "
                         "matching on a match stream; the outputs are double-buffered)")
    ap.add_argument("--unique", type=int, default=12, help="distinct rendered multi-frames")
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--cpu-sample", type=int, default=12, help="multi-frames timed on the CPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stage-timing", type=int, default=1)
    ap.add_argument("--ba-calls", type=int, default=20, help="timed LocalBA calls (config C)")
    ap.add_argument("--gba-calls", type=int, default=2, help="timed GlobalBA calls (config E)")
    ap.add_argument("--gba-kf", type=int, default=200)
    ap.add_argument("--gba-points", type=int, default=50000)
    ap.add_argument("--gba-edges", type=int, default=400000)
    ap.add_argument("--d-multiframes", type=int, default=16,
                    help="config D multi-frames per step (8 cams 1024^2, camera per GPU); 0 = off")
    ap.add_argument("--bow-reps", type=int, default=10, help="timed DBoW2 transform launches; 0 = off")
    ap.add_argument("--tri-reps", type=int, default=20,
                    help="timed SearchForTriangulationRaw keyframes (5 neighbours each); 0 = off")
    ap.add_argument("--d-unique", type=int, default=2, help="distinct rendered config D multi-frames")
    ap.add_argument("--latency-reps", type=int, default=20,
                    help="single multi-frame extraction latency samples; 0 = off")
    ap.add_argument("--selftest-dist", action="store_true",
                    help="CPU (gloo) rehearsal of the multi-rank launch and collectives only")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` outside torchrun: start N fresh ranks as child processes (nothing
        # has touched the GPU in this process yet) and exit with their status
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.selftest_dist:
        return selftest_dist(rank, world)

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import mcs_amd
    from mcs_amd import synth
    L = mcs_amd.lib()
    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.current_stream()

    W, H, NC = 754, 480, 3
    M = args.multiframes
    U = min(args.unique, M)
    uimgs, imgs, masks, midx, pairs = synth.config_b_batch(M, U, rank, W, H, NC)
    F = M * NC

    params = mcs_amd.ExtractorParams(nfeatures=args.nfeatures, fast_threshold=20)
    ex = mcs_amd.Extractor(params, W, H, max_frames=F, device=local_rank)
    cap = ex.capacity
    d_img = torch.from_numpy(imgs).to(dev)
    d_mask = torch.from_numpy(masks).to(dev)
    ex.set_masks_device(d_mask.data_ptr(), NC, stream.cuda_stream)
    d_midx = torch.from_numpy(midx).to(dev)
    d_kps = torch.zeros((F, cap * 7), dtype=torch.int32, device=dev)
    d_cnt = torch.zeros(F, dtype=torch.int32, device=dev)
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device=dev)
    d_pairs = torch.from_numpy(pairs).to(dev)
    NP = len(pairs)
    d_m = [torch.zeros((NP, cap), dtype=torch.int32, device=dev) for _ in range(4)]
    # --pipeline: a second output set, so that step s+1 extracts while step s's pairs are matched
    bufs = [(d_kps, d_cnt, d_desc)]
    if args.pipeline:
        bufs.append((torch.zeros_like(d_kps), torch.zeros_like(d_cnt), torch.zeros_like(d_desc)))

    ev_m0 = torch.cuda.Event(enable_timing=True)
    ev_m1 = torch.cuda.Event(enable_timing=True)
    # --split K (default 2): the batch as K parts of consecutive multi-frames, each with its own
    # extractor (its own workspace) on its own stream; a part's pairs are matched as soon as it
    # is extracted (MFMA work beside the other parts' VALU-bound extraction), the pairs across a
    # part boundary once both sides are.  Same kernels, same outputs.
    K = max(1, min(args.split, M // 2))
    split = K > 1
    if split:
        mb = [M * k // K for k in range(K + 1)]            # part k = multi-frames [mb[k], mb[k+1])
        exs = [ex] + [mcs_amd.Extractor(params, W, H, max_frames=(mb[k + 1] - mb[k]) * NC, device=local_rank)
                      for k in range(1, K)]
        for e in exs[1:]:
            e.set_masks_device(d_mask.data_ptr(), NC, stream.cuda_stream)
        sts = [stream] + [torch.cuda.Stream(device=dev) for _ in range(1, K)]
        ev_go = torch.cuda.Event()
        ev_done = [torch.cuda.Event() for _ in range(K)]
        ev_end = [torch.cuda.Event() for _ in range(K)]

    def match(p0, n, st, b=0):
        _, cnt_b, desc_b = bufs[b]
        rc = L.mcs_hamming_top2_batch_device(desc_b.data_ptr(), cnt_b.data_ptr(),
                                             d_pairs.data_ptr() + 8 * p0, n, cap, 32,
                                             *[t.data_ptr() + 4 * p0 * cap for t in d_m], st)
        if rc != 0:
            raise RuntimeError("matcher failed %d" % rc)

    def extract_part(k, st, b=0):
        kps_b, cnt_b, desc_b = bufs[b]
        f0, nf = mb[k] * NC, (mb[k + 1] - mb[k]) * NC
        exs[k].extract_batch_device(d_img.data_ptr() + f0 * W * H, nf, d_midx.data_ptr() + 4 * f0,
                                    kps_b.data_ptr() + 4 * f0 * cap * 7, cnt_b.data_ptr() + 4 * f0,
                                    desc_b.data_ptr() + f0 * cap * 32, st.cuda_stream)

    # --pipeline: the parts' extraction streams run from step to step without waiting for the
    # matching, which follows on its own stream; output set s % 2 is reused by step s + 2 only
    # after step s's matching (ev_free)
    if args.pipeline:
        if not split:
            mb, exs, sts, K = [0, M], [ex], [stream], 1
        mst = torch.cuda.Stream(device=dev)
        ev_x = [[torch.cuda.Event() for _ in range(K)] for _ in range(2)]
        ev_free = [torch.cuda.Event() for _ in range(2)]
        free_rec = [False, False]
        pstep = [0]

    def step_pipelined():
        b = pstep[0] % 2
        pstep[0] += 1
        for k in range(K):
            if free_rec[b]:
                sts[k].wait_event(ev_free[b])
            extract_part(k, sts[k], b)
            ev_x[b][k].record(sts[k])
        mst.wait_event(ev_x[b][0])
        match(0, (mb[1] - 1) * NC, mst.cuda_stream, b)
        for k in range(1, K):
            mst.wait_event(ev_x[b][k])
            p0 = (mb[k] - 1) * NC
            match(p0, (mb[k + 1] - 1) * NC - p0, mst.cuda_stream, b)
        ev_free[b].record(mst)
        free_rec[b] = True
        return b

    def step(timed, allow_split=True):
        if args.pipeline and allow_split:
            return step_pipelined()
        if split and allow_split:
            ev_go.record(stream)
            for k in range(1, K):
                sts[k].wait_event(ev_go)
            for k in range(K):
                extract_part(k, sts[k])
                ev_done[k].record(sts[k])
            if timed:
                ev_m0.record(stream)
            match(0, (mb[1] - 1) * NC, stream.cuda_stream)      # part 0's own pairs
            for k in range(1, K):   # the boundary pair (mb[k] - 1, mb[k]) and part k's own pairs
                sts[k].wait_event(ev_done[k - 1])
                p0 = (mb[k] - 1) * NC
                match(p0, (mb[k + 1] - 1) * NC - p0, sts[k].cuda_stream)
                ev_end[k].record(sts[k])
                stream.wait_event(ev_end[k])
            if timed:
                ev_m1.record(stream)
            return
        ex.extract_batch_device(d_img.data_ptr(), F, d_midx.data_ptr(), d_kps.data_ptr(),
                                d_cnt.data_ptr(), d_desc.data_ptr(), stream.cuda_stream)
        if timed:
            ev_m0.record(stream)
        match(0, NP, stream.cuda_stream)
        if timed:
            ev_m1.record(stream)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # timed region: the production path, no stage events between the kernels
    t0 = time.perf_counter()
    last_b = 0
    for _ in range(args.steps):
        last_b = step(True) or 0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    # matcher device time (events on the launch stream around the match launch alone): in split
    # mode the timed step's events also wrap the wait on the second half's extraction, so the
    # figure comes from the one-stream stage-timing steps below instead
    match_ms_last = None if (split or args.pipeline) else ev_m0.elapsed_time(ev_m1)
    # per-stage kernel times for the roofline: a few extra, untimed steps with the stage
    # events on (which run the stages back to back on one stream)
    stages, ncalls = {}, 0
    if args.stage_timing:
        ex.enable_timing(True)
        for _ in range(max(2, min(5, args.steps))):
            step(True, False)    # the stages back to back on one stream, the whole batch
        torch.cuda.synchronize()
        stages, ncalls = ex.read_timing()
        ex.enable_timing(False)
        match_ms_last = ev_m0.elapsed_time(ev_m1)

    kp_per_step = int(d_cnt.sum().item())
    dt_max, kp_tot = reduce_over_ranks(dt, kp_per_step * args.steps, dev, world)
    latency = single_multiframe_latency(ex, d_img, d_midx, d_kps, d_cnt, d_desc, NC, stream,
                                        args.latency_reps) if args.latency_reps > 0 else None
    value = kp_tot / dt_max / 1e3

    wh, _ = ex.levels()
    bpf = alg_bytes_pyr_fast(wh)
    roofline = None
    stage_ms = {}
    if ncalls:
        stage_ms = {k: v / ncalls for k, v in stages.items()}
        # pyramid + FAST = k_pyr_rows<true> x (L-1) (resize + fused blur) + k_fast_rows (all
        # levels, one launch); the level-0 blur launch is not part of the algorithmic bytes
        #  and is not timed
        t_pf = (stage_ms["pyramid"] + stage_ms["fast"]) / 1e3
        achieved = bpf * F / t_pf / 1e9
        roofline = {"kernel": "pyramid+fast: k_pyr_rows<true> x %d (resize + 5x5 blur) + "
                              "k_fast_rows (FAST-9/16 + cell-local NMS + mask)" % (len(wh) - 1),
                    "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": None, "alg_bytes_per_call": bpf * F}
        roofline.update(pmc_traffic(bpf * F))
        roofline.update(sq_issue())
    roofline_od, roofline_oct = (stage_rooflines(ex, F, stage_ms, kp_per_step, params.desc_size)
                                 if ncalls else (None, None))

    # ---- LocalBA (config C): 10 local MultiKeyFrames + 3 fixed observers, 3k points, ~20k edges
    localba = None
    cpu_ba = None
    if args.ba_calls > 0:
        from mcs_amd import ba as mba
        pr = mba.make_problem(seed=1 + rank)
        solver = mba.Solver(device=local_rank)
        for _ in range(3):   # warm-up (code objects, grow-only buffers, clocks)
            solver.local_ba(pr)
        solver.read_host_timing(reset=True)
        t0 = time.perf_counter()
        iters = 0
        for _ in range(args.ba_calls):
            r = solver.local_ba(pr)
            iters += r["report1"].iterations + r["report2"].iterations
        tba = time.perf_counter() - t0
        host_ms, _ = solver.read_host_timing(reset=True)
        it_rate = torch.tensor([iters / tba], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(it_rate, op=dist.ReduceOp.SUM)
        localba = {"iters_per_s": round(float(it_rate.item()), 1),
                   "calls_per_s_per_gpu": round(args.ba_calls / tba, 2),
                   "ms_per_call": round(tba / args.ba_calls * 1e3, 3),
                   "iterations_per_call": [r["report1"].iterations, r["report2"].iterations],
                   "host_ms_per_call": {k: round(v / args.ba_calls, 4) for k, v in host_ms.items()},
                   "problem": "config C: %d poses (%d fixed), %d points, %d edges, 3 cams" % (
                       len(pr["poses"]), int(pr["pose_fixed"].sum()), len(pr["points"]),
                       len(pr["edge_pose"]))}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from tests import oracle_bind as ob
            cpus = baseline_cpus(1)
            with pinned_thread(cpus[0] if cpus else None):
                t0 = time.perf_counter()
                o = ob.local_ba(pr)
                tc = time.perf_counter() - t0
            cpu_ba = {"value": round((o["report1"].iterations + o["report2"].iterations) / tc, 2),
                      "unit": "LocalBA iters/s", "cores": 1, "kind": "port",
                      "sample": "1 LocalBA call (config C), oracle restatement, single thread; " +
                                pin_note(cpus)}

    bow, cpu_bow = run_bow(args, rank, world, dev, stream, d_desc, kp_per_step)
    tri, cpu_tri = run_triangulation(args, rank, world, dev, stream, d_kps, d_cnt, d_desc, cap, NC, U)
    gba, cpu_gba = run_global_ba(args, rank, world, local_rank, dev)
    cfg_d = run_config_d(args, rank, world, local_rank, dev, stream)

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        S = min(args.cpu_sample, U)
        v, sample, cores, ref, stages = cpu_baseline(uimgs, masks, NC, args.nfeatures, S)
        cpu = {"value": round(v, 3), "unit": "kfeatures/s", "cores": cores, "kind": "port",
               "sample": sample,
               "stage_ms_per_camera_frame": stages,
               "note": "upper bound on the GPU/CPU ratio: a scalar portable-x86-64 restatement "
                       "(no -march, no SIMD intrinsics, -ffp-contract=off), not the reference's "
                       "OpenCV SSE/AVX build"}
        cpu.update(host_cpu_info())
        # the stage-timed steps (one stream, output set 0) ran last when stage timing is on;
        # otherwise the last timed step's output set
        chk = bufs[0] if args.stage_timing else bufs[last_b]
        parity = check_against_cpu_baseline(ref, chk[0], chk[1], chk[2], d_m, NC,
                                            "last stage-timed step" if args.stage_timing else "last timed step")

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "kfeatures/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (Lafida-calibrated fisheye renders, resident in HBM)",
            "config": {"workload": "config B: 3-cam Lafida rig 754x480, 2000 feat/cam, "
                                   "extract + consecutive-multi-frame top-2 Hamming match",
                       "camera_frames_per_step_per_gpu": F,
                       "keypoints_per_step_per_gpu": kp_per_step,
                       "match_pairs_per_step_per_gpu": NP,
                       "parallelism": "dp%d (independent multi-frame segments)" % world,
                       "schedule": ("%d parts of the step's multi-frames on %d streams "
                                    "(%d extractors), each part's pairs matched after it" % (K, K, K)
                                    if split else "one stream") +
                                   ("; steps pipelined: step s+1 extracts while step s's pairs are "
                                    "matched on a match stream (double-buffered keypoints and "
                                    "descriptors)" if args.pipeline else "")},
            "roofline": roofline,
            "roofline_orient_desc": roofline_od,
            "roofline_octree": roofline_oct,
            "cpu_baseline": cpu,
            "parity_check": parity,
            "localba": localba,
            "cpu_baseline_localba": cpu_ba,
            "globalba": gba,
            "cpu_baseline_globalba": cpu_gba,
            "config_d": cfg_d,
            "bow": bow,
            "cpu_baseline_bow": cpu_bow,
            "triangulation": tri,
            "cpu_baseline_triangulation": cpu_tri,
            "latency": latency,
            "stage_ms_per_step": {k: round(v, 4) for k, v in stage_ms.items()},
            "match_ms_per_step": None if match_ms_last is None else round(match_ms_last, 4),
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
