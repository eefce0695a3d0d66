"""Generate tests/golden/mcsjacs1.npz: literal evaluations of the reference's mcsJacs1.

mcsJacs1 (/root/reference/src/g2o_MultiCol_vertices_edges.cpp:134-1145) is ~1000 lines of
machine-generated straight-line double arithmetic (`const double tN = <expr>;`, then
`jacs(i, j) = <expr>;`).  This script reads that function as TEXT from the reference checkout
(run it in the build container, where /root/reference exists), evaluates every statement in
order with Python floats (IEEE double, the same left-to-right operator precedence as C++;
sqrt / atan / pow from the C library through `math`), and stores inputs + the full 2 x 32
`jacs` matrix per sample.  No reference source is stored: the fixture is numbers only.

Samples: edges of the synthetic Lafida-rig LocalBA problem (`mcs_amd.ba.make_problem`), poses
and points perturbed off the ground truth so no residual is zero.  The GPU Jacobians are
asserted against `-jacs` (linearizeOplus sign, :84-126) in tests/test_ba_golden.py.

    python tests/golden/gen_mcsjacs1.py [--ref /root/reference] [--n 96]
"""
import argparse
import math
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "multicol-slam-annotation_amd"))
sys.path.insert(0, HERE)
from safe_exec import safe_compile_eval, safe_eval  # noqa: E402

_INT_LIT = re.compile(r"(?<![\w.])\d+(?![\w.])")


def _function_body(src, name):
    i = src.index("void " + name + "(")
    j = src.index("{", i)
    depth, k = 0, j
    while True:
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                return src[j + 1:k]
        k += 1


def _to_py(expr):
    expr = re.sub(r"pt3\((\d)\)", r"pt3[\1]", expr)
    expr = re.sub(r"(M_t|M_c|camModelData)\((\d+),\s*0\)", r"\1[\2]", expr)
    expr = re.sub(r"\b(sqrt|atan|pow)\(", r"math.\1(", expr)
    ints = _INT_LIT.findall(re.sub(r"\[\d+\]", "", expr))
    if ints:
        # an int literal would behave differently only in int/int division; forbid any
        raise ValueError("integer literal in expression: %s" % expr[:120])
    return expr


def compile_mcsjacs1(ref_root):
    path = os.path.join(ref_root, "src", "g2o_MultiCol_vertices_edges.cpp")
    src = open(path, encoding="latin-1").read()
    body = _function_body(src, "mcsJacs1")
    body = re.sub(r"//[^\n]*", "", body)
    prog = []
    for st in body.split(";"):
        st = " ".join(st.split())
        if not st:
            continue
        if st.startswith("jacs = "):
            continue  # zeros(): the output array starts zeroed
        m = re.fullmatch(r"const double (\w+) = (.+)", st)
        if m:
            prog.append((m.group(1), None, safe_compile_eval(_to_py(m.group(2)), m.group(1))))
            continue
        m = re.fullmatch(r"jacs\((\d), (\d+)\) = (.+)", st)
        if m:
            prog.append((None, (int(m.group(1)), int(m.group(2))),
                         safe_compile_eval(_to_py(m.group(3)), "jacs")))
            continue
        raise ValueError("unparsed statement: %s" % st[:120])
    return prog


def eval_mcsjacs1(prog, pt3, M_t, M_c, camModelData):
    env = {"math": math, "pt3": [float(v) for v in pt3], "M_t": [float(v) for v in M_t],
           "M_c": [float(v) for v in M_c], "camModelData": [float(v) for v in camModelData]}
    jacs = np.zeros((2, 32))
    for name, ij, code in prog:
        v = safe_eval(code, env)
        if name is not None:
            env[name] = float(v)
        else:
            jacs[ij] = float(v)
    return jacs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--n", type=int, default=96)
    ap.add_argument("--out", default=os.path.join(HERE, "mcsjacs1.npz"))
    a = ap.parse_args()
    from mcs_amd import ba
    prog = compile_mcsjacs1(a.ref)
    pr = ba.make_problem(n_local=6, n_fixed=2, n_points=400, target_edges=3000, seed=11)
    ne = len(pr["edge_pose"])
    sel = np.linspace(0, ne - 1, a.n).astype(np.int64)
    poses = pr["poses"][pr["edge_pose"][sel]]
    points = pr["points"][pr["edge_point"][sel]]
    mc = pr["mc"][pr["edge_cam"][sel]]
    cam = pr["cam"][pr["edge_cam"][sel]]
    meas = pr["edge_meas"][sel]
    jacs = np.stack([eval_mcsjacs1(prog, points[i], poses[i], mc[i], cam[i]) for i in range(a.n)])
    assert np.isfinite(jacs).all()
    np.savez_compressed(a.out, poses=poses, points=points, mc=mc, cam=cam, meas=meas, jacs=jacs,
                        n_statements=len(prog))
    print("wrote %s: %d samples, %d statements" % (a.out, a.n, len(prog)))


if __name__ == "__main__":
    main()
