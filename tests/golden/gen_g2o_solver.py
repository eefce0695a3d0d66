"""Generate tests/golden/g2o_solver.npz: the reference's own g2o solver control and robust
kernel, evaluated from its TEXT (no reference source is stored: the fixture is numbers only).

Translated from /root/reference/ThirdParty/g2o/g2o/core/ by tests/golden/cxx_subset.py (AST-
whitelisted, run without builtins):
  SparseOptimizer::optimize                        sparse_optimizer.cpp:354-419
  OptimizationAlgorithmLevenberg ctor, solve,      optimization_algorithm_levenberg.cpp:44-55,
    computeLambdaInit, computeScale                  61-164, 166-180, 182-189
  SparseOptimizerTerminateAction ctor (initializer list), operator(), setOptimizerStopFlag
                                                   sparse_optimizer_terminate_action.cpp:9-72
  RobustKernelHuber::setDelta / robustify          robust_kernel_impl.cpp:65-91, with the member
                                                   types of robust_kernel_impl.h (float dsqr)
The objects those functions call (the sparse optimizer's error evaluation and state stack, the
block solver) are scripted stand-ins: every LM trial's outcome (robust chi2 after the update,
the model-decrease terms that computeScale sums, whether the linear solve succeeded) comes from
a random scenario, exactly as the product's test hook mcs_ba_lm_replay takes it; the stand-ins
below cite the g2o lines whose behaviour they restate (push / pop / discardTop, terminate(),
postIteration, setForceStopFlag).  The product's replay must reproduce every lambda, nu,
accept / reject decision, nBad, stop flag and iteration count (tests/test_g2o_golden.py).

    python tests/golden/gen_g2o_solver.py [--ref /root/reference]
"""
import argparse
import math
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from cxx_subset import function_body, member_types, translate  # noqa: E402
from safe_exec import safe_exec  # noqa: E402

INT_MAX = 2 ** 31 - 1


def ctor_initializers(src, signature):
    """`Class::Class() : a(x), b(y) {` -> C++ assignment statements 'a = x;' ..."""
    i = src.index(signature) + len(signature)
    j = src.index("{", i)
    init = src[i:j]
    init = init[init.index(":") + 1:] if ":" in init else ""
    out, depth, cur = [], 0, ""
    for ch in init:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    out.append(cur)
    stmts = []
    for it in out:
        it = " ".join(it.split())
        m = re.fullmatch(r"(_\w+)\((.*)\)", it)
        if m:
            stmts.append("%s = %s;" % (m.group(1), m.group(2)))
    return "\n".join(stmts)


def _cpow(x, y):
    """C pow (glibc, through math.pow) with C's overflow result instead of Python's exception."""
    try:
        return math.pow(x, y)
    except OverflowError:
        odd = float(y).is_integer() and int(y) % 2 == 1
        return math.copysign(math.inf, x) if odd else math.inf


def _env():
    def _deref_set(cell, v):
        cell[0][cell[1]] = v

    def _ref(M, k):
        return [M, k]
    return {"_pow": _cpow, "_fabs": math.fabs, "_sqrt": math.sqrt, "_isfinite": math.isfinite,
            "_min": min, "_max": max, "_time": lambda: 0.0, "_nop": lambda *a: None,
            "_DBL_MAX": sys.float_info.max, "_INT_MAX": INT_MAX, "_f32": lambda x: float(np.float32(x)),
            "_ref": _ref, "_deref_set": _deref_set, "_deref": lambda c: c[0][c[1]],
            "range": range, "len": len, "cerr": None, "endl": None}


class RefCode:
    """The translated reference functions."""

    def __init__(self, ref):
        core = os.path.join(ref, "ThirdParty", "g2o", "g2o", "core")
        env = _env()
        self.n_statements = 0

        def add(path, sig, name, params, members=(), float_members=(), body=None):
            src = open(os.path.join(core, path), encoding="latin-1").read()
            b = body if body is not None else function_body(src, sig)
            py = translate(b, name, params, members=members, float_members=float_members)
            self.n_statements += b.count(";")
            g = safe_exec(py, env, "<ref:%s %s>" % (path, name))
            return g[name]

        lm = "optimization_algorithm_levenberg.cpp"
        self.lm_ctor = add(lm, "OptimizationAlgorithmLevenberg::OptimizationAlgorithmLevenberg(Solver* solver)",
                           "lm_ctor", ["solver"])
        self.lm_solve = add(lm, "OptimizationAlgorithm::SolverResult OptimizationAlgorithmLevenberg::solve(",
                            "lm_solve", ["iteration", "online"])
        self.lm_lambda_init = add(lm, "double OptimizationAlgorithmLevenberg::computeLambdaInit()",
                                  "lm_lambda_init", [])
        self.lm_scale = add(lm, "double OptimizationAlgorithmLevenberg::computeScale()", "lm_scale", [])
        self.opt_optimize = add("sparse_optimizer.cpp", "int SparseOptimizer::optimize(int iterations, bool online)",
                                "opt_optimize", ["iterations", "online"])
        ta = "sparse_optimizer_terminate_action.cpp"
        ta_src = open(os.path.join(core, ta), encoding="latin-1").read()
        init = ctor_initializers(ta_src, "SparseOptimizerTerminateAction::SparseOptimizerTerminateAction()")
        init = init.replace("std::numeric_limits<int>::max()", "_INT_MAX")
        self.term_ctor = add(ta, None, "term_ctor", [], body=init)
        self.term_action = add(ta, "HyperGraphAction* SparseOptimizerTerminateAction::operator()(",
                               "term_action", ["graph", "parameters"])
        self.term_set_stop = add(ta, "void SparseOptimizerTerminateAction::setOptimizerStopFlag(",
                                 "term_set_stop", ["optimizer", "stop"])
        rk = "robust_kernel_impl.cpp"
        mt = member_types(open(os.path.join(core, "robust_kernel_impl.h"), encoding="latin-1").read(),
                          "RobustKernelHuber")
        fl = [k for k, v in mt.items() if v == "float"]
        self.huber_member_types = mt
        self.huber_set_delta = add(rk, "void RobustKernelHuber::setDelta(double delta)", "huber_set_delta",
                                   ["delta"], members=list(mt) + ["_delta"], float_members=fl)
        self.huber_robustify = add(rk, "void RobustKernelHuber::robustify(double e, Eigen::Vector3d& rho)",
                                   "huber_robustify", ["e", "rho"], members=list(mt) + ["_delta"])


class Scenario:
    """Stand-ins for the objects the translated code calls, driven by scripted trials."""

    def __init__(self, R, chi0, maxdiag_pt, maxdiag_pose, trials, max_iterations,
                 gain_threshold, terminate_max_iter):
        self.R, self.trials, self.t = R, trials, 0
        self.rec = []
        self.state_chi = chi0            # robust chi2 of the current estimate
        self.stack = []
        self.force = None                # SparseOptimizer::_forceStopFlag (sparse_optimizer.h:290)
        # OptimizationAlgorithmLevenberg members (ctor) + the objects it calls
        L = {"_properties": {"makeProperty": lambda name, default: {"value": (lambda d=default: d)}}}
        R.lm_ctor(L, None)
        opt = {
            # computeActiveErrors / activeRobustChi2: the chi2 of the current estimate
            "computeActiveErrors": lambda: None,
            "activeRobustChi2": lambda: self.state_chi,
            # push / pop / discardTop: the estimate stack (optimizable_graph.cpp push/pop/discardTop)
            "push": self._push, "pop": self._pop, "discardTop": self._discard,
            "update": self._update,
            # terminate() (sparse_optimizer.h:188)
            "terminate": lambda: bool(self.force[0][self.force[1]]) if self.force else False,
            "forceStopFlag": lambda: self.force,
            "setForceStopFlag": self._set_force,
            "indexMapping": lambda: {"size": lambda: 2,
                                     0: {"dimension": lambda: 1, "hessian": lambda i, j: maxdiag_pose},
                                     1: {"dimension": lambda: 1, "hessian": lambda i, j: maxdiag_pt}},
        }
        solver = {"buildStructure": lambda: True, "buildSystem": lambda: None,
                  "setLambda": self._set_lambda, "solve": self._solve, "restoreDiagonal": lambda: None,
                  "x": lambda: None}
        L["_optimizer"] = opt
        L["_solver"] = solver
        L["computeLambdaInit"] = lambda: R.lm_lambda_init(L)
        # computeScale sums x_j (lambda x_j + b_j) over the update vector (:182-189); the
        # product sums the pose and the point blocks separately and adds them, which is the
        # scripted value here (tests/golden: lm_scale_case pins the formula itself)
        L["computeScale"] = lambda: self.cur[2] + self.cur[1]
        self.L = L
        # the terminate action (cOptimizer: gain 1e-6, max 15, src/cOptimizer.cpp:577-581)
        TA = {}
        R.term_ctor(TA)
        TA["_gainThreshold"] = gain_threshold
        TA["_maxIterations"] = terminate_max_iter
        TA["setOptimizerStopFlag"] = lambda o, s: R.term_set_stop(TA, o, s)
        self.TA = TA
        # SparseOptimizer members used by optimize()
        S = {"_ivMap": {"size": lambda: 1}, "_algorithm": {"init": lambda online: True,
                                                           "solve": lambda i, online: R.lm_solve(L, i, online),
                                                           "printVerbose": lambda *a: None},
             "_batchStatistics": {"clear": lambda: None, "resize": lambda n: None},
             "_computeBatchStatistics": False, "verbose": lambda: False,
             "terminate": opt["terminate"], "preIteration": lambda i: None,
             # postIteration (optimizable_graph.cpp:784-793): every post-iteration action
             "postIteration": lambda i: R.term_action(TA, opt, {"iteration": i}),
             "computeActiveErrors": lambda: None, "activeRobustChi2": opt["activeRobustChi2"]}
        self.S = S
        self.max_iterations = max_iterations
        self.iter_no = 0

    def _set_force(self, cell):
        self.force = cell

    def _push(self):
        self.stack.append(self.state_chi)

    def _pop(self):
        self.state_chi = self.stack.pop()
        self._record(accepted=0)

    def _discard(self):
        self.stack.pop()
        self._record(accepted=1)

    def _set_lambda(self, lam, backup):
        if self.t >= len(self.trials):
            raise RuntimeError("scenario ran out of scripted trials")
        self.cur = self.trials[self.t]
        self.lam_used = lam

    def _solve(self):
        return self.cur[3] == 0.0

    def _update(self, x):
        self.state_chi = self.cur[0]

    def _record(self, accepted):
        L = self.L
        self.rec.append([self.lam_used, L["_currentLambda"], L["_ni"], accepted])
        self.t += 1

    def run(self):
        iters = self.R.opt_optimize(self.S, self.max_iterations, False)
        stop = bool(self.force[0][self.force[1]]) if self.force else False
        return iters, stop


def scenario_trials(rng, kind):
    """Scripted trial outcomes {chi2, point decrease, pose decrease, failed}."""
    n = 200
    out = np.zeros((n, 4))
    chi = 1e4 * rng.uniform(0.5, 2.0)
    for t in range(n):
        r = rng.random()
        if kind == "converge":
            step = chi * (rng.uniform(0.05, 0.5) if t < 8 else rng.uniform(1e-9, 1e-4))
        elif kind == "stall":
            step = chi * rng.uniform(0, 2e-4)
        else:
            step = chi * rng.uniform(-0.3, 0.4)
        if r < 0.15:
            step = -abs(step) - chi * 0.01          # worse: reject
        elif r < 0.2:
            step = 0.0                              # no change: rho == 0
        trial = chi - step
        failed = 1.0 if rng.random() < 0.05 else 0.0
        sp = abs(step) * rng.uniform(0.2, 1.5) * (1 if rng.random() > 0.03 else -1)
        sl = abs(step) * rng.uniform(0.0, 0.5)
        out[t] = [trial, sl, sp, failed]
        if step > 0 and not failed:
            chi = trial
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "g2o_solver.npz"))
    a = ap.parse_args()
    R = RefCode(a.ref)
    rng = np.random.default_rng(2026)
    kinds = ["converge", "stall", "wild"]
    sc_in, sc_trials, sc_out, sc_meta = [], [], [], []
    for s in range(60):
        kind = kinds[s % 3]
        trials = scenario_trials(rng, kind)
        # scenario-specific edge cases
        if s == 3:
            trials[:12, 0] = trials[0, 0] * 2       # ten failures in a row: max trials
            trials[:12, 3] = 0
        if s == 4:
            trials[:, 3] = 1.0                       # the solve always fails
        max_it = [10, 15, 5, 1, 10][s % 5]
        chi0 = float(trials[0, 0] * rng.uniform(1.0, 3.0))
        mp, mq = float(rng.uniform(1, 1e6)), float(rng.uniform(1, 1e6))
        sim = Scenario(R, chi0, mp, mq, trials, max_it, 1e-6, 15)
        iters, stop = sim.run()
        rec = np.array(sim.rec) if sim.rec else np.zeros((0, 4))
        sc_in.append([chi0, mp, mq])
        sc_trials.append(trials)
        out = np.zeros((200, 4))
        out[:len(rec)] = rec
        sc_out.append(out)
        sc_meta.append([len(rec), iters, int(stop), max_it])
    # Huber: deltas the reference uses and squared errors around delta^2 (double and float)
    deltas = [math.sqrt(5.991), 1.345 * 2, 1.345, 1.345 * 1.5, 0.7]
    hub_e, hub_d, hub_r0, hub_r1 = [], [], [], []
    for d in deltas:
        d2 = d * d
        f2 = float(np.float32(d2))
        es = [0.0, 1e-9, 0.5 * d2, d2, f2, np.nextafter(f2, 0), np.nextafter(f2, np.inf),
              np.nextafter(d2, 0), np.nextafter(d2, np.inf), 2 * d2, 10 * d2, 1e6]
        es += list(rng.uniform(0, 4 * d2, 40)) + list(10 ** rng.uniform(-6, 6, 40))
        K = {}
        R.huber_set_delta(K, d)
        for e in es:
            rho = [0.0, 0.0, 0.0]
            R.huber_robustify(K, float(e), rho)
            hub_e.append(float(e))
            hub_d.append(d)
            hub_r0.append(rho[0])
            hub_r1.append(rho[1])
    # computeScale's own formula on a vector (the product splits it into pose / point blocks)
    x = rng.normal(size=40)
    b = rng.normal(size=40)
    lam = 3.7
    L = {"_currentLambda": lam, "_solver": {"vectorSize": lambda: 40, "x": lambda: x, "b": lambda: b}}
    scale = R.lm_scale(L)
    np.savez_compressed(a.out, lm_in=np.array(sc_in), lm_trials=np.array(sc_trials), lm_out=np.array(sc_out),
                        lm_meta=np.array(sc_meta, np.int64), huber_e=np.array(hub_e), huber_delta=np.array(hub_d),
                        huber_rho0=np.array(hub_r0), huber_rho1=np.array(hub_r1),
                        scale_x=x, scale_b=b, scale_lambda=lam, scale_value=scale,
                        huber_dsqr_is_float=int(R.huber_member_types.get("dsqr") == "float"),
                        n_statements=R.n_statements)
    print("wrote %s: %d scenarios (%d trials replayed), %d Huber evaluations, %d statements" % (
        a.out, len(sc_in), int(sum(m[0] for m in sc_meta)), len(hub_e), R.n_statements))


if __name__ == "__main__":
    main()
