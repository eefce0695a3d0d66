"""Generate tests/golden/g2o_schur.npz: the per-landmark block of g2o's BlockSolver::solve
(ThirdParty/g2o/g2o/core/block_solver.hpp:381-403) -- Dinv = D->inverse(), db = Dinv * db,
BDinv = (*Bi) * Dinv -- evaluated in the operation order of the reference's vendored Eigen
3.2.10.  No reference source is stored: the fixture is numbers only.

What is read from the reference text (and checked, so a different Eigen would stop the script):
  * Eigen/src/LU/Inverse.h:117-159 -- cofactor_3x3's expression, which cofactor lands in which
    entry of the result (compute_inverse_size3_helper), and the column-0 cofactors that form the
    determinant (compute_inverse<..., 3>);  the (row, col) <- cofactor(i, j) table is PARSED
    from the text and drives the evaluation below;
  * Eigen/src/Core/Redux.h:77-106 -- redux_novec_unroller's halving (the determinant's sum of
    three products: a 3-vector of doubles is not packet-aligned in Eigen 3.2,
    util/XprHelper.h:134-154, so the unvectorised unroller applies: c0 + (c1 + c2));
  * Eigen/src/Core/products/CoeffBasedProduct.h:240-258 -- the small fixed-size product's
    coefficient loop (k ascending, res = l0 r0 then res += lk rk);
  * Eigen/src/Core/util/Macros.h -- the version (3.2.10).
Python floats are IEEE doubles without FMA contraction: the text's order as written.  (The
reference builds with -march=native, so whether GCC contracts a * b + c into an FMA depends on
the build machine; like tests/golden/gen_mcsjacs1.py, this pins the text's order.)

    python tests/golden/gen_g2o_schur.py [--ref /root/reference]
"""
import argparse
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def read(ref, rel):
    with open(os.path.join(ref, rel)) as f:
        return f.read()


def parse_eigen(ref):
    eig = "ThirdParty/Eigen/Eigen/src/"
    mac = read(ref, eig + "Core/util/Macros.h")
    ver = tuple(int(re.search(r"#define EIGEN_%s_VERSION (\d+)" % k, mac).group(1))
                for k in ("WORLD", "MAJOR", "MINOR"))
    assert ver == (3, 2, 10), ver
    inv = read(ref, eig + "LU/Inverse.h")
    # cofactor_3x3<MatrixType, i, j>: i1 = (i+1)%3, ... ; m(i1,j1) m(i2,j2) - m(i1,j2) m(i2,j1)
    flat = " ".join(inv.split())
    for k, e in (("i1", "(i+1) % 3"), ("i2", "(i+2) % 3"), ("j1", "(j+1) % 3"), ("j2", "(j+2) % 3")):
        assert "%s = %s" % (k, e) in flat, k
    assert "return m.coeff(i1, j1) * m.coeff(i2, j2) - m.coeff(i1, j2) * m.coeff(i2, j1);" in flat
    helper = inv[inv.index("inline void compute_inverse_size3_helper"):]
    helper = helper[:helper.index("\n}\n")]
    table = {}
    assert "result.row(0) = cofactors_col0 * invdet;" in helper
    for r, c, i, j in re.findall(r"result\.coeffRef\((\d),(\d)\)\s*=\s*cofactor_3x3<MatrixType,(\d),(\d)>\(matrix\)\s*\*\s*invdet;", helper):
        table[(int(r), int(c))] = (int(i), int(j))
    run3 = inv[inv.index("struct compute_inverse<MatrixType, ResultType, 3>"):]
    run3 = run3[:run3.index("};")]
    col0 = {}
    for k, i, j in re.findall(r"cofactors_col0\.coeffRef\((\d)\)\s*=\s*cofactor_3x3<MatrixType,(\d),(\d)>\(matrix\);", run3):
        col0[int(k)] = (int(i), int(j))
    assert col0 == {0: (0, 0), 1: (1, 0), 2: (2, 0)}, col0
    assert "const Scalar det = (cofactors_col0.cwiseProduct(matrix.col(0))).sum();" in run3
    assert "const Scalar invdet = Scalar(1) / det;" in run3
    for k in range(3):   # result.row(0) = cofactors_col0 * invdet
        table[(0, k)] = col0[k]
    assert len(table) == 9, table
    red = read(ref, eig + "Core/Redux.h")
    assert "HalfLength = Length/2" in red
    assert ("return func(redux_novec_unroller<Func, Derived, Start, HalfLength>::run(mat,func),"
            in red)
    cbp = read(ref, eig + "Core/products/CoeffBasedProduct.h")
    assert "res += lhs.coeff(row, UnrollingIndex-1) * rhs.coeff(UnrollingIndex-1, col);" in cbp
    assert "res = lhs.coeff(row, 0) * rhs.coeff(0, col);" in cbp
    xpr = read(ref, eig + "Core/util/XprHelper.h")
    assert "(((MaxCols*MaxRows*int(sizeof(Scalar))) % 16) == 0)" in xpr   # 3 doubles: unaligned
    return table, col0


def redux_novec(vals):
    """redux_novec_unroller (Redux.h:77-106): func(first half, second half), halves Length/2."""
    if len(vals) == 1:
        return vals[0]
    h = len(vals) // 2
    return redux_novec(vals[:h]) + redux_novec(vals[h:])


def eigen_inverse3(m, table, col0):
    """compute_inverse<..., 3>::run on m (3x3 nested lists)."""
    def cof(i, j):
        i1, i2, j1, j2 = (i + 1) % 3, (i + 2) % 3, (j + 1) % 3, (j + 2) % 3
        return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1]
    c = [cof(*col0[k]) for k in range(3)]
    det = redux_novec([c[k] * m[k][0] for k in range(3)])   # cwiseProduct(col(0)).sum()
    invdet = 1.0 / det
    out = [[0.0] * 3 for _ in range(3)]
    for (r, cc), (i, j) in table.items():   # row 0: cofactors_col0 * invdet; others per the table
        out[r][cc] = cof(i, j) * invdet
    return out


def coeff_product(lhs, rhs):
    """CoeffBasedProduct (DefaultTraversal, complete unrolling): res = l0 r0; res += lk rk."""
    n, k, p = len(lhs), len(rhs), len(rhs[0])
    out = [[0.0] * p for _ in range(n)]
    for r in range(n):
        for c in range(p):
            res = lhs[r][0] * rhs[0][c]
            for t in range(1, k):
                res += lhs[r][t] * rhs[t][c]
            out[r][c] = res
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "g2o_schur.npz"))
    args = ap.parse_args()
    table, col0 = parse_eigen(args.ref)
    rng = np.random.default_rng(20261017)
    n = 1500
    H = rng.normal(size=(n, 3, 3))
    # mostly Hessian-like (A^T A + noise: near-symmetric, positive), some general and some
    # ill-conditioned blocks, magnitudes over many decades
    A = rng.normal(size=(n, 4, 3))
    spd = np.einsum("nki,nkj->nij", A, A)
    kind = rng.integers(0, 3, n)
    H = np.where(kind[:, None, None] == 0, spd, H)
    H = np.where(kind[:, None, None] == 1, spd + 1e-9 * rng.normal(size=(n, 3, 3)), H)
    scale = 10.0 ** rng.uniform(-6, 8, n)
    H = H * scale[:, None, None]
    ill = rng.random(n) < 0.1
    H[ill, 2] = H[ill, 1] * (1 + 1e-10)   # nearly singular rows
    lam = 1e-5 * np.abs(H).max() ** 0.5
    b = rng.normal(size=(n, 3)) * scale[:, None]
    hpl = rng.normal(size=(n, 6, 3)) * 10.0 ** rng.uniform(-3, 5, (n, 1, 1))
    Dinv = np.zeros((n, 3, 3))
    db = np.zeros((n, 3))
    Y = np.zeros((n, 6, 3))
    for t in range(n):
        D = [[float(H[t, i, j]) + (lam if i == j else 0.0) for j in range(3)] for i in range(3)]
        Di = eigen_inverse3(D, table, col0)
        Dinv[t] = Di
        db[t] = [r[0] for r in coeff_product(Di, [[float(v)] for v in b[t]])]   # db = Dinv * db
        Y[t] = coeff_product([list(map(float, row)) for row in hpl[t]], Di)     # BDinv = Bi * Dinv
    np.savez_compressed(args.out, H=H.reshape(n, 9), lam=np.float64(lam), b=b, hpl=hpl.reshape(n, 18),
                        Dinv=Dinv.reshape(n, 9), db=db, Y=Y.reshape(n, 18),
                        table=np.array([[r, c, i, j] for (r, c), (i, j) in sorted(table.items())], np.int32))
    print("wrote", args.out, n, "blocks; lambda", lam)


if __name__ == "__main__":
    main()
