"""Generate golden vectors for the oracle — run in the build container only.

Sources:
  * the reference's vendored Sophus sympy package (Thirdparty/Sophus/py/sophus/se3.py:8-80,
    so3.py:8-30), evaluated with 30-digit precision, for SE3/SO3 exp and log at the tangents of
    the Sophus C++ tests (Thirdparty/Sophus/test/core/test_se3.cpp:33-50) plus seeded random ones;
  * the same package's symbolic derivatives of exp (Se3.calc_Dxi_exp_x_matrix, se3.py:153-157):
    T(x)^-1 dT/dx_i = hat(Jr(x) e_i) gives SE(3)'s right Jacobian column by column, the quantity
    Pose3utils' RightJacobianPose3 / RightJacobianPose3Inv (src/Pose3utils.cc:32-46) compute in closed
    form, at the same tangents plus small-angle ones (both branches of LeftJacobianPose3Q, :11 and :17,
    and LeftJacobianRot3's identity branch, :50);
  * an independent numpy/mpmath-free restatement of GaussianProcess::QueryPose's 12x12 products
    (src/GaussianProcess.cc:5-42), exercising the four-scalar identity of SURVEY.md §0.4.

The reference tree is NOT available on the GPU box; the outputs are committed as
tests/golden/sophus_golden.json and tests/golden/gp_golden.json (data only).

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SOPHUS_PY = "/root/reference/Thirdparty/Sophus/py"


def sophus_vectors():
    sys.path.insert(0, SOPHUS_PY)
    import sympy
    import sophus

    tangents = [
        [1, 0, 0, 0, 0, 1e-5],          # rotZ(1e-5)-like small angle
        [0, 1, 0, 1, 0, 0],
        [-1, 1, 0, 0, 0, 1],
        [20, -1, 0, -1, 1, 0],
        [30, 5, -1, 20, -1, 0],
        [1e-8, 0, 0, 0, 0, 1e-4],
        [0.3, -0.2, 0.1, 3.14159, 0, 0],  # near rotX(pi)
    ]
    rng = np.random.default_rng(20250912)
    for _ in range(8):
        v = rng.normal(0, 1, 6)
        v[3:] *= 0.5
        tangents.append(v.tolist())
    out = []
    for v in tangents:
        vs = sympy.Matrix([sympy.Float(x, 30) for x in v])
        T = sophus.Se3.exp(vs)
        q = T.so3.q
        qv = [float(sympy.N(q.vec[i], 30)) for i in range(3)] + [float(sympy.N(q.real, 30))]
        t = [float(sympy.N(T.t[i], 30)) for i in range(3)]
        xi = T.log()
        out.append({"xi": [float(x) for x in v], "q": qv, "t": t, "log": [float(sympy.N(xi[i], 30)) for i in range(6)]})
    so3 = []
    for v in ([0.1, -0.2, 0.3], [1e-4, 0, 0], [2.0, 1.0, -0.5], [0, 0, 3.0]):
        vs = sympy.Matrix([sympy.Float(x, 30) for x in v])
        R = sophus.So3.exp(vs)
        q = [float(sympy.N(R.q.vec[i], 30)) for i in range(3)] + [float(sympy.N(R.q.real, 30))]
        w = R.log()
        so3.append({"w": v, "q": q, "log": [float(sympy.N(w[i], 30)) for i in range(3)]})
    return {"source": "Thirdparty/Sophus/py/sophus (sympy, 30 digits)", "se3": out, "so3": so3}


def se3_jacobian_vectors():
    sys.path.insert(0, SOPHUS_PY)
    import sympy
    import sophus

    x = sympy.Matrix(sympy.symbols("x0:6", real=True))
    Tm = sophus.Se3.exp(x).matrix()
    D = [sophus.Se3.calc_Dxi_exp_x_matrix(x, i) for i in range(6)]
    tangents = [
        [1, 0, 0, 0, 0, 1e-5],
        [0, 1, 0, 1, 0, 0],
        [-1, 1, 0, 0, 0, 1],
        [20, -1, 0, -1, 1, 0],
        [30, 5, -1, 20, -1, 0],
        [0.3, -0.2, 0.1, 3.14159, 0, 0],
        [0.5, -0.3, 0.2, 2e-6, -1e-6, 3e-6],     # |w| < 1e-5: LeftJacobianPose3Q's series branch
        [0.2, 0.1, -0.3, 1e-9, 0, 0],            # |w|^2 <= eps: LeftJacobianRot3's identity branch
        [-0.4, 0.9, 0.05, 0.02, -0.01, 0.03],
    ]
    rng = np.random.default_rng(777)
    for _ in range(4):
        v = rng.normal(0, 1, 6)
        v[3:] *= 0.6
        tangents.append(v.tolist())
    out = []
    for v in tangents:
        sub = {x[i]: sympy.Float(repr(float(v[i])), 80) for i in range(6)}
        T = Tm.subs(sub).evalf(80)
        Ti = T.inv()
        J = []
        for i in range(6):
            M = (Ti * D[i].subs(sub).evalf(80)).evalf(80)
            col = sophus.Se3.vee(M)
            J.append([float(sympy.N(col[r], 30)) for r in range(6)])
        Jr = np.array(J).T   # column i = vee(T^-1 dT/dx_i)
        out.append({"xi": [float(t) for t in v], "Jr": Jr.ravel().tolist()})
    return {"source": "Thirdparty/Sophus/py/sophus se3.py Se3.calc_Dxi_exp_x_matrix (sympy, 80 digits): "
                      "Jr(x) e_i = vee(exp(x)^-1 d exp(x) / dx_i)", "se3_right_jacobian": out}


def gp_vectors():
    """QueryPose's Pt1/At1 from explicit 12x12 products with a dense SPD Qc (numpy)."""
    rng = np.random.default_rng(7)
    cases = []
    for trial in range(6):
        A = rng.normal(size=(6, 6))
        Qc = A @ A.T + 0.5 * np.eye(6) if trial % 2 else np.diag([0.02, 0.02, 0.02, 0.002, 0.002, 0.002])
        t1 = 100.0 + trial * 0.1
        T = 0.1 if trial < 4 else 0.05
        t2 = t1 + T
        t = t1 + rng.uniform(0.05, 0.95) * T
        I6 = np.eye(6)

        def Qi(dt):
            return np.block([[dt ** 3 / 3 * Qc, dt ** 2 / 2 * Qc], [dt ** 2 / 2 * Qc, dt * Qc]])

        def QiInv(dt):
            Qi_ = np.linalg.inv(Qc)
            return np.block([[12 / dt ** 3 * Qi_, -6 / dt ** 2 * Qi_], [-6 / dt ** 2 * Qi_, 4 / dt * Qi_]])

        def Phi(a, b):
            return np.block([[I6, (b - a) * I6], [np.zeros((6, 6)), I6]])

        Pt = Qi(t - t1) @ Phi(t, t2).T @ QiInv(t2 - t1)
        At = Phi(t1, t) - Pt @ Phi(t1, t2)
        cases.append({"qc": Qc.ravel().tolist(), "t1": t1, "t2": t2, "t": t,
                      "Pt1": Pt[:6].ravel().tolist(), "At1": At[:6].ravel().tolist()})
    return {"source": "numpy restatement of GaussianProcess::QueryPose 12x12 products", "cases": cases}


if __name__ == "__main__":
    with open(os.path.join(HERE, "sophus_golden.json"), "w") as f:
        json.dump(sophus_vectors(), f, indent=1)
    with open(os.path.join(HERE, "gp_golden.json"), "w") as f:
        json.dump(gp_vectors(), f, indent=1)
    with open(os.path.join(HERE, "se3_jacobian_golden.json"), "w") as f:
        json.dump(se3_jacobian_vectors(), f, indent=1)
    print("wrote", os.listdir(HERE))
