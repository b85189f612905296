"""Host-side mirror of the reference's QPSolver class (include/QPSolver.h:10-56), running
every numerical step on the GPU through the single-instance C ABI.

Same method names, argument meaning and behaviour as the reference:
  QPSolver(Ts, N, Ac, Bc, Q, R, P, x_min, x_max, u_min, u_max)   src/QPSolver.cpp:3-19
  discretizeSystem()                                               src/QPSolver.cpp:21-29
  buildQPParams(xi0, xi_ref) -> (H, f, A_eq, b_eq, lb, ub, A_ineq, lbA_ineq, ubA_ineq)
                                                                   src/QPSolver.cpp:31-81
  solveQP(H, f, A_total, lb, ub, lbA_total, ubA_total) -> (True, U_opt)
                                                                   src/QPSolver.cpp:83-106
  updateState(u), getState()                                       src/QPSolver.cpp:108-116
Differences, all deliberate:
  * solveQP returns True like the reference (status printed, not raised: :98-105), and keeps
    the solver status in ``last_status``.  When the harness-stacked problem [A_eq; A_ineq]
    is infeasible (it always is), the equality block is dropped and the
    corrected QP is solved (``corrected = True``) instead of leaving U_opt undefined.
  * A_total is read column-major (what Eigen hands out), i.e. as intended, not scrambled.
  * ``xi`` starts at zero exactly like the reference (src/QPSolver.cpp:12).
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from ._lib import A_COLMAJOR, MPCQP_OK, STATUS, check, lib


def _f(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, order="F"))


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def discretize(Ac, Bc, Ts, quadrature: bool = False):
    """QPSolver::discretizeSystem (src/QPSolver.cpp:21-29); quadrature=True gives
    linear_mpc_example's integrated Bd (src/linear_mpc_example.cpp:35-46)."""
    Ac = np.asarray(Ac, float)
    Bc = np.asarray(Bc, float)
    nx, nu = Bc.shape
    Ad = np.zeros(nx * nx)
    Bd = np.zeros(nx * nu)
    fAc, fBc = _f(Ac), _f(Bc)  # keep the buffers alive across the call
    fn = "mpcqp_discretize_quadrature" if quadrature else "mpcqp_discretize"
    check(fn, getattr(lib(), fn)(nx, nu, float(Ts), _p(fAc), _p(fBc), _p(Ad), _p(Bd)))
    return Ad.reshape(nx, nx, order="F"), Bd.reshape(nx, nu, order="F")


def build_qp(Ad, Bd, Q, R, P, x_min, x_max, u_min, u_max, xi0, xi_ref, N):
    Ad = np.asarray(Ad, float)
    Bd = np.asarray(Bd, float)
    nx, nu = Bd.shape
    nV, NE, NI = nu * N, nx * N, 2 * nx * N
    o = dict(H=np.zeros(nV * nV), f=np.zeros(nV), A_eq=np.zeros(NE * nV), b_eq=np.zeros(NE),
             lb=np.zeros(nV), ub=np.zeros(nV), A_ineq=np.zeros(NI * nV), lbA=np.zeros(NI),
             ubA=np.zeros(NI))
    keep = [_f(a) for a in (Ad, Bd, Q, R, P, x_min, x_max, xi0, xi_ref)]
    check("mpcqp_build_qp", lib().mpcqp_build_qp(
        nx, nu, N, *[_p(k) for k in keep[:7]], float(u_min), float(u_max), _p(keep[7]),
        _p(keep[8]), _p(o["H"]), _p(o["f"]), _p(o["A_eq"]), _p(o["b_eq"]), _p(o["lb"]),
        _p(o["ub"]), _p(o["A_ineq"]), _p(o["lbA"]), _p(o["ubA"])))
    o["H"] = o["H"].reshape(nV, nV, order="F")
    o["A_eq"] = o["A_eq"].reshape(NE, nV, order="F")
    o["A_ineq"] = o["A_ineq"].reshape(NI, nV, order="F")
    return o


def solve_dense(H, f, A=None, lb=None, ub=None, lbA=None, ubA=None, n_wsr=0, want_y=False):
    """-> (status, x, cost, iters, y).  A is a 2-D array (passed column-major)."""
    H = np.asarray(H, float)
    nV = H.shape[0]
    nC = 0 if A is None else np.asarray(A).shape[0]
    x = np.zeros(nV)
    y = np.zeros(nV + nC) if want_y else None
    cost = C.c_double(0.0)
    nwsr = C.c_int(int(n_wsr))
    keep = dict(H=_f(H), f=_f(f), A=None if A is None else _f(A),
                lb=None if lb is None else _f(lb), ub=None if ub is None else _f(ub),
                lbA=None if lbA is None else _f(lbA), ubA=None if ubA is None else _f(ubA))
    st = lib().mpcqp_solve_dense(nV, nC, _p(keep["H"]), _p(keep["f"]), _p(keep["A"]), A_COLMAJOR,
                                 _p(keep["lb"]), _p(keep["ub"]), _p(keep["lbA"]), _p(keep["ubA"]),
                                 C.byref(nwsr), _p(x), _p(y), C.byref(cost))
    if st in (5, 6, 7):
        check("mpcqp_solve_dense", st)
    return st, x, cost.value, nwsr.value, y


class QPSolver:
    """Reference-compatible QPSolver (include/QPSolver.h:10-56) over the GPU C ABI."""

    def __init__(self, Ts, N, Ac, Bc, Q, R, P, x_min, x_max, u_min, u_max, verbose=False,
                 quadrature=False):
        self.Ts, self.N = float(Ts), int(N)
        self.Ac, self.Bc = np.asarray(Ac, float), np.asarray(Bc, float)
        self.Q, self.R, self.P = (np.asarray(a, float) for a in (Q, R, P))
        self.x_min, self.x_max = np.asarray(x_min, float), np.asarray(x_max, float)
        self.u_min, self.u_max = float(u_min), float(u_max)
        self.NX, self.NU = self.Ac.shape[0], self.Bc.shape[1]
        self.xi = np.zeros(self.NX)  # src/QPSolver.cpp:12 (not the harness's x0)
        self.verbose = verbose
        self.last_status = MPCQP_OK
        self.last_iters = 0
        self.corrected = False
        # quadrature=True: linear_mpc_example's discretisation (src/linear_mpc_example.cpp:35-46)
        self.quadrature = bool(quadrature)
        self.discretizeSystem()

    def discretizeSystem(self):
        self.Ad, self.Bd = discretize(self.Ac, self.Bc, self.Ts, quadrature=self.quadrature)

    def setState(self, xi):
        """mpc_test carries its own xi from (2,0,0,0) (src/linear_mpc_example.cpp:124,182); the
        reference QPSolver has no setter (its xi starts at zero, src/QPSolver.cpp:12)"""
        self.xi = np.asarray(xi, float).reshape(self.NX).copy()

    def buildQPParams(self, xi0, xi_ref):
        o = build_qp(self.Ad, self.Bd, self.Q, self.R, self.P, self.x_min, self.x_max,
                     self.u_min, self.u_max, xi0, xi_ref, self.N)
        return (o["H"], o["f"], o["A_eq"], o["b_eq"], o["lb"], o["ub"], o["A_ineq"], o["lbA"],
                o["ubA"])

    def solveQP(self, H, f, A_total, lb, ub, lbA_total, ubA_total):
        st, x, _, it, _ = solve_dense(H, f, A_total, lb, ub, lbA_total, ubA_total, n_wsr=50000)
        self.corrected = False
        neq = self.NX * self.N
        if st == 2 and np.asarray(A_total).shape[0] == neq + 2 * self.NX * self.N:
            # the harness's [A_eq; A_ineq] stack is infeasible by construction: solve the
            # corrected QP (bounds + A_ineq) -- SURVEY.md 0.5
            st, x, _, it, _ = solve_dense(H, f, np.asarray(A_total)[neq:], lb, ub,
                                          np.asarray(lbA_total)[neq:], np.asarray(ubA_total)[neq:],
                                          n_wsr=50000)
            self.corrected = True
        self.last_status, self.last_iters = st, it
        if st != MPCQP_OK:
            print(f"QP solve failed, status: {STATUS.get(st, st)}", file=sys.stderr)
        return True, x.reshape(self.NU, self.N, order="F")

    def updateState(self, u):
        x = np.ascontiguousarray(self.xi, dtype=np.float64).copy()
        uu = np.ascontiguousarray(np.asarray(u, float).reshape(-1))
        fAd, fBd = _f(self.Ad), _f(self.Bd)
        check("mpcqp_plant_step", lib().mpcqp_plant_step(
            self.NX, self.NU, _p(fAd), _p(fBd), _p(x), _p(uu)))
        self.xi = x
        if self.verbose:
            print(" ".join(f"{v:g}" for v in self.xi))

    def getState(self):
        if self.verbose:
            print(" ".join(f"{v:g}" for v in self.xi))
        return self.xi.copy()
