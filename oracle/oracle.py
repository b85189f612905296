"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY.  Loaded by tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg as the checker / baseline; the product path (libmpcqp.so over HIP)
never imports this module.  Parity status: unpinned w.r.t. the reference binary (see
mpcqp_oracle.h); cross-checked against tests/golden/ (numpy/scipy restatement + SURVEY
section 8c known-answer values).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_up = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")


class Friction(C.Structure):
    _fields_ = [("enabled", C.c_int), ("nu", C.c_int), ("N", C.c_int), ("nfeet", C.c_int),
                ("mu", C.c_double), ("contact_mask", C.c_uint64), ("elide_fz", C.c_int)]


class SrbmCfg(C.Structure):
    _fields_ = [("nx", C.c_int), ("nu", C.c_int), ("N", C.c_int), ("model", C.c_int),
                ("friction", C.c_int), ("Ts", C.c_double), ("mass", C.c_double),
                ("mu", C.c_double), ("Ib", C.c_double * 9), ("fz_min", C.c_double),
                ("fz_max", C.c_double), ("fxy_max", C.c_double), ("u_min", C.c_double),
                ("u_max", C.c_double), ("Q", C.c_void_p), ("R", C.c_void_p),
                ("P", C.c_void_p), ("max_iter", C.c_int), ("crash_kmax", C.c_int),
                ("crash_pmax", C.c_int), ("crash_kmax_wg", C.c_int), ("crash_pmax_wg", C.c_int),
                ("crash_split", C.c_int), ("elide_fz", C.c_int)]


def crash_params(p):
    """p["crash"]: the library's (kmax, pmax, kmax_wg, pmax_wg, split) (BatchEngine.crash), or a
    (kmax, pmax) pair for every instance; absent: the plain dual loop"""
    c = tuple(p.get("crash", (0, 0)))
    if len(c) == 2:
        return c + (c[0], c[1], 1 << 30)
    return c


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class DenseCfg(C.Structure):
    _fields_ = [("nx", C.c_int), ("nu", C.c_int), ("N", C.c_int), ("Ts", C.c_double),
                ("Q", C.c_void_p), ("R", C.c_void_p), ("P", C.c_void_p), ("u_min", C.c_double),
                ("u_max", C.c_double), ("max_iter", C.c_int), ("crash_kmax", C.c_int),
                ("crash_pmax", C.c_int)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.orc_expm.argtypes = [C.c_int, _dp, _dp]
        L.orc_matpow.argtypes = [C.c_int, _dp, C.c_int, _dp]
        L.orc_discretize.argtypes = [C.c_int, C.c_int, C.c_double, _dp, _dp, _dp, _dp]
        L.orc_discretize_quadrature.argtypes = [C.c_int, C.c_int, C.c_double, _dp, _dp, _dp, _dp]
        L.orc_build_qp.argtypes = [C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _dp,
                                   C.c_double, C.c_double, _dp, _dp] + [_dp] * 9
        L.orc_solve_qp.argtypes = [C.c_int, _dp, _dp, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, _dp,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_model_literal.argtypes = [C.c_double] * 4 + [_dp, _dp]
        L.orc_model_srbm.argtypes = [_dp, C.c_double, _dp, _dp, _dp]
        L.orc_gait_contact_mask.argtypes = [C.c_int, C.c_double, C.c_double, C.c_float, C.c_float]
        L.orc_gait_contact_mask.restype = C.c_uint64
        L.orc_srbm_batch.argtypes = [C.POINTER(SrbmCfg), C.c_int, _dp, _dp, _dp, _up, _dp, _dp,
                                     _ip, _ip, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.orc_dense_batch.argtypes = [C.POINTER(DenseCfg), C.c_int, _dp, _dp, _dp, _dp, _dp, _ip,
                                      _ip, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_srbm_bounds.argtypes = [C.POINTER(SrbmCfg), C.c_uint64, _dp, _dp]
        L.orc_srbm_plant.argtypes = [C.POINTER(SrbmCfg), _dp, _dp, _dp]
        L.orc_fk_feet.argtypes = [_dp, _dp, _dp]
        L.orc_kf_update.argtypes = [C.c_double, _dp, _dp, _dp, _dp, C.c_void_p, _dp, _dp]
        _lib = L
    return _lib


def _f(a):
    """column-major (Fortran) flatten to a C-contiguous float64 buffer"""
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, order="F"))


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def expm(A):
    A = np.asarray(A, float)
    n = A.shape[0]
    E = np.zeros(n * n)
    lib().orc_expm(n, _f(A), E)
    return E.reshape(n, n, order="F")


def matpow(A, p):
    A = np.asarray(A, float)
    n = A.shape[0]
    out = np.zeros(n * n)
    lib().orc_matpow(n, _f(A), int(p), out)
    return out.reshape(n, n, order="F")


def discretize(Ac, Bc, Ts, quadrature=False):
    Ac = np.asarray(Ac, float)
    Bc = np.asarray(Bc, float)
    nx, nu = Bc.shape
    Ad = np.zeros(nx * nx)
    Bd = np.zeros(nx * nu)
    fn = lib().orc_discretize_quadrature if quadrature else lib().orc_discretize
    rc = fn(nx, nu, float(Ts), _f(Ac), _f(Bc), Ad, Bd)
    assert rc == 0
    return Ad.reshape(nx, nx, order="F"), Bd.reshape(nx, nu, order="F")


def build_qp(Ad, Bd, Q, R, P, x_min, x_max, u_min, u_max, xi0, xi_ref, N):
    """QPSolver::buildQPParams restated; returns dict of the reference's outputs."""
    Ad = np.asarray(Ad, float)
    Bd = np.asarray(Bd, float)
    nx, nu = Bd.shape
    nV = nu * N
    out = dict(H=np.zeros(nV * nV), f=np.zeros(nV), A_eq=np.zeros(nx * N * nV),
               b_eq=np.zeros(nx * N), lb=np.zeros(nV), ub=np.zeros(nV),
               A_ineq=np.zeros(2 * nx * N * nV), lbA=np.zeros(2 * nx * N),
               ubA=np.zeros(2 * nx * N))
    rc = lib().orc_build_qp(nx, nu, N, _f(Ad), _f(Bd), _f(Q), _f(R), _f(P), _f(x_min),
                            _f(x_max), float(u_min), float(u_max), _f(xi0), _f(xi_ref),
                            out["H"], out["f"], out["A_eq"], out["b_eq"], out["lb"], out["ub"],
                            out["A_ineq"], out["lbA"], out["ubA"])
    assert rc == 0
    out["H"] = out["H"].reshape(nV, nV, order="F")
    out["A_eq"] = out["A_eq"].reshape(nx * N, nV, order="F")
    out["A_ineq"] = out["A_ineq"].reshape(2 * nx * N, nV, order="F")
    return out


def solve_qp(H, f, lb=None, ub=None, A=None, lbA=None, ubA=None, friction=None, max_iter=0):
    """Corrected dense QP (Goldfarb-Idnani).  A given as a 2-D numpy array (row i = constraint i).
    Returns (status, x, cost, iters, lam_bounds, lam_rows)."""
    H = np.asarray(H, float)
    n = H.shape[0]
    mA = 0 if A is None else int(np.asarray(A).shape[0])
    Arm = None if A is None else np.ascontiguousarray(np.asarray(A, float))
    lb_ = None if lb is None else np.ascontiguousarray(np.asarray(lb, float))
    ub_ = None if ub is None else np.ascontiguousarray(np.asarray(ub, float))
    lbA_ = None if lbA is None else np.ascontiguousarray(np.asarray(lbA, float))
    ubA_ = None if ubA is None else np.ascontiguousarray(np.asarray(ubA, float))
    x = np.zeros(n)
    cost = C.c_double(0)
    iters = C.c_int(0)
    lamb = np.zeros(n)
    lamr = np.zeros(max(mA, 1))
    fr = None
    if friction is not None:
        fr = Friction(1, friction["nu"], friction["N"], friction.get("nfeet", 2),
                      friction["mu"], int(friction["contact_mask"]),
                      int(friction.get("elide_fz", 0)))
    st = lib().orc_solve_qp(n, _f(H), np.ascontiguousarray(np.asarray(f, float)), mA, _ptr(Arm),
                            0, _ptr(lb_), _ptr(ub_), _ptr(lbA_), _ptr(ubA_),
                            None if fr is None else C.cast(C.pointer(fr), C.c_void_p),
                            int(max_iter), x, C.cast(C.pointer(cost), C.c_void_p),
                            C.cast(C.pointer(iters), C.c_void_p), _ptr(lamb), _ptr(lamr))
    return st, x, cost.value, iters.value, lamb, lamr[:mA]


def model_literal(dx, dy, dz, m):
    Ac = np.zeros(169)
    Bc = np.zeros(39)
    lib().orc_model_literal(dx, dy, dz, m, Ac, Bc)
    return Ac.reshape(13, 13, order="F"), Bc.reshape(13, 3, order="F")


def model_srbm(lin, m, Ib):
    Ac = np.zeros(169)
    Bc = np.zeros(78)
    lib().orc_model_srbm(np.ascontiguousarray(np.asarray(lin, float)[:7]), m, _f(Ib), Ac, Bc)
    return Ac.reshape(13, 13, order="F"), Bc.reshape(13, 6, order="F")


def gait_contact_mask(N, Ts, phase0, swing=0.5, stance=0.5):
    return int(lib().orc_gait_contact_mask(N, Ts, phase0, swing, stance))


def make_cfg(p):
    """p: dict from mpcqp.model (the host-side model description)."""
    cfg = SrbmCfg()
    cfg.nx, cfg.nu, cfg.N = p["nx"], p["nu"], p["N"]
    cfg.model = p["model"]
    cfg.friction = p["friction"]
    cfg.Ts, cfg.mass, cfg.mu = p["Ts"], p["mass"], p["mu"]
    for i, v in enumerate(np.asarray(p["Ib"], float).reshape(-1, order="F")):
        cfg.Ib[i] = v
    cfg.fz_min, cfg.fz_max, cfg.fxy_max = p["fz_min"], p["fz_max"], p["fxy_max"]
    cfg.u_min, cfg.u_max = p["u_min"], p["u_max"]
    keep = [_f(p["Q"]), _f(p["R"]), _f(p["P"])]
    cfg.Q, cfg.R, cfg.P = [k.ctypes.data for k in keep]
    cfg.max_iter = p.get("max_iter", 0)
    (cfg.crash_kmax, cfg.crash_pmax, cfg.crash_kmax_wg, cfg.crash_pmax_wg,
     cfg.crash_split) = crash_params(p)
    # the library leaves out each contact foot's fz >= fz_min (<= 0) bound, which its friction
    # pyramid implies (gi_setup, gi_solver.hpp); p["elide_fz"] = 0 keeps it (same minimiser,
    # more dual passes)
    cfg.elide_fz = int(p.get("elide_fz", 1))
    return cfg, keep


def srbm_batch(p, x0, xref, lin, contact, nthreads=0, want_hf=False, want_flops=False):
    cfg, keep = make_cfg(p)
    B = int(x0.shape[0])
    nV = p["nu"] * p["N"]
    U = np.zeros(B * nV)
    cost = np.zeros(B)
    status = np.zeros(B, np.int32)
    iters = np.zeros(B, np.int32)
    H = np.zeros(B * nV * nV) if want_hf else None
    f = np.zeros(B * nV) if want_hf else None
    sfl = np.zeros(B) if want_flops else None
    lib().orc_srbm_batch(C.byref(cfg), B, np.ascontiguousarray(x0, dtype=np.float64).reshape(-1),
                         np.ascontiguousarray(xref, dtype=np.float64).reshape(-1),
                         np.ascontiguousarray(lin, dtype=np.float64).reshape(-1),
                         np.ascontiguousarray(contact, dtype=np.uint64), U, cost, status, iters,
                         _ptr(H), _ptr(f), int(nthreads), _ptr(sfl))
    del keep
    out = dict(U=U.reshape(B, nV), cost=cost, status=status, iters=iters)
    if want_hf:
        out["H"] = H.reshape(B, nV, nV).transpose(0, 2, 1)  # column-major per instance
        out["f"] = f.reshape(B, nV)
    if want_flops:
        out["solver_flops"] = sfl
    return out


def srbm_bounds(p, contact):
    cfg, keep = make_cfg(p)
    nV = p["nu"] * p["N"]
    lb = np.zeros(nV)
    ub = np.zeros(nV)
    lib().orc_srbm_bounds(C.byref(cfg), int(contact), lb, ub)
    del keep
    return lb, ub


def srbm_plant(p, lin, x, u):
    """x+ = Ad x + Bd u of the SRBM at lin (exact ZOH via the Eigen-expm restatement)."""
    cfg, keep = make_cfg(p)
    xx = np.ascontiguousarray(x, dtype=np.float64).copy()
    rc = lib().orc_srbm_plant(C.byref(cfg), np.ascontiguousarray(lin, dtype=np.float64),
                              xx, np.ascontiguousarray(u, dtype=np.float64))
    del keep
    assert rc == 0, rc
    return xx


def kf_update(dt, xhat, P, eePos, eeVel, contact, quat, acc):
    """stateEstimator::update restated (one robot) -> (xhat, P)"""
    x = np.ascontiguousarray(xhat, dtype=np.float64).copy()
    Pm = np.asfortranarray(np.asarray(P, dtype=np.float64)).reshape(-1, order="F").copy()
    ct = np.ascontiguousarray(contact, dtype=np.uint8)
    rc = lib().orc_kf_update(float(dt), x, Pm, np.ascontiguousarray(eePos, dtype=np.float64),
                             np.ascontiguousarray(eeVel, dtype=np.float64),
                             C.c_void_p(ct.ctypes.data), np.ascontiguousarray(quat, dtype=np.float64),
                             np.ascontiguousarray(acc, dtype=np.float64))
    assert rc == 0, rc
    return x, Pm.reshape(12, 12, order="F")


def fk_feet(q, rpy):
    out = np.zeros(6)
    lib().orc_fk_feet(np.ascontiguousarray(q, dtype=np.float64),
                      np.ascontiguousarray(rpy, dtype=np.float64), out)
    return out


def dense_batch(p, x0, xref, AB, nthreads=0, want_hf=False):
    """config E (dense continuous model per instance): discretize -> literal dense condensing ->
    box-constrained Goldfarb-Idnani.  AB [B, nx*(nx+nu)] = [Ac | Bc] column-major."""
    keep = [_f(p["Q"]), _f(p["R"]), _f(p["P"])]
    _, _, ck, cp, _ = crash_params(p)  # the dense model runs the workgroup solver
    cfg = DenseCfg(p["nx"], p["nu"], p["N"], p["Ts"], keep[0].ctypes.data, keep[1].ctypes.data,
                   keep[2].ctypes.data, p["u_min"], p["u_max"], p.get("max_iter", 0), ck, cp)
    B = int(x0.shape[0])
    nV = p["nu"] * p["N"]
    U = np.zeros(B * nV)
    cost = np.zeros(B)
    status = np.zeros(B, np.int32)
    iters = np.zeros(B, np.int32)
    H = np.zeros(B * nV * nV) if want_hf else None
    f = np.zeros(B * nV) if want_hf else None
    lib().orc_dense_batch(C.byref(cfg), B, np.ascontiguousarray(x0, dtype=np.float64).reshape(-1),
                          np.ascontiguousarray(xref, dtype=np.float64).reshape(-1),
                          np.ascontiguousarray(AB, dtype=np.float64).reshape(-1), U, cost, status,
                          iters, _ptr(H), _ptr(f), int(nthreads))
    del keep
    out = dict(U=U.reshape(B, nV), cost=cost, status=status, iters=iters)
    if want_hf:
        out["H"] = H.reshape(B, nV, nV).transpose(0, 2, 1)
        out["f"] = f.reshape(B, nV)
    return out
