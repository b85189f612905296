"""TRON1 model constants and the benchmark configurations.

Constants are the reference's:
  mass 9.585, body inertia                       include/mpcQP.h:18-22
  Ts = 0.001, Q, R = 0.1 I, P = 20 Q, u in +-8    include/mpcQP.h:37, 54-60
  gait swing = stance = 0.5 s (float)            include/MPCParam.h:48-49
  static foot offsets                            include/MPCParam.h:13-38, 64-72
Build-chosen (the reference's SRBM path is a placeholder): per-foot normal
force fz in [0, 4 m g], friction mu = 0.6, tangential box |fx|,|fy| <= mu * fz_max, and
R = 1e-5 I for the 6-input force model: with the reference's R = 0.1 I at Ts = 1 ms the
optimum does not carry the body weight (mean fz 18 N against m g = 94 N) and no constraint
is ever active; with 1e-5 the forces are physical (mean fz 86-92 N) and the bounds and
friction cone bind.  The literal 13x3 model keeps the reference's R = 0.1 I.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import CONS_BOX, CONS_FRICTION, MODEL_DENSE, MODEL_LITERAL, MODEL_SRBM, Model

MASS = 9.585
INERTIA = np.array([[140110.479e-06, 534.939e-06, 28184.116e-06],
                    [534.939e-06, 110641.449e-06, -27.278e-06],
                    [28184.116e-06, -27.278e-06, 98944.542e-06]])
GRAVITY = 9.8
TS = 0.001
Q_DIAG = np.array([1, 1, 10, 100, 100, 100, 50, 50, 50, 100, 100, 100, 0.1], dtype=float)
SWING_TIME = np.float32(0.5)
STANCE_TIME = np.float32(0.5)
MU = 0.6
R_SRBM = 1e-5

# kinematicValues, include/MPCParam.h:13-38
_K = dict(abad=(0.05556, 0.105, -0.2602), hip=(-0.077, 0.02050, 0.0),
          knee=(-0.1500, -0.02050, -0.25981), foot=(0.145, 0.0, -0.2598),
          contact=(0.0, 0.0, -0.032))


def static_foot_offsets():
    """MPCParam::MPCParam, include/MPCParam.h:64-72 -> (left, right) body-frame offsets.
    (The reference's left foot gets y = -0.105: kept as is.)"""
    a, h, k, f, c = (_K[n] for n in ("abad", "hip", "knee", "foot", "contact"))
    x = a[0] + h[0] + k[0] + f[0] + c[0]
    z = a[2] + h[2] + k[2] + f[2] + c[2]
    left = np.array([x, -a[1] - h[1] - k[1] + f[1] + c[1], z])
    right = np.array([x, a[1] + h[1] + k[1] + f[1] + c[1], z])
    return left, right


# Config E (BASELINE configs[4]): the whole-body linearisation of TRON1 -- 24 states (6 base + 6
# joint positions, 12 velocities), 6 joint torques, N = 16.  The reference computes its
# whole-body kinematics with Pinocchio (include/pinocchio_kinematics.h) and has no whole-body
# MPC, so the weights, torque limit and sample time are build-chosen; the
# per-instance continuous model [Ac | Bc] comes from workload.whole_body_models.
TS_E = 0.01
TAU_MAX_E = 5.0  # about ten active torque bounds per QP at the optimum
Q_DIAG_E = np.array([200.0] * 6 + [50.0] * 6 + [2.0] * 6 + [1.0] * 6)
R_E = 1e-3


def model_params(config: str = "B", N: int | None = None) -> dict:
    """Host description of one benchmark configuration.

    A0  reference qp_test plant (4/2/15) -- single-instance API only, see qp_harness()
    A   13/6/10 SRBM, box, one QP          B  13/6/10 SRBM, box (the metric model)
    C   13/6/20 SRBM, box + friction       L  13/3/20 reference-literal mpcQP model
    E   24/6/16 whole-body dense model, torque box (one workgroup per QP, MFMA condensing)
    """
    fzmax = 4.0 * MASS * GRAVITY
    if config == "E":
        Nh = 16 if N is None else N
        Q = np.diag(Q_DIAG_E)
        return dict(config="E", nx=24, nu=6, N=Nh, model=MODEL_DENSE, friction=CONS_BOX,
                    constraints=CONS_BOX, Ts=TS_E, mass=MASS, mu=MU, Ib=INERTIA.copy(),
                    fz_min=0.0, fz_max=fzmax, fxy_max=MU * fzmax, u_min=-TAU_MAX_E,
                    u_max=TAU_MAX_E, Q=Q, R=R_E * np.eye(6), P=10.0 * Q, max_iter=0,
                    max_free=0)
    if config in ("A", "B", "C", "D"):
        nu, model = 6, MODEL_SRBM
        Nh = 20 if config == "C" else 10
        cons = CONS_FRICTION if config == "C" else CONS_BOX
    elif config == "L":
        nu, model, Nh, cons = 3, MODEL_LITERAL, 20, CONS_BOX
    else:
        raise ValueError(config)
    if N is not None:
        Nh = N
    nx = 13
    Q = np.diag(Q_DIAG)
    return dict(config=config, nx=nx, nu=nu, N=Nh, model=model, friction=cons,
                constraints=cons, Ts=TS, mass=MASS, mu=MU, Ib=INERTIA.copy(), fz_min=0.0,
                fz_max=fzmax, fxy_max=MU * fzmax, u_min=-8.0, u_max=8.0, Q=Q,
                R=(R_SRBM if model == MODEL_SRBM else 0.1) * np.eye(nu), P=20.0 * Q, max_iter=0,
                max_free=0)  # 0: nu*N, every contact schedule (overflow to the workgroup kernel)


def to_struct(p: dict):
    """-> (mpcqp_model ctypes struct, keep-alive list)"""
    m = Model()
    m.nx, m.nu, m.N = p["nx"], p["nu"], p["N"]
    m.model, m.constraints = p["model"], p["constraints"]
    m.Ts, m.mass, m.mu = p["Ts"], p["mass"], p["mu"]
    for i, v in enumerate(np.asarray(p["Ib"], float).reshape(-1, order="F")):
        m.Ib[i] = v
    m.fz_min, m.fz_max, m.fxy_max = p["fz_min"], p["fz_max"], p["fxy_max"]
    m.u_min, m.u_max = p["u_min"], p["u_max"]
    keep = [np.ascontiguousarray(np.asarray(p[k], float).reshape(-1, order="F"))
            for k in ("Q", "R", "P")]
    m.Q, m.R, m.P = [C.c_void_p(k.ctypes.data) for k in keep]
    m.max_iter = p.get("max_iter", 0)
    m.max_free = p.get("max_free", 0)
    return m, keep
