"""Seeded synthetic per-instance inputs.

Batch = S states x C candidate gait phases.  Per state:
  roll, pitch ~ U(-0.1, 0.1); yaw ~ U(-pi, pi); x, y ~ U(-1, 1); z ~ U(0.76, 0.86);
  omega ~ N(0, 0.2); vx ~ U(-1, 1); vy ~ U(-0.3, 0.3); vz ~ N(0, 0.05); g = -9.8
  foot lever arms r_s = Rz(yaw) (static offset_s + N(0, 0.03))  (world frame, foot - CoM)
  xref as include/mpcQP.h:77-97 (yaw rate 0.1) with a per-state forward speed ~ U(0, 1)
Per candidate: gait phase offset ~ U(0, 1 s); contact per horizon step from
MPC::calculateGait (include/MPCController.h:61-75).
"""
from __future__ import annotations

import math

import numpy as np

from .model import GRAVITY, INERTIA, MASS, STANCE_TIME, SWING_TIME, static_foot_offsets

DEFAULT_SEED = 20250404


def gait_contact_mask(N: int, Ts: float, phase0: float, swing=SWING_TIME, stance=STANCE_TIME) -> int:
    """bit 2k = left foot in contact at step k, bit 2k+1 = right (calculateGait per step)."""
    cycle = float(np.float32(swing) + np.float32(stance))
    mask = 0
    for k in range(N):
        ph = math.fmod(phase0 + float(k) * Ts, cycle)
        mask |= (1 << (2 * k + 1)) if ph < float(swing) else (1 << (2 * k))
    return mask


def double_support_mask(N: int, Ts: float, phase0: float, duty: float = 0.6,
                        cycle: float = 1.0) -> int:
    """Walking gait with double-support phases (build-chosen; the reference's calculateGait
    never puts both feet down): each foot is in contact for `duty` of the cycle, the right
    foot half a cycle behind the left, so both are down for (2 duty - 1) of the cycle."""
    mask = 0
    for k in range(N):
        t = phase0 + float(k) * Ts
        if math.fmod(t, cycle) < duty * cycle:
            mask |= 1 << (2 * k)
        if math.fmod(t + 0.5 * cycle, cycle) < duty * cycle:
            mask |= 1 << (2 * k + 1)
    return mask


def standing_mask(N: int) -> int:
    """both feet in contact at every horizon step (a standing TRON1: nf = 6 N)"""
    return (1 << (2 * N)) - 1


GAITS = ("alternating", "standing", "double", "mixed")


def contact_masks(gait: str, N: int, Ts: float, phase) -> np.ndarray:
    """contact masks of a [S, C] array of candidate phases for one of GAITS:
    alternating  MPC::calculateGait (include/MPCController.h:61-75), one stance foot per step
    standing     both feet down (nf = 6 N)
    double       double_support_mask (duty 0.6: 20 % of the cycle with both feet down)
    mixed        per candidate c: alternating (c % 4 in {0, 1}), double (2) or standing (3)"""
    S, C = phase.shape
    out = np.zeros((S, C), dtype=np.uint64)
    for s in range(S):
        for c in range(C):
            g = gait
            if gait == "mixed":
                g = ("alternating", "alternating", "double", "standing")[c % 4]
            ph = float(phase[s, c])
            if g == "alternating":
                m = gait_contact_mask(N, Ts, ph)
            elif g == "standing":
                m = standing_mask(N)
            elif g == "double":
                m = double_support_mask(N, Ts, ph)
            else:
                raise ValueError(gait)
            out[s, c] = m
    return out


def whole_body_models(S: int, rng) -> np.ndarray:
    """S linearised whole-body models of a TRON1-like robot, [Ac | Bc] (24 x 30, column-major
    flattened): q = (base xyz, base rpy, 6 joints), v = dq, and
        dv = M^-1 (Sel tau - K dq - D v)
    with a random SPD mass matrix around the reference's body mass / inertia
    (include/mpcQP.h:18-22) and light legs, a contact / gravity stiffness K and damping D
    (build-chosen: the reference's whole-body path is Pinocchio FK only), torques on the six
    joints."""
    n = 12
    Md = np.concatenate([np.full(3, MASS), np.diag(INERTIA), np.full(6, 0.05)])
    A = rng.normal(0.0, 0.3, (S, n, n))
    M = 0.02 * A @ A.transpose(0, 2, 1) + np.diag(Md)[None]
    Kd = np.concatenate([np.full(3, 2000.0), np.full(3, 200.0), np.full(6, 20.0)])
    Kr = rng.normal(0.0, 1.0, (S, n, n))
    K = np.diag(Kd)[None] + (Kr + Kr.transpose(0, 2, 1))
    Dd = np.concatenate([np.full(3, 40.0), np.full(3, 4.0), np.full(6, 0.5)])
    D = np.diag(Dd)[None] + 0.1 * np.abs(rng.normal(0.0, 1.0, (S, 1, 1))) * np.eye(n)[None]
    Minv = np.linalg.inv(M)
    Ac = np.zeros((S, 24, 24))
    Ac[:, :n, n:] = np.eye(n)
    Ac[:, n:, :n] = -Minv @ K
    Ac[:, n:, n:] = -Minv @ D
    Bc = np.zeros((S, 24, 6))
    Bc[:, n:, :] = Minv[:, :, 6:]  # Sel = [0; I6]: the joint torques
    AB = np.concatenate([Ac, Bc], axis=2)  # [Ac | Bc], 24 x 30
    return np.ascontiguousarray(AB.transpose(0, 2, 1).reshape(S, -1))  # column-major per model


def make_dense_batch(p: dict, B: int, seed: int = DEFAULT_SEED, candidates: int = 16):
    """config E: S states x C candidates; per state a linearised whole-body model and a
    deviation x0 (base pose +-0.02, joints +-0.3 rad, velocities +-1), per candidate a joint
    target held over the horizon (xref, N(0, 0.1) rad)"""
    rng = np.random.default_rng(seed)
    nx, N = p["nx"], p["N"]
    C = max(1, min(candidates, B))
    S = (B + C - 1) // C
    AB = whole_body_models(S, rng)
    x0 = np.concatenate([rng.uniform(-0.02, 0.02, (S, 6)), rng.uniform(-0.3, 0.3, (S, 6)),
                         rng.uniform(-1.0, 1.0, (S, 12))], axis=1)
    tgt = rng.normal(0.0, 0.1, (S, C, 6))
    xref = np.zeros((S, C, N + 1, nx))
    xref[:, :, :, 6:12] = tgt[:, :, None, :]
    rep = lambda a: np.repeat(a, C, axis=0)[:B]
    return dict(x0=np.ascontiguousarray(rep(x0)),
                xref=np.ascontiguousarray(xref.reshape(S * C, N + 1, nx)[:B]),
                lin=np.ascontiguousarray(rep(AB)), contact=np.zeros(B, dtype=np.uint64))


def make_batch(p: dict, B: int, seed: int = DEFAULT_SEED, candidates: int = 16,
               gait: str = "alternating"):
    """-> dict(x0 [B,13], xref [B,N+1,13], lin [B,8], contact [B] uint64).  `gait` picks the
    contact schedules of the candidates (GAITS); the default is the reference's calculateGait.
    The dense model (config E) takes make_dense_batch."""
    if p.get("model") == 2:
        return make_dense_batch(p, B, seed, candidates)
    rng = np.random.default_rng(seed)
    N, nx, Ts = p["N"], p["nx"], p["Ts"]
    C = max(1, min(candidates, B))
    S = (B + C - 1) // C
    roll = rng.uniform(-0.1, 0.1, S)
    pitch = rng.uniform(-0.1, 0.1, S)
    yaw = rng.uniform(-math.pi, math.pi, S)
    pos = np.stack([rng.uniform(-1, 1, S), rng.uniform(-1, 1, S), rng.uniform(0.76, 0.86, S)], 1)
    om = rng.normal(0.0, 0.2, (S, 3))
    vel = np.stack([rng.uniform(-1, 1, S), rng.uniform(-0.3, 0.3, S), rng.normal(0, 0.05, S)], 1)
    vxr = rng.uniform(0.0, 1.0, S)
    off_l, off_r = static_foot_offsets()
    nl = rng.normal(0.0, 0.03, (S, 3))
    nr = rng.normal(0.0, 0.03, (S, 3))
    phase = rng.uniform(0.0, 1.0, (S, C))

    x0 = np.zeros((S, nx))
    x0[:, 0], x0[:, 1], x0[:, 2] = roll, pitch, yaw
    x0[:, 3:6] = pos
    x0[:, 6:9] = om
    x0[:, 9:12] = vel
    x0[:, 12] = -GRAVITY
    # reference trajectory, include/mpcQP.h:77-97
    t = np.arange(N + 1) * Ts
    xref = np.repeat(x0[:, None, :], N + 1, axis=1)
    xref[:, :, 2] = yaw[:, None] + t[None, :] * 0.1
    xref[:, :, 3] = pos[:, 0:1] + t[None, :] * vxr[:, None]
    xref[:, 1:, 9] = vxr[:, None]
    # lever arms
    cy, sy = np.cos(yaw), np.sin(yaw)
    lin = np.zeros((S, 8))
    lin[:, 0] = yaw
    for j, (off, nz) in enumerate(((off_l, nl), (off_r, nr))):
        o = off[None, :] + nz
        lin[:, 1 + 3 * j] = cy * o[:, 0] - sy * o[:, 1]
        lin[:, 2 + 3 * j] = sy * o[:, 0] + cy * o[:, 1]
        lin[:, 3 + 3 * j] = o[:, 2]
    if p["model"] == 1:  # literal model: lin = support-foot offset (dx, dy, dz)
        lit = np.zeros((S, 8))
        lit[:, 0:3] = lin[:, 1:4]
        lin = lit
    contact = contact_masks(gait, N, Ts, phase)
    rep = lambda a: np.repeat(a, C, axis=0)[:B]
    return dict(x0=np.ascontiguousarray(rep(x0)), xref=np.ascontiguousarray(rep(xref)),
                lin=np.ascontiguousarray(rep(lin)), contact=np.ascontiguousarray(contact.reshape(-1)[:B]))


def qp_harness_inputs(k: int = 0):
    """The reference's qp_test plant and tick-k circle reference (src/qpSolver_test.cpp:6-50)."""
    Ts, N = 0.01, 15
    Ac = np.array([[0, 1, 0, 0], [0, -0.1, 0, 0], [0, 0, 0, 1], [0, 0, 0, -0.1]], float)
    Bc = np.array([[0, 0], [5, 0], [0, 0], [0, 5]], float)
    Q = np.diag([50.0, 5.0, 50.0, 5.0])
    R = 0.1 * np.eye(2)
    P = 20 * Q
    x_min = np.array([-5.0, -3.0, -5.0, -3.0])
    xr = np.zeros((4, N + 1))
    for i in range(N + 1):
        th = 0.5 * (k * Ts + i * Ts)
        xr[0, i] = 2.0 * math.cos(th)
        xr[2, i] = 2.0 * math.sin(th)
        xr[1, i] = -2.0 * 0.5 * math.sin(th)
        xr[3, i] = 2.0 * 0.5 * math.cos(th)
    return dict(Ts=Ts, N=N, Ac=Ac, Bc=Bc, Q=Q, R=R, P=P, x_min=x_min, x_max=-x_min,
                u_min=-8.0, u_max=8.0, xi0=np.array([2.0, 0.0, 0.0, 0.0]), xi_ref=xr)


def mpc_test_inputs(k: int = 0):
    """linear_mpc_example's plant and tick-k circle reference (src/linear_mpc_example.cpp:12-33,
    108-145): the qp_test plant written as damping / mass (-0.02 / 0.2 = -0.09999999999999999,
    1 / 0.2 = 5), xi from (2, 0, 0, 0) carried tick to tick, t = k Ts + i Ts."""
    h = qp_harness_inputs(k)
    damping, mass = 0.02, 0.2
    h["Ac"] = np.array([[0, 1, 0, 0], [0, -damping / mass, 0, 0], [0, 0, 0, 1],
                        [0, 0, 0, -damping / mass]], float)
    h["Bc"] = np.array([[0, 0], [1 / mass, 0], [0, 0], [0, 1 / mass]], float)
    return h


def make_gait_states(p: dict, S: int, seed: int = DEFAULT_SEED, candidates: int = 16):
    """Per-state data for the on-device input generation (mpcqp_batch_solve_gait), drawn
    exactly as make_batch draws them: state [S,13], feet [S,6], cmd [S,2] = (0.1 rad/s yaw
    rate, per-state forward speed), phase [S,C]."""
    rng = np.random.default_rng(seed)
    Cc = max(1, candidates)
    roll = rng.uniform(-0.1, 0.1, S)
    pitch = rng.uniform(-0.1, 0.1, S)
    yaw = rng.uniform(-math.pi, math.pi, S)
    pos = np.stack([rng.uniform(-1, 1, S), rng.uniform(-1, 1, S), rng.uniform(0.76, 0.86, S)], 1)
    om = rng.normal(0.0, 0.2, (S, 3))
    vel = np.stack([rng.uniform(-1, 1, S), rng.uniform(-0.3, 0.3, S), rng.normal(0, 0.05, S)], 1)
    vxr = rng.uniform(0.0, 1.0, S)
    off_l, off_r = static_foot_offsets()
    nl = rng.normal(0.0, 0.03, (S, 3))
    nr = rng.normal(0.0, 0.03, (S, 3))
    phase = rng.uniform(0.0, 1.0, (S, Cc))
    state = np.zeros((S, 13))
    state[:, 0], state[:, 1], state[:, 2] = roll, pitch, yaw
    state[:, 3:6], state[:, 6:9], state[:, 9:12] = pos, om, vel
    state[:, 12] = -GRAVITY
    cy, sy = np.cos(yaw), np.sin(yaw)
    feet = np.zeros((S, 6))
    for j, (off, nz) in enumerate(((off_l, nl), (off_r, nr))):
        o = off[None, :] + nz
        feet[:, 3 * j] = cy * o[:, 0] - sy * o[:, 1]
        feet[:, 3 * j + 1] = sy * o[:, 0] + cy * o[:, 1]
        feet[:, 3 * j + 2] = o[:, 2]
    cmd = np.stack([np.full(S, 0.1), vxr], 1)
    return dict(state=state, feet=feet, cmd=cmd, phase=phase)


def gait_inputs(p: dict, g: dict):
    """Host mirror of what mpcqp_batch_solve_gait builds on chip: x0, xref (include/mpcQP.h:
    74-97), lin = {yaw, r_L, r_R, 0} and contact (MPC::calculateGait) per instance s*C + c."""
    state, feet, cmd, phase = g["state"], g["feet"], g["cmd"], g["phase"]
    S, Cc = phase.shape
    N, Ts = p["N"], p["Ts"]
    x0 = np.repeat(state, Cc, axis=0)
    t = np.arange(N + 1) * Ts
    xr = np.repeat(state[:, None, :], N + 1, axis=1)
    xr[:, :, 2] = state[:, 2:3] + t[None, :] * cmd[:, 0:1]
    xr[:, :, 3] = state[:, 3:4] + t[None, :] * cmd[:, 1:2]
    xr[:, 1:, 9] = cmd[:, 1:2]
    xr[:, :, 12] = -9.8
    lin = np.zeros((S, 8))
    lin[:, 0] = state[:, 2]
    lin[:, 1:7] = feet
    contact = np.array([[gait_contact_mask(N, Ts, float(phase[s, c])) for c in range(Cc)]
                        for s in range(S)], dtype=np.uint64).reshape(-1)
    return dict(x0=x0, xref=np.repeat(xr, Cc, axis=0), lin=np.repeat(lin, Cc, axis=0),
                contact=contact)
