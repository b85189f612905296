"""Algorithmic flop count of the closed-form fused path (k_mpc_pair / k_mpc), phase by phase.

This is the work the headline kernel's algorithm needs, counted the textbook way (an FMA is two
flops, a triangle is a triangle), NOT SURVEY.md 8d's count: 8d prices the reference's dense
path (Pade expm, matrix powers, Phi chain, the block-Toeplitz B'QB, src/QPSolver.cpp:21-106),
which the closed form does not execute (A^3 = 0 for both TRON1 models, DESIGN.md section 4
"Closed-form discretisation and condensing").  bench.py divides this count by the kernel's
time for `roofline.frac` and reports the 8d figure beside it as `work_rate_vs_survey_8d`.

Per QP, with nf free forces, SD support rows of each of X0 = Bc Ts and X1 = A X0 (SRBM: 6,
literal 13x3 model: 3), N steps, NU inputs per step:

  model       Iw^-1 = Rz Ib^-1 Rz' (two 3x3 products), X0 / X1 on their support rows, A x0,
              A^2 x0 (the nonzeros of the row products only)
  S blocks    S^Q_00, S^Q_11, S^P_00, S^P_11: NU(NU+1)/2 entries each, SD weighted terms
  u / v       W_m e_m per (m, support row), then u_m = X0' W_m e_m, v_m = X1' W_m e_m
  gradient    f_i = 2 sum_{m > k_i} (u_m + beta v_m) over the free inputs
  H_FF        nf(nf+1)/2 entries, each c S0 + s_ij S1 + S2 + b_ij S3 (+ R), times 2; the beta
              sums once per block pair
  Cholesky    nf^3/3
  J = L^-T    nf^3/3 (triangular inverse)
  t, x, f     t = L^-1 g, x = -J t (two triangular mat-vecs), -|t|^2/2
  dual pass   with q constraints active before the pass (an add): r = R^-1 d1 (q^2),
              |d1|^2 and |d2|^2 (4 nf), z = J2 d2 (2 nf (nf - q)), the step and the x / u
              updates (2 nf + 3 q), the Householder add J2 <- J2 (I - beta v v')
              (4 nf (nf - q)); a friction row's normal has two nonzeros (+2 nf)

  crash set   (k_mpc_pair's crash start, one working set of k bounds solved): the Gram
              M = J_A J_A' (k(k+1)/2 entries of nf-long dots), Gauss-Jordan with one right-hand
              side ((k-1) k (k+1)), w (k), y = J_A' w (2 k nf), x = x0 - J y (2 nf^2), the
              x / f updates (nf + 2k)

A pass and a working-set solve cost different amounts, and an instance's `iters` counts both,
so the headline kernel's solver flops are not a function of `iters`: k_mpc_pair counts them
itself, per working set and pass, when its context asks for it (mpcqp_count_solver_flops, a
diagnostic pointer; bench.py's pass after the timed steps), with exactly these formulas; the
oracle applies the same formulas to its own decisions (oracle.srbm_batch(want_flops=True)).
Kernels without the crash start (configs C, L: k_mpc) report dual passes only, which
`batch_flops` prices from `iters`.

The SIMD kernel executes more FP64 instructions than this (lane l owns row l, so every
triangular sweep runs its square; pad lanes; EXEC-masked halves): `roofline.pipe_frac`
(rocprofv3 SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes) is that executed rate, and
`lane_efficiency` = this count / the executed count.
"""
from __future__ import annotations

import numpy as np

SUPPORT_ROWS = {0: 6, 1: 3}  # XSupport<MODEL>: rows of X0 (and of X1) that can be nonzero


def free_counts(p: dict, contact) -> np.ndarray:
    """free variables of each instance: the forces of the feet in contact (SRBM), every input
    (the literal model)"""
    N = p["N"]
    if p["model"] == 1:
        return np.full(len(contact), p["nu"] * N, dtype=np.int64)
    mask = (1 << (2 * N)) - 1 if N < 32 else (1 << 64) - 1
    c = np.asarray(contact, dtype=np.uint64) & np.uint64(mask)
    return 3 * np.array([bin(int(v)).count("1") for v in c], dtype=np.int64)


def fixed_phases(p: dict, nf: int) -> dict:
    """flops of the phases that do not depend on the solver's passes, for one QP"""
    nu, N, sd = p["nu"], p["N"], SUPPORT_ROWS[p["model"]]
    nsym = nu * (nu + 1) // 2
    npair = N * (N + 1) // 2
    return dict(
        model=2 * 2 * 27 + nu * (sd * 4 + sd) + nu * 2 * sd + 2 * 13 * 2,
        s_blocks=4 * nsym * sd * 3,
        u_v=N * 2 * sd * 8 + N * nu * 2 * sd * 2,
        gradient=nf * (N + 2),  # (nf / N per step) x sum_k (2 (N - k) + 1)
        h_ff=(nf * (nf + 1) // 2) * 8 + npair * 25,
        cholesky=nf ** 3 / 3.0,
        inverse=nf ** 3 / 3.0,
        unconstrained=2 * nf * nf + 2 * nf,
    )


def pass_flops(nf: int, q: int, friction: bool = False) -> float:
    """one dual add pass with q constraints already active"""
    r = max(0, nf - q)
    return q * q + 4 * nf + 2 * nf * r + 2 * nf + 3 * q + 4 * nf * r + (2 * nf if friction else 0)


def crash_ws_flops(nf: int, k: int) -> float:
    """one crash working-set solve with k bounds (the kernel's and the oracle's formula)"""
    return k * (k + 1) * nf + (k - 1) * k * (k + 1) + 2 * k * nf + 2 * nf * nf + nf + 3 * k


def fixed_flops(p: dict, contact, max_nf: int | None = None):
    """-> (flops of the phases before the solver over the instances the one-wave kernel solved,
    their count): add the kernel-counted solver flops for the headline kernel's total"""
    nf = free_counts(p, contact)
    keep = nf > 0 if max_nf is None else (nf > 0) & (nf <= max_nf)
    vals, counts = np.unique(nf[keep], return_counts=True)
    return float(sum(c * sum(fixed_phases(p, int(f)).values()) for f, c in zip(vals, counts))), \
        int(keep.sum())


def instance_flops(p: dict, nf: int, iters: int) -> float:
    if nf <= 0:
        return 0.0
    fx = sum(fixed_phases(p, nf).values())
    fr = bool(p.get("constraints"))
    return fx + sum(pass_flops(nf, min(q, nf - 1), fr) for q in range(int(iters)))


def batch_flops(p: dict, contact, iters, status=None, max_nf: int | None = None):
    """-> (total flops of the instances the one-wave kernel solved, their count).  Instances
    with more than max_nf free variables went to the overflow workgroup kernel and are not
    counted against the one-wave kernel's time; infeasible / failed instances (status != 0)
    stop early and are counted with their passes."""
    nf = free_counts(p, contact)
    it = np.asarray(iters, dtype=np.int64)
    keep = np.ones(len(nf), bool) if max_nf is None else nf <= max_nf
    keep &= nf > 0
    tot = 0.0
    # group by (nf, iters): few distinct pairs
    pairs, counts = np.unique(np.stack([nf[keep], it[keep]], 1), axis=0, return_counts=True)
    for (f, i), c in zip(pairs, counts):
        tot += c * instance_flops(p, int(f), int(i))
    return tot, int(keep.sum())


def phase_table(p: dict, nf: int, mean_iters: float) -> dict:
    """per-phase flops of one QP at the mean pass count"""
    t = fixed_phases(p, nf)
    fr = bool(p.get("constraints"))
    whole = int(mean_iters)
    dual = sum(pass_flops(nf, q, fr) for q in range(whole))
    dual += (mean_iters - whole) * pass_flops(nf, whole, fr)
    t["dual_loop"] = dual
    t["total"] = sum(t.values())
    return t
