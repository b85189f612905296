"""The oracle's two round-5 rules for friction problems (oracle/mpcqp_oracle.c, mirrored by the
GPU solvers, DESIGN.md section 4 "Round 5"), against its own plain form:
  * elide_fz: a contact foot's fz >= fz_min (<= 0) bound is left out -- its friction pyramid
    implies it -- so the optimum is the same and the dual loop takes fewer passes;
  * the tie-stable selection key (violations within ~2^-32 relative tie, lowest id wins): the
    iteration counts no longer depend on input perturbations at the rounding level.
CPU only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mpc-limx-control_amd"))

import mpcqp  # noqa: E402

TOL_U = 1e-8


def _close(U, U0):
    return np.abs(U - U0).max(axis=1) <= TOL_U * np.maximum(1.0, np.abs(U0).max(axis=1))


def test_elide_fz_same_optimum_fewer_passes(orc):
    p = mpcqp.model_params("C")
    assert p["friction"] and p["fz_min"] <= 0.0
    batch = mpcqp.make_batch(p, 512, seed=81)
    args = (batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    plain = orc.srbm_batch(dict(p, elide_fz=0), *args, nthreads=4)
    el = orc.srbm_batch(dict(p, elide_fz=1), *args, nthreads=4)
    assert np.all(plain["status"] == 0) and np.all(el["status"] == 0)
    assert np.all(_close(el["U"], plain["U"]))
    np.testing.assert_allclose(el["cost"], plain["cost"], rtol=1e-9, atol=1e-9)
    assert el["iters"].mean() < 0.7 * plain["iters"].mean()  # 5.9 -> 3.2 at 4,096


def test_elide_fz_is_the_default_and_box_problems_are_unchanged(orc):
    pc = mpcqp.model_params("C")
    batch = mpcqp.make_batch(pc, 64, seed=82)
    args = (batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    d = orc.srbm_batch(pc, *args, nthreads=2)
    e = orc.srbm_batch(dict(pc, elide_fz=1), *args, nthreads=2)
    np.testing.assert_array_equal(d["iters"], e["iters"])
    pb = mpcqp.model_params("B")  # box only: no pyramid, nothing to leave out
    bb = mpcqp.make_batch(pb, 128, seed=82)
    argb = (bb["x0"], bb["xref"], bb["lin"], bb["contact"])
    b0 = orc.srbm_batch(dict(pb, elide_fz=0), *argb, nthreads=2)
    b1 = orc.srbm_batch(dict(pb, elide_fz=1), *argb, nthreads=2)
    np.testing.assert_array_equal(b0["iters"], b1["iters"])
    np.testing.assert_array_equal(b0["U"], b1["U"])


def test_tie_stable_selection_under_perturbation(orc):
    """x0 perturbed at 1e-11 relative: with the quantised key every instance keeps its pass
    count (without it ~0.1 % changed at 4,096: exact ties between a pyramid's +- rows)"""
    p = mpcqp.model_params("C")
    batch = mpcqp.make_batch(p, 1024, seed=83)
    a = orc.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"], nthreads=4)
    x0 = batch["x0"] * (1.0 + 1e-11 * np.random.default_rng(5).standard_normal(batch["x0"].shape))
    b = orc.srbm_batch(p, x0, batch["xref"], batch["lin"], batch["contact"], nthreads=4)
    assert np.mean(a["iters"] == b["iters"]) >= 0.999


def test_elide_fz_needs_a_positive_friction_coefficient(orc):
    """at mu = 0 the pyramid rows only pin fx, fy (mu fz -+ fx >= 0 no longer sums to fz >= 0),
    so the fz lower bound is kept: a body moving up (the optimum pulls it down) still gets
    fz >= fz_min, and the elision flag changes nothing"""
    p = mpcqp.model_params("C")
    p["mu"] = 0.0
    batch = mpcqp.make_batch(p, 256, seed=83)
    batch["x0"][:, 11] = 3.0  # v_z up
    args = (batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    plain = orc.srbm_batch(dict(p, elide_fz=0), *args, nthreads=4)
    el = orc.srbm_batch(dict(p, elide_fz=1), *args, nthreads=4)
    assert np.all(plain["status"] == 0) and np.all(el["status"] == 0)
    fz = el["U"].reshape(len(el["U"]), p["N"], 2, 3)[..., 2]
    assert fz.min() >= p["fz_min"] - 1e-8
    assert np.all(_close(el["U"], plain["U"]))
    np.testing.assert_array_equal(el["iters"], plain["iters"])
