"""Pin the CPU oracle (oracle/) against the golden fixtures (independent numpy/scipy
restatement, tests/golden/make_golden.py) and the SURVEY.md section 8c known-answer values.

Tolerances (fp64): Ad, Bd <= 1e-13; H, f <= 1e-12 norm-wise relative; constraint arrays
<= 1e-12; QP optimum ||dU||_inf <= 1e-8 max(1, ||U||_inf)  (SURVEY.md 8c parity definition).
"""
import numpy as np
import pytest

from conftest import rel_err

TOL_DISC = 1e-13
TOL_COND = 1e-12
TOL_U = 1e-8


def test_survey_known_answers(golden, orc):
    """values computed from the reference harness inputs (src/qpSolver_test.cpp)."""
    g = golden("a0_harness.npz")
    Ad, Bd = orc.discretize(g["Ac"], g["Bc"], float(g["Ts"]))
    assert Ad[0, 1] == pytest.approx(0.00999500166625008, rel=1e-14)
    assert Ad[1, 1] == pytest.approx(0.999000499833375, rel=1e-14)
    assert Bd[0, 0] == pytest.approx(2.4991668749583e-4, rel=1e-12)
    assert Bd[1, 0] == pytest.approx(0.04997500833125042, rel=1e-14)
    o = orc.build_qp(Ad, Bd, g["Q"], g["R"], g["P"], g["x_min"], g["x_max"], -8, 8,
                     g["k0_xi0"], g["k0_xi_ref"], int(g["N"]))
    H, f = o["H"], o["f"]
    assert H[0, 0] == pytest.approx(1.1570659340730662, rel=1e-13)
    assert H[29, 29] == pytest.approx(0.6996252082430875, rel=1e-13)
    assert np.trace(H) == pytest.approx(27.269776932317207, rel=1e-13)
    np.testing.assert_allclose(f[:4], [1.09250943846621, -19.409062898877156, 1.0842076517155157,
                                       -18.72605026985299], rtol=1e-12)
    ev = np.linalg.eigvalsh(H)
    assert ev[0] == pytest.approx(0.2063, abs=1e-4) and ev[-1] == pytest.approx(9.8599, abs=1e-4)
    st, U, cost, it, _, _ = orc.solve_qp(H, f, o["lb"], o["ub"], o["A_ineq"], o["lbA"], o["ubA"])
    assert st == 0
    np.testing.assert_allclose(U[:4], [-0.10043946404952889, 6.34455273069966,
                                       -0.1003577489861012, 4.457591003585556], rtol=1e-10)
    assert cost == pytest.approx(-184.6412614841987, rel=1e-12)


def test_discretize_matches_scipy_expm(golden, orc):
    g = golden("a0_harness.npz")
    Ad, Bd = orc.discretize(g["Ac"], g["Bc"], float(g["Ts"]))
    assert rel_err(Ad, g["Ad"]) <= TOL_DISC
    assert rel_err(Bd, g["Bd"]) <= TOL_DISC


def test_quadrature_bd_linear_mpc_example(golden, orc):
    """src/linear_mpc_example.cpp:35-46 uses a different (approximate) Bd -- reproduced."""
    g = golden("a0_harness.npz")
    Ad, Bd = orc.discretize(g["Ac"], g["Bc"], float(g["Ts"]), quadrature=True)
    assert rel_err(Ad, g["Ad_quad"]) <= TOL_DISC
    assert rel_err(Bd, g["Bd_quad"]) <= 1e-12
    assert Bd[0, 0] == pytest.approx(5.0e-4, rel=1e-2)  # SURVEY CS-2: 5.0e-4 vs exact 2.4992e-4


@pytest.mark.parametrize("k", [0, 1, 250])
def test_build_qp_reference_layout(golden, orc, k):
    g = golden("a0_harness.npz")
    o = orc.build_qp(g["Ad"], g["Bd"], g["Q"], g["R"], g["P"], g["x_min"], g["x_max"], -8, 8,
                     g[f"k{k}_xi0"], g[f"k{k}_xi_ref"], int(g["N"]))
    for key in ("H", "f", "A_eq", "b_eq", "lb", "ub", "A_ineq"):
        assert rel_err(o[key], g[f"k{k}_{key}"]) <= TOL_COND, key
    # lbA/ubA: finite rows equal, zero rows carry exactly -/+INFTY (src/QPSolver.cpp:72-73)
    for key in ("lbA", "ubA"):
        a, b = o[key], g[f"k{k}_{key}"]
        fin = np.abs(b) < 1e19
        assert rel_err(a[fin], b[fin]) <= TOL_COND
        np.testing.assert_array_equal(a[~fin], b[~fin])
    assert o["A_ineq"].shape == (2 * 4 * 15, 30) and o["A_eq"].shape == (60, 30)
    # every other block of A_ineq is zero (src/QPSolver.cpp:71-80)
    assert np.all(o["A_ineq"][4:8] == 0) and np.all(o["lbA"][4:8] == -1e20)


@pytest.mark.parametrize("k", [0, 1, 250])
def test_corrected_qp_optimum(golden, orc, k):
    g = golden("a0_harness.npz")
    st, U, cost, it, lamb, lamr = orc.solve_qp(g[f"k{k}_H"], g[f"k{k}_f"], g[f"k{k}_lb"],
                                               g[f"k{k}_ub"], g[f"k{k}_A_ineq"],
                                               g[f"k{k}_lbA"], g[f"k{k}_ubA"])
    assert st == 0
    U0 = g[f"k{k}_U"]
    assert np.abs(U - U0).max() <= TOL_U * max(1.0, np.abs(U0).max())
    assert cost == pytest.approx(float(g[f"k{k}_cost"]), rel=1e-10, abs=1e-10)
    # qpOASES-convention multipliers: H x + f = y_b + A' y_A
    H, f, A = g[f"k{k}_H"], g[f"k{k}_f"], g[f"k{k}_A_ineq"]
    np.testing.assert_allclose(H @ U + f, lamb + A.T @ lamr, atol=1e-9)


@pytest.mark.parametrize("k", [0, 1, 250])
def test_faithful_stack_is_infeasible(golden, orc, k):
    """The reference hands qpOASES [A_eq; A_ineq] with A_eq as equalities -- infeasible
    (SURVEY.md 0.5).  Both the oracle and an LP feasibility check (HiGHS) agree."""
    g = golden("a0_harness.npz")
    assert not bool(g[f"k{k}_faithful_feasible"])
    A = np.vstack([g[f"k{k}_A_eq"], g[f"k{k}_A_ineq"]])
    lbA = np.concatenate([g[f"k{k}_b_eq"], g[f"k{k}_lbA"]])
    ubA = np.concatenate([g[f"k{k}_b_eq"], g[f"k{k}_ubA"]])
    st, *_ = orc.solve_qp(g[f"k{k}_H"], g[f"k{k}_f"], g[f"k{k}_lb"], g[f"k{k}_ub"], A, lbA, ubA)
    assert st == 2  # INFEASIBLE


def test_qp_test_closed_loop(golden, orc):
    """qp_test's 500-tick loop (src/qpSolver_test.cpp:38-90) with the corrected QP, including
    the plant-state-starts-at-zero quirk (src/QPSolver.cpp:12)."""
    g = golden("a0_harness.npz")
    import mpcqp
    N = int(g["N"])
    plant = np.zeros(4)
    xi = np.array([2.0, 0, 0, 0])
    for k in range(500):
        h = mpcqp.qp_harness_inputs(k)
        o = orc.build_qp(g["Ad"], g["Bd"], g["Q"], g["R"], g["P"], g["x_min"], g["x_max"], -8, 8,
                         xi, h["xi_ref"], N)
        st, U, *_ = orc.solve_qp(o["H"], o["f"], o["lb"], o["ub"], o["A_ineq"], o["lbA"], o["ubA"])
        assert st == 0
        plant = g["Ad"] @ plant + g["Bd"] @ U[:2]
        xi = plant.copy()
        if k in (0, 99, 499):
            np.testing.assert_allclose(xi, g["loop_states"][k], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(xi, g["loop_states"][-1], rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("fname", ["srbm_B.npz", "srbm_C.npz", "literal_L.npz"])
def test_srbm_pipeline(golden, orc, fname):
    import mpcqp
    g = golden(fname)
    p = mpcqp.model_params(str(g["config"]))
    o = orc.srbm_batch(p, g["x0"], g["xref"], g["lin"], g["contact"], nthreads=2, want_hf=True)
    assert np.all(o["status"] == 0)
    nH = g["H"].shape[0]
    for i in range(nH):
        assert rel_err(o["H"][i], g["H"][i]) <= TOL_COND
    for i in range(g["f"].shape[0]):
        assert rel_err(o["f"][i], g["f"][i]) <= TOL_COND
        U0 = g["U"][i]
        assert np.abs(o["U"][i] - U0).max() <= TOL_U * max(1.0, np.abs(U0).max()), i
        assert o["cost"][i] == pytest.approx(float(g["cost"][i]), rel=1e-9, abs=1e-9)


def test_model_builders_match_golden(golden, orc):
    import mpcqp
    g = golden("srbm_B.npz")
    p = mpcqp.model_params("B")
    for i in range(4):
        Ac, Bc = orc.model_srbm(g["lin"][i], p["mass"], p["Ib"])
        Ad, Bd = orc.discretize(Ac, Bc, p["Ts"])
        assert rel_err(Ad, g["Ad"][i]) <= TOL_DISC and rel_err(Bd, g["Bd"][i]) <= TOL_DISC
    gl = golden("literal_L.npz")
    pl = mpcqp.model_params("L")
    Ac, Bc = orc.model_literal(*gl["lin"][0][:3], pl["mass"])
    assert Bc[9, 0] == -pl["mass"] and Ac[11, 12] == -1.0  # include/mpcQP.h:165,178
    Ad, Bd = orc.discretize(Ac, Bc, pl["Ts"])
    assert rel_err(Ad, gl["Ad"][0]) <= TOL_DISC and rel_err(Bd, gl["Bd"][0]) <= TOL_DISC


def test_matpow_binary_powering(orc):
    rng = np.random.default_rng(0)
    A = rng.normal(size=(5, 5)) / 3
    for p in (0, 1, 2, 3, 7, 16):
        np.testing.assert_allclose(orc.matpow(A, p), np.linalg.matrix_power(A, p), rtol=1e-12,
                                   atol=1e-14)


@pytest.mark.parametrize("scale", [1e-3, 0.1, 0.5, 1.5, 8.0, 60.0])
def test_expm_all_pade_degrees(orc, scale):
    """Eigen's degree selection: 3/5/7/9/13 (+ scaling) across norms."""
    import scipy.linalg as sl
    rng = np.random.default_rng(1)
    A = rng.normal(size=(7, 7))
    A *= scale / np.abs(A).sum(0).max()
    assert rel_err(orc.expm(A), sl.expm(A)) <= 1e-12


def test_mpc_test_closed_loop(golden, orc):
    """linear_mpc_example's 500-tick loop (src/linear_mpc_example.cpp:108-195): the oracle's
    quadrature Bd (:35-46) against the fixture's scipy one, xi carried from (2,0,0,0) by
    xi = Ad xi + Bd u (:124,182), corrected QP per tick, against the certified trajectory."""
    g = golden("mpc_test_loop.npz")
    import mpcqp
    h = mpcqp.mpc_test_inputs(0)
    Ad, Bd = orc.discretize(h["Ac"], h["Bc"], h["Ts"], quadrature=True)
    np.testing.assert_allclose(Ad, g["Ad"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(Bd, g["Bd"], rtol=0, atol=1e-14)
    N = int(g["N"])
    xi = h["xi0"].copy()
    for k in range(500):
        hk = mpcqp.mpc_test_inputs(k)
        o = orc.build_qp(Ad, Bd, h["Q"], h["R"], h["P"], h["x_min"], h["x_max"], -8, 8, xi,
                         hk["xi_ref"], N)
        st, U, *_ = orc.solve_qp(o["H"], o["f"], o["lb"], o["ub"], o["A_ineq"], o["lbA"], o["ubA"])
        assert st == 0
        xi = Ad @ xi + Bd @ U[:2]
        if k in (0, 99, 499):
            np.testing.assert_allclose(U[:2], g["loop_u"][k], rtol=1e-7, atol=1e-9)
            np.testing.assert_allclose(xi, g["loop_states"][k], rtol=1e-7, atol=1e-9)
