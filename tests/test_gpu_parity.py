"""GPU parity: libmpcqp.so (HIP, gfx950) through its C ABI vs the golden fixtures and the CPU
oracle on identical seeded inputs.  Floating point throughout (fp64, the reference's Eigen
MatrixXd arithmetic); tolerances are stated per quantity:
  Ad, Bd                    <= 1e-13 norm-wise relative
  H, f, constraint arrays   <= 1e-12 norm-wise relative
  QP optimum U              ||dU||_inf <= 1e-8 * max(1, ||U||_inf)      
  cost                      <= 1e-9 relative
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

TOL_DISC = 1e-13
TOL_COND = 1e-12
TOL_U = 1e-8


def u_close(U, U0):
    return np.abs(np.asarray(U) - U0).max() <= TOL_U * max(1.0, np.abs(U0).max())


# ------------------------------------------------------------- single-instance reference API
def test_discretize_reference_plant(gpu, golden):
    from mpcqp.qpsolver import discretize
    g = golden("a0_harness.npz")
    Ad, Bd = discretize(g["Ac"], g["Bc"], float(g["Ts"]))
    assert rel_err(Ad, g["Ad"]) <= TOL_DISC and rel_err(Bd, g["Bd"]) <= TOL_DISC
    assert Bd[0, 0] == pytest.approx(2.4991668749583e-4, rel=1e-12)  # SURVEY 8c KAT


def test_discretize_quadrature_linear_mpc_example(gpu, golden, orc):
    """src/linear_mpc_example.cpp:35-46 (the mpc_test harness's Bd) vs the golden fixture"""
    from mpcqp.qpsolver import discretize
    g = golden("a0_harness.npz")
    Ad, Bd = discretize(g["Ac"], g["Bc"], float(g["Ts"]), quadrature=True)
    assert rel_err(Ad, g["Ad_quad"]) <= TOL_DISC and rel_err(Bd, g["Bd_quad"]) <= TOL_DISC
    rng = np.random.default_rng(8)
    Ac, Bc = rng.normal(size=(13, 13)), rng.normal(size=(13, 6))
    Ad, Bd = discretize(Ac, Bc, 0.01, quadrature=True)
    Ad0, Bd0 = orc.discretize(Ac, Bc, 0.01, quadrature=True)
    assert rel_err(Ad, Ad0) <= TOL_DISC and rel_err(Bd, Bd0) <= TOL_DISC


@pytest.mark.parametrize("scale", [1e-3, 0.1, 0.5, 1.5, 8.0, 60.0])
def test_discretize_all_pade_degrees(gpu, orc, scale):
    from mpcqp.qpsolver import discretize
    rng = np.random.default_rng(int(scale * 1000))
    for nx, nu in ((4, 2), (13, 6), (24, 6)):
        Ac = rng.normal(size=(nx, nx))
        Bc = rng.normal(size=(nx, nu))
        M = np.zeros((nx + nu, nx + nu))
        M[:nx, :nx], M[:nx, nx:] = Ac, Bc
        Ts = scale / np.abs(M).sum(0).max()
        Ad, Bd = discretize(Ac, Bc, Ts)
        Ad0, Bd0 = orc.discretize(Ac, Bc, Ts)
        assert rel_err(Ad, Ad0) <= 1e-12 and rel_err(Bd, Bd0) <= 1e-12, (nx, nu)


@pytest.mark.parametrize("k", [0, 1, 250])
def test_build_qp_reference_layout(gpu, golden, k):
    from mpcqp.qpsolver import build_qp
    g = golden("a0_harness.npz")
    o = build_qp(g["Ad"], g["Bd"], g["Q"], g["R"], g["P"], g["x_min"], g["x_max"], -8, 8,
                 g[f"k{k}_xi0"], g[f"k{k}_xi_ref"], int(g["N"]))
    for key in ("H", "f", "A_eq", "b_eq", "lb", "ub", "A_ineq"):
        assert rel_err(o[key], g[f"k{k}_{key}"]) <= TOL_COND, key
    for key in ("lbA", "ubA"):
        a, b = o[key], g[f"k{k}_{key}"]
        fin = np.abs(b) < 1e19
        assert rel_err(a[fin], b[fin]) <= TOL_COND
        np.testing.assert_array_equal(a[~fin], b[~fin])


@pytest.mark.parametrize("k", [0, 1, 250])
def test_solve_dense_corrected_and_faithful(gpu, golden, orc, k):
    from mpcqp.qpsolver import solve_dense
    g = golden("a0_harness.npz")
    H, f, lb, ub = g[f"k{k}_H"], g[f"k{k}_f"], g[f"k{k}_lb"], g[f"k{k}_ub"]
    A, lbA, ubA = g[f"k{k}_A_ineq"], g[f"k{k}_lbA"], g[f"k{k}_ubA"]
    st, x, cost, it, y = solve_dense(H, f, A, lb, ub, lbA, ubA, want_y=True)
    assert st == 0
    assert u_close(x, g[f"k{k}_U"])
    assert cost == pytest.approx(float(g[f"k{k}_cost"]), rel=1e-9)
    st0, x0, c0, it0, lb0, lr0 = orc.solve_qp(H, f, lb, ub, A, lbA, ubA)
    assert it == it0
    np.testing.assert_allclose(H @ x + f, y[:30] + A.T @ y[30:], atol=1e-9)
    np.testing.assert_allclose(y[:30], lb0, atol=1e-8)
    # the reference's stacked [A_eq; A_ineq] problem is infeasible: reported, not hidden
    Af = np.vstack([g[f"k{k}_A_eq"], A])
    bl = np.concatenate([g[f"k{k}_b_eq"], lbA])
    bu = np.concatenate([g[f"k{k}_b_eq"], ubA])
    st2, *_ = solve_dense(H, f, Af, lb, ub, bl, bu)
    assert st2 == 2


def test_qpsolver_class_closed_loop(gpu, golden):
    """qp_test (src/qpSolver_test.cpp:26-90) through the reference-shaped QPSolver mirror."""
    from mpcqp.qpsolver import QPSolver
    import mpcqp
    g = golden("a0_harness.npz")
    h = mpcqp.qp_harness_inputs(0)
    qp = QPSolver(h["Ts"], h["N"], h["Ac"], h["Bc"], h["Q"], h["R"], h["P"], h["x_min"],
                  h["x_max"], h["u_min"], h["u_max"])
    xi = h["xi0"].copy()
    for k in range(100):
        hk = mpcqp.qp_harness_inputs(k)
        H, f, A_eq, b_eq, lb, ub, A_ineq, lbA, ubA = qp.buildQPParams(xi, hk["xi_ref"])
        A_total = np.vstack([A_eq, A_ineq])
        ok, U_opt = qp.solveQP(H, f, A_total, lb, ub, np.concatenate([b_eq, lbA]),
                               np.concatenate([b_eq, ubA]))
        assert ok and qp.corrected and qp.last_status == 0
        qp.updateState(U_opt[:, 0])
        xi = qp.getState()
    np.testing.assert_allclose(xi, g["loop_states"][99], rtol=1e-7, atol=1e-9)


def test_qpsolver_mpc_test_closed_loop(gpu, golden):
    """mpc_test (src/linear_mpc_example.cpp:108-195) through the QPSolver mirror: quadrature
    Bd (mpcqp_discretize_quadrature), xi carried from (2,0,0,0), the stacked [A_eq; A_ineq] the
    harness builds (corrected on the GPU), 500 ticks against the certified trajectory."""
    from mpcqp.qpsolver import QPSolver
    import mpcqp
    g = golden("mpc_test_loop.npz")
    h = mpcqp.mpc_test_inputs(0)
    qp = QPSolver(h["Ts"], h["N"], h["Ac"], h["Bc"], h["Q"], h["R"], h["P"], h["x_min"],
                  h["x_max"], h["u_min"], h["u_max"], quadrature=True)
    np.testing.assert_allclose(qp.Bd, g["Bd"], rtol=0, atol=1e-14)
    xi = h["xi0"].copy()
    qp.setState(xi)
    for k in range(500):
        hk = mpcqp.mpc_test_inputs(k)
        H, f, A_eq, b_eq, lb, ub, A_ineq, lbA, ubA = qp.buildQPParams(xi, hk["xi_ref"])
        A_total = np.vstack([A_eq, A_ineq])
        ok, U_opt = qp.solveQP(H, f, A_total, lb, ub, np.concatenate([b_eq, lbA]),
                               np.concatenate([b_eq, ubA]))
        assert ok and qp.corrected and qp.last_status == 0
        qp.updateState(U_opt[:, 0])
        xi = qp.getState()
        if k in (0, 99, 250, 499):
            np.testing.assert_allclose(U_opt[:, 0], g["loop_u"][k], rtol=1e-7, atol=1e-9)
            np.testing.assert_allclose(xi, g["loop_states"][k], rtol=1e-7, atol=1e-9)


# ------------------------------------------------------------------------- batched engine
def run_batch(p, batch, want_hf=False, expect_fast=True):
    """fused fast path (discretize + condense_solve); with want_hf also the generic path
    (full H, f to HBM + stand-alone solve), whose results are returned under 'gen_*'."""
    from mpcqp.engine import BatchEngine
    eng = BatchEngine(p)
    assert eng.fast_path == expect_fast
    d = eng.upload(batch)
    out = {}
    if want_hf:
        H, f = eng.condense(d)
        eng.solve_qp(d, H, f)
        eng.sync()
        out["H"] = H.cpu().numpy().transpose(0, 2, 1)  # stored column-major per instance
        out["f"] = f.cpu().numpy()
        for k in ("U", "cost", "status", "iters"):
            out["gen_" + k] = d[k].cpu().numpy().copy()
    eng.solve(d)
    eng.sync()
    for k in ("U", "cost", "status", "iters"):
        out[k] = d[k].cpu().numpy()
    out["crash"] = eng.crash  # the oracle reproduces the iteration counts with p["crash"] = this
    eng.close()
    return out


def with_crash(p, crash):
    """the oracle configured with the library kernel's crash start (iteration counts)"""
    q = dict(p)
    q["crash"] = tuple(crash)
    return q


@pytest.mark.parametrize("fname", ["srbm_B.npz", "srbm_C.npz", "literal_L.npz"])
def test_batch_vs_golden(gpu, golden, fname):
    import mpcqp
    g = golden(fname)
    p = mpcqp.model_params(str(g["config"]))
    batch = dict(x0=g["x0"], xref=g["xref"], lin=g["lin"], contact=g["contact"])
    o = run_batch(p, batch, want_hf=True)
    assert np.all(o["status"] == 0) and np.all(o["gen_status"] == 0)
    for i in range(g["f"].shape[0]):
        assert u_close(o["gen_U"][i], g["U"][i]), i
    for i in range(g["H"].shape[0]):
        assert rel_err(o["H"][i], g["H"][i]) <= TOL_COND
    for i in range(g["f"].shape[0]):
        assert rel_err(o["f"][i], g["f"][i]) <= TOL_COND
        assert u_close(o["U"][i], g["U"][i]), i
        assert o["cost"][i] == pytest.approx(float(g["cost"][i]), rel=1e-9, abs=1e-9)


@pytest.mark.parametrize("config,B", [("B", 2048), ("C", 512), ("L", 512)])
def test_batch_vs_oracle(gpu, orc, config, B):
    import mpcqp
    p = mpcqp.model_params(config)
    batch = mpcqp.make_batch(p, B, seed=99)
    o = run_batch(p, batch, want_hf=True)
    ref = orc.srbm_batch(with_crash(p, o["crash"]), batch["x0"], batch["xref"], batch["lin"],
                         batch["contact"], want_hf=True)
    assert (o["crash"][0] > 0) == (config == "B")  # the paired kernel's crash start
    np.testing.assert_array_equal(o["status"], ref["status"])
    np.testing.assert_array_equal(o["gen_status"], ref["status"])
    assert np.all(o["status"] == 0)
    bad_g = [i for i in range(B) if not u_close(o["gen_U"][i], ref["U"][i])]
    assert not bad_g, bad_g[:10]
    for i in range(0, B, max(1, B // 64)):
        assert rel_err(o["H"][i], ref["H"][i]) <= TOL_COND
        assert rel_err(o["f"][i], ref["f"][i]) <= TOL_COND
    bad = [i for i in range(B) if not u_close(o["U"][i], ref["U"][i])]
    assert not bad, bad[:10]
    np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
    # same algorithm, same order: iteration counts agree except on rounding-level ties (the
    # paired kernel's crash start included: the oracle runs it with the same caps)
    assert np.mean(o["iters"] == ref["iters"]) >= 0.99


def test_full_size_metric_batch_properties(gpu, orc):
    """BASELINE metric config (13/6/10, batch 65536): size-independent properties --
    every instance solved, KKT-consistent sample against the oracle, bitwise determinism
    across two runs, and the min-cost key equals the host argmin of the returned costs."""
    import mpcqp
    from mpcqp.engine import BatchEngine, decode_key, encode_key
    p = mpcqp.model_params("B")
    B = 65536
    batch = mpcqp.make_batch(p, B)
    eng = BatchEngine(p)
    d = eng.upload(batch)
    eng.solve(d)
    key = int(eng.select_min(d).item())
    U1 = d["U"].cpu().numpy().copy()
    c1 = d["cost"].cpu().numpy().copy()
    st = d["status"].cpu().numpy()
    eng.solve(d)
    eng.sync()
    U2 = d["U"].cpu().numpy()
    eng.close()
    assert np.all(st == 0)
    np.testing.assert_array_equal(U1, U2)  # deterministic
    host_key = min(encode_key(c, i) for i, c in enumerate(c1))
    assert key == host_key
    cbest, ibest = decode_key(key)
    assert ibest == int(np.lexsort((np.arange(B), c1.astype(np.float32)))[0])
    idx = np.random.default_rng(5).choice(B, 192, replace=False)
    sub = {k: batch[k][idx] for k in batch}
    ref = orc.srbm_batch(p, sub["x0"], sub["xref"], sub["lin"], sub["contact"])
    for j, i in enumerate(idx):
        assert u_close(U1[i], ref["U"][j]), i


def test_select_min_repeated_calls(gpu):
    """k_select_min reduces in one launch (last block re-arms the context's ticket): repeated
    calls on one context with different batch sizes (1 block up to the 1024-block clamp with a
    grid-stride loop: 1,100,000 instances; B = 0), index bases and failed instances each return
    the host key"""
    import torch
    import mpcqp
    from mpcqp.engine import BatchEngine, encode_key
    p = mpcqp.model_params("B")
    eng = BatchEngine(p)
    rng = np.random.default_rng(17)
    dev = torch.device("cuda:0")
    key = torch.zeros(1, dtype=torch.int64, device=dev)
    for B in (0, 1, 255, 256, 257, 4096, 65536, 300000, 1_100_000, 3):
        cost = rng.normal(size=B) * 100.0
        status = np.where(rng.random(B) < 0.1, 3, 0).astype(np.int32)
        base = int(rng.integers(0, 1 << 20))
        d = dict(B=B, cost=torch.tensor(cost, device=dev),
                 status=torch.tensor(status, device=dev), key=key)
        torch.cuda.synchronize()
        k = eng.select_min(d, index_base=base)
        eng.sync()
        got = int(k.item())
        ok = np.nonzero(status == 0)[0]
        want = min((encode_key(cost[i], base + int(i)) for i in ok), default=0x7FFFFFFFFFFFFFFF)
        assert got == want, B
    eng.close()


def test_select_record_and_reduce(gpu):
    """selection records (k_select_min with the winner's U row) and the device record
    reduction of the one-collective multi-GPU selection: batch sizes through the
    kSelMaxBlocks clamp and the grid-stride path (1,100,000 > 1024 x 1024), an all-invalid
    shard (key INT64_MAX, U = 0), and the reduction over several ranks' records equal the
    host restatements (mpcqp.dist.host_record / host_reduce_records)."""
    import torch
    import mpcqp
    from mpcqp.dist import NO_KEY, host_record, host_reduce_records
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    nV = p["nu"] * p["N"]
    eng = BatchEngine(p)
    rng = np.random.default_rng(29)
    dev = torch.device("cuda:0")
    recs = []
    for r, B in enumerate((1, 4097, 1_100_000, 5, 300)):
        cost = rng.normal(size=B) * 100.0
        status = np.where(rng.random(B) < 0.2, 3, 0).astype(np.int32)
        if r == 3:
            status[:] = 2  # nothing valid on this shard
        U = rng.normal(size=(B, nV))
        base = r * 2_000_000
        d = dict(B=B, cost=torch.tensor(cost, device=dev), status=torch.tensor(status, device=dev),
                 U=torch.tensor(U, device=dev))
        rec = torch.full((1 + nV,), -1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        eng.select_record(d, rec, index_base=base)
        eng.sync()
        got = rec.cpu().numpy()
        want = host_record(cost, status, U, base)
        np.testing.assert_array_equal(got, want)
        if r == 3:
            assert got[0] == NO_KEY and not got[1:].any()
        recs.append(want)
    g = torch.tensor(np.stack(recs), device=dev)
    best = torch.zeros(1 + nV, dtype=torch.int64, device=dev)
    eng.reduce_records(g, best)
    eng.sync()
    ref = np.zeros(1 + nV, np.int64)
    host_reduce_records(np.stack(recs), ref)
    np.testing.assert_array_equal(best.cpu().numpy(), ref)
    # all ranks invalid -> the no-selection record
    g2 = torch.tensor(np.stack([recs[3], recs[3]]), device=dev)
    eng.reduce_records(g2, best)
    eng.sync()
    b2 = best.cpu().numpy()
    assert b2[0] == NO_KEY and not b2[1:].any()
    eng.close()


def test_edge_cases(gpu):
    """empty batch, infeasible bounds, no free variable, non-PD Hessian, too many free vars"""
    from mpcqp.qpsolver import solve_dense
    import mpcqp
    from mpcqp.engine import BatchEngine
    # empty batch
    p = mpcqp.model_params("B")
    eng = BatchEngine(p)
    d = eng.upload({k: v[:0] for k, v in mpcqp.make_batch(p, 4).items()})
    eng.solve(d)
    eng.sync()
    eng.close()
    H = np.diag([2.0, 4.0, 1.0])
    f = np.array([1.0, -2.0, 0.5])
    st, *_ = solve_dense(H, f, None, np.array([0.0, 1.0, 0.0]), np.array([1.0, 0.0, 1.0]))
    assert st == 2  # lb > ub
    st, x, cost, it, _ = solve_dense(H, f, None, np.array([0.5, 1.0, -1.0]),
                                     np.array([0.5, 1.0, -1.0]))
    assert st == 0 and np.allclose(x, [0.5, 1.0, -1.0])
    assert cost == pytest.approx(0.5 * x @ H @ x + f @ x)
    st, *_ = solve_dense(np.diag([1.0, -1.0, 1.0]), f, None, None, None)
    assert st == 4  # not positive definite
    # unbounded-below directions are impossible for PD H; a bounds-only QP hits the box
    st, x, *_ = solve_dense(H, np.array([-100.0, 100.0, 0.0]), None, -np.ones(3), np.ones(3))
    assert st == 0 and np.allclose(x, [1.0, -1.0, 0.0])
    # equality row: x0 + x1 = 1
    st, x, *_ = solve_dense(H, f, np.array([[1.0, 1.0, 0.0]]), None, None, np.array([1.0]),
                            np.array([1.0]))
    assert st == 0 and x[0] + x[1] == pytest.approx(1.0, abs=1e-12)
    # a non-diagonal Q runs the generic kernels (same answers, see test_generic_path_*)
    # more free variables than the batched context was sized for -> BAD_DIMS per instance
    p2 = mpcqp.model_params("B")
    p2["max_free"] = 12
    batch = mpcqp.make_batch(p2, 8)
    eng = BatchEngine(p2)
    d = eng.upload(batch)
    eng.solve(d)
    eng.sync()
    assert np.all(d["status"].cpu().numpy() == 1)
    eng.close()


def test_generic_path_non_diagonal_weights(gpu, orc):
    """a full (non-diagonal) Q takes the generic runtime-dimension kernels; results still
    match the oracle"""
    import mpcqp
    p = mpcqp.model_params("B")
    rng = np.random.default_rng(3)
    M = rng.normal(size=(13, 13)) * 0.05
    p["Q"] = p["Q"] + M @ M.T
    p["P"] = 20.0 * p["Q"]
    batch = mpcqp.make_batch(p, 128, seed=5)
    o = run_batch(p, batch, expect_fast=False)
    ref = orc.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    assert np.all(o["status"] == 0)
    for i in range(128):
        assert u_close(o["U"][i], ref["U"][i]), i


def test_pair_kernel_matches_single_and_oracle(gpu, orc, monkeypatch):
    """Two QPs per wavefront (csrc/mpc_pair.hpp, nf <= 30) against the one-QP-per-wave kernel
    (MPCQP_PAIR=0) and the oracle: odd batch (the last wave's upper half is idle), contact
    masks with fewer stance forces (nf < 30, uneven iteration counts inside a wave) and with
    both feet down at one step (nf > max_free -> BAD_DIMS beside a solved neighbour; the
    context is capped at 30 free forces, so nothing overflows to the workgroup kernel)."""
    import mpcqp
    p = mpcqp.model_params("B")
    p["max_free"] = 30
    B = 333
    batch = mpcqp.make_batch(p, B, seed=7)
    ct = batch["contact"].astype(np.uint64).copy()
    rng = np.random.default_rng(11)
    for i in range(B):
        if i % 5 == 1:  # lift the stance foot for a few random steps
            for k in rng.choice(p["N"], 3, replace=False):
                ct[i] &= ~np.uint64(3 << (2 * int(k)))
        if i % 7 == 3:  # double support at one step: 33 free forces
            ct[i] |= np.uint64(3 << (2 * int(rng.integers(p["N"]))))
    batch["contact"] = ct
    from mpcqp.engine import BatchEngine
    monkeypatch.setenv("MPCQP_PAIR", "0")
    assert BatchEngine(p).fused_kernel == "k_mpc"
    single = run_batch(p, batch)
    monkeypatch.delenv("MPCQP_PAIR")
    assert BatchEngine(p).fused_kernel == "k_mpc_pair"
    pair = run_batch(p, batch)
    nfree = np.array([3 * bin(int(c)).count("1") for c in ct])
    bad_dims = nfree > p["max_free"]
    assert bad_dims.sum() > 20 and (nfree < 30).sum() > 20
    np.testing.assert_array_equal(pair["status"], single["status"])
    assert np.all(pair["status"][bad_dims] == 1) and np.all(pair["status"][~bad_dims] == 0)
    # iteration counts: the one-QP kernel runs the plain dual loop, the paired kernel its crash
    # start first -- each against the oracle configured the same way (below)
    assert single["crash"][:2] == (0, 0) and pair["crash"][0] > 0
    # blocked MFMA factorisation in the one-QP kernel vs column sweeps in the paired one
    sc = np.maximum(1.0, np.abs(single["U"]).max(axis=1, keepdims=True))
    assert np.all(np.abs(pair["U"] - single["U"]) <= 1e-10 * sc)
    np.testing.assert_allclose(pair["cost"], single["cost"], rtol=1e-10, atol=1e-10)
    ok = ~bad_dims
    ref = orc.srbm_batch(p, batch["x0"][ok], batch["xref"][ok], batch["lin"][ok], ct[ok])
    refc = orc.srbm_batch(with_crash(p, pair["crash"]), batch["x0"][ok], batch["xref"][ok],
                          batch["lin"][ok], ct[ok])
    assert np.all(ref["status"] == 0) and np.all(refc["status"] == 0)
    Uo = pair["U"][ok]
    bad = [j for j in range(Uo.shape[0]) if not u_close(Uo[j], ref["U"][j])]
    assert not bad, bad[:10]
    np.testing.assert_allclose(pair["cost"][ok], ref["cost"], rtol=1e-9, atol=1e-9)
    assert np.mean(single["iters"][ok] == ref["iters"]) >= 0.99
    assert np.mean(pair["iters"][ok] == refc["iters"]) >= 0.99
    assert len(set(pair["iters"][ok].tolist())) > 2  # uneven work inside the waves


def test_pair_kernel_full_size_vs_single(gpu, monkeypatch):
    """metric batch (65536): the paired kernel's schedule-sorted instance assignment writes
    every instance exactly once (outputs pre-filled with sentinels) and agrees with the
    one-QP kernel everywhere: status and iteration counts equal, U / cost to 1e-10 relative
    (the one-QP kernel factors H_FF with the blocked MFMA algorithm of chol_reg.hpp, the
    paired kernel column by column: same operations, different summation order)."""
    import torch
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    B = 65536
    batch = mpcqp.make_batch(p, B, seed=23)
    res = {}
    for pair in (False, True):
        if pair:
            monkeypatch.delenv("MPCQP_PAIR", raising=False)
        else:
            monkeypatch.setenv("MPCQP_PAIR", "0")
        eng = BatchEngine(p)
        assert eng.fused_kernel == ("k_mpc_pair" if pair else "k_mpc")
        d = eng.upload(batch)
        d["U"].fill_(float("nan"))
        d["cost"].fill_(float("nan"))
        d["status"].fill_(99)
        d["iters"].fill_(-1)
        torch.cuda.synchronize()
        eng.solve(d)
        eng.sync()
        res[pair] = {k: d[k].cpu().numpy().copy() for k in ("U", "cost", "status", "iters")}
        eng.close()
    a, b = res[True], res[False]
    assert np.all(a["status"] == 0) and np.all(b["status"] == 0)
    assert np.all(np.isfinite(a["U"])) and np.all(np.isfinite(a["cost"]))
    # the crash start solves the same QPs in fewer passes: the tail above all
    assert a["iters"].mean() < 0.6 * b["iters"].mean()
    assert a["iters"].max() <= 10 < b["iters"].max()
    scale = np.maximum(1.0, np.abs(b["U"]).max(axis=1, keepdims=True))
    assert np.all(np.abs(a["U"] - b["U"]) <= 1e-10 * scale)
    np.testing.assert_allclose(a["cost"], b["cost"], rtol=1e-10, atol=1e-10)


def test_pair_kernel_literal_model(gpu, orc, monkeypatch):
    """reference-literal 13/3/10 (nf = 30) through the paired kernel vs the one-QP kernel"""
    import mpcqp
    p = mpcqp.model_params("L", N=10)
    B = 257
    batch = mpcqp.make_batch(p, B, seed=3)
    monkeypatch.setenv("MPCQP_PAIR", "0")
    single = run_batch(p, batch)
    monkeypatch.delenv("MPCQP_PAIR")
    pair = run_batch(p, batch)
    np.testing.assert_array_equal(pair["status"], single["status"])
    sc = np.maximum(1.0, np.abs(single["U"]).max(axis=1, keepdims=True))
    assert np.all(np.abs(pair["U"] - single["U"]) <= 1e-10 * sc)
    ref = orc.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    refc = orc.srbm_batch(with_crash(p, pair["crash"]), batch["x0"], batch["xref"], batch["lin"],
                          batch["contact"])
    for i in range(B):
        assert u_close(pair["U"][i], ref["U"][i]), i
    assert np.mean(single["iters"] == ref["iters"]) >= 0.99
    assert np.mean(pair["iters"] == refc["iters"]) >= 0.99


def test_friction_rows_mixed_contact_vs_oracle(gpu, orc):
    """Config C (friction pyramid) with double-support and flight steps mixed into the gait:
    the one-QP solver evaluates each foot-step's four friction rows on the lane of its
    vertical force (neighbours' forces by DPP), which must give the oracle's optimum and
    iteration counts whatever the stance pattern (nf up to 64)."""
    import mpcqp
    p = mpcqp.model_params("C")
    p["max_free"] = 64
    B = 256
    batch = mpcqp.make_batch(p, B, seed=21)
    ct = batch["contact"].astype(np.uint64).copy()
    rng = np.random.default_rng(4)
    for i in range(B):
        ks = rng.choice(p["N"], 3, replace=False)
        ct[i] |= np.uint64(3 << (2 * int(ks[0])))      # double support
        ct[i] &= ~np.uint64(3 << (2 * int(ks[1])))     # flight
        if i % 2:
            ct[i] |= np.uint64(3 << (2 * int(ks[2])))  # a second double-support step
    nfree = np.array([3 * bin(int(c)).count("1") for c in ct])
    keep = nfree <= 64
    batch = {k: v[keep] for k, v in batch.items()}
    batch["contact"] = ct[keep]
    o = run_batch(p, batch)
    ref = orc.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    np.testing.assert_array_equal(o["status"], ref["status"])
    assert np.all(o["status"] == 0) and o["status"].size > 200
    bad = [i for i in range(o["U"].shape[0]) if not u_close(o["U"][i], ref["U"][i])]
    assert not bad, bad[:10]
    np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
    assert np.mean(o["iters"] == ref["iters"]) >= 0.99


def _prefilled(eng, batch):
    import torch
    d = eng.upload(batch)
    d["U"].fill_(float("nan"))
    d["cost"].fill_(float("nan"))
    d["status"].fill_(99)
    d["iters"].fill_(-1)
    torch.cuda.synchronize()
    return d


@pytest.mark.parametrize("config,B", [("B", 512), ("C", 384)])
def test_overflow_workgroup_kernel_vs_oracle(gpu, orc, config, B):
    """Every contact schedule (qpOASES takes the dense nV = NU*N problem
    whatever the bounds, src/QPSolver.cpp:87-96): alternating, double-support and standing
    candidates (gait "mixed") plus random extra double-support and flight steps.  Instances
    beyond the one-wave kernel's capacity (30 free forces for the paired kernel at N = 10, 64
    for k_mpc at N = 20) go through the overflow list: at N = 10 to the one-QP-per-wave
    k_mpc_list (up to 6N = 60 free forces), at N = 20 to the 4-wave workgroup kernel (up to
    120); every instance is written exactly once (sentinel pre-fill) and matches the oracle."""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params(config)
    batch = mpcqp.make_batch(p, B, seed=41, gait="mixed")
    ct = batch["contact"].astype(np.uint64).copy()
    rng = np.random.default_rng(43)
    for i in range(B):
        if i % 3 == 1:
            ct[i] |= np.uint64(3 << (2 * int(rng.integers(p["N"]))))   # double support
        if i % 5 == 2:
            ct[i] &= ~np.uint64(3 << (2 * int(rng.integers(p["N"]))))  # flight
    batch["contact"] = ct
    nfree = np.array([3 * bin(int(c)).count("1") for c in ct])
    cap = 30 if config == "B" else 64
    assert (nfree > cap).sum() > B // 5 and (nfree <= cap).sum() > B // 5
    assert nfree.max() == 6 * p["N"]  # standing candidates
    eng = BatchEngine(p)
    crash = eng.crash
    d = _prefilled(eng, batch)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    eng.close()
    ref = orc.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], ct)
    refc = orc.srbm_batch(with_crash(p, crash), batch["x0"], batch["xref"], batch["lin"], ct)
    assert np.all(ref["status"] == 0)
    np.testing.assert_array_equal(o["status"], ref["status"])
    assert np.all(np.isfinite(o["U"])) and np.all(o["iters"] >= 0)
    bad = [i for i in range(B) if not u_close(o["U"][i], ref["U"][i])]
    assert not bad, (bad[:10], nfree[bad[:10]])
    np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
    # iteration counts: the oracle run with the library's caps (the SRBM overflow kernels are
    # built without the workgroup crash unless MPCQP_WG_SRBM_CRASH=1, and never run it with
    # friction rows: config C)
    assert crash[2] == 0 or config == "B"
    big = nfree > cap
    assert np.mean(o["iters"][big] == refc["iters"][big]) >= 0.95


def test_overflow_full_size_mixed_gait(gpu, orc):
    """config C at batch 65,536 with the mixed gait (a quarter standing, nf = 120): every
    instance solved and written once, repeated calls re-arm the overflow list (identical
    results), a random sample matches the oracle"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("C")
    B = 65536
    batch = mpcqp.make_batch(p, B, seed=47, gait="mixed")
    eng = BatchEngine(p)
    d = _prefilled(eng, batch)
    eng.solve(d)
    eng.sync()
    U1 = d["U"].cpu().numpy().copy()
    st = d["status"].cpu().numpy().copy()
    it = d["iters"].cpu().numpy().copy()
    eng.solve(d)
    eng.sync()
    U2 = d["U"].cpu().numpy()
    eng.close()
    assert np.all(st == 0) and np.all(it >= 0) and np.all(np.isfinite(U1))
    np.testing.assert_array_equal(U1, U2)
    idx = np.random.default_rng(6).choice(B, 160, replace=False)
    sub = {k: batch[k][idx] for k in batch}
    ref = orc.srbm_batch(p, sub["x0"], sub["xref"], sub["lin"], sub["contact"])
    for j, i in enumerate(idx):
        assert u_close(U1[i], ref["U"][j]), i


# ------------------------------------------------------------- config E: the dense model
def test_dense_staged_solve_refused(gpu):
    """a dense (config E) context frees all 96 inputs, beyond the 64 of the stand-alone
    solve, so the staged entry points return BAD_DIMS instead of OK with every instance failing;
    mpcqp_batch_solve still serves it (k_dense_wg)"""
    import mpcqp
    from mpcqp._lib import MpcqpError
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("E")
    batch = mpcqp.make_batch(p, 4, seed=3)
    eng = BatchEngine(p)
    d = eng.upload(batch)
    H, f = eng.condense(d)
    with pytest.raises(MpcqpError) as e:
        eng.solve_qp(d, H, f)
    assert e.value.code == 1
    AB = eng.discretize(d)
    with pytest.raises(MpcqpError) as e:
        eng.condense_solve(d, AB)
    assert e.value.code == 1
    eng.solve(d)
    eng.sync()
    assert np.all(d["status"].cpu().numpy() == 0)
    eng.close()


def test_literal_empty_input_box_refused(gpu):
    """the literal model with u_min == u_max (every input fixed) is refused at
    create: the fused kernels read fixed inputs as 0"""
    import mpcqp
    from mpcqp._lib import MpcqpError
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("L", N=10)
    p["u_min"] = p["u_max"] = 2.0
    with pytest.raises(MpcqpError) as e:
        BatchEngine(p)
    assert e.value.code == 6


def test_dense_condense_vs_oracle(gpu, orc):
    """config E (24/6/16 whole-body model, dense Q/R/P): the generic condensing kernel
    (k_condense: Pade expm + Phi chain, full H to HBM) against the oracle's literal dense
    B'QB (src/QPSolver.cpp:31-81) at <= 1e-12"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("E")
    batch = mpcqp.make_batch(p, 48, seed=5)
    eng = BatchEngine(p)
    d = eng.upload(batch)
    H, f = eng.condense(d)
    eng.sync()
    Hg = H.cpu().numpy().transpose(0, 2, 1)
    fg = f.cpu().numpy()
    eng.close()
    ref = orc.dense_batch(p, batch["x0"], batch["xref"], batch["lin"], want_hf=True)
    for i in range(48):
        assert rel_err(Hg[i], ref["H"][i]) <= TOL_COND, i
        assert rel_err(fg[i], ref["f"][i]) <= TOL_COND, i


def test_dense_fused_vs_oracle(gpu, orc):
    """config E through the fused workgroup kernel (k_dense_wg: expm, MFMA condensing, 96-free-
    variable Goldfarb-Idnani): every instance solved and written once, U / cost / iterations
    against the oracle"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("E")
    B = 256
    batch = mpcqp.make_batch(p, B, seed=9)
    eng = BatchEngine(p)
    assert eng.fused_kernel == "k_dense_wg"
    crash = eng.crash
    d = _prefilled(eng, batch)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    eng.close()
    ref = orc.dense_batch(p, batch["x0"], batch["xref"], batch["lin"])
    assert np.all(ref["status"] == 0)
    np.testing.assert_array_equal(o["status"], ref["status"])
    assert ref["iters"].mean() > 3  # torque bounds bind
    bad = [i for i in range(B) if not u_close(o["U"][i], ref["U"][i])]
    assert not bad, bad[:10]
    np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
    # iteration counts against the oracle run with the workgroup solver's crash start
    assert crash[2] > 0
    refc = orc.dense_batch(with_crash(p, crash), batch["x0"], batch["xref"], batch["lin"])
    assert np.mean(o["iters"] == refc["iters"]) >= 0.95


def test_dense_full_weights_vs_oracle(gpu, orc):
    """config E with full symmetric Q and P (off-diagonal weights, Q rank-deficient PSD): the
    host factors them by Jacobi (Q = F F') for the Toeplitz condensing; U / cost / status
    against the oracle, which forms B'QB directly"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("E")
    rng = np.random.default_rng(31)
    nx = p["nx"]
    A = rng.standard_normal((nx, nx - 4))
    Q = 200.0 * (A @ A.T) / nx  # full, PSD of rank nx - 4 (zero eigenvalues)
    Bm = rng.standard_normal((nx, nx - 6))
    P = 100.0 * (Bm @ Bm.T) / nx + np.diag(np.r_[np.zeros(6), np.diag(p["P"])[6:]])  # full, PD
    p["Q"], p["P"] = 0.5 * (Q + Q.T), 0.5 * (P + P.T)
    B = 128
    batch = mpcqp.make_batch(p, B, seed=17)
    eng = BatchEngine(p)
    assert eng.fused_kernel == "k_dense_wg"
    d = _prefilled(eng, batch)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    eng.close()
    ref = orc.dense_batch(p, batch["x0"], batch["xref"], batch["lin"])
    np.testing.assert_array_equal(o["status"], ref["status"])
    assert np.all(ref["status"] == 0)
    bad = [i for i in range(B) if not u_close(o["U"][i], ref["U"][i])]
    assert not bad, bad[:10]
    np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)


def test_dense_full_size_properties(gpu, orc):
    """config E at its BASELINE batch (16,384): all solved, deterministic, sample vs oracle"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("E")
    B = 16384
    batch = mpcqp.make_batch(p, B, seed=13)
    eng = BatchEngine(p)
    d = _prefilled(eng, batch)
    eng.solve(d)
    eng.sync()
    U1 = d["U"].cpu().numpy().copy()
    st = d["status"].cpu().numpy().copy()
    eng.solve(d)
    eng.sync()
    U2 = d["U"].cpu().numpy()
    eng.close()
    assert np.all(st == 0)
    np.testing.assert_array_equal(U1, U2)
    idx = np.random.default_rng(2).choice(B, 96, replace=False)
    sub = {k: batch[k][idx] for k in batch}
    ref = orc.dense_batch(p, sub["x0"], sub["xref"], sub["lin"])
    for j, i in enumerate(idx):
        assert u_close(U1[i], ref["U"][j]), i


@pytest.mark.parametrize("config,gait,B,max_free", [
    ("B", None, 4097, None), ("B", "standing", 512, None), ("C", None, 384, None),
    ("C", "mixed", 384, None), ("L", None, 300, None), ("E", None, 64, None),
    ("B", None, 4097, 30), ("B", None, 33, 30), ("C", None, 384, 60)])
def test_solve_select_fused_record(gpu, config, gait, B, max_free):
    """mpcqp_batch_solve_select: the record the fused kernels build (keys min-ed per workgroup,
    the batch's last workgroup copies the winner's U; the workgroup kernel finalizes when
    instances overflow to it) equals k_select_min's record of the same solve and the host
    restatement, bit for bit; repeated calls re-arm (same record), index_base offsets the key.
    E runs the two-launch fallback, and so do contexts that cannot overflow (max_free within the
    one-wave kernel's capacity: no workgroup kernel)."""
    import torch
    import mpcqp
    from mpcqp.dist import host_record
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params(config)
    if max_free is not None:
        p["max_free"] = max_free
    nV = p["nu"] * p["N"]
    batch = mpcqp.make_batch(p, B, seed=41, gait=gait) if gait else mpcqp.make_batch(p, B, seed=41)
    eng = BatchEngine(p)
    d = _prefilled(eng, batch)
    dev = torch.device("cuda:0")
    for base in (0, 123_457, 0):
        rec = torch.full((1 + nV,), -1, dtype=torch.int64, device=dev)
        eng.solve_select(d, rec, index_base=base)
        eng.sync()
        got = rec.cpu().numpy()
        cost, status, U = (d[k].cpu().numpy() for k in ("cost", "status", "U"))
        assert np.all(status == 0)
        np.testing.assert_array_equal(got, host_record(cost, status, U, base))
        rec2 = torch.full((1 + nV,), -1, dtype=torch.int64, device=dev)
        eng.select_record(d, rec2, index_base=base)
        eng.sync()
        np.testing.assert_array_equal(got, rec2.cpu().numpy())
    eng.close()


@pytest.mark.parametrize("crash_p", ["0", "1", "2"])
def test_pair_crash_fallback_paths(gpu, orc, monkeypatch, crash_p):
    """the paired kernel's crash start capped at 0 / 1 / 2 working sets (MPCQP_CRASH_P): 0 is
    the plain dual loop (iteration counts equal the one-QP kernel's), 1 and 2 give up on most
    constrained instances and fall back to the dual loop from the unconstrained minimum (counts
    = working sets tried + dual passes).  U / cost equal the oracle's optimum everywhere, the
    iteration counts the oracle's run with the same caps."""
    import mpcqp
    p = mpcqp.model_params("B")
    B = 1024
    batch = mpcqp.make_batch(p, B, seed=41)
    monkeypatch.setenv("MPCQP_CRASH_P", crash_p)
    o = run_batch(p, batch)
    assert o["crash"][1] == int(crash_p)
    ref = orc.srbm_batch(with_crash(p, o["crash"]), batch["x0"], batch["xref"], batch["lin"],
                         batch["contact"])
    assert np.all(o["status"] == 0) and np.all(ref["status"] == 0)
    bad = [i for i in range(B) if not u_close(o["U"][i], ref["U"][i])]
    assert not bad, bad[:10]
    np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
    assert np.mean(o["iters"] == ref["iters"]) >= 0.99
    if crash_p == "0":
        plain = orc.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
        assert np.mean(o["iters"] == plain["iters"]) >= 0.99
    else:  # some instances fell back: more iterations than working sets
        assert (o["iters"] > int(crash_p)).any()


@pytest.mark.parametrize("crash_p", ["0", "1"])
def test_wg_crash_fallback_paths(gpu, orc, monkeypatch, crash_p):
    """the workgroup solver's crash start capped at 0 / 1 working sets (MPCQP_CRASH_P_WG) at B
    standing (every instance in the overflow kernel, NF = 64; built without the crash unless
    MPCQP_WG_SRBM_CRASH=1) and config E (NF = 96): 0 is the plain dual loop, 1 gives up on most
    instances; U / cost equal the oracle's optimum, the iteration counts the oracle run with the
    library's reported caps"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    monkeypatch.setenv("MPCQP_CRASH_P_WG", crash_p)
    for config, gait, B in (("B", "standing", 256), ("E", None, 96)):
        p = mpcqp.model_params(config)
        batch = mpcqp.make_batch(p, B, seed=53, gait=gait) if gait else \
            mpcqp.make_batch(p, B, seed=53)
        eng = BatchEngine(p)
        crash = eng.crash
        # the SRBM overflow kernels are built without the crash (crash[2] = 0: env ignored)
        assert crash[3] == (int(crash_p) if crash[2] > 0 else 0)
        assert crash[2] > 0 or config == "B"
        d = _prefilled(eng, batch)
        eng.solve(d)
        eng.sync()
        o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
        eng.close()
        args = (batch["x0"], batch["xref"], batch["lin"]) if config == "E" else \
            (batch["x0"], batch["xref"], batch["lin"], batch["contact"])
        fn = orc.dense_batch if config == "E" else orc.srbm_batch
        ref = fn(p, *args)
        refc = fn(with_crash(p, crash), *args)
        assert np.all(o["status"] == 0) and np.all(ref["status"] == 0)
        bad = [i for i in range(B) if not u_close(o["U"][i], ref["U"][i])]
        assert not bad, (config, bad[:10])
        np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
        assert np.mean(o["iters"] == refc["iters"]) >= 0.95, config
        if crash_p == "0":
            assert np.mean(o["iters"] == ref["iters"]) >= 0.95, config


@pytest.mark.gpu
def test_pair_kernel_ill_conditioned_vs_oracle(gpu, orc):
    """The paired kernel's pivot scales come from v_rsq_f64 + one Newton step (~1e-14 relative,
    wave_ops.hpp rsqrt_nr) and its J from the folded sweep: on a badly conditioned H_FF (R 1e-9 I
    against Q up to 1e4: condition ~1e9) the optimum still matches the oracle's (exact sqrt and
    divisions) to 1e-10 (3.9e-13 measured) -- guards tightening tolerances later"""
    import mpcqp
    p = mpcqp.model_params("B")
    p["R"] = 1e-9 * np.eye(p["nu"])
    p["Q"] = np.diag([1, 1, 1e4, 1e4, 1e4, 1e4, 50, 50, 50, 1e4, 1e4, 1e4, 0.1])
    p["P"] = 20.0 * p["Q"]
    batch = mpcqp.make_batch(p, 2048, seed=2026)
    out = run_batch(p, batch)
    ref = orc.srbm_batch(with_crash(p, out["crash"]), batch["x0"], batch["xref"], batch["lin"],
                         batch["contact"])
    ok = (ref["status"] == 0) & (out["status"] == 0)
    assert ok.mean() > 0.99
    sc = np.maximum(1.0, np.abs(ref["U"][ok]).max(axis=1))
    err = (np.abs(out["U"][ok] - ref["U"][ok]).max(axis=1) / sc).max()
    print(f"ill-conditioned H_FF: max rel U error {err:.3e}")
    assert err <= 1e-10, err  # (3.9e-13 measured at r05)
    np.testing.assert_allclose(out["cost"][ok], ref["cost"][ok], rtol=1e-8, atol=1e-8)
