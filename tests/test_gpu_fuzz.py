"""Randomised parity: the fused fast path under perturbed physical parameters, odd batch sizes
and every contact pattern, against the CPU oracle on the same inputs.

Each case draws (seeded) a configuration (B, C or L), a body mass, inertia, friction
coefficient, force / torque bounds (a positive minimum normal force included), sampling time,
diagonal weights, a batch size that is not a multiple of the wavefront pairing or of the
candidate group, and a gait.  The host-computed kernel constants (bound values, violation
thresholds, selection keys), the pairing of instances into wavefronts, the overflow routing and
the crash start all see values the fixed-config tests never use.  Tolerances are those of
test_gpu_parity.py: ||dU||_inf <= 1e-8 max(1, ||U||_inf), cost 1e-9 relative; statuses equal.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL_U = 1e-8


def _draw(seed):
    import mpcqp
    rng = np.random.default_rng(7000 + seed)
    config = ("B", "C", "L", "B", "C", "B", "L", "B")[seed % 8]
    p = mpcqp.model_params(config)
    nx, nu = p["nx"], p["nu"]
    p["mass"] *= rng.uniform(0.7, 1.4)
    p["Ib"] = np.asarray(p["Ib"], float) * rng.uniform(0.7, 1.4)
    p["Ts"] *= rng.uniform(0.6, 1.8)
    if config == "L":
        lim = rng.uniform(3.0, 15.0)
        p["u_min"], p["u_max"] = -lim, lim
    else:
        p["mu"] = rng.uniform(0.3, 1.0)
        p["fz_max"] *= rng.uniform(0.5, 1.5)
        p["fxy_max"] = p["mu"] * p["fz_max"] * rng.uniform(0.8, 1.2)
        if seed % 3 == 2:
            p["fz_min"] = rng.uniform(1.0, 20.0)  # a minimum normal force in stance
    qd = np.diag(p["Q"]) * rng.uniform(0.3, 3.0, nx)
    p["Q"] = np.diag(qd)
    p["P"] = np.diag(qd * rng.uniform(5.0, 30.0))
    p["R"] = np.asarray(p["R"], float) * rng.uniform(0.5, 2.0)
    B = int(rng.choice([1, 3, 31, 33, 63, 127, 129, 255, 333, 511]))
    gait = "alternating" if config == "L" else str(rng.choice(
        ["alternating", "double", "mixed", "standing"]))
    if config == "C" and gait in ("mixed", "standing"):
        B = min(B, 129)  # standing at N = 20: ~70 dual passes per instance in the oracle
    batch = mpcqp.make_batch(p, B, seed=8000 + seed, gait=gait)
    return p, batch, gait


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_params_vs_oracle(gpu, orc, seed):
    from mpcqp.engine import BatchEngine
    p, batch, gait = _draw(seed)
    eng = BatchEngine(p)
    crash = eng.crash
    d = eng.upload(batch)
    d["U"].fill_(float("nan"))
    d["status"].fill_(99)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    fast = eng.fast_path
    eng.close()
    q = dict(p)
    q["crash"] = tuple(crash)
    ref = orc.srbm_batch(q, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    tag = (p["config"], gait, batch["x0"].shape[0], fast)
    np.testing.assert_array_equal(o["status"], ref["status"], err_msg=str(tag))
    ok = ref["status"] == 0
    assert ok.mean() >= 0.9, tag
    for i in np.flatnonzero(ok):
        scale = max(1.0, np.abs(ref["U"][i]).max())
        assert np.abs(o["U"][i] - ref["U"][i]).max() <= TOL_U * scale, (tag, i)
    np.testing.assert_allclose(o["cost"][ok], ref["cost"][ok], rtol=1e-9, atol=1e-9,
                               err_msg=str(tag))
    assert np.mean(o["iters"][ok] == ref["iters"][ok]) >= 0.95, tag


def test_zero_friction_coefficient_vs_oracle(gpu, orc):
    """mu = 0: the friction rows pin fx, fy only, so the fz lower bound must stay in the problem
    (the implied-bound elision requires mu > 0); with the body moving up the unconstrained
    optimum pulls it down, and the solvers must still return fz >= fz_min"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("C")
    p["mu"] = 0.0
    batch = mpcqp.make_batch(p, 256, seed=9001)
    batch["x0"][:, 11] = 3.0
    eng = BatchEngine(p)
    d = eng.upload(batch)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    eng.close()
    ref = orc.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    np.testing.assert_array_equal(o["status"], ref["status"])
    assert np.all(o["status"] == 0)
    fz = o["U"].reshape(len(o["U"]), p["N"], 2, 3)[..., 2]
    assert fz.min() >= p["fz_min"] - 1e-8
    for i in range(len(o["U"])):
        scale = max(1.0, np.abs(ref["U"][i]).max())
        assert np.abs(o["U"][i] - ref["U"][i]).max() <= TOL_U * scale, i
    np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)


def _draw_dense(seed):
    """config E with the sampling time, torque bound and diagonal weights perturbed, odd batch"""
    import mpcqp
    rng = np.random.default_rng(9100 + seed)
    p = mpcqp.model_params("E")
    nx = p["nx"]
    p["Ts"] *= rng.uniform(0.5, 2.0)
    lim = p["u_max"] * rng.uniform(0.5, 2.0)
    p["u_min"], p["u_max"] = -lim, lim
    qd = np.diag(p["Q"]) * rng.uniform(0.3, 3.0, nx)
    p["Q"] = np.diag(qd)
    p["P"] = np.diag(qd * rng.uniform(3.0, 20.0))
    p["R"] = np.asarray(p["R"], float) * rng.uniform(0.5, 2.0)
    B = int(rng.choice([1, 7, 33, 65, 127, 191]))
    return p, mpcqp.make_batch(p, B, seed=9200 + seed)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_dense_vs_oracle(gpu, orc, seed):
    """config E (the dense whole-body model: expm, Toeplitz condensing, 96-variable solve) with
    the sampling time, torque bound and diagonal weights perturbed and odd batch sizes; U / cost
    / status against the oracle, iteration counts with the workgroup crash caps"""
    from mpcqp.engine import BatchEngine
    p, batch = _draw_dense(seed)
    B, lim = batch["x0"].shape[0], p["u_max"]
    eng = BatchEngine(p)
    crash = eng.crash
    d = eng.upload(batch)
    d["U"].fill_(float("nan"))
    d["status"].fill_(99)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    eng.close()
    q = dict(p)
    q["crash"] = tuple(crash)
    ref = orc.dense_batch(q, batch["x0"], batch["xref"], batch["lin"])
    tag = (B, float(p["Ts"]), float(lim))
    np.testing.assert_array_equal(o["status"], ref["status"], err_msg=str(tag))
    ok = ref["status"] == 0
    assert ok.mean() >= 0.9, tag
    for i in np.flatnonzero(ok):
        scale = max(1.0, np.abs(ref["U"][i]).max())
        assert np.abs(o["U"][i] - ref["U"][i]).max() <= TOL_U * scale, (tag, i)
    np.testing.assert_allclose(o["cost"][ok], ref["cost"][ok], rtol=1e-9, atol=1e-9,
                               err_msg=str(tag))
    assert np.mean(o["iters"][ok] == ref["iters"][ok]) >= 0.95, tag


@pytest.mark.parametrize("config,max_iter", [("B", 2), ("C", 2), ("C", 4), ("L", 2), ("L", 5)])
def test_iteration_cap_vs_oracle(gpu, orc, config, max_iter):
    """mpcqp_model.max_iter small enough to bind: the same instances stop at the cap
    (ST_ITER_LIMIT) in the kernels and the oracle -- the crash start's working sets count as
    iterations and the dual loop stops once the count reaches the cap -- and the others match"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params(config)
    p["max_iter"] = max_iter
    batch = mpcqp.make_batch(p, 512, seed=9300 + max_iter)
    eng = BatchEngine(p)
    crash = eng.crash
    d = eng.upload(batch)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    eng.close()
    q = dict(p)
    q["crash"] = tuple(crash)
    ref = orc.srbm_batch(q, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    assert np.mean(o["status"] == ref["status"]) >= 0.99
    both = (o["status"] == 0) & (ref["status"] == 0)
    assert both.mean() > 0.25
    for i in np.flatnonzero(both):
        scale = max(1.0, np.abs(ref["U"][i]).max())
        assert np.abs(o["U"][i] - ref["U"][i]).max() <= TOL_U * scale, i
    if config != "B":
        assert np.any(ref["status"] == 3)  # the cap binds


@pytest.mark.parametrize("config,N", [("B", 5), ("B", 8), ("B", 15), ("C", 12), ("L", 6), ("L", 13)])
def test_other_horizons_vs_oracle(gpu, orc, config, N):
    """horizons without a compile-time kernel run the generic runtime-dimension kernels (batched
    condensing + the one-wave solver, up to 64 free variables): U / cost / status against the
    oracle, iteration counts equal"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params(config, N=N)
    if config != "L":
        p["max_free"] = min(64, 3 * N)  # the alternating gait: one stance foot per step
    batch = mpcqp.make_batch(p, 97, seed=9400 + N)
    eng = BatchEngine(p)
    d = eng.upload(batch)
    eng.solve(d)
    eng.sync()
    o = {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}
    eng.close()
    ref = orc.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    np.testing.assert_array_equal(o["status"], ref["status"])
    assert np.all(o["status"] == 0)
    for i in range(len(o["U"])):
        scale = max(1.0, np.abs(ref["U"][i]).max())
        assert np.abs(o["U"][i] - ref["U"][i]).max() <= TOL_U * scale, i
    np.testing.assert_allclose(o["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
    assert np.mean(o["iters"] == ref["iters"]) >= 0.95
