"""inputs generated on device (mpcqp_batch_solve_gait), per-state
selection, the SRBM plant step and the batched closed loop (mpcqp_rollout).

CPU: the host mirror of the generated inputs (workload.gait_inputs) equals make_batch's inputs
for the same seed.  GPU: the generated path equals the explicit-input path on the mirrored
inputs; the selection follows the host rule; the plant step equals the oracle's exact-ZOH step
(orc_srbm_plant, Eigen-expm restatement); every rollout tick is re-derived by the oracle from
the GPU's own state.  Tolerances (fp64): U <= 1e-10 abs (same QP, inputs built by identical
formulas), plant step <= 1e-12 relative, rollout ticks <= 1e-9 relative."""
import numpy as np
import pytest


def test_gait_inputs_mirror_make_batch():
    import mpcqp
    for cfg in ("B", "C"):
        p = mpcqp.model_params(cfg)
        g = mpcqp.make_gait_states(p, 8, seed=7, candidates=16)
        a = mpcqp.gait_inputs(p, g)
        b = mpcqp.make_batch(p, 8 * 16, seed=7, candidates=16)
        for k in ("x0", "xref", "lin"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        np.testing.assert_array_equal(a["contact"], b["contact"])


def _host_select(cost, status, C):
    S = cost.shape[0] // C
    best = np.full(S, -1)
    for s in range(S):
        c32 = cost[s * C:(s + 1) * C].astype(np.float32)
        ok = np.nonzero(status[s * C:(s + 1) * C] == 0)[0]
        if ok.size:
            best[s] = ok[np.lexsort((ok, c32[ok]))[0]]
    return best


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["B", "C"])
def test_solve_gait_matches_explicit(gpu, cfg):
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params(cfg)
    g = mpcqp.make_gait_states(p, 256, seed=11, candidates=16)
    eng = BatchEngine(p)
    dg = eng.upload_gait(g)
    eng.solve_gait(dg)
    d = eng.upload(mpcqp.gait_inputs(p, g))
    eng.solve(d)
    eng.sync()
    np.testing.assert_array_equal(dg["status"].cpu().numpy(), d["status"].cpu().numpy())
    np.testing.assert_allclose(dg["U"].cpu().numpy(), d["U"].cpu().numpy(), rtol=0, atol=1e-10)
    np.testing.assert_allclose(dg["cost"].cpu().numpy(), d["cost"].cpu().numpy(), rtol=1e-12,
                               atol=1e-12)
    # per-state selection
    eng.select_state(dg)
    eng.sync()
    cost = dg["cost"].cpu().numpy()
    st = dg["status"].cpu().numpy()
    best = dg["best"].cpu().numpy()
    np.testing.assert_array_equal(best, _host_select(cost, st, 16))
    U = dg["U"].cpu().numpy().reshape(256, 16, -1)
    np.testing.assert_array_equal(dg["Ubest"].cpu().numpy(), U[np.arange(256), best])
    eng.close()


@pytest.mark.gpu
def test_solve_gait_metric_batch_matches_explicit(gpu):
    """metric batch (4096 states x 16 candidates = 65536): the on-chip generated path writes
    every instance (outputs pre-filled with sentinels) and equals the explicit-input path"""
    import torch
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    g = mpcqp.make_gait_states(p, 4096, seed=29, candidates=16)
    eng = BatchEngine(p)
    dg = eng.upload_gait(g)
    dg["U"].fill_(float("nan"))
    dg["status"].fill_(99)
    torch.cuda.synchronize()
    eng.solve_gait(dg)
    d = eng.upload(mpcqp.gait_inputs(p, g))
    eng.solve(d)
    eng.sync()
    st = dg["status"].cpu().numpy()
    assert st.shape == (65536,) and np.all(st == 0)
    np.testing.assert_array_equal(st, d["status"].cpu().numpy())
    np.testing.assert_allclose(dg["U"].cpu().numpy(), d["U"].cpu().numpy(), rtol=0, atol=1e-10)
    np.testing.assert_allclose(dg["cost"].cpu().numpy(), d["cost"].cpu().numpy(), rtol=1e-12,
                               atol=1e-12)
    eng.close()


@pytest.mark.gpu
def test_plant_srbm_matches_oracle(gpu, orc):
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    S, Cc = 64, 4
    g = mpcqp.make_gait_states(p, S, seed=3, candidates=Cc)
    eng = BatchEngine(p)
    dg = eng.upload_gait(g)
    eng.solve_gait(dg)
    eng.select_state(dg)
    eng.sync()
    Ub = dg["Ubest"].cpu().numpy()
    eng.plant(dg)
    eng.sync()
    xs = dg["state"].cpu().numpy()
    for s in range(S):
        lin = np.concatenate([[g["state"][s, 2]], g["feet"][s], [0.0]])
        x1 = orc.srbm_plant(p, lin, g["state"][s], Ub[s, :6])
        np.testing.assert_allclose(xs[s], x1, rtol=1e-12, atol=1e-12)
        dp = x1[3:6] - g["state"][s, 3:6]
        np.testing.assert_allclose(dg["feet"].cpu().numpy()[s],
                                   g["feet"][s] - np.tile(dp, 2), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(dg["phase"].cpu().numpy(), g["phase"] + p["Ts"], rtol=0,
                               atol=1e-15)
    eng.close()


@pytest.mark.gpu
def test_rollout_ticks_rederived_by_oracle(gpu, orc):
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    S, Cc, K = 24, 8, 6
    g = mpcqp.make_gait_states(p, S, seed=5, candidates=Cc)
    eng = BatchEngine(p)
    dg = eng.upload_gait(g)
    traj, choice = eng.rollout(dg, K)
    eng.sync()
    traj = traj.cpu().numpy()
    choice = choice.cpu().numpy()
    state, feet, phase = g["state"].copy(), g["feet"].copy(), g["phase"].copy()
    for k in range(K):
        gi = mpcqp.gait_inputs(p, dict(state=state, feet=feet, cmd=g["cmd"], phase=phase))
        ref = orc.srbm_batch(p, gi["x0"], gi["xref"], gi["lin"], gi["contact"])
        hb = _host_select(ref["cost"], ref["status"], Cc)
        for s in range(S):
            if choice[k, s] != hb[s]:  # only an fp32 near-tie may differ
                c = ref["cost"][s * Cc:(s + 1) * Cc]
                assert abs(c[choice[k, s]] - c[hb[s]]) <= 1e-6 * max(1.0, abs(c[hb[s]])), (k, s)
        nxt = np.empty_like(state)
        for s in range(S):
            u = ref["U"][s * Cc + choice[k, s]][:6]
            lin = np.concatenate([[state[s, 2]], feet[s], [0.0]])
            nxt[s] = orc.srbm_plant(p, lin, state[s], u)
        np.testing.assert_allclose(traj[k], nxt, rtol=1e-9, atol=1e-9)
        # continue from the GPU's own state (re-derivation, not a free-running comparison)
        dp = traj[k][:, 3:6] - state[:, 3:6]
        feet = feet - np.tile(dp, (1, 2))
        state = traj[k].copy()
        phase = phase + p["Ts"]
    eng.close()


def _closed_loop_iters(p, g, K, warm, orc=None):
    """K ticks of solve_gait -> select_state -> plant on one context (the mpcqp_rollout loop),
    optionally warm-started; every tick's U / cost re-derived by the oracle when orc is given.
    Returns the per-tick iteration totals."""
    import mpcqp
    from mpcqp.engine import BatchEngine
    eng = BatchEngine(p)
    eng.set_warm_start(warm)
    dg = eng.upload_gait(g)
    totals = []
    for k in range(K):
        if orc is not None:
            gi = mpcqp.gait_inputs(p, dict(state=dg["state"].cpu().numpy(),
                                           feet=dg["feet"].cpu().numpy(), cmd=g["cmd"],
                                           phase=dg["phase"].cpu().numpy()))
        eng.solve_gait(dg)
        eng.select_state(dg)
        eng.sync()
        it = dg["iters"].cpu().numpy()
        totals.append(int(it.sum()))
        if orc is not None:
            ref = orc.srbm_batch(p, gi["x0"], gi["xref"], gi["lin"], gi["contact"])
            st = dg["status"].cpu().numpy()
            np.testing.assert_array_equal(st, ref["status"])
            U = dg["U"].cpu().numpy()
            err = np.abs(U - ref["U"]).max(axis=1) / np.maximum(1.0, np.abs(ref["U"]).max(axis=1))
            assert err.max() <= 1e-8, (k, err.max())
            np.testing.assert_allclose(dg["cost"].cpu().numpy(), ref["cost"], rtol=1e-9, atol=1e-9)
        eng.plant(dg)
    eng.sync()
    eng.close()
    return np.array(totals)


@pytest.mark.gpu
def test_rollout_warm_start_matches_oracle_and_saves_passes(gpu, orc):
    """Warm start of the closed loop (mpcqp_set_warm_start) at config C:
    every tick's plans equal the oracle's cold solve of the same inputs (unique optimum), the
    first tick is cold (identical iteration count), and the warm ticks take fewer dual passes
    than the cold loop over the same ticks (tools/warm_start_ab.py: up to 53 % fewer with every
    contact foot's fz >= 0 bound in the set; since that bound is left out -- its pyramid implies
    it, gi_setup -- the cold loop needs ~45 % fewer passes itself and warm saves ~6 % more
    here: 5,824 vs 6,224 passes over ticks 1-7)."""
    import mpcqp
    p = mpcqp.model_params("C")
    S, Cc, K = 32, 8, 8
    g = mpcqp.make_gait_states(p, S, seed=9, candidates=Cc)
    warm = _closed_loop_iters(p, g, K, True, orc)
    cold = _closed_loop_iters(p, g, K, False)
    assert warm[0] == cold[0]
    assert warm[1:].sum() < 0.97 * cold[1:].sum(), (warm, cold)


@pytest.mark.gpu
def test_rollout_warm_start_seeds_the_pair_crash(gpu, orc):
    """Warm start at config B (the paired kernel): the previous tick's
    active bounds, one horizon step later, join the crash start's first working set
    (mpc_pair.hpp).  Every tick's plans equal the oracle's cold solve of the same inputs (the
    unique optimum), tick 0 is cold (identical iteration count), and ticks 1-7 take >= 20 %
    fewer working sets + passes than the cold loop (0.73x measured: 16,108 vs 22,056 at 256
    states x 16 candidates, tools/warm_iters.py)."""
    import mpcqp
    p = mpcqp.model_params("B")
    S, Cc, K = 64, 16, 8
    g = mpcqp.make_gait_states(p, S, seed=11, candidates=Cc)
    warm = _closed_loop_iters(p, g, K, True, orc)
    cold = _closed_loop_iters(p, g, K, False)
    assert warm[0] == cold[0]
    assert warm[1:].sum() <= 0.8 * cold[1:].sum(), (warm, cold)


@pytest.mark.gpu
def test_pair_kernel_solver_flops_count_matches_oracle(gpu, orc):
    """k_mpc_pair's diagnostic solver-flops counter (mpcqp_count_solver_flops: crash working-set
    solves and dual passes, per instance with its own free count) against the oracle's count of
    the same formulas over its own decisions with the kernel's crash caps (iteration counts
    agree on >= 99 % of instances, so the totals agree closely)"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    b = mpcqp.make_batch(p, 4096, seed=91)
    eng = BatchEngine(p)
    d = eng.upload(b)
    eng.count_solver_flops(True)
    eng.solve(d)
    got, launches = eng.solver_flops()
    eng.count_solver_flops(False)
    assert launches == 1
    eng.solve(d)  # counting off: nothing added
    assert eng.solver_flops() == (0.0, 0)
    pc = dict(p)
    pc["crash"] = eng.crash
    ref = orc.srbm_batch(pc, b["x0"], b["xref"], b["lin"], b["contact"], want_flops=True)
    eng.close()
    want = float(ref["solver_flops"].sum())
    assert want > 0 and abs(got - want) <= 0.01 * want, (got, want)
