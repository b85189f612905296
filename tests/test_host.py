"""Host-side logic: workload generator, gait schedule, selection key, model constants."""
import numpy as np
import pytest


def test_static_foot_offsets_match_mpcparam():
    """include/MPCParam.h:64-72 (left y is -0.105: the reference's sign kept)"""
    import mpcqp
    l, r = mpcqp.static_foot_offsets()
    np.testing.assert_allclose(l, [-0.02644, -0.105, -0.81181], atol=1e-12)
    np.testing.assert_allclose(r, [-0.02644, 0.105, -0.81181], atol=1e-12)


@pytest.mark.parametrize("phase", [0.0, 0.25, 0.4999, 0.495, 0.9955, 0.7, 0.123456])
def test_gait_mask_matches_oracle(orc, phase):
    import mpcqp
    for N, Ts in ((10, 0.001), (20, 0.001), (16, 0.01)):
        assert mpcqp.gait_contact_mask(N, Ts, phase) == orc.gait_contact_mask(N, Ts, phase)


def test_gait_one_foot_in_contact_every_step():
    """calculateGait (include/MPCController.h:61-75) has no double stance"""
    import mpcqp
    for ph in np.linspace(0, 1, 37):
        m = mpcqp.gait_contact_mask(10, 0.001, float(ph))
        for k in range(10):
            assert ((m >> (2 * k)) & 1) + ((m >> (2 * k + 1)) & 1) == 1


def test_workload_deterministic_and_shaped():
    import mpcqp
    p = mpcqp.model_params("B")
    a = mpcqp.make_batch(p, 100, seed=3)
    b = mpcqp.make_batch(p, 100, seed=3)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])
    assert a["x0"].shape == (100, 13) and a["xref"].shape == (100, 11, 13)
    assert a["lin"].shape == (100, 8) and a["contact"].dtype == np.uint64
    assert np.all(a["x0"][:, 12] == -9.8)
    # xref step 0 equals the state except vx (include/mpcQP.h:89-93)
    np.testing.assert_array_equal(a["xref"][:, 0, :], a["x0"])
    # candidates of one state share x0 and differ in phase
    np.testing.assert_array_equal(a["x0"][0], a["x0"][15])


def test_selection_key_orders_like_cost():
    from mpcqp.engine import decode_key, encode_key
    rng = np.random.default_rng(0)
    costs = np.concatenate([rng.normal(0, 100, 500), [0.0, -0.0, 1e-30, -1e-30, 3.5, 3.5]])
    keys = [encode_key(c, i) for i, c in enumerate(costs)]
    assert all(0 <= k < 2 ** 63 for k in keys)
    order_k = np.argsort(np.array(keys, dtype=np.int64), kind="stable")
    f32 = costs.astype(np.float32)
    order_c = np.lexsort((np.arange(len(costs)), f32))
    np.testing.assert_array_equal(f32[order_k], f32[order_c])
    for i in (0, 7, 501):
        c, idx = decode_key(keys[i])
        assert idx == i and c == pytest.approx(float(f32[i]))


def test_srbm_bounds_oracle_vs_golden(golden, orc):
    import mpcqp
    for fname in ("srbm_B.npz", "srbm_C.npz", "literal_L.npz"):
        g = golden(fname)
        p = mpcqp.model_params(str(g["config"]))
        for i in range(g["lb"].shape[0]):
            lb, ub = orc.srbm_bounds(p, int(g["contact"][i]))
            np.testing.assert_array_equal(lb, g["lb"][i])
            np.testing.assert_array_equal(ub, g["ub"][i])
