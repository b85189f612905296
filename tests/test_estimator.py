"""batched leg kinematics (mpcqp_fk_feet) and the 12-state Kalman
filter of stateEstimator::update (mpcqp_kf_update, include/stateEstimator.h:217-337).

Pinning: FK at q = 0 equals MPCParam's static_foot_offset_{left,right} (include/MPCParam.h:
64-72) -- the reference's own formula; joint axes beyond that are build-chosen (the URDF is not
in the repository): parity unpinned there, checked against the oracle's restatement.  The KF is
restated as written (oracle/mpcqp_oracle.c, orc_kf_update); no reference vectors exist for it
(parity unpinned w.r.t. the binary).  Tolerances (fp64): FK <= 1e-14 abs, KF <= 1e-10
relative (14x14 LU with different elimination order)."""
import numpy as np
import pytest


def _robots(R, seed):
    rng = np.random.default_rng(seed)
    q = rng.uniform(-0.6, 0.6, (R, 6))
    rpy = np.stack([rng.uniform(-0.2, 0.2, R), rng.uniform(-0.2, 0.2, R),
                    rng.uniform(-np.pi, np.pi, R)], 1)
    xhat = rng.normal(0, 0.3, (R, 12))
    A = rng.normal(0, 0.3, (R, 12, 12))
    P = np.einsum("rij,rkj->rik", A, A) + 0.1 * np.eye(12)
    eeP = rng.normal(0, 0.4, (R, 6))
    eeV = rng.normal(0, 0.2, (R, 6))
    contact = rng.integers(0, 2, (R, 2)).astype(np.uint8)
    qu = rng.normal(0, 1, (R, 4))
    qu[:, 3] += 3.0
    qu /= np.linalg.norm(qu, axis=1, keepdims=True)
    acc = rng.normal(0, 1, (R, 3)) + np.array([0, 0, 9.8])
    return q, rpy, xhat, P, eeP, eeV, contact, qu, acc


def test_fk_zero_is_static_offsets(orc):
    import mpcqp
    l, r = mpcqp.static_foot_offsets()
    f = orc.fk_feet(np.zeros(6), np.zeros(3))
    np.testing.assert_allclose(f, np.concatenate([l, r]), rtol=0, atol=1e-15)


def test_kf_oracle_keeps_covariance_symmetric(orc):
    _, _, xhat, P, eeP, eeV, contact, qu, acc = _robots(4, 1)
    for r in range(4):
        x1, P1 = orc.kf_update(0.002, xhat[r], P[r], eeP[r], eeV[r], contact[r], qu[r], acc[r])
        np.testing.assert_array_equal(P1, P1.T)
        assert np.all(np.isfinite(x1))


@pytest.mark.gpu
def test_fk_feet_matches_oracle(gpu, orc):
    import mpcqp
    from mpcqp.estimator import fk_feet
    torch = gpu
    R = 300
    q, rpy, *_ = _robots(R, 2)
    dq = torch.from_numpy(q).cuda()
    f = fk_feet(dq, torch.from_numpy(rpy).cuda()).cpu().numpy()
    for r in range(R):
        np.testing.assert_allclose(f[r], orc.fk_feet(q[r], rpy[r]), rtol=0, atol=1e-14)
    # a [R,13] state as the attitude source (row stride 13), and q = 0 -> static offsets
    st = np.zeros((R, 13))
    st[:, 0:3] = rpy
    f2 = fk_feet(dq, torch.from_numpy(st).cuda()).cpu().numpy()
    np.testing.assert_array_equal(f2, f)
    z = fk_feet(torch.zeros((2, 6), dtype=torch.float64).cuda(),
                torch.zeros((2, 3), dtype=torch.float64).cuda()).cpu().numpy()
    l, rr = mpcqp.static_foot_offsets()
    np.testing.assert_allclose(z, np.tile(np.concatenate([l, rr]), (2, 1)), rtol=0, atol=1e-15)


@pytest.mark.gpu
def test_kf_update_matches_oracle(gpu, orc):
    from mpcqp.estimator import kf_update
    torch = gpu
    R = 256
    _, _, xhat, P, eeP, eeV, contact, qu, acc = _robots(R, 3)
    P[:8] *= 1e-4  # small covariances: the det(P(0:2,0:2)) <= 1e-6 branch too
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    dx = dev(xhat)
    dP = dev(np.ascontiguousarray(P.transpose(0, 2, 1)))  # column-major per robot
    kf_update(0.002, dx, dP, dev(eeP), dev(eeV), dev(contact), dev(qu), dev(acc))
    torch.cuda.synchronize()
    gx = dx.cpu().numpy()
    gP = dP.cpu().numpy().transpose(0, 2, 1)
    branches = set()
    for r in range(R):
        x1, P1 = orc.kf_update(0.002, xhat[r], P[r], eeP[r], eeV[r], contact[r], qu[r], acc[r])
        np.testing.assert_allclose(gx[r], x1, rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(gP[r], P1, rtol=1e-10, atol=1e-12 * np.abs(P1).max())
        branches.add(bool(P1[0, 2] == 0.0))
    assert branches == {True, False}
