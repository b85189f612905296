"""Producers either side of the MPC step, batched on the GPU:
leg kinematics (foot lever arms for the gait path) and the 12-state Kalman filter of
stateEstimator::update (include/stateEstimator.h:217-337).  Inputs are torch tensors on the
device (plumbing); the compute is libmpcqp.so's k_fk_feet / k_kf_update."""
from __future__ import annotations

import ctypes as C

from ._lib import check, lib


def _p(t):
    return C.c_void_p(t.data_ptr())


def _stream(t):
    import torch
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def fk_feet(q, rpy, feet=None):
    """q [R,6] (abad, hip, knee; left then right), rpy [R,3] or a state [R,13] -> feet [R,6]
    (foot contact points minus base, world frame)"""
    import torch
    R = q.shape[0]
    if feet is None:
        feet = torch.empty((R, 6), dtype=torch.float64, device=q.device)
    stride = rpy.shape[1]
    check("mpcqp_fk_feet", lib().mpcqp_fk_feet(_stream(q), R, _p(q), _p(rpy), stride, _p(feet)))
    return feet


def kf_update(dt, xhat, P, eePos, eeVel, contact, quat, acc):
    """one estimator step for R robots, in place on xhat [R,12] and P [R,12,12] (stored
    column-major per robot: pass P as the transpose view's contiguous copy, see tests)"""
    R = xhat.shape[0]
    check("mpcqp_kf_update", lib().mpcqp_kf_update(
        _stream(xhat), R, float(dt), _p(xhat), _p(P), _p(eePos), _p(eeVel), _p(contact),
        _p(quat), _p(acc)))
