"""Multi-GPU min-cost selection.

The batch of (state, gait-candidate) QPs is sharded in contiguous ranges over the ranks (one
process per GPU); the solves need no communication.  The only exchange is the selection of the
global minimum-cost candidate: every rank reduces its shard to one 8-byte key on device
(mpcqp_batch_select_min), ONE MIN all-reduce (RCCL over xGMI for backend "nccl", gloo on CPU)
finds the global key, and the owning rank broadcasts its U row (nu*N doubles).

key = (order-preserving bits of float32(cost)) << 31 | global index  -- non-negative int64, so
a signed MIN is the lexicographic (cost, index) minimum: ties go to the lowest index, as in the
host reference (encode_key).
"""
from __future__ import annotations

import numpy as np

from .engine import decode_key, encode_key


def select_global(dist, key_tensor, U_local, per_rank: int, ubest):
    """All-reduce the local key (int64 tensor of shape [1]) with MIN, then broadcast the
    winner's U row into `ubest` on every rank.  Shards are equal (`per_rank` instances, rank r
    owns global indices [r*per_rank, (r+1)*per_rank)).  Returns (cost_f32, global_index)."""
    dist.all_reduce(key_tensor, op=dist.ReduceOp.MIN)
    cost, gidx = decode_key(int(key_tensor.item()))
    owner = gidx // per_rank
    if owner == dist.get_rank():
        ubest.copy_(U_local[gidx - owner * per_rank])
    dist.broadcast(ubest, src=owner)
    return cost, gidx


def host_keys(costs, status, index_base: int = 0):
    """host restatement of k_select_min over one shard (min key, INT64_MAX if none valid)"""
    best = 0x7FFFFFFFFFFFFFFF
    for i, (c, s) in enumerate(zip(costs, status)):
        if s == 0:
            best = min(best, encode_key(float(c), index_base + i))
    return best


def host_select(costs, status):
    """reference: global (float32 cost, lowest index) minimum over valid instances"""
    c = np.asarray(costs, dtype=np.float64).astype(np.float32)
    ok = np.asarray(status) == 0
    idx = np.nonzero(ok)[0]
    j = idx[np.lexsort((idx, c[idx]))[0]]
    return float(c[j]), int(j)
