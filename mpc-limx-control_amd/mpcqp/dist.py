"""Multi-GPU min-cost selection.

The batch of (state, gait-candidate) QPs is sharded in contiguous ranges over the ranks (one
process per GPU, ranges aligned to whole states); the solves need no communication.  The only
exchange is the selection of the global minimum-cost candidate, in ONE collective:

  1. each rank reduces its shard on device to a record [key | winner's U]
     (mpcqp_batch_select_record: key = order-preserving bits of float32(cost) << 31 | global
     index; U row nu*N doubles; an all-invalid shard gives key INT64_MAX and U = 0),
  2. one all-gather of the records (RCCL over xGMI for backend "nccl", gloo on CPU),
  3. every rank picks the minimum key's record on device (mpcqp_reduce_records).

No `.item()`, no host synchronisation and no owner broadcast inside the step.  Keys are
non-negative int64, so the minimum is the lexicographic (fp32 cost, global index) minimum:
ties go to the lowest index, as in the host reference (host_select).
"""
from __future__ import annotations

import numpy as np

from .engine import decode_key, encode_key

NO_KEY = 0x7FFFFFFFFFFFFFFF


def select_global(dist, record, gathered, best, reduce):
    """record: int64 [1 + nV] of this rank; gathered: int64 [world, 1 + nV] buffer; best:
    int64 [1 + nV] output (same on every rank); reduce(gathered, best): the device (or host)
    record reduction.  One collective."""
    dist.all_gather_into_tensor(gathered.view(-1), record)
    reduce(gathered, best)
    return best


class PipelinedSelect:
    """select_global over a stream of independent batches with the collective of batch s in
    flight while batch s + 1 solves.

    Two record / gather buffers alternate.  submit() starts batch s's all-gather asynchronously
    (the backend orders it after the solve that wrote the record: RCCL waits on the current
    stream) and then completes batch s - 1: work.wait() makes the current stream wait for that
    collective, and the device reduction into `best` follows it.  So solve(s + 1), enqueued
    after submit(s), waits only for the all-gather of s - 1, and the all-gather of s overlaps
    it.  drain() completes the last batch.  Still one collective per batch; every batch's
    selection is complete when drain() returns.  Buffer reuse is safe: record[i] is rewritten
    by solve(s + 2), which the stream orders after wait(s); gathered[i] is refilled by the
    all-gather of s + 2, which RCCL orders after the reduction of s on the current stream.
    done: the number of batches whose selection has been reduced into `best`."""

    def __init__(self, dist, records, gathered, best, reduce):
        self.dist, self.records, self.gathered = dist, records, gathered
        self.best, self.reduce = best, reduce
        self.i = 0
        self.pending = None
        self.done = 0

    def record(self):
        """the record buffer the next batch's solve writes"""
        return self.records[self.i]

    def submit(self):
        i = self.i
        work = self.dist.all_gather_into_tensor(self.gathered[i].view(-1), self.records[i],
                                                async_op=True)
        self.drain()
        self.pending = (work, i)
        self.i ^= 1

    def drain(self):
        if self.pending is not None:
            work, j = self.pending
            work.wait()
            self.reduce(self.gathered[j], self.best)
            self.pending = None
            self.done += 1
        return self.best


def decode_record(best) -> tuple:
    """(float32 cost or inf, global index or -1, U row float64) from a selection record"""
    b = np.asarray(best, dtype=np.int64)
    key = int(b[0])
    U = b[1:].view(np.float64).copy()
    if key == NO_KEY:
        return float("inf"), -1, U
    c, i = decode_key(key)
    return c, i, U


def host_record(costs, status, U, index_base: int = 0):
    """host restatement of mpcqp_batch_select_record over one shard"""
    U = np.asarray(U, dtype=np.float64)
    nV = U.shape[1] if U.ndim == 2 else 0
    rec = np.zeros(1 + nV, dtype=np.int64)
    key = host_keys(costs, status, index_base)
    rec[0] = key
    if key != NO_KEY:
        li = (key & 0x7FFFFFFF) - index_base
        rec[1:] = U[li].view(np.int64)
    return rec


def host_reduce_records(gathered, best):
    """host restatement of mpcqp_reduce_records (numpy or CPU torch int64 arrays)"""
    g = gathered.numpy() if hasattr(gathered, "numpy") else np.asarray(gathered)
    j = int(np.argmin(g[:, 0].astype(np.uint64)))
    if hasattr(best, "copy_"):
        import torch
        best.copy_(torch.from_numpy(g[j].copy()))
    else:
        best[...] = g[j]
    return best


def host_keys(costs, status, index_base: int = 0):
    """host restatement of k_select_min over one shard (min key, INT64_MAX if none valid)"""
    best = NO_KEY
    for i, (c, s) in enumerate(zip(costs, status)):
        if s == 0:
            best = min(best, encode_key(float(c), index_base + i))
    return best


def host_select(costs, status):
    """reference: global (float32 cost, lowest index) minimum over valid instances
    ((inf, -1) if none is valid)"""
    c = np.asarray(costs, dtype=np.float64).astype(np.float32)
    ok = np.asarray(status) == 0
    idx = np.nonzero(ok)[0]
    if idx.size == 0:
        return float("inf"), -1
    j = idx[np.lexsort((idx, c[idx]))[0]]
    return float(c[j]), int(j)
