"""Multi-GPU selection path on CPU: world_size-2/3 gloo ranks run the same select_global as
bench.py (one all-gather of the [key | U] selection records, then the record reduction) over
shards solved by the oracle, and must reproduce the single-process global argmin; an
all-infeasible batch selects nothing (key INT64_MAX, index -1, U = 0) on every rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, seed, out_q, infeasible=False):
    sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import mpcqp
    import oracle
    from mpcqp.dist import decode_record, host_record, host_reduce_records, select_global

    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = mpcqp.model_params("B")
    batch = mpcqp.make_batch(p, B, seed=seed + rank)   # each rank its own shard (weak scaling)
    o = oracle.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    status = np.full_like(o["status"], 2) if infeasible else o["status"]
    nV = p["nu"] * p["N"]
    rec = torch.from_numpy(host_record(o["cost"], status, o["U"], rank * B))
    gathered = torch.zeros((world, 1 + nV), dtype=torch.int64)
    best = torch.zeros(1 + nV, dtype=torch.int64)
    select_global(dist, rec, gathered, best, host_reduce_records)
    cost, gidx, ub = decode_record(best.numpy())
    out_q.put((rank, cost, gidx, ub))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_min_cost_selection_matches_single_process(world):
    import mpcqp
    import oracle
    from mpcqp.dist import host_select

    B, seed = 48, 777
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, seed, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    # single-process reference over the concatenated batch
    p = mpcqp.model_params("B")
    costs, stats, Us = [], [], []
    for r in range(world):
        b = mpcqp.make_batch(p, B, seed=seed + r)
        o = oracle.srbm_batch(p, b["x0"], b["xref"], b["lin"], b["contact"])
        costs.append(o["cost"]); stats.append(o["status"]); Us.append(o["U"])
    costs, stats, Us = np.concatenate(costs), np.concatenate(stats), np.concatenate(Us)
    c0, i0 = host_select(costs, stats)
    for rank, cost, gidx, ub in res:
        assert gidx == i0 and cost == pytest.approx(c0)
        np.testing.assert_array_equal(ub, Us[i0])   # every rank received the winner's U


def test_gloo_selection_all_infeasible_selects_nothing():
    """no valid instance on any rank: every rank gets (inf, -1, U = 0), no collective fails"""
    world, B, seed = 2, 16, 99
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, seed, q, True))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, cost, gidx, ub in res:
        assert gidx == -1 and cost == float("inf")
        assert not ub.any()


def test_host_record_roundtrip():
    from mpcqp.dist import NO_KEY, decode_record, host_record, host_reduce_records, host_select
    rng = np.random.default_rng(5)
    recs, costs, stats, Us = [], [], [], []
    for r in range(4):
        c = rng.normal(size=32)
        st = (rng.random(32) < 0.3).astype(np.int32) * 2
        U = rng.normal(size=(32, 7))
        recs.append(host_record(c, st, U, r * 32))
        costs.append(c); stats.append(st); Us.append(U)
    best = np.zeros(8, np.int64)
    host_reduce_records(np.stack(recs), best)
    c0, i0 = host_select(np.concatenate(costs), np.concatenate(stats))
    cost, gidx, ub = decode_record(best)
    assert gidx == i0 and cost == pytest.approx(c0)
    np.testing.assert_array_equal(ub, np.concatenate(Us)[i0])
    none = host_record(np.zeros(3), np.ones(3, np.int32), np.ones((3, 7)))
    assert none[0] == NO_KEY and not none[1:].any()


def _pipe_worker(rank, world, port, B, T, out_q):
    sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from mpcqp.dist import PipelinedSelect, decode_record, host_record, host_reduce_records

    dist.init_process_group("gloo", rank=rank, world_size=world)
    nV = 60
    recs = [torch.zeros(1 + nV, dtype=torch.int64) for _ in range(2)]
    gathered = [torch.zeros((world, 1 + nV), dtype=torch.int64) for _ in range(2)]
    best = torch.zeros(1 + nV, dtype=torch.int64)
    pipe = PipelinedSelect(dist, recs, gathered, best, host_reduce_records)
    got = []
    for t in range(T):  # batch t: costs seeded by (t, rank); every rank writes its own record
        rng = np.random.default_rng(1000 * t + rank)
        cost = rng.normal(size=B)
        status = np.where(rng.random(B) < 0.2, 2, 0).astype(np.int32)
        U = rng.normal(size=(B, nV))
        pipe.record().copy_(torch.from_numpy(host_record(cost, status, U, rank * B)))
        pipe.submit()  # completes batch t - 1
        if t > 0:
            got.append(decode_record(best.numpy())[:2])
    pipe.drain()
    got.append(decode_record(best.numpy())[:2])
    out_q.put((rank, got, pipe.done))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_pipelined_selection_completes_every_batch():
    """mpcqp.dist.PipelinedSelect (bench.py's N > 1 step: batch s's all-gather in flight while
    batch s + 1 solves): after submit(s) the reduced record is batch s - 1's global argmin, and
    drain() completes the last batch, on every rank."""
    from mpcqp.dist import host_select

    world, B, T = 2, 40, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_pipe_worker, args=(r, world, port, B, T, q)) for r in range(world)]
    for pr in ps:
        pr.start()
    res = {}
    for _ in range(world):
        r, got, done = q.get(timeout=120)
        res[r] = (got, done)
    for pr in ps:
        pr.join(timeout=60)
    for t in range(T):
        costs, status = [], []
        for r in range(world):
            rng = np.random.default_rng(1000 * t + r)
            costs.append(rng.normal(size=B))
            status.append(np.where(rng.random(B) < 0.2, 2, 0).astype(np.int32))
        c, i = host_select(np.concatenate(costs), np.concatenate(status))
        for r in range(world):
            got, done = res[r]
            assert done == T
            assert got[t][1] == i and np.float32(got[t][0]) == np.float32(c), (t, r, got[t], c, i)
