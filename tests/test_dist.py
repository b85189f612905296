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
