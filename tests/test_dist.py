"""Multi-GPU selection path on CPU: world_size-2 gloo ranks run the same select_global as
bench.py (one MIN all-reduce of the 8-byte key + broadcast of the winner's U) over shards
solved by the oracle, and must reproduce the single-process global argmin."""
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


def _worker(rank, world, port, B, seed, out_q):
    sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import mpcqp
    import oracle
    from mpcqp.dist import host_keys, select_global

    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = mpcqp.model_params("B")
    batch = mpcqp.make_batch(p, B, seed=seed + rank)   # each rank its own shard (weak scaling)
    o = oracle.srbm_batch(p, batch["x0"], batch["xref"], batch["lin"], batch["contact"])
    key = torch.tensor([host_keys(o["cost"], o["status"], rank * B)], dtype=torch.int64)
    ubest = torch.zeros(p["nu"] * p["N"], dtype=torch.float64)
    cost, gidx = select_global(dist, key, torch.from_numpy(o["U"]), B, ubest)
    out_q.put((rank, cost, gidx, ubest.numpy().copy()))
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
