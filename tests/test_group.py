"""The library's multi-GPU group (include/mpcqp.h mpcqp_group_*, csrc/group.hip).

CPU: the shard arithmetic every multi-GPU path shares (mpcqp_shard, host code in the library)
against a restatement and the cover / balance properties; the group entry points refuse bad
arguments without touching a device.  GPU: a one-rank group (mpcqp_group_create_rank with the
library's own RCCL communicator, and mpcqp_group_create over device 0) gives, step after step,
the record and per-instance outputs of one context's mpcqp_batch_solve_select bit for bit."""
import ctypes as C

import numpy as np
import pytest


def shard_ref(total, world, rank):
    base, rem = divmod(total, world)
    return rank * base + min(rank, rem), base + (1 if rank < rem else 0)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
def test_shard_matches_restatement_and_covers(world):
    from mpcqp.group import shard
    for total in (world, world + 1, 255, 256, 4096, 4097, 32768):
        got = [shard(total, world, r) for r in range(world)]
        assert got == [shard_ref(total, world, r) for r in range(world)]
        assert got[0][0] == 0 and sum(n for _, n in got) == total
        assert all(a[0] + a[1] == b[0] for a, b in zip(got, got[1:]))
        assert max(n for _, n in got) - min(n for _, n in got) <= 1


def test_group_entry_points_refuse_bad_arguments():
    import mpcqp
    from mpcqp import model as M
    L = mpcqp.lib()
    f, n = C.c_int(), C.c_int()
    assert L.mpcqp_shard(10, 0, 0, C.byref(f), C.byref(n)) == 6
    assert L.mpcqp_shard(10, 2, 2, C.byref(f), C.byref(n)) == 6
    assert L.mpcqp_shard(-1, 2, 0, C.byref(f), C.byref(n)) == 6
    m, keep = M.to_struct(mpcqp.model_params("B"))
    g = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)  # one rank per device
    assert L.mpcqp_group_create(C.byref(m), 2, devs, C.byref(g)) == 6 and not g.value
    assert L.mpcqp_group_create(C.byref(m), 0, devs, C.byref(g)) == 6
    uid = (C.c_ubyte * 128)()
    assert L.mpcqp_group_create_rank(C.byref(m), 0, 2, 2, uid, C.byref(g)) == 6
    assert L.mpcqp_group_destroy(None) == 6
    assert L.mpcqp_group_ctx(None, 0) is None
    del keep


@pytest.mark.gpu
@pytest.mark.parametrize("gait", ["alternating", "mixed"])
def test_group_rank_device_path_matches_solve_select(gpu, gait):
    """one-rank group from a unique id (the torchrun form bench.py --capi-group uses): three
    pipelined steps over both record buffers, each record and the outputs bit-identical to a
    plain context's mpcqp_batch_solve_select on the same shard"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    from mpcqp.group import Group, unique_id
    torch = gpu
    p = mpcqp.model_params("B")
    B, base = 16 * 97, 4096
    batch = mpcqp.make_batch(p, B, seed=77, gait=gait)
    ref = BatchEngine(p)
    dr = ref.upload(batch)
    rec = torch.zeros(1 + ref.nV, dtype=torch.int64, device="cuda:0")
    ref.solve_select(dr, rec, index_base=base)
    ref.sync()
    grp = Group(p, rank=(0, 1, 0, unique_id()))
    assert (grp.local, grp.nranks, grp.first_rank) == (1, 1, 0)
    eng = BatchEngine.wrap(p, grp.ctx(0), 0)
    d = eng.upload(batch)
    torch.cuda.synchronize()
    bests = [torch.full((1 + ref.nV,), -5, dtype=torch.int64, device="cuda:0") for _ in range(3)]
    for b_ in bests:
        grp.solve_select([dict(d, base=base)], [b_])
    grp.sync()
    for b_ in bests:
        assert torch.equal(b_, rec)
    for k in ("U", "cost", "status", "iters"):
        assert torch.equal(d[k], dr[k]), k
    eng.close()
    grp.close()
    ref.close()


@pytest.mark.gpu
def test_group_host_path_matches_solve_select(gpu):
    """single-process group over device 0, host arrays (the C++ controller's form)"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    from mpcqp.group import Group
    torch = gpu
    p = mpcqp.model_params("B")
    S, Cn = 61, 16
    batch = mpcqp.make_batch(p, S * Cn, seed=5150, gait="mixed")
    ref = BatchEngine(p)
    dr = ref.upload(batch)
    rec = torch.zeros(1 + ref.nV, dtype=torch.int64, device="cuda:0")
    ref.solve_select(dr, rec)
    ref.sync()
    grp = Group(p, devices=[0])
    for _ in range(2):
        out = grp.solve_select_host(S, Cn, batch)
        assert np.array_equal(out["best"], rec.cpu().numpy())
        assert np.array_equal(out["U"], dr["U"].cpu().numpy())
        assert np.array_equal(out["cost"], dr["cost"].cpu().numpy())
        assert np.array_equal(out["status"], dr["status"].cpu().numpy())
        assert np.array_equal(out["iters"], dr["iters"].cpu().numpy())
    grp.close()
    ref.close()
