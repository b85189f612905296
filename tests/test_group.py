"""The library's multi-GPU group (include/mpcqp.h mpcqp_group_*, csrc/group.hip).

CPU: the shard arithmetic every multi-GPU path shares (mpcqp_shard, host code in the library)
against a restatement and the cover / balance properties; the group entry points refuse bad
arguments without touching a device.  GPU: a one-rank group (mpcqp_group_create_rank with the
library's own RCCL communicator, and mpcqp_group_create over device 0) gives, step after step,
the record and per-instance outputs of one context's mpcqp_batch_solve_select bit for bit; a
group over EVERY visible device (skipped on a one-GPU box) gives the whole batch's record on
every member; the solve waits for the stream that produced its inputs; a step that fails
part-way leaves the group failed (communicators aborted, later calls refused)."""
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


@pytest.mark.gpu
def test_group_host_path_page_locked_matches(gpu):
    """the group's host path with the caller's arrays page-locked (mpcqp_host_register on
    page-aligned copies): each member's shard is DMA'd straight from and into them, and every
    output equals the staged path's bit for bit"""
    import ctypes as C
    import mpcqp
    from mpcqp._lib import lib
    from mpcqp.group import Group
    p = mpcqp.model_params("B")
    S, Cn = 300, 16
    batch = mpcqp.make_batch(p, S * Cn, seed=5151, gait="mixed")
    grp = Group(p, devices=[0])
    ref = grp.solve_select_host(S, Cn, batch)
    B, nV = S * Cn, p["nu"] * p["N"]
    locked = {k: mpcqp.page_aligned(batch[k]) for k in ("x0", "xref", "lin", "contact")}
    out = dict(U=mpcqp.page_aligned(np.full((B, nV), np.nan)),
               cost=mpcqp.page_aligned(np.full(B, np.nan)),
               status=mpcqp.page_aligned(np.full(B, 99, np.int32)),
               iters=mpcqp.page_aligned(np.full(B, -1, np.int32)))
    arrs = list(locked.values()) + list(out.values())
    for a in arrs:
        assert lib().mpcqp_host_register(C.c_void_p(a.ctypes.data), C.c_size_t(a.nbytes)) == 0
    try:
        for _ in range(2):
            got = grp.solve_select_host(S, Cn, locked, out=out)
            for k in ("U", "cost", "status", "iters", "best"):
                assert np.array_equal(got[k], ref[k]), k
    finally:
        for a in arrs:
            assert lib().mpcqp_host_unregister(C.c_void_p(a.ctypes.data)) == 0
    grp.close()


def _group_matches_whole_batch(torch, gait, devices, seed):
    """a single-process group over `devices` (one rank each): each member's best record equals
    one context's mpcqp_batch_solve_select over the WHOLE batch, bit for bit, over three steps
    (both record buffers, one reused), and the per-instance outputs of each shard equal that
    context's"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    from mpcqp.group import Group, shard
    nr = len(devices)
    p = mpcqp.model_params("B")
    Cn = 16
    S = 37 * nr + 3  # uneven shards
    batch = mpcqp.make_batch(p, S * Cn, seed=seed, gait=gait)
    ref = BatchEngine(p, device=0)
    dr = ref.upload(batch)
    rec = torch.zeros(1 + ref.nV, dtype=torch.int64, device="cuda:0")
    ref.solve_select(dr, rec)
    ref.sync()
    grp = Group(p, devices=list(devices))
    assert (grp.local, grp.nranks, grp.first_rank) == (nr, nr, 0)
    engs, shards = [], []
    for r in range(nr):
        f, n = shard(S, nr, r)
        sub = {k: v[f * Cn:(f + n) * Cn] for k, v in batch.items()}
        e = BatchEngine.wrap(p, grp.ctx(r), devices[r])
        d = e.upload(sub)
        engs.append(e)
        shards.append(dict(d, base=f * Cn))
    steps = [[torch.full((1 + ref.nV,), -5, dtype=torch.int64, device=f"cuda:{devices[r]}")
              for r in range(nr)] for _ in range(3)]
    for best in steps:
        grp.solve_select(shards, best)
    grp.sync()
    want = rec.cpu()
    for best in steps:
        for b_ in best:
            assert torch.equal(b_.cpu(), want)
    for r in range(nr):
        f, n = shard(S, nr, r)
        for k in ("U", "cost", "status", "iters"):
            assert torch.equal(shards[r][k].cpu(), dr[k][f * Cn:(f + n) * Cn].cpu()), (r, k)
    # the host path over the same group: the whole batch's outputs and record
    out = grp.solve_select_host(S, Cn, batch)
    assert np.array_equal(out["best"], want.numpy())
    for k in ("U", "cost", "status", "iters"):
        assert np.array_equal(out[k], dr[k].cpu().numpy()), k
    for e in engs:
        e.close()
    grp.close()
    ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("gait", ["alternating", "mixed"])
def test_group_all_devices_matches_whole_batch(gpu, gait):
    """mpcqp_group_create over every visible device (ncclCommInitAll, the grouped all-gather of
    the local members, the cross-rank reduction): _group_matches_whole_batch.  Needs >= 2
    devices (src/mpc_control_fake_state.cpp:108-149 at batch scale)."""
    torch = gpu
    ndev = torch.cuda.device_count()
    if ndev < 2:
        pytest.skip("one visible device: the multi-device group needs >= 2")
    _group_matches_whole_batch(torch, gait, list(range(ndev)), 8080)


@pytest.mark.gpu
@pytest.mark.parametrize("gait", ["alternating", "mixed"])
def test_group_three_ranks_loopback_matches_whole_batch(gpu, gait, monkeypatch):
    """three ranks on device 0 over the test transport (MPCQP_GROUP_LOOPBACK=1: the all-gather as
    device copies, no RCCL): the multi-member orchestration -- uneven shards, per-member solve /
    collective streams, the record double-buffering across steps, the cross-rank reduction, the
    host path's per-member staging -- gives every rank the whole batch's record
    (_group_matches_whole_batch); what it cannot cover is RCCL itself"""
    monkeypatch.setenv("MPCQP_GROUP_LOOPBACK", "1")
    _group_matches_whole_batch(gpu, gait, [0, 0, 0], 8181)


@pytest.mark.gpu
def test_group_solve_waits_for_the_input_stream(gpu):
    """inputs written on a torch stream that is still busy (a spin kernel ahead of the copies):
    the group's own solve stream waits for it (mpcqp_group_wait_stream, Group.solve_select's
    default) with no host synchronisation, and the step's results are the inputs' results"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    from mpcqp.group import Group, unique_id
    torch = gpu
    p = mpcqp.model_params("B")
    B = 16 * 64
    batch = mpcqp.make_batch(p, B, seed=91)
    ref = BatchEngine(p)
    dr = ref.upload(batch)
    rec = torch.zeros(1 + ref.nV, dtype=torch.int64, device="cuda:0")
    ref.solve_select(dr, rec)
    ref.sync()
    grp = Group(p, rank=(0, 1, 0, unique_id()))
    eng = BatchEngine.wrap(p, grp.ctx(0), 0)
    d = eng.upload(mpcqp.make_batch(p, B, seed=92))  # other inputs, overwritten below
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.cuda._sleep(50_000_000)  # ~20 ms of spinning ahead of the input copies
        for k in ("x0", "xref", "lin", "contact"):
            d[k].copy_(dr[k])
        best = torch.full((1 + ref.nV,), -5, dtype=torch.int64, device="cuda:0")
        grp.solve_select([dict(d, base=0)], [best])
    grp.sync()
    side.synchronize()
    assert torch.equal(best, rec)
    for k in ("U", "cost", "status", "iters"):
        assert torch.equal(d[k], dr[k]), k
    eng.close()
    grp.close()
    ref.close()


@pytest.mark.gpu
def test_group_failed_step_aborts_and_refuses(gpu, monkeypatch):
    """a step that fails after its solves were enqueued (fault injection at step 1) aborts the
    communicator and leaves the group failed: that step and every later call but info / failed
    / destroy return MPCQP_ERR_DEVICE; bad arguments before anything is enqueued do not"""
    import ctypes as C

    import mpcqp
    from mpcqp.engine import BatchEngine
    from mpcqp.group import Group, unique_id
    torch = gpu
    monkeypatch.setenv("MPCQP_GROUP_INJECT_FAIL", "1")
    p = mpcqp.model_params("B")
    batch = mpcqp.make_batch(p, 16 * 8, seed=3)
    grp = Group(p, rank=(0, 1, 0, unique_id()))
    eng = BatchEngine.wrap(p, grp.ctx(0), 0)
    d = eng.upload(batch)
    best = torch.zeros(1 + eng.nV, dtype=torch.int64, device="cuda:0")
    L = mpcqp.lib()
    # a bad argument (no contact for the SRBM model): refused up front, the group unchanged
    bad = dict(d, base=0, contact=None)
    with pytest.raises(RuntimeError):
        grp.solve_select([bad], [best])
    assert not grp.failed
    grp.solve_select([dict(d, base=0)], [best])  # step 0
    grp.sync()
    with pytest.raises(RuntimeError):
        grp.solve_select([dict(d, base=0)], [best])  # step 1: injected failure
    assert grp.failed
    with pytest.raises(RuntimeError):
        grp.solve_select([dict(d, base=0)], [best])
    assert L.mpcqp_group_wait(grp.g) == 5 and L.mpcqp_group_sync(grp.g) == 5
    loc = C.c_int()
    assert L.mpcqp_group_info(grp.g, C.byref(loc), None, None) == 0 and loc.value == 1
    eng.close()
    grp.close()
