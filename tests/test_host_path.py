"""The controller's host-pointer tick (mpcqp_batch_solve_host, what ConvexMpc::solve and
compat/MPCController.h call once per MPC tick; include/MPCController.h:178-180): pinned staging,
one copy each way, the step captured into a HIP graph per batch size and overflow-list parity.
Checked bit-for-bit against the device-pointer path on the same inputs (same kernels), and the
overflow instances against the oracle (U <= 1e-8 max(1, |U|))."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def host_solve(eng, p, b):
    from mpcqp._lib import lib
    B = b["x0"].shape[0]
    nV = p["nu"] * p["N"]
    ins = [np.ascontiguousarray(b[k]) for k in ("x0", "xref", "lin", "contact")]
    out = dict(U=np.full(B * nV, np.nan), cost=np.full(B, np.nan), status=np.full(B, 99, np.int32),
               iters=np.full(B, -1, np.int32))
    ptr = lambda a: C.c_void_p(a.ctypes.data)
    rc = lib().mpcqp_batch_solve_host(eng.ctx, B, *[ptr(a) for a in ins],
                                      *[ptr(out[k]) for k in ("U", "cost", "status", "iters")])
    assert rc == 0
    out["U"] = out["U"].reshape(B, nV)
    return out


def device_solve(eng, b):
    d = eng.upload(b)
    eng.solve(d)
    eng.sync()
    return {k: d[k].cpu().numpy() for k in ("U", "cost", "status", "iters")}


def same(a, b):
    for k in ("U", "cost", "status", "iters"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.mark.parametrize("B", [1, 16, 37])
def test_host_tick_equals_device_path(gpu, B):
    """repeated host ticks (graph replays) equal the device path exactly"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    b = mpcqp.make_batch(p, B, seed=101 + B)
    eng = BatchEngine(p)
    ref = device_solve(eng, b)
    for _ in range(3):
        same(host_solve(eng, p, b), ref)
    eng.close()


def test_host_tick_overflow_parities(gpu, orc):
    """double-support instances need the workgroup kernel: the host path then captures one
    graph per overflow-list parity; host ticks interleaved with device-path solves on the same
    context keep the lists consistent, and the overflow instances match the oracle"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    B = 16
    b = mpcqp.make_batch(p, B, seed=5, gait="mixed")
    nf = np.array([3 * bin(int(c)).count("1") for c in b["contact"]])
    assert (nf > 30).any() and (nf <= 30).any()
    eng = BatchEngine(p)
    ref = device_solve(eng, b)
    for i in range(5):
        same(host_solve(eng, p, b), ref)
        if i % 2:
            same(device_solve(eng, b), ref)
    o = orc.srbm_batch(p, b["x0"], b["xref"], b["lin"], b["contact"])
    assert np.all(ref["status"] == 0) and np.all(o["status"] == 0)
    sc = np.maximum(1.0, np.abs(o["U"]).max(axis=1))
    assert np.all(np.abs(ref["U"] - o["U"]).max(axis=1) <= 1e-8 * sc)
    eng.close()


def test_host_tick_batch_size_change(gpu):
    """a new batch size re-captures; going back re-captures again (one cached size)"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    eng = BatchEngine(p)
    for B in (16, 3, 64, 16):
        b = mpcqp.make_batch(p, B, seed=B)
        same(host_solve(eng, p, b), device_solve(eng, b))
    eng.close()


def test_host_graph_survives_buffer_reallocation(gpu):
    """a host-path graph holds the overflow-list and staging addresses it was
    captured with; a device solve at a larger batch (or mpcqp_ctx_reserve) reallocates them.
    Host tick B = 16 on a mixed gait -> device solve B = 4,096 (grows the lists) -> host tick
    B = 16 again must re-capture, not replay against freed memory"""
    import mpcqp
    from mpcqp._lib import lib
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    b16 = mpcqp.make_batch(p, 16, seed=5, gait="mixed")
    big = mpcqp.make_batch(p, 4096, seed=6, gait="mixed")
    eng = BatchEngine(p)
    ref16 = device_solve(eng, b16)
    same(host_solve(eng, p, b16), ref16)
    ref_big = device_solve(eng, big)  # grows the overflow lists past the captured ones
    for _ in range(3):
        same(host_solve(eng, p, b16), ref16)
    assert lib().mpcqp_ctx_reserve(eng.ctx, 8192) == 0  # grows the host staging too
    for _ in range(3):
        same(host_solve(eng, p, b16), ref16)
    same(device_solve(eng, big), ref_big)
    eng.close()


def test_host_tick_overflow_flips(gpu):
    """a walking schedule flips the overflow prediction from tick to tick;
    the graphs for (no overflow) and (overflow, list parity 0 / 1) are cached side by side and
    every tick still equals the device path"""
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    mixed = mpcqp.make_batch(p, 16, seed=7, gait="mixed")
    alt = mpcqp.make_batch(p, 16, seed=7)
    nf_alt = np.array([3 * bin(int(c)).count("1") for c in alt["contact"]])
    assert (nf_alt <= 30).all()
    eng = BatchEngine(p)
    ref_m, ref_a = device_solve(eng, mixed), device_solve(eng, alt)
    for i in range(8):
        if i % 3 == 2:
            same(host_solve(eng, p, alt), ref_a)
        else:
            same(host_solve(eng, p, mixed), ref_m)
    eng.close()


def _locked(arrs, fn):
    """mpcqp_host_register / _unregister over numpy arrays (the caller's own buffers)"""
    from mpcqp._lib import lib
    for a in arrs:
        r = getattr(lib(), fn)(C.c_void_p(a.ctypes.data), *([C.c_size_t(a.nbytes)] if fn.endswith("_register") else []))
        assert r == 0, (fn, r)


@pytest.mark.parametrize("B,gait", [(4096, "alternating"), (40960 + 48, "alternating"),
                                    (20480, "mixed")])
def test_host_direct_path_equals_device_path(gpu, B, gait):
    """page-locked caller arrays (mpcqp_host_register) and B >= 4,096: the direct path (DMA
    straight from / into the caller's arrays, chunks of >= 8,192 pipelined over three streams;
    40,960 + 48 instances: a ragged last chunk; the mixed gait: the overflow launch per chunk)
    equals the device path bit for bit, and so does the staged path of the same context once
    the arrays are unregistered"""
    from mpcqp._lib import lib
    import mpcqp
    from mpcqp.engine import BatchEngine
    p = mpcqp.model_params("B")
    b = mpcqp.make_batch(p, B, seed=202 + B, gait=gait)
    eng = BatchEngine(p)
    ref = device_solve(eng, b)
    nV = p["nu"] * p["N"]
    # registered buffers start on a page and own their pages (mpcqp_host_register's contract)
    ins = [mpcqp.page_aligned(b[k]) for k in ("x0", "xref", "lin", "contact")]
    out = dict(U=mpcqp.page_aligned(np.full(B * nV, np.nan)),
               cost=mpcqp.page_aligned(np.full(B, np.nan)),
               status=mpcqp.page_aligned(np.full(B, 99, np.int32)),
               iters=mpcqp.page_aligned(np.full(B, -1, np.int32)))
    locked = ins + list(out.values())
    _locked(locked, "mpcqp_host_register")
    ptr = lambda a: C.c_void_p(a.ctypes.data)
    for _ in range(2):
        for v in out.values():
            v.fill(0)
        rc = lib().mpcqp_batch_solve_host(eng.ctx, B, *[ptr(a) for a in ins],
                                          *[ptr(out[k]) for k in ("U", "cost", "status", "iters")])
        assert rc == 0
        got = dict(out, U=out["U"].reshape(B, nV))
        same(got, ref)
    _locked(locked, "mpcqp_host_unregister")
    same(host_solve(eng, p, b), ref)
    eng.close()


def test_host_register_needs_page_aligned_start():
    """mpcqp_host_register refuses a start inside a page (before touching the device): two
    registrations may never share a page"""
    from mpcqp._lib import lib
    import mpcqp
    a = mpcqp.page_aligned(np.zeros(4096))
    assert a.ctypes.data % 4096 == 0
    assert lib().mpcqp_host_register(C.c_void_p(a.ctypes.data + 8), C.c_size_t(64)) == 6


def test_host_alloc_roundtrip(gpu):
    """mpcqp_host_alloc / _free: page-locked memory from the library, usable as a host array"""
    from mpcqp._lib import lib
    pv = C.c_void_p()
    assert lib().mpcqp_host_alloc(C.c_size_t(1 << 20), C.byref(pv)) == 0 and pv.value
    buf = (C.c_double * (1 << 17)).from_address(pv.value)
    buf[0], buf[-1] = 1.5, -2.5
    assert buf[0] == 1.5 and buf[-1] == -2.5
    assert lib().mpcqp_host_free(pv) == 0
    assert lib().mpcqp_host_free(None) == 6 and lib().mpcqp_host_register(None, 8) == 6
