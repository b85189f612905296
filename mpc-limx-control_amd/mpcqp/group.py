"""The C-ABI multi-GPU group (include/mpcqp.h mpcqp_group_*), from Python.

The group is the library's own form of SURVEY.md 8e: one context per device, an RCCL
communicator owned by the library, and per step ONE ncclAllGather of the [key | U] selection
records followed by the on-device reduction (csrc/group.hip).  A C++ controller links it
directly; `bench.py --capi-group` drives it under torchrun, where
torch.distributed only hands the RCCL unique id from rank 0 to the others (no collective of the
step goes through torch).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import model as _model
from ._lib import check, lib

UID_BYTES = 128


def shard(total_states: int, nranks: int, rank: int):
    """(first state, states) of `rank`: mpcqp_shard (contiguous whole states; the first
    total_states % nranks ranks take one more).  Host arithmetic, no device."""
    f, n = C.c_int(), C.c_int()
    check("mpcqp_shard", lib().mpcqp_shard(int(total_states), int(nranks), int(rank),
                                           C.byref(f), C.byref(n)))
    return f.value, n.value


def unique_id() -> bytes:
    """RCCL unique id for mpcqp_group_create_rank (call on one rank, hand it to all)"""
    buf = (C.c_ubyte * UID_BYTES)()
    check("mpcqp_group_unique_id", lib().mpcqp_group_unique_id(buf))
    return bytes(buf)


def _ptrs(ts, ctype=C.c_void_p):
    arr = (ctype * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = t.data_ptr() if t is not None else None
    return arr


class Group:
    """mpcqp_group: devices=[...] (one process drives them all: ncclCommInitAll), or
    rank=(device, nranks, rank, uid) (one process per device)."""

    def __init__(self, params: dict, devices=None, rank=None):
        self.p = params
        self.nV = params["nu"] * params["N"]
        m, keep = _model.to_struct(params)
        g = C.c_void_p()
        L = lib()
        if devices is not None:
            devs = (C.c_int * len(devices))(*devices)
            check("mpcqp_group_create", L.mpcqp_group_create(C.byref(m), len(devices), devs,
                                                             C.byref(g)))
        else:
            dev, nranks, r, uid = rank
            ub = (C.c_ubyte * UID_BYTES).from_buffer_copy(uid)
            check("mpcqp_group_create_rank",
                  L.mpcqp_group_create_rank(C.byref(m), int(dev), int(nranks), int(r), ub,
                                            C.byref(g)))
        del keep
        self.g = g
        loc, nr, first = C.c_int(), C.c_int(), C.c_int()
        check("mpcqp_group_info", L.mpcqp_group_info(g, C.byref(loc), C.byref(nr),
                                                     C.byref(first)))
        self.local, self.nranks, self.first_rank = loc.value, nr.value, first.value

    def ctx(self, i: int = 0):
        return C.c_void_p(lib().mpcqp_group_ctx(self.g, i))

    def close(self):
        if self.g:
            lib().mpcqp_group_destroy(self.g)
            self.g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve_select(self, shards, best, after_current_stream=True):
        """shards: one dict per local member (torch tensors on its device: x0, xref, lin,
        contact, U, cost, status, iters, and "base": the global index of its first instance);
        best: one int64 [1 + nV] tensor per member.  Asynchronous (group_sync / group_wait).
        The group's solve streams first wait (on device) for torch's current stream of each
        member's device, which produced the shards (mpcqp_group_wait_stream), unless
        after_current_stream is False."""
        n = self.local
        if after_current_stream:
            import torch
            streams = (C.c_void_p * n)(*[torch.cuda.current_stream(s["x0"].device).cuda_stream
                                         for s in shards])
            check("mpcqp_group_wait_stream", lib().mpcqp_group_wait_stream(self.g, streams))
        Bs = (C.c_int * n)(*[int(s["x0"].shape[0]) for s in shards])
        bases = (C.c_int64 * n)(*[int(s["base"]) for s in shards])
        col = lambda k: _ptrs([s[k] for s in shards])
        check("mpcqp_group_solve_select",
              lib().mpcqp_group_solve_select(self.g, Bs, bases, col("x0"), col("xref"), col("lin"),
                                             col("contact"), col("U"), col("cost"), col("status"),
                                             col("iters"), _ptrs(best)))

    @property
    def failed(self) -> bool:
        return bool(lib().mpcqp_group_failed(self.g))

    def wait(self):
        check("mpcqp_group_wait", lib().mpcqp_group_wait(self.g))

    def sync(self):
        check("mpcqp_group_sync", lib().mpcqp_group_sync(self.g))

    def solve_select_host(self, S: int, Cn: int, batch: dict, out: dict | None = None):
        """single-process group: the global host batch of S states x Cn candidates -> dict(U,
        cost, status, iters, best) (numpy), synchronous.  `out` may hold the U / cost / status /
        iters arrays to write (e.g. page-locked with mpcqp_host_register, with the batch's input
        arrays: the library then DMAs straight from and into them)"""
        B = S * Cn
        ins = [np.ascontiguousarray(batch[k]) for k in ("x0", "xref", "lin", "contact")]
        out = out or {}
        U = out.get("U", np.zeros((B, self.nV)))
        cost = out.get("cost", np.zeros(B))
        st = out.get("status", np.zeros(B, np.int32))
        it = out.get("iters", np.zeros(B, np.int32))
        best = np.zeros(1 + self.nV, np.int64)
        ptr = lambda a: C.c_void_p(a.ctypes.data)
        check("mpcqp_group_solve_select_host",
              lib().mpcqp_group_solve_select_host(self.g, S, Cn, *[ptr(a) for a in ins], ptr(U),
                                                  ptr(cost), ptr(st), ptr(it), ptr(best)))
        return dict(U=U, cost=cost, status=st, iters=it, best=best)
