"""Batched engine: device-resident inputs/outputs (torch tensors for HBM allocation and
streams -- plumbing only) driven through the C ABI of libmpcqp.so.

Mirrors the reference's per-tick step (mpcQP ctor, include/mpcQP.h:35-119: linearise ->
discretise -> condense -> solve -> U_opt.col(0)) for a whole batch of states x gait candidates.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import model as _model
from ._lib import check, lib


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class BatchEngine:
    """One mpcqp_ctx on one GPU.  Arrays are torch tensors on `device`."""

    def __init__(self, params: dict, device: int = 0, stream=None):
        import torch  # plumbing: device memory + streams

        self.torch = torch
        self.p = params
        self.device = device
        self.nV = params["nu"] * params["N"]
        m, keep = _model.to_struct(params)
        ctx = C.c_void_p()
        check("mpcqp_ctx_create", lib().mpcqp_ctx_create(C.byref(m), device, C.byref(ctx)))
        del keep
        self.ctx = ctx
        self.own = True
        if stream is None:  # share torch's stream so uploads/memsets are ordered before us
            stream = torch.cuda.current_stream(device).cuda_stream
        check("mpcqp_set_stream", lib().mpcqp_set_stream(self.ctx, C.c_void_p(stream)))

    @classmethod
    def wrap(cls, params: dict, ctx, device: int = 0):
        """an engine over a context someone else owns (a member of mpcqp.group.Group: its
        stream stays the group's; close() leaves the context alone)"""
        import torch
        e = cls.__new__(cls)
        e.torch, e.p, e.device, e.nV = torch, params, device, params["nu"] * params["N"]
        e.ctx, e.own = ctx, False
        return e

    def close(self):
        if self.ctx:
            if self.own:
                lib().mpcqp_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- buffers ---------------------------------------------------------------------------
    def upload(self, batch: dict):
        t = self.torch
        dev = f"cuda:{self.device}"
        out = {k: t.from_numpy(np.ascontiguousarray(batch[k])).to(dev)
               for k in ("x0", "xref", "lin")}
        out["contact"] = t.from_numpy(np.ascontiguousarray(batch["contact"]).view(np.int64)).to(dev)
        B = batch["x0"].shape[0]
        out["U"] = t.zeros((B, self.nV), dtype=t.float64, device=dev)
        out["cost"] = t.zeros(B, dtype=t.float64, device=dev)
        out["status"] = t.zeros(B, dtype=t.int32, device=dev)
        out["iters"] = t.zeros(B, dtype=t.int32, device=dev)
        out["key"] = t.zeros(1, dtype=t.int64, device=dev)
        out["B"] = B
        self.reserve(B)
        return out

    def set_warm_start(self, on: bool = True):
        """seed each gait solve with the previous tick's active sets (mpcqp_set_warm_start)"""
        check("mpcqp_set_warm_start", lib().mpcqp_set_warm_start(self.ctx, int(bool(on))))

    def reserve(self, B: int):
        """size the context's scratch for B instances: no allocation on the solve path"""
        check("mpcqp_ctx_reserve", lib().mpcqp_ctx_reserve(self.ctx, int(B)))

    # -- stages ----------------------------------------------------------------------------
    def condense(self, d, H=None, f=None):
        t = self.torch
        B = d["B"]
        if H is None:
            H = t.empty((B, self.nV, self.nV), dtype=t.float64, device=d["x0"].device)
            f = t.empty((B, self.nV), dtype=t.float64, device=d["x0"].device)
        check("mpcqp_batch_condense", lib().mpcqp_batch_condense(
            self.ctx, B, _ptr(d["x0"]), _ptr(d["xref"]), _ptr(d["lin"]), _ptr(H), _ptr(f)))
        return H, f

    def solve_qp(self, d, H, f):
        check("mpcqp_batch_solve_qp", lib().mpcqp_batch_solve_qp(
            self.ctx, d["B"], _ptr(H), _ptr(f), _ptr(d["contact"]), _ptr(d["U"]),
            _ptr(d["cost"]), _ptr(d["status"]), _ptr(d["iters"])))

    @property
    def fast_path(self) -> bool:
        return bool(lib().mpcqp_ctx_fast_path(self.ctx))

    @property
    def pair_nf(self) -> int:
        """free variables per instance the one-wave fused kernel solves (more: the overflow
        workgroup kernel)"""
        return int(lib().mpcqp_ctx_one_wave_nf(self.ctx))

    @property
    def crash(self) -> tuple:
        """(kmax, pmax) of the one-wave kernel's crash start, (kmax, pmax) of the workgroup
        solver's, and the free count above which an instance is the workgroup solver's; zeros
        where the dual loop starts cold.  The oracle reproduces the iteration counts with
        p["crash"] set to this tuple."""
        import ctypes as C
        if not hasattr(lib(), "mpcqp_ctx_crash_params"):  # an A/B build of older sources
            return (0, 0, 0, 0, 0)
        v = [C.c_int(0) for _ in range(4)]
        check("mpcqp_ctx_crash_params",
              lib().mpcqp_ctx_crash_params(self.ctx, *[C.byref(x) for x in v]))
        # (one-wave kmax, pmax, workgroup kmax, pmax, the free count above which an instance is
        #  the workgroup solver's)
        return tuple(x.value for x in v) + (self.pair_nf,)

    @property
    def fused_kernel(self) -> str:
        """name of the kernel mpcqp_batch_solve launches: k_mpc_pair (two QPs per wave),
        k_mpc (one QP per wave) or the generic k_condense + k_solve pair"""
        return {3: "k_dense_wg", 2: "k_mpc_pair", 1: "k_mpc"}.get(
            lib().mpcqp_ctx_fast_path(self.ctx), "k_condense+k_solve")

    @property
    def overflow_kernel(self) -> str:
        """the overflow launch after the one-wave kernel (slot 3 of the library's timing):
        k_mpc_list (one QP per wavefront), k_mpc_wg (one workgroup per QP) or none"""
        L = lib()
        if not hasattr(L, "mpcqp_ctx_overflow_kernel"):  # A/B builds of older sources
            return "k_mpc_wg"
        return {1: "k_mpc_list", 2: "k_mpc_wg"}.get(L.mpcqp_ctx_overflow_kernel(self.ctx), "none")

    def discretize(self, d, AB=None):
        """stage 1: linearise + exp(M Ts) -> [Ad | Bd] per instance"""
        t = self.torch
        if AB is None:
            nx, nu = self.p["nx"], self.p["nu"]
            AB = t.empty((d["B"], nx * (nx + nu)), dtype=t.float64, device=d["x0"].device)
        check("mpcqp_batch_discretize", lib().mpcqp_batch_discretize(
            self.ctx, d["B"], _ptr(d["lin"]), _ptr(AB)))
        return AB

    def condense_solve(self, d, AB):
        """stage 2: Phi, H_FF, f and the QP solve fused on chip"""
        check("mpcqp_batch_condense_solve", lib().mpcqp_batch_condense_solve(
            self.ctx, d["B"], _ptr(AB), _ptr(d["x0"]), _ptr(d["xref"]), _ptr(d["contact"]),
            _ptr(d["U"]), _ptr(d["cost"]), _ptr(d["status"]), _ptr(d["iters"])))

    def solve(self, d):
        """linearise + discretise + condense + solve, all on device (async on the ctx stream)"""
        check("mpcqp_batch_solve", lib().mpcqp_batch_solve(
            self.ctx, d["B"], _ptr(d["x0"]), _ptr(d["xref"]), _ptr(d["lin"]),
            _ptr(d["contact"]), _ptr(d["U"]), _ptr(d["cost"]), _ptr(d["status"]),
            _ptr(d["iters"])))

    def solve_select(self, d, rec, index_base: int = 0):
        """solve + this shard's selection record in one pass (mpcqp_batch_solve_select): rec
        (int64 device [1 + nV]) <- [min key | winner's U bits], as solve() + select_record()"""
        check("mpcqp_batch_solve_select", lib().mpcqp_batch_solve_select(
            self.ctx, d["B"], _ptr(d["x0"]), _ptr(d["xref"]), _ptr(d["lin"]),
            _ptr(d["contact"]), _ptr(d["U"]), _ptr(d["cost"]), _ptr(d["status"]),
            _ptr(d["iters"]), int(index_base), _ptr(rec)))
        return rec

    # -- device-generated inputs and the closed loop ----------------
    def upload_gait(self, g: dict):
        """g: state [S,13], feet [S,6], cmd [S,2], phase [S,C] (numpy) -> device dict"""
        t = self.torch
        dev = f"cuda:{self.device}"
        out = {k: t.from_numpy(np.ascontiguousarray(g[k], dtype=np.float64)).to(dev)
               for k in ("state", "feet", "cmd", "phase")}
        S, Cc = g["phase"].shape
        B = S * Cc
        out["U"] = t.zeros((B, self.nV), dtype=t.float64, device=dev)
        out["cost"] = t.zeros(B, dtype=t.float64, device=dev)
        out["status"] = t.zeros(B, dtype=t.int32, device=dev)
        out["iters"] = t.zeros(B, dtype=t.int32, device=dev)
        out["best"] = t.zeros(S, dtype=t.int32, device=dev)
        out["best_cost"] = t.zeros(S, dtype=t.float64, device=dev)
        out["Ubest"] = t.zeros((S, self.nV), dtype=t.float64, device=dev)
        out["S"], out["C"], out["B"] = S, Cc, B
        out["swing"] = float(g.get("swing", _model.SWING_TIME))
        out["stance"] = float(g.get("stance", _model.STANCE_TIME))
        return out

    def solve_gait(self, g):
        """x0 / xref / lin / contact generated on chip from the per-state data, then the step"""
        check("mpcqp_batch_solve_gait", lib().mpcqp_batch_solve_gait(
            self.ctx, g["S"], g["C"], _ptr(g["state"]), _ptr(g["feet"]), _ptr(g["cmd"]),
            _ptr(g["phase"]), g["swing"], g["stance"], _ptr(g["U"]), _ptr(g["cost"]),
            _ptr(g["status"]), _ptr(g["iters"])))

    def select_state(self, g):
        check("mpcqp_batch_select_state", lib().mpcqp_batch_select_state(
            self.ctx, g["S"], g["C"], _ptr(g["cost"]), _ptr(g["status"]), _ptr(g["U"]),
            _ptr(g["best"]), _ptr(g["best_cost"]), _ptr(g["Ubest"])))

    def plant(self, g):
        check("mpcqp_batch_plant_srbm", lib().mpcqp_batch_plant_srbm(
            self.ctx, g["S"], g["C"], _ptr(g["state"]), _ptr(g["feet"]), _ptr(g["phase"]),
            _ptr(g["best"]), _ptr(g["Ubest"])))

    def rollout(self, g, K: int, record: bool = True):
        """K closed-loop ticks on device; returns (traj [K,S,13], choice [K,S]) if record"""
        t = self.torch
        dev = g["state"].device
        traj = t.empty((K, g["S"], 13), dtype=t.float64, device=dev) if record else None
        choice = t.empty((K, g["S"]), dtype=t.int32, device=dev) if record else None
        check("mpcqp_rollout", lib().mpcqp_rollout(
            self.ctx, g["S"], g["C"], int(K), _ptr(g["state"]), _ptr(g["feet"]), _ptr(g["cmd"]),
            _ptr(g["phase"]), g["swing"], g["stance"], _ptr(traj), _ptr(choice)))
        return traj, choice

    def select_min(self, d, index_base: int = 0):
        check("mpcqp_batch_select_min", lib().mpcqp_batch_select_min(
            self.ctx, d["B"], _ptr(d["cost"]), _ptr(d["status"]), int(index_base),
            _ptr(d["key"])))
        return d["key"]

    def select_record(self, d, rec, index_base: int = 0):
        """rec: int64 device tensor [1 + nV] <- [min key | winner's U bits] of this shard"""
        check("mpcqp_batch_select_record", lib().mpcqp_batch_select_record(
            self.ctx, d["B"], _ptr(d["cost"]), _ptr(d["status"]), _ptr(d["U"]), int(index_base),
            _ptr(rec)))
        return rec

    def reduce_records(self, gathered, best):
        """gathered: int64 [n, 1 + nV] (one record per rank) -> best [1 + nV], on device"""
        check("mpcqp_reduce_records", lib().mpcqp_reduce_records(
            self.ctx, int(gathered.shape[0]), _ptr(gathered), _ptr(best)))
        return best

    def sync(self):
        check("mpcqp_sync", lib().mpcqp_sync(self.ctx))

    def enable_timing(self, on=True):
        check("mpcqp_enable_timing", lib().mpcqp_enable_timing(self.ctx, 1 if on else 0))

    def count_solver_flops(self, on=True):
        """(diagnostic) k_mpc_pair adds its crash working-set and dual-pass flops to a counter"""
        check("mpcqp_count_solver_flops", lib().mpcqp_count_solver_flops(self.ctx, 1 if on else 0))

    def solver_flops(self):
        """(flops summed since the previous call, paired-kernel launches counted); waits"""
        n = C.c_int(0)
        v = float(lib().mpcqp_solver_flops(self.ctx, C.byref(n)))
        return v, n.value

    def last_kernel_ms(self, which: int) -> float:
        """which: 0 stage 1, 1 the whole solve, 2 the one-wave fused kernel, 3 the overflow
        workgroup kernel (mpcqp.h)"""
        return float(lib().mpcqp_last_kernel_ms(self.ctx, which))

    def kernel_ms_sum(self, which: int):
        """(sum of ms, launches) of slot `which` since the previous call (the last 64 at most)"""
        n = C.c_int(0)
        ms = float(lib().mpcqp_kernel_ms_sum(self.ctx, which, C.byref(n)))
        return ms, n.value


def decode_key(key: int):
    """(float32 cost, global index) from a select_min key"""
    idx = key & 0x7FFFFFFF
    ob = (key >> 31) & 0xFFFFFFFF
    bits = (ob & 0x7FFFFFFF) if (ob & 0x80000000) else (~ob & 0xFFFFFFFF)
    cost = np.frombuffer(np.uint32(bits).tobytes(), dtype=np.float32)[0]
    return float(cost), int(idx)


def encode_key(cost: float, index: int) -> int:
    """host restatement of the device key (for the CPU reference of the selection)"""
    u = int(np.frombuffer(np.float32(cost).tobytes(), dtype=np.uint32)[0])
    ob = (~u & 0xFFFFFFFF) if (u & 0x80000000) else (u | 0x80000000)
    return (ob << 31) | (index & 0x7FFFFFFF)
