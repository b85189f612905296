#!/usr/bin/env python3
"""Benchmark: QP solves/s for the TRON1 13-state / 6-input / N=10 SRBM MPC (BASELINE.json
metric): global batch 65,536 on 1/2/4/8 MI355X, STRONG scaling (65,536/N instances per GPU),
one process per GPU.  Config D (weak scaling, 65,536 per GPU: 524,288 on 8 GPUs) is reported
beside it in `config.weak`; the other single-GPU configs (B@4,096, C, L, standing/double
support) in `config.per_config` (N = 1 only).

One step = one pass of the hot path over the rank's shard, inputs resident in HBM:
  k_mpc_pair (linearise + discretise + condense + Goldfarb-Idnani solve, fused, two QPs per
  wavefront) -> k_mpc_list (the overflow list's instances, one QP per wavefront; empty for the
  alternating gait) whose last workgroup writes the per-rank selection record [min key | U]
  (mpcqp_batch_solve_select, the default `--select fused`: 0.376 vs 0.383 ms per step at
  65,536, 69 vs 76 us at 4,096; `--select separate` adds the k_select_min launch instead)
  -> [N>1] ONE RCCL all-gather of the records (8 + 480 B per rank) -> k_reduce_records.
No host synchronisation inside the step.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch G] [--config B|C|L]

`--gpus N` with N > 1 and no WORLD_SIZE in the environment launches N ranks itself
(`python -m torch.distributed.run --nproc-per-node N ...` as a child process; this parent makes
no GPU call).  Under torchrun (the driver's launch) RANK/LOCAL_RANK/WORLD_SIZE come from the
environment.  Rank 0 prints ONE JSON line (driver contract; DESIGN.md sections 5-6).

`--selection-dry-run` (test harness, CPU): the solve is replaced by seeded synthetic
cost/status/U per shard and the ranks run the same launcher, sharding and one-collective
selection over gloo; tests/test_bench_launcher.py checks n_gpus and the global argmin.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))

FP64_PEAK_TFLOPS = 78.6  # MI355X dense FP64 (vector = matrix), AMD spec; SURVEY.md 8d
HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E (/opt/skills/guides/MI355X_MICROARCH.md)
METRIC = "QP solves/sec, 13-state N=10 SRBM MPC, batch=65536 at 1/2/4/8 MI355X"
CANDIDATES = 16  # gait candidates per state: shards are aligned to whole states


def algorithmic_flops(nx: int, nu: int, N: int):
    """SURVEY.md section 8d structure-exploiting flop model, split per kernel."""
    n = nx + nu
    nV = nu * N
    F_disc = 8 * n ** 3 + (2.0 / 3.0) * n ** 3
    F_pow = (N - 1) * 2 * nx ** 3
    F_phi = (N - 1) * 2 * nx ** 2 * nu
    F_W = (N * (N + 1) / 2) * 2 * nx ** 2 * nu
    F_H = sum((i + 1) * (N - i) for i in range(N)) * 2 * nu ** 2 * nx
    F_f = N * 2 * nx ** 2 + (N * (N + 1) / 2) * 2 * nx * nu
    F_chol = nV ** 3 / 3.0
    F_iter = 4 * nV ** 2
    return dict(disc=F_disc, condense=F_disc + F_pow + F_phi + F_W + F_H + F_f,
                solve_fixed=F_chol, per_iter=F_iter)


def algorithmic_bytes(nx: int, nu: int, N: int):
    """read x0, xref, 7 linearisation scalars, contact; write U, cost, status."""
    nV = nu * N
    return (nx + nx * (N + 1) + 7 + 2 * N + nV + 1) * 8 + 4


def config_bytes(p):
    """Per-QP algorithmic bytes of any config: x0, xref, the linearisation (8 doubles for the
    SRBM / literal models, the NX x (NX + NU) [Ac | Bc] for a dense model), the contact word; U,
    cost, status, iterations out."""
    nx, nu, N = p["nx"], p["nu"], p["N"]
    lin = nx * (nx + nu) if p["model"] == 2 else 8
    return (nx + nx * (N + 1) + lin + 1 + nu * N + 1) * 8 + 2 * 4


def flops_per_qp(p, mean_iters):
    """SURVEY.md 8d's count (the reference's dense path), per QP"""
    fl = algorithmic_flops(p["nx"], p["nu"], p["N"])
    return fl["condense"] + fl["solve_fixed"] + fl["per_iter"] * float(mean_iters)


def algorithmic_work(p, contact, iters, max_nf, solver=None):
    """-> (algorithmic flops per launch of the fused kernel, instances it solved, basis).
    Closed-form models (SRBM, literal): the fixed phases (mpcqp/flops.py) over the instances the
    one-wave kernel solved (nf <= max_nf; the rest are the overflow kernel's), plus the solver's
    flops -- counted by the paired kernel itself per crash working set and dual pass when
    `solver` = (flops summed, launches) from mpcqp_solver_flops is given (a working set and a pass
    cost different amounts, so `iters` alone cannot price them), otherwise priced from `iters` as
    dual passes (kernels without the crash start).  The dense model (config E) runs the
    reference's algorithm: SURVEY.md 8d's count."""
    from mpcqp import flops
    it = np.asarray(iters)
    if p["model"] not in (0, 1):
        return (flops_per_qp(p, float(it.mean())) * len(it), len(it),
                "SURVEY.md 8d (the dense model runs the reference's Pade expm and condensing)")
    if solver is not None and solver[1] > 0:
        fx, n = flops.fixed_flops(p, contact, max_nf)
        return (fx + solver[0] / solver[1], n,
                "closed-form fixed phases (mpcqp/flops.py) + the kernel's own count of its crash "
                "working-set solves and dual passes (mpcqp_count_solver_flops)")
    fl, n = flops.batch_flops(p, contact, it, max_nf=max_nf)
    return fl, n, "closed-form fixed phases + dual passes priced from iters (mpcqp/flops.py)"


def count_solver_flops(eng, step, sync, launches=3):
    """(flops, paired-kernel launches) of the kernel's own solver-flops counter over a few more
    steps after the timed ones (None where the context has no paired kernel)"""
    if eng.fused_kernel != "k_mpc_pair":
        return None
    eng.count_solver_flops(True)
    for _ in range(launches):
        step()
    sync()
    out = eng.solver_flops()
    eng.count_solver_flops(False)
    return out


def hbm_fields(traffic, kernel_ms, alg_bytes):
    """HBM rate of the measured traffic (PMC bytes per launch) against the 8 TB/s peak"""
    if not traffic:
        return dict(hbm_gbps=None, hbm_frac=None)
    gbps = traffic / (kernel_ms * 1e-3) / 1e9
    return dict(hbm_gbps=gbps, hbm_frac=gbps / HBM_PEAK_GBPS,
                algorithmic_gbps=alg_bytes / (kernel_ms * 1e-3) / 1e9,
                traffic_over_algorithmic=traffic / alg_bytes)


def _profile_json(name):
    try:
        return json.load(open(os.path.join(ROOT, "profiles", name)))
    except (OSError, ValueError):
        return None


def lib_build_id():
    from mpcqp._lib import lib
    return lib().mpcqp_build_id().decode()


def pmc_traffic(config: str, batch: int):
    """HBM bytes per fused-kernel launch from the committed rocprofv3 PMC summary
    (tools/profile_run.sh + tools/summarize_profile.py), if it matches this workload; with the
    summary's tag and the source hash of the library it was measured on."""
    t = _profile_json("pmc_traffic.json")
    if not t or t.get("config") != config or t.get("batch") != batch:
        return None, None, None
    return t.get("hbm_bytes_per_launch"), t.get("tag"), t.get("lib_build_id")


def pmc_executed(config: str, batch: int):
    """Executed FP64 work of the fused kernel from the committed PMC pass
    (SQ_INSTS_VALU_{FMA,MUL,ADD}_F64 and MFMA ops; tools/pmc_flops.sh), if it matches."""
    t = _profile_json("pmc_flops.json")
    if not t or t.get("config") != config or t.get("batch") != batch:
        return None
    return t


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """(CPUs in sched_getaffinity, cgroup CPU quota in whole CPUs or None).  On the GPU box the
    affinity mask names every core of the host while the job's cgroup grants a share of them
    (cpu.max): running one OpenMP thread per affinity core there oversubscribes the quota."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(float(q) / float(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    return affinity, quota


def cpu_baseline(p, batch, budget_s=12.0):
    """The oracle (C restatement of the reference path, OpenMP over the batch) on ALL the host
    cores this process may run on, plus a 1-thread run beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # CPU baseline leg only

    affinity, quota = host_cpus()
    threads = max(1, min(affinity, quota or affinity))
    n0 = min(max(256, 4 * threads), batch["x0"].shape[0])
    sub = {k: v[:n0] for k, v in batch.items()}
    t = time.perf_counter()
    oracle.srbm_batch(p, sub["x0"], sub["xref"], sub["lin"], sub["contact"], nthreads=threads)
    rate0 = n0 / max(1e-6, time.perf_counter() - t)
    n = int(min(batch["x0"].shape[0], max(n0, rate0 * budget_s / 2)))
    sub = {k: v[:n] for k, v in batch.items()}
    # repeat the sample until ~budget_s of CPU work is timed (10-30 s guideline)
    done, dt, passes = 0, 0.0, 0
    while passes == 0 or (dt < budget_s and passes < 8):
        t = time.perf_counter()
        oracle.srbm_batch(p, sub["x0"], sub["xref"], sub["lin"], sub["contact"], nthreads=threads)
        dt += time.perf_counter() - t
        done += n
        passes += 1
    n1 = min(n, max(16, int(done / dt / threads * 2.0)))  # ~2 s single-thread sample
    t = time.perf_counter()
    oracle.srbm_batch(p, sub["x0"][:n1], sub["xref"][:n1], sub["lin"][:n1], sub["contact"][:n1],
                      nthreads=1)
    one = n1 / (time.perf_counter() - t)
    return dict(value=done / dt, unit="QP/s", cores=threads, kind="port",
                nproc=os.cpu_count(), affinity_cpus=affinity, cgroup_cpu_quota=quota,
                cpu_model=cpu_model(), single_thread_value=one,
                sample=f"first {n} instances of the rank-0 shard x {passes} passes, "
                       f"oracle/mpcqp_oracle.c (reference-literal dense condensing + "
                       f"Goldfarb-Idnani), OpenMP {threads} threads = every CPU the job may "
                       f"use (min of sched_getaffinity {affinity} and the cgroup quota "
                       f"{quota}), {dt:.1f} s; 1 thread: {n1} instances")


def host_staged_rate(eng, batch, p, reps=5, locked=False):
    """QP/s through mpcqp_batch_solve_host: host arrays in, H2D + fused kernel + D2H, synchronous
    (the PCIe-inclusive number; never `value`).  locked: the caller's arrays are
    page-locked once beforehand (mpcqp_host_register, as a controller allocating its buffers
    once would), so the library DMAs straight from / into them in pipelined chunks; otherwise
    pageable arrays through the context's pinned staging (a host memcpy each way)."""
    import ctypes as C

    from mpcqp._lib import lib
    from mpcqp import page_aligned, page_aligned_empty
    B = batch["x0"].shape[0]
    nV = p["nu"] * p["N"]
    # registered buffers start on a page and own their pages (include/mpcqp.h)
    alloc = page_aligned_empty if locked else np.zeros
    U = alloc(B * nV, np.float64)
    cost = alloc(B, np.float64)
    st = alloc(B, np.int32)
    it = alloc(B, np.int32)
    ins = [(page_aligned if locked else np.ascontiguousarray)(batch[k])
           for k in ("x0", "xref", "lin", "contact")]
    ptr = lambda a: C.c_void_p(a.ctypes.data)
    arrs = ins + [U, cost, st, it]
    if locked:
        for a in arrs:
            assert lib().mpcqp_host_register(ptr(a), C.c_size_t(a.nbytes)) == 0
    call = lambda: lib().mpcqp_batch_solve_host(eng.ctx, B, *[ptr(a) for a in ins], ptr(U),
                                                 ptr(cost), ptr(st), ptr(it))
    try:
        assert call() == 0
        t = time.perf_counter()
        for _ in range(reps):
            call()
        return B * reps / (time.perf_counter() - t)
    finally:
        if locked:
            for a in arrs:
                lib().mpcqp_host_unregister(ptr(a))


def per_tick_latency(p, seed, ticks=1000, warmup=50, device=0):
    """The controller's real path: one MPC tick host-to-host, as
    ConvexMpc::solve / MPC::computeSupportFootForce make it (include/mpcqp/convex_mpc.hpp ->
    mpcqp_batch_solve_host: host arrays in, the fused step, U / cost / status / iterations back,
    synchronous), for 1 state x {1, 16} gait candidates, against the 1 ms control period
    (include/MPCParam.h:44).  ctypes adds ~1 us per call over the C++ caller."""
    import ctypes as C

    import mpcqp
    from mpcqp._lib import lib
    from mpcqp.engine import BatchEngine
    out = dict(path="mpcqp_batch_solve_host (ConvexMpc::solve), host arrays in/out, synchronous",
               period_us=1000.0, ticks=ticks)
    eng = BatchEngine(p, device=device)
    eng.reserve(CANDIDATES)
    nV = p["nu"] * p["N"]
    full = mpcqp.make_batch(p, CANDIDATES, seed=seed)
    for Cn in (1, CANDIDATES):
        ins = [np.ascontiguousarray(full[k][:Cn]) for k in ("x0", "xref", "lin", "contact")]
        U = np.zeros(Cn * nV)
        cost = np.zeros(Cn)
        st = np.zeros(Cn, np.int32)
        it = np.zeros(Cn, np.int32)
        args = [eng.ctx, Cn] + [C.c_void_p(a.ctypes.data) for a in ins + [U, cost, st, it]]
        fn = lib().mpcqp_batch_solve_host
        for _ in range(warmup):
            assert fn(*args) == 0
        ts = np.empty(ticks)
        for i in range(ticks):
            t0 = time.perf_counter_ns()
            fn(*args)
            ts[i] = (time.perf_counter_ns() - t0) * 1e-3
        assert np.all(st == 0)
        out[f"C{Cn}"] = dict(p50_us=float(np.percentile(ts, 50)), p99_us=float(np.percentile(ts, 99)),
                             mean_us=float(ts.mean()), max_us=float(ts.max()),
                             max_solver_iters=int(it.max()))
    # ticks whose contact schedules alternate between a walking gait's candidates (no instance
    # can overflow) and a mixed set with double support / standing ones (the overflow launch
    # runs): the host path's graph cache is keyed by (overflow, list parity), so a flip replays
    # a cached graph instead of re-capturing
    mixed = mpcqp.make_batch(p, CANDIDATES, seed=seed + 1, gait="mixed")
    sets = []
    for src in (full, mixed):
        ins = [np.ascontiguousarray(src[k][:CANDIDATES]) for k in ("x0", "xref", "lin", "contact")]
        outs = [np.zeros(CANDIDATES * nV), np.zeros(CANDIDATES), np.zeros(CANDIDATES, np.int32),
                np.zeros(CANDIDATES, np.int32)]
        sets.append((ins, outs, [eng.ctx, CANDIDATES] +
                     [C.c_void_p(a.ctypes.data) for a in ins + outs]))
    fn = lib().mpcqp_batch_solve_host
    for i in range(warmup):
        assert fn(*sets[i & 1][2]) == 0
    ts = np.empty(ticks)
    for i in range(ticks):
        t0 = time.perf_counter_ns()
        fn(*sets[i & 1][2])
        ts[i] = (time.perf_counter_ns() - t0) * 1e-3
    assert all(np.all(o[2] == 0) for _, o, _ in sets)

    def stats(x):
        return dict(p50_us=float(np.percentile(x, 50)), p99_us=float(np.percentile(x, 99)),
                    mean_us=float(x.mean()), max_us=float(x.max()))
    out["C16_flip"] = dict(walking_ticks=stats(ts[0::2]), mixed_ticks=stats(ts[1::2]),
                           note="16 candidates per tick, alternating between the walking gait "
                                "(no overflow launch) and a mixed set with standing candidates "
                                "(the overflow workgroup kernel runs)")
    eng.close()
    return out


def gait_fused_rate(eng, p, B, seed, reps=10):
    """QP/s of mpcqp_batch_solve_gait: the same step with x0/xref/lin/contact generated on
    chip from per-state data (B/16 states x 16 gait candidates)."""
    import torch

    import mpcqp
    if not eng.fast_path or p["model"] != 0:
        return None
    g = eng.upload_gait(mpcqp.make_gait_states(p, B // CANDIDATES, seed=seed,
                                               candidates=CANDIDATES))
    eng.solve_gait(g)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        eng.solve_gait(g)
    e1.record()
    torch.cuda.synchronize()
    return g["B"] * reps / (e0.elapsed_time(e1) * 1e-3)


def time_config(config, B, seed, steps=10, warmup=2, gait=None, device=0):
    """One single-GPU config: fused-kernel ms (HIP events on the engine's stream), QP/s, mean
    solver iterations, solved fraction and the SURVEY 8d algorithmic-flop fraction."""
    import torch

    import mpcqp
    from mpcqp.engine import BatchEngine

    p = mpcqp.model_params(config)
    batch = mpcqp.make_batch(p, B, seed=seed, gait=gait) if gait else \
        mpcqp.make_batch(p, B, seed=seed)
    eng = BatchEngine(p, device=device)
    d = eng.upload(batch)
    for _ in range(warmup):
        eng.solve(d)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for e0, e1 in ev:
        e0.record(stream)
        eng.solve(d)
        e1.record(stream)
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    st = d["status"].cpu().numpy()
    it = d["iters"].cpu().numpy()
    f_qp = flops_per_qp(p, it.mean())
    ach8d = f_qp * B / (ms * 1e-3) / 1e12
    out = dict(batch=B, nx=p["nx"], nu=p["nu"], N=p["N"],
               constraints="box+friction" if p["constraints"] else "box",
               gait=gait or "alternating (calculateGait, swing = stance = 0.5 s)",
               R=float(p["R"][0, 0]), kernel=eng.fused_kernel, kernel_ms=ms,
               qps=B / (ms * 1e-3), mean_solver_iters=float(it.mean()),
               max_solver_iters=int(it.max()), solved_frac=float(np.mean(st == 0)))
    if p["model"] in (0, 1):
        # closed-form path: its own algorithmic count over every instance of the call (ms is
        # the whole solve call, overflow launch included); the paired kernel counts its solver
        # flops itself, in two more launches after the timed ones
        solver = None
        if eng.fused_kernel == "k_mpc_pair":
            eng.count_solver_flops(True)
            for _ in range(2):
                eng.solve(d)
            solver = eng.solver_flops()
            eng.count_solver_flops(False)
        fl, _, basis = algorithmic_work(p, batch["contact"], it, None, solver)
        out.update(algorithmic_flops_per_qp=fl / B, achieved_tflops=fl / (ms * 1e-3) / 1e12,
                   frac=fl / (ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, flops_basis=basis,
                   work_rate_vs_survey_8d=dict(flops_per_qp=f_qp, tflops=ach8d,
                                               frac=ach8d / FP64_PEAK_TFLOPS))
    else:
        # the dense model (config E) runs the reference's algorithm (Pade expm, condensing):
        # SURVEY.md 8d's count is its count
        out.update(algorithmic_flops_per_qp=f_qp, achieved_tflops=ach8d,
                   frac=ach8d / FP64_PEAK_TFLOPS, flops_basis="SURVEY.md 8d")
    ex = _profile_json(f"pmc_flops_{config}.json")
    if ex and ex.get("batch") == B and gait is None:
        # executed FP64 work of this kernel (64 lanes x SQ_INSTS_VALU_FLOPS_FP64 + 512 x MFMA
        # ops, an upper bound) from the committed PMC pass, over this run's kernel time
        out["executed_tflops"] = ex["executed_flops_per_launch"] / (ms * 1e-3) / 1e12
        out["pipe_frac"] = out["executed_tflops"] / FP64_PEAK_TFLOPS
        out["mfma_tflops"] = ex["mfma_flops_per_launch"] / (ms * 1e-3) / 1e12
        out["mfma_busy_frac"] = ex.get("mfma_busy_frac")
        out["lane_efficiency"] = out["achieved_tflops"] / out["executed_tflops"]
        out["pmc_source"] = f"profiles/pmc_flops_{config}.json ({ex.get('tag')})"
        out["pmc_matches_library"] = ex.get("lib_build_id") == lib_build_id()
    tr = _profile_json(f"pmc_traffic_{config}.json")
    if tr and tr.get("batch") == B and gait is None and tr.get("hbm_bytes_per_launch"):
        # HBM bytes of this kernel (2 x FETCH_SIZE + WRITE_SIZE, separate PMC passes) against
        # its algorithmic inputs + outputs
        alg = config_bytes(p) * B
        out["traffic_bytes_per_launch"] = tr["hbm_bytes_per_launch"]
        out["algorithmic_bytes_per_launch"] = alg
        out["traffic_over_algorithmic"] = tr["hbm_bytes_per_launch"] / alg
        out.update(hbm_fields(tr["hbm_bytes_per_launch"], ms, alg))
        out["traffic_source"] = f"profiles/pmc_traffic_{config}.json ({tr.get('tag')})"
        out["traffic_matches_library"] = tr.get("lib_build_id") == lib_build_id()
    eng.close()
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """Start N ranks as children (torch.distributed.run) and exit with their status.  The
    parent never touches the GPU (no exec from a GPU-initialised process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def shard(total_states, world, rank):
    """contiguous range of whole states for `rank` -> (first state, number of states): the
    library's mpcqp_shard, the arithmetic its multi-GPU group uses"""
    from mpcqp.group import shard as lib_shard
    return lib_shard(total_states, world, rank)


def slice_batch(batch, i0, n):
    return {k: np.ascontiguousarray(v[i0:i0 + n]) for k, v in batch.items()}


def synthetic_shard(B, nV, seed, rank, index_base):
    """--selection-dry-run: seeded cost/status/U of a shard (a function of the global index,
    so the global argmin does not depend on how the batch is split)"""
    gi = index_base + np.arange(B)
    rng = np.random.default_rng([seed] + [int(x) for x in gi[:1]])
    cost = np.cos(gi * 0.7071 + seed) * 1e3 + np.sin(gi * 1.3) * 10.0
    status = np.where((gi % 7) == 3, 3, 0).astype(np.int32)
    U = (gi[:, None] * 1e-3 + np.arange(nV)[None, :]).astype(np.float64)
    del rng
    return cost, status, U


def main():
    argv = sys.argv[1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--global-batch", type=int, default=65536,
                    help="instances over all GPUs (strong scaling: split over the ranks)")
    ap.add_argument("--weak-batch", type=int, default=65536,
                    help="instances per GPU of the weak-scaling (config D) line; 0 = skip")
    ap.add_argument("--config", default="B")
    ap.add_argument("--seed", type=int, default=20250404)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-config", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the PCIe-inclusive, generated-input and per-tick lines (profiling "
                         "runs: the host path launches the headline kernel too)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-kernel timing pass after the timed steps")
    ap.add_argument("--selection-dry-run", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--select", choices=("fused", "separate"), default="fused",
                    help="selection record from the solve kernels (fused) or k_select_min")
    ap.add_argument("--capi-group", action="store_true",
                    help="drive the step through the library's multi-GPU group (include/mpcqp.h "
                         "mpcqp_group_*: its own RCCL communicator, one all-gather per step); "
                         "torch.distributed only hands rank 0's RCCL id to the other ranks")
    ap.add_argument("--serial-select", action="store_true",
                    help="N > 1: wait for each step's all-gather before the next solve (default: "
                         "the collective of step s overlaps the solve of step s + 1)")
    args = ap.parse_args()
    fused = args.select == "fused"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    import mpcqp
    from mpcqp.dist import PipelinedSelect, decode_record, host_record, host_reduce_records

    dry = args.selection_dry_run
    if dry:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)

    p = mpcqp.model_params(args.config)
    nV = p["nu"] * p["N"]
    G = args.global_batch
    S_total = G // CANDIDATES
    if S_total * CANDIDATES != G or S_total < world:
        raise SystemExit(f"--global-batch must be a multiple of {CANDIDATES} with >= 1 state "
                         "per rank")
    s0, ns = shard(S_total, world, rank)
    i0, B = s0 * CANDIDATES, ns * CANDIDATES
    # what the process group actually formed, per rank (a SCALE run checks
    # itself): world size after init, each rank's device and its shard of the global batch
    me = dict(rank=rank, local_rank=local, device=str(dev), shard=[i0, i0 + B], states=[s0, s0 + ns])
    if not dry:
        me["device_name"] = torch.cuda.get_device_name(dev)
        me["pci_bus_id"] = torch.cuda.get_device_properties(dev).pci_bus_id \
            if hasattr(torch.cuda.get_device_properties(dev), "pci_bus_id") else None
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
        formed = dict(backend=dist.get_backend(), world_size=dist.get_world_size(), ranks=ranks)
    else:
        formed = dict(backend=None, world_size=1, ranks=[me])

    group = None
    if args.capi_group and not dry:
        from mpcqp.group import Group, unique_id
        uid = [unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        group = Group(p, rank=(local, world, rank, uid[0]))

    def run_line(batch_local, index_base, steps, warmup, serial=False):
        """time `steps` steps of solve + selection on this rank's shard; returns
        (elapsed max over ranks, kernel ms, select ms, best record, status, iters, eng).
        N > 1: one all-gather of the ranks' records per step (mpcqp.dist.PipelinedSelect: step
        s's collective in flight while step s + 1 solves, unless serial; all of them complete
        inside the timed region)."""
        Bl = batch_local["x0"].shape[0] if not dry else batch_local["B"]
        recs = [torch.zeros(1 + nV, dtype=torch.int64, device=dev) for _ in range(2)]
        gathered = [torch.zeros((world, 1 + nV), dtype=torch.int64, device=dev) for _ in range(2)]
        # one rank: the record the solve writes IS the selection (no copy launch per step)
        best = torch.zeros(1 + nV, dtype=torch.int64, device=dev) if world > 1 else recs[0]
        reduce = host_reduce_records if dry else None
        if dry:
            cost, status, U = batch_local["cost"], batch_local["status"], batch_local["U"]
            eng = None

            def solve_into(rec):
                rec.copy_(torch.from_numpy(host_record(cost, status, U, index_base)))
        elif group is not None:
            # the C-ABI group (csrc/group.hip): solve + the library's own RCCL all-gather of the
            # records + the device reduction, pipelined inside the library
            from mpcqp.engine import BatchEngine
            eng = BatchEngine.wrap(p, group.ctx(0), local)
            d = eng.upload(batch_local)
            torch.cuda.synchronize()
            shard_io = [dict(d, base=index_base)]
            best = torch.zeros(1 + nV, dtype=torch.int64, device=dev)
        else:
            from mpcqp.engine import BatchEngine
            eng = BatchEngine(p, device=local)
            d = eng.upload(batch_local)
            reduce = eng.reduce_records

            def solve_into(rec):
                if fused:
                    eng.solve_select(d, rec, index_base=index_base)
                else:
                    eng.solve(d)
                    eng.select_record(d, rec, index_base=index_base)
        pipe = PipelinedSelect(dist, recs, gathered, best, reduce) \
            if world > 1 and group is None else None

        def step():
            if group is not None:
                group.solve_select(shard_io, [best])
                return
            if pipe is None:  # world == 1: best is recs[0]
                solve_into(recs[0])
                return
            solve_into(pipe.record())
            pipe.submit()
            if serial:
                pipe.drain()

        def sync():
            if group is not None:
                group.sync()
            if pipe is not None:
                pipe.drain()
            if not dry:
                torch.cuda.synchronize()

        for _ in range(warmup):
            step()
        sync()
        if world > 1:
            dist.barrier()
        sync()
        # the timed region is the steps alone: no event record between or around them (each
        # record is a marker packet on the stream, ~4 us apiece at small shards)
        t0 = time.perf_counter()
        for s in range(steps):
            step()
        sync()
        if world > 1:
            dist.barrier()
        sync()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        mpc_ms = sel_ms = None
        kern = {}
        if group is not None:
            # the library's events around each solve call (slot 1) and kernel (2: the one-wave
            # kernel, 3: the overflow launch), a pass of `steps` more steps after the timed ones
            eng.enable_timing(True)
            for _ in range(steps):
                step()
            sync()
            for w, name in ((2, eng.fused_kernel), (3, eng.overflow_kernel)):
                ms, n = eng.kernel_ms_sum(w)
                if n:
                    kern[name] = dict(ms=ms / n, launches=n)
            ms, n = eng.kernel_ms_sum(1)
            mpc_ms = ms / max(1, n)
            sel_ms = 0.0
            eng.enable_timing(False)
            kern["_solver_flops"] = count_solver_flops(eng, step, sync)
            status = d["status"].cpu().numpy()
            iters = d["iters"].cpu().numpy()
        elif not dry:
            # solve and selection durations: torch events around the calls, a separate pass of
            # `steps` more steps after the timed ones
            stream = torch.cuda.current_stream()
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
            rec = recs[0]
            for s in range(steps):
                e = evs[s]
                e[0].record(stream)
                if fused:  # selection record built by the solve kernels' last workgroup
                    eng.solve_select(d, rec, index_base=index_base)
                else:
                    eng.solve(d)
                e[1].record(stream)
                e[2].record(stream)
                if not fused:
                    eng.select_record(d, rec, index_base=index_base)
                e[3].record(stream)
            sync()
            mpc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
            sel_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in evs]))
            if not args.no_kernel_timing:
                # each kernel alone: HIP events inside the library around each launch (on the ctx
                # stream; slot 2 the one-wave fused kernel, 3 the overflow workgroup kernel), over
                # `steps` more steps right after the timed ones -- event records between the two
                # kernels cost ~25 us per step, so they stay out of the timed region
                eng.enable_timing(True)
                for _ in range(steps):
                    step()
                sync()
                for w, name in ((2, eng.fused_kernel), (3, eng.overflow_kernel)):
                    ms, n = eng.kernel_ms_sum(w)
                    if n:
                        kern[name] = dict(ms=ms / n, launches=n)
                eng.enable_timing(False)
                kern["_solver_flops"] = count_solver_flops(eng, step, sync)
            status = d["status"].cpu().numpy()
            iters = d["iters"].cpu().numpy()
        else:
            status, iters = batch_local["status"], np.zeros(Bl, np.int32)
        return elapsed, mpc_ms, sel_ms, best.cpu().numpy(), status, iters, eng, kern

    # ---- strong scaling: the global batch split over the ranks (the metric) ----------------
    if dry:
        cost, status, U = synthetic_shard(B, nV, args.seed, rank, i0)
        local_batch = dict(B=B, cost=cost, status=status, U=U)
    else:
        full = mpcqp.make_batch(p, G, seed=args.seed)
        local_batch = slice_batch(full, i0, B)
        del full
    # per-config lines (N = 1) run first: a fresh process's first few hundred milliseconds of
    # GPU work run while the clocks ramp (the headline kernel's first ~60 launches fall from
    # ~400 to ~355 us), and a short warm-up W would otherwise time them
    per = None
    if world == 1 and not dry and not args.no_per_config:
        per = {}
        for name, conf, Bc, gait in (("B@4096", "B", 4096, None),
                                     ("C@65536", "C", 65536, None),
                                     ("L@65536", "L", 65536, None),
                                     ("B-standing@65536", "B", 65536, "standing"),
                                     ("C-mixed@65536", "C", 65536, "mixed"),
                                     ("E@16384", "E", 16384, None)):
            try:
                per[name] = time_config(conf, Bc, args.seed, gait=gait)
            except Exception as exc:  # report, never hide
                per[name] = dict(error=f"{type(exc).__name__}: {exc}")
    elapsed, mpc_ms, sel_ms, best, status, iters, eng, kern = run_line(
        local_batch, i0, args.steps, args.warmup, serial=args.serial_select)
    bcost, bidx, bU = decode_record(best)
    # N > 1: the same steps with each all-gather waited for before the next solve (reported
    # beside the overlapped value, never as it)
    serial_ms = None
    if world > 1 and not args.serial_select and group is None:
        el_s, *rest = run_line(local_batch, i0, args.steps, args.warmup, serial=True)
        if rest[5] is not None:
            rest[5].close()
        serial_ms = el_s / args.steps * 1e3

    # ---- weak scaling (config D at N = 8): 65,536 per GPU, independent shards -------------
    weak = None
    if args.weak_batch and world > 1 and not dry:
        Bw = args.weak_batch
        wb = mpcqp.make_batch(p, Bw, seed=args.seed + 1000 + rank)
        el_w, ms_w, _, best_w, st_w, _, eng_w, _ = run_line(wb, rank * Bw, args.steps,
                                                            args.warmup)
        eng_w.close()
        cw, iw, _ = decode_record(best_w)
        weak = dict(batch_per_gpu=Bw, global_batch=Bw * world, value=Bw * world /
                    (el_w / args.steps), ms_per_step=el_w / args.steps * 1e3,
                    kernel_ms=ms_w, solved_frac_rank0=float(np.mean(st_w == 0)),
                    selected=dict(index=iw, cost=cw), scaling="weak",
                    note="config D at N = 8 (524,288 instances); shards seeded per rank")

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = G / (elapsed / args.steps)
        solved = float(np.mean(status == 0))
        out = dict(metric=METRIC, value=value, unit="QP/s", n_gpus=world, steps=args.steps,
                   warmup=args.warmup, ms_per_step=ms_per_step, higher_is_better=True,
                   scaling="strong", vs_baseline=None, dtype="f64",
                   data="synthetic (seeded SURVEY.md 8d TRON1 states x 16 gait candidates)")
        cfg = dict(workload=f"TRON1 SRBM MPC {p['nx']}x{p['nu']} N={p['N']} "
                            f"({'box+friction' if p['constraints'] else 'box'}, R = "
                            f"{p['R'][0, 0]:g} I), linearise+discretise+condense+solve + "
                            f"min-cost selection, global batch {G} split over {world} GPU(s)",
                   global_batch=G, batch_per_gpu=B, horizon=p["N"], nx=p["nx"], nu=p["nu"],
                   config=args.config, parallelism=f"dp{world}",
                   selection=(("record fused into the solve kernels (last workgroup)" if fused
                               else "k_select_min record") +
                              (" + one all-gather of [key | U] records + k_reduce_records"
                               if world > 1 else " (single GPU)")),
                   selected=dict(index=bidx, cost=bcost))
        if group is not None:
            cfg["selection"] = ("C-ABI group (mpcqp_group_solve_select, csrc/group.hip): fused "
                                "record + ncclAllGather from libmpcqp.so's own communicator + "
                                "k_reduce_records, the collective of step s beside the solve of "
                                "step s + 1")
            cfg["capi_group"] = True
        if world > 1:
            cfg["selection_overlap"] = (
                "serial: each all-gather waited for before the next solve" if args.serial_select
                else "step s's all-gather in flight during step s + 1's solve (mpcqp.dist."
                     "PipelinedSelect); every selection completes inside the timed region")
            cfg["serial_select_ms_per_step"] = serial_ms
            cfg["pipelined_ms_per_step"] = elapsed / args.steps * 1e3
        cfg["process_group"] = formed
        covered = sorted(tuple(r["shard"]) for r in formed["ranks"])
        cfg["shards_cover_global_batch"] = (covered[0][0] == 0 and covered[-1][1] == G and all(
            a[1] == b[0] for a, b in zip(covered, covered[1:])))
    if rank == 0 and dry:
        cfg["dry_run"] = "selection only: synthetic costs, gloo, no solve"
        out["config"] = cfg
        print(json.dumps(out), flush=True)
    elif rank == 0:
        f_qp = flops_per_qp(p, iters.mean())
        # the dominant kernel's own launches (library events around it); the events around the
        # whole solve in the timed steps (mpc_ms) also hold the overflow launch
        k_ms = kern[eng.fused_kernel]["ms"] if eng.fused_kernel in kern else mpc_ms
        # the work of the instances that kernel solved (an overflow instance is the workgroup
        # kernel's, timed apart): the closed-form path's own algorithmic count, the solver's
        # part counted by the kernel (its pass after the timed steps)
        solver = kern.pop("_solver_flops", None)
        fl, n_solved, basis = algorithmic_work(p, local_batch.get("contact"), iters, eng.pair_nf,
                                               solver)
        achieved = fl / (k_ms * 1e-3) / 1e12
        traffic, traffic_tag, traffic_lib = pmc_traffic(args.config, B)
        build = lib_build_id()
        kms = {k: v["ms"] for k, v in kern.items()}
        kms["mpcqp_batch_solve" + ("_select" if fused else "") +
            " (events around the call, a pass after the timed steps)"] = mpc_ms
        if not fused:
            kms["k_select_min"] = sel_ms
        cfg.update(solved_frac=solved, mean_solver_iters=float(iters.mean()),
                   max_solver_iters=int(iters.max()),
                   fast_path=eng.fast_path, select=args.select, kernel_ms=kms,
                   kernel_launches={k: v["launches"] for k, v in kern.items()})
        alg_bytes = (config_bytes(p) if p["model"] == 2 else
                     algorithmic_bytes(p["nx"], p["nu"], p["N"])) * B
        roof = dict(bound="fp64-valu",
                    compute_unit=("fp64 VALU (k_mpc_pair issues no MFMA)"
                                  if eng.fused_kernel == "k_mpc_pair" else "fp64 VALU + MFMA"),
                    kernel=eng.fused_kernel, kernel_ms=k_ms, achieved=achieved,
                    peak=FP64_PEAK_TFLOPS, unit="TFLOP/s", frac=achieved / FP64_PEAK_TFLOPS,
                    traffic=traffic,
                    flops_basis=basis + " (DESIGN.md section 4 'Roofline accounting')",
                    solver_flops_per_launch=(solver[0] / solver[1]) if solver and solver[1]
                    else None,
                    algorithmic_flops_per_qp=fl / max(1, n_solved), instances=n_solved,
                    work_rate_vs_survey_8d=dict(
                        flops_per_qp=f_qp, tflops=f_qp * B / (k_ms * 1e-3) / 1e12,
                        frac=f_qp * B / (k_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                        note="SURVEY.md 8d prices the reference's dense path (expm, powers, "
                             "Phi chain, B'QB); the closed form does not execute it, so this "
                             "is a work rate, not a roofline fraction"),
                    traffic_source=(f"profiles/{traffic_tag}_summary.json (rocprofv3 PMC, "
                                    "2 x FETCH_SIZE + WRITE_SIZE)") if traffic else None,
                    traffic_lib_build_id=traffic_lib, lib_build_id=build,
                    traffic_matches_library=(traffic_lib == build) if traffic else None,
                    algorithmic_bytes_per_launch=alg_bytes,
                    mfma_busy_frac=None)
        roof.update(hbm_fields(traffic, k_ms, alg_bytes))
        ex = pmc_executed(args.config, B)
        if ex:
            per_launch = ex["executed_flops_per_launch"]
            roof["executed_tflops"] = per_launch / (k_ms * 1e-3) / 1e12
            roof["pipe_frac"] = roof["executed_tflops"] / FP64_PEAK_TFLOPS
            roof["lane_efficiency"] = achieved / roof["executed_tflops"]
            roof["mfma_busy_frac"] = ex.get("mfma_busy_frac")
            roof["executed_source"] = f"profiles/{ex.get('file', 'pmc_flops.json')} " \
                                      "(64 lanes x SQ_INSTS_VALU_FLOPS_FP64, a per-wave-" \
                                      "instruction count: EXEC-masked lanes included, an " \
                                      "upper bound; + MFMA ops; SQ_VALU_MFMA_BUSY_CYCLES for " \
                                      "mfma_busy_frac)"
            roof["executed_tag"] = ex.get("tag")
            roof["executed_matches_library"] = ex.get("lib_build_id") == build
        out["roofline"] = roof
        if weak:
            cfg["weak"] = weak
        if world == 1 and not args.no_host_path:
            cfg["pcie_inclusive_qps"] = host_staged_rate(eng, local_batch, p, locked=True)
            cfg["pcie_inclusive_qps_pageable"] = host_staged_rate(eng, local_batch, p)
            cfg["pcie_inclusive_note"] = (
                "mpcqp_batch_solve_host, host arrays in / out, synchronous: pcie_inclusive_qps "
                "with the caller's arrays page-locked once (mpcqp_host_register: DMA straight "
                "from / into them, chunks pipelined over three streams), _pageable through the "
                "context's pinned staging (a host memcpy each way)")
            cfg["gait_fused_qps"] = gait_fused_rate(eng, p, B, args.seed)
            cfg["per_tick_latency"] = per_tick_latency(p, args.seed, device=local)
        out["config"] = cfg
        eng.close()
        if per is not None:
            cfg["per_config"] = per
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(p, local_batch)
        print(json.dumps(out), flush=True)
    elif eng is not None:
        eng.close()
    if group is not None:
        group.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
