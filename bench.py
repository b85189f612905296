#!/usr/bin/env python3
"""Benchmark: QP solves/s for the TRON1 13-state / 6-input / N=10 SRBM MPC (BASELINE.json
metric), batch 65,536 per GPU, 1..8 MI355X (one process per GPU, weak scaling: config D is
524,288 = 65,536 x 8).

One step = one pass of the hot path over the whole per-GPU batch, inputs resident in HBM:
  k_mpc_pair (linearise + discretise + condense + Goldfarb-Idnani solve, fused, two QPs per
  wavefront; k_mpc, one QP per wavefront, where nf > 30) -> k_select_min (min-cost key)
  -> [N>1] RCCL MIN all-reduce of the 8-byte key + broadcast of the winner's U (480 B).

Prints ONE JSON line on rank 0 (driver contract).
  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config B|C|L]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))

FP64_PEAK_TFLOPS = 78.6  # MI355X dense FP64 (vector = matrix), AMD spec; SURVEY.md 8d


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


def pmc_traffic(config: str, batch: int):
    """HBM bytes per fused-kernel launch from the committed rocprofv3 PMC summary
    (tools/profile_run.sh + tools/summarize_profile.py), if it matches this workload."""
    try:
        t = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    except (OSError, ValueError):
        return None, None
    if t.get("config") != config or t.get("batch") != batch:
        return None, None
    return t.get("hbm_bytes_per_launch"), t.get("tag")


def cpu_baseline(p, batch, budget_s=12.0):
    """The oracle (C restatement of the reference path, OpenMP over the batch) on the host."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # CPU baseline leg only

    threads = max(1, min(16, os.cpu_count() or 1))
    n0 = min(256, batch["x0"].shape[0])
    sub = {k: v[:n0] for k, v in batch.items()}
    t = time.perf_counter()
    oracle.srbm_batch(p, sub["x0"], sub["xref"], sub["lin"], sub["contact"], nthreads=threads)
    rate0 = n0 / max(1e-6, time.perf_counter() - t)
    n = int(min(batch["x0"].shape[0], max(n0, rate0 * budget_s)))
    sub = {k: v[:n] for k, v in batch.items()}
    # repeat the sample until ~budget_s of CPU work is timed (10-30 s guideline)
    o, done, dt, passes = None, 0, 0.0, 0
    while passes == 0 or (dt < budget_s and passes < 8):
        t = time.perf_counter()
        r = oracle.srbm_batch(p, sub["x0"], sub["xref"], sub["lin"], sub["contact"],
                              nthreads=threads)
        dt += time.perf_counter() - t
        done += n
        passes += 1
        o = o if o is not None else r
    n1 = min(n, max(16, int(done / dt / threads * 2.0)))  # ~2 s single-thread sample
    t = time.perf_counter()
    oracle.srbm_batch(p, sub["x0"][:n1], sub["xref"][:n1], sub["lin"][:n1], sub["contact"][:n1],
                      nthreads=1)
    one = n1 / (time.perf_counter() - t)
    return dict(value=done / dt, unit="QP/s", cores=threads, kind="port",
                single_thread_value=one,
                sample=f"first {n} instances of the rank-0 batch x {passes} passes, "
                       f"oracle/mpcqp_oracle.c (reference-literal dense condensing + "
                       f"Goldfarb-Idnani), OpenMP {threads} threads, {dt:.1f} s"), o


def host_staged_rate(eng, batch, p, reps=5):
    """QP/s through mpcqp_batch_solve_host: host arrays in, H2D + fused kernel + D2H, synchronous
    (the PCIe-inclusive number; never `value`)."""
    import ctypes as C

    from mpcqp._lib import lib
    B = batch["x0"].shape[0]
    nV = p["nu"] * p["N"]
    U = np.zeros(B * nV)
    cost = np.zeros(B)
    st = np.zeros(B, np.int32)
    it = np.zeros(B, np.int32)
    ins = [np.ascontiguousarray(batch[k]) for k in ("x0", "xref", "lin", "contact")]
    ptr = lambda a: C.c_void_p(a.ctypes.data)
    call = lambda: lib().mpcqp_batch_solve_host(eng.ctx, B, *[ptr(a) for a in ins], ptr(U),
                                                 ptr(cost), ptr(st), ptr(it))
    assert call() == 0
    t = time.perf_counter()
    for _ in range(reps):
        call()
    return B * reps / (time.perf_counter() - t)


def gait_fused_rate(eng, p, B, seed, reps=10):
    """QP/s of mpcqp_batch_solve_gait: the same step with x0/xref/lin/contact generated on
    chip from per-state data (B/16 states x 16 gait candidates)."""
    import torch

    import mpcqp
    if not eng.fast_path or p["model"] != 0:
        return None
    Cc = 16
    g = eng.upload_gait(mpcqp.make_gait_states(p, B // Cc, seed=seed, candidates=Cc))
    eng.solve_gait(g)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        eng.solve_gait(g)
    e1.record()
    torch.cuda.synchronize()
    return g["B"] * reps / (e0.elapsed_time(e1) * 1e-3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="instances per GPU")
    ap.add_argument("--config", default="B")
    ap.add_argument("--seed", type=int, default=20250404)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import mpcqp
    from mpcqp.dist import select_global
    from mpcqp.engine import BatchEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))

    p = mpcqp.model_params(args.config)
    B = args.batch
    batch = mpcqp.make_batch(p, B, seed=args.seed + rank)
    eng = BatchEngine(p, device=local)
    d = eng.upload(batch)
    nV = eng.nV
    ubest = torch.zeros(nV, dtype=torch.float64, device=f"cuda:{local}")

    def step():
        eng.solve(d)
        key = eng.select_min(d, index_base=rank * B)
        if world > 1:
            select_global(dist, key, d["U"], B, ubest)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s in range(args.steps):
        e = ev[s]
        e[0].record(stream)
        eng.solve(d)
        e[1].record(stream)
        e[2].record(stream)
        key = eng.select_min(d, index_base=rank * B)
        e[3].record(stream)
        if world > 1:
            select_global(dist, key, d["U"], B, ubest)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    mpc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    sel_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in ev]))
    status = d["status"].cpu().numpy()
    iters = d["iters"].cpu().numpy()
    solved = float(np.mean(status == 0))

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        total = B * world
        fl = algorithmic_flops(p["nx"], p["nu"], p["N"])
        f_qp = fl["condense"] + fl["solve_fixed"] + fl["per_iter"] * float(iters.mean())
        dom_flops = f_qp * B
        achieved = dom_flops / (mpc_ms * 1e-3) / 1e12
        traffic, traffic_tag = pmc_traffic(args.config, B)
        out = dict(
            metric="QP solves/sec, 13-state N=10 SRBM MPC, batch=65536 at 1/2/4/8 MI355X",
            value=total / (elapsed / args.steps), unit="QP/s", n_gpus=world, steps=args.steps,
            warmup=args.warmup, ms_per_step=ms_per_step, higher_is_better=True,
            scaling="weak", vs_baseline=None, dtype="f64",
            data="synthetic (seeded SURVEY.md 8d TRON1 states x 16 gait candidates)",
            config=dict(workload=f"TRON1 SRBM MPC {p['nx']}x{p['nu']} N={p['N']} "
                                 f"({'box+friction' if p['constraints'] else 'box'}), "
                                 f"linearise+discretise+condense+solve, batch {B} per GPU",
                        batch_per_gpu=B, global_batch=total, horizon=p["N"], nx=p["nx"],
                        nu=p["nu"], config=args.config, parallelism=f"dp{world}",
                        solved_frac=solved, mean_solver_iters=float(iters.mean()),
                        fast_path=eng.fast_path,
                        kernel_ms={eng.fused_kernel: mpc_ms, "k_select_min": sel_ms}),
            roofline=dict(bound="mfma", kernel=eng.fused_kernel, achieved=achieved,
                          peak=FP64_PEAK_TFLOPS, unit="TFLOP/s",
                          frac=achieved / FP64_PEAK_TFLOPS, traffic=traffic,
                          traffic_source=(f"profiles/{traffic_tag}_summary.json (rocprofv3 PMC, "
                                          "2 x FETCH_SIZE + WRITE_SIZE)") if traffic else None,
                          algorithmic_bytes_per_launch=algorithmic_bytes(
                              p["nx"], p["nu"], p["N"]) * B,
                          algorithmic_flops_per_qp=f_qp,
                          basis="SURVEY.md 8d algorithmic flops (F_fixed + F_iter x mean iters); "
                                "the closed-form path executes fewer, so frac can exceed 1",
                          whole_step_tflops=dom_flops / (ms_per_step * 1e-3) / 1e12),
        )
        out["config"]["pcie_inclusive_qps"] = host_staged_rate(eng, batch, p)
        out["config"]["gait_fused_qps"] = gait_fused_rate(eng, p, B, args.seed)
        if not args.no_cpu_baseline:
            cb, _ = cpu_baseline(p, batch)
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
