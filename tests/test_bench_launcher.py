"""bench.py's own multi-rank launcher: `bench.py --gpus 2`
without WORLD_SIZE starts two ranks through torch.distributed.run, shards the global batch on
whole states, and selects the global minimum with ONE all-gather of the selection records.
Run on CPU over gloo with --selection-dry-run (seeded synthetic costs replace the GPU solve),
so the launcher, the sharding and the selection are exactly the code the GPU run executes."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT


def _run(world, G, seed=11):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world),
           "--selection-dry-run", "--steps", "2", "--warmup", "1", "--global-batch", str(G),
           "--seed", str(seed)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # ONE JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("world,G", [(1, 4096), (2, 4096), (3, 4097 * 16)])
def test_bench_launcher_global_argmin(world, G):
    """(3, 4097 x 16): an uneven state split, 1366 / 1366 / 1365 states over three ranks"""
    sys.path.insert(0, ROOT)
    import bench
    from mpcqp.dist import host_select

    seed = 11
    r = _run(world, G, seed)
    assert r["n_gpus"] == world
    assert r["scaling"] == "strong" and r["config"]["global_batch"] == G
    assert r["config"]["parallelism"] == f"dp{world}"
    # host reference over the whole batch: the synthetic costs are a function of the index
    cost, status, _ = bench.synthetic_shard(G, 60, seed, 0, 0)
    c0, i0 = host_select(cost, status)
    assert r["config"]["selected"]["index"] == i0
    assert r["config"]["selected"]["cost"] == pytest.approx(c0)


def test_shards_cover_whole_states():
    sys.path.insert(0, ROOT)
    import bench
    for S, w in ((4096, 8), (4097, 8), (10, 3)):
        cover = []
        for r in range(w):
            s0, n = bench.shard(S, w, r)
            cover.extend(range(s0, s0 + n))
        assert cover == list(range(S))


def test_bench_line_records_the_formed_group():
    """the line names the world size the process group formed, each rank's
    device and shard, and both the pipelined and the serial-selection step times"""
    r = _run(2, 4096)
    cfg = r["config"]
    pg = cfg["process_group"]
    assert pg["world_size"] == 2 and pg["backend"] == "gloo"
    ranks = sorted(pg["ranks"], key=lambda x: x["rank"])
    assert [x["rank"] for x in ranks] == [0, 1]
    assert [x["local_rank"] for x in ranks] == [0, 1]
    assert all(x["device"] == "cpu" for x in ranks)  # dry run; cuda:<local_rank> on the GPU box
    assert ranks[0]["shard"] == [0, 2048] and ranks[1]["shard"] == [2048, 4096]
    assert cfg["shards_cover_global_batch"] is True
    assert cfg["pipelined_ms_per_step"] == pytest.approx(r["ms_per_step"])
    assert cfg["serial_select_ms_per_step"] > 0
