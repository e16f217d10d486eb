"""bench.py's launcher on the CPU (`--gpus N` must never silently measure one GPU).

- `--gpus 2` with no WORLD_SIZE spawns 2 rank processes (torch.multiprocessing spawn); with --host-walk (test only:
  gloo, the compiled host image walked by infw_debug_walk) they shard a fixed job, rank 1 imports rank 0's compiled
  table image, the counters go through StatsExchange, and the line reports rccl_world_size 2 with the same
  stats_digest as one process and as the spawn path at N = 1 — and as the counters of the whole job walked here.
- Under torch.distributed.run, --gpus must equal WORLD_SIZE.
- Without a HIP device, --gpus 2 refuses instead of running one rank.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JOB = 30011


def _bench(*a, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *a], cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=600)


def _line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_gpus_2_spawns_two_ranks_same_digest():
    common = ["--host-walk", "--steps", "2", "--warmup", "1", "--global-packets", str(JOB)]
    two = _line(_bench("--gpus", "2", *common))
    one = _line(_bench("--gpus", "1", *common))
    sp1 = _line(_bench("--gpus", "1", "--spawn", *common))
    assert two["rccl_world_size"] == 2 and two["backend"] == "gloo" and not two["valid_measurement"]
    assert [r["rank"] for r in two["per_rank"]] == [0, 1]
    assert [r["tables"] for r in two["per_rank"]] == ["compiled", "imported"]
    assert sum(r["packets_per_step"] for r in two["per_rank"]) == JOB
    assert one["rccl_world_size"] is None and sp1["rccl_world_size"] == 1
    assert two["config"]["stats_digest"] == one["config"]["stats_digest"] == sp1["config"]["stats_digest"]
    four = _line(_bench("--gpus", "4", *common))  # the driver's scaling run uses 1, 2, 4, 8 ranks
    assert four["rccl_world_size"] == 4 and four["config"]["stats_digest"] == one["config"]["stats_digest"]
    assert [r["tables"] for r in four["per_rank"]] == ["compiled"] + ["imported"] * 3
    eight = _line(_bench("--gpus", "8", *common))  # the 8-GPU node's rank count (image verified on 7 imports)
    assert eight["rccl_world_size"] == 8 and eight["config"]["stats_digest"] == one["config"]["stats_digest"]
    assert [r["tables"] for r in eight["per_rank"]] == ["compiled"] + ["imported"] * 7
    assert sum(r["packets_per_step"] for r in eight["per_rank"]) == JOB
    # the digest is the whole job's counters, walked here in one piece
    import infw
    from bench import host_counters, stats_digest
    from infw import workloads as W
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16)
    wl.load_into(c)
    c.commit()
    t = wl.tuples(0, JOB)
    assert stats_digest(host_counters(c.debug_walk(t), t[:, 5])) == two["config"]["stats_digest"]


def test_in_process_shape_same_digest_as_ranks():
    """--in-process (one context, N slots, a host thread per slot; counters summed per rule over the slots) on a CPU
    box: with --host-walk each slot's thread walks its shard through the shared host image concurrently; for the
    same fixed job the digest equals the rank path's at any N."""
    common = ["--host-walk", "--steps", "2", "--warmup", "1", "--global-packets", str(JOB)]
    ranks = _line(_bench("--gpus", "2", *common))
    for n in (1, 2, 8):
        ip = _line(_bench("--gpus", str(n), "--in-process", *common))
        assert ip["mode"] == "in-process" and ip["device_slots"] == n and not ip["valid_measurement"]
        assert sum(s["packets_per_step"] for s in ip["per_slot"]) == JOB
        assert ip["config"]["stats_digest"] == ranks["config"]["stats_digest"], n


def test_bench_options_reach_the_context():
    """--opt NAME=VALUE sets a per-context option on every context the bench creates; a bad one fails loudly."""
    common = ["--host-walk", "--steps", "1", "--warmup", "0", "--global-packets", str(JOB)]
    base = _line(_bench(*common))
    forced = _line(_bench(*common, "--opt", "short_table=1", "--opt", "dt_parts=4"))
    assert forced["config"]["stats_digest"] == base["config"]["stats_digest"]  # forms never change results
    bad = _bench(*common, "--opt", "no_such_option=1")
    assert bad.returncode != 0 and "unknown option" in bad.stderr


def test_torchrun_world_size_must_match_gpus():
    p = _bench("--gpus", "3", "--host-walk", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "--gpus 3 but WORLD_SIZE=2" in p.stderr


def test_gpus_n_without_devices_refuses():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("HIP devices present")
    p = _bench("--gpus", "2", "--steps", "1")
    assert p.returncode != 0 and "--gpus 2 but" in p.stderr and "HIP device" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def test_host_counters_match_stats_from_results():
    from bench import host_counters
    from parity import stats_from_results
    rng = np.random.default_rng(3)
    res = (rng.integers(0, 1200, 5000).astype(np.uint32) << 8) | rng.integers(0, 4, 5000).astype(np.uint32)
    pl = rng.integers(60, 9000, 5000).astype(np.uint32)
    assert np.array_equal(host_counters(res, pl), stats_from_results(res, pl))
