"""The library's own multi-GPU shape on the device: ONE process, ONE context over N device slots, one host thread
and HIP stream per slot classifying its shard concurrently (bench.py --in-process), the counters summed per rule over
the slots like the per-CPU read of statistics.go:126-157 over kernel.c:36-41's PERCPU map.  Rehearsed on one GPU with
every slot on device 0 (--slots-on-gpu0) at N = 1, 2, 8: for configs[3]'s fixed-job sharding the stats digest must
equal the RCCL rank path's (bench.py --spawn, an RCCL group of one) for the same job."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JOB = (1 << 24) + 4099
COMMON = ["--steps", "2", "--warmup", "1", "--global-packets", str(JOB), "--prefixes", "100000", "--templates", "512",
          "--no-cpu-baseline", "--no-line-rates"]


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _bench(*a):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *a], cwd=ROOT, env=e, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])


@pytest.fixture(scope="module")
def rccl_digest():
    line = _bench("--gpus", "1", "--spawn", *COMMON)
    assert line["rccl_world_size"] == 1
    return line["config"]["stats_digest"], line["config"]["packets_counted_in_stats"]


@pytest.mark.parametrize("n", [1, 2, 8])
def test_in_process_slots_equal_rank_path(rccl_digest, n):
    line = _bench("--in-process", "--slots-on-gpu0", "--gpus", str(n), *COMMON)
    assert line["mode"] == "in-process" and line["device_slots"] == n and line["n_gpus"] == 1
    assert [s["slot"] for s in line["per_slot"]] == list(range(n))
    assert sum(s["packets_per_step"] for s in line["per_slot"]) == JOB
    assert all(s["kernel_ms_avg"] > 0 for s in line["per_slot"])
    assert line["config"]["tables"]["n_device_slots"] == n
    digest, counted = rccl_digest
    assert line["config"]["stats_digest"] == digest and line["config"]["packets_counted_in_stats"] == counted
    assert line["value"] > 0
