"""Multi-GPU plumbing on the device (one MI355X).

- bench.py through its spawn launcher at N = 1 (`--gpus 1 --spawn`): one rank process, an RCCL (nccl backend)
  process group of one, the HIP kernel's counters through StatsExchange's asynchronous all-reduce — the line's
  stats_digest equals the standalone run's, and it reports rccl_world_size 1 and the rank's kernel time.
- A context over four device slots (devices=[0, 0, 0, 0], what a node-wide daemon driving every GPU from one
  process uses; one card here) built by importing a compiled image (infw_table_import: no compile), then
  incrementally committed: every slot classifies like the oracle after each epoch, the slots upload / patch on
  their own host threads (info: n_device_slots, device_ms_max).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import infw
from infw import workloads as W
from infw.batch import SoaBatch
from parity import gpu_run, oracle_for

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def test_spawn_rccl_world1_digest_equals_standalone():
    common = ["--steps", "3", "--warmup", "1", "--batch", str(1 << 22), "--prefixes", "50000", "--templates", "256",
              "--no-cpu-baseline"]
    solo = _bench("--gpus", "1", *common)
    spawned = _bench("--gpus", "1", "--spawn", *common)
    assert solo["rccl_world_size"] is None and spawned["rccl_world_size"] == 1
    assert spawned["config"]["stats_digest"] == solo["config"]["stats_digest"]
    assert spawned["config"]["packets_counted_in_stats"] == solo["config"]["packets_counted_in_stats"] > 0
    assert len(spawned["per_rank"]) == 1 and spawned["per_rank"][0]["kernel_ms_avg"] > 0
    assert spawned["n_gpus"] == 1 and spawned["value"] > 0


def test_four_slot_context_from_imported_image():
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=128)
    src = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 64)
    wl.load_into(src)
    src.commit()
    clf = infw.Classifier(devices=[0, 0, 0, 0], max_entries=wl.n_entries + 64)
    clf.import_image(src.export_image())
    info = clf.info()
    assert info["imported"] == 1 and info["n_device_slots"] == 4 and info["device_ms_max"] > 0
    m = oracle_for(wl)
    dev = torch.device("cuda", 0)
    n = 1 << 15
    batches = []
    for d in range(4):
        b = SoaBatch.empty(n, dev)
        wl.gen_device(b, d * n, 0)
        batches.append(b)
    keys = wl.keys_bytes().reshape(-1, 24)
    tmpl = wl.templates_bytes().reshape(-1, 1200)
    for epoch in range(3):
        for d in range(4):
            gres, _ = gpu_run(clf, batches[d], n, dev_index=d)
            hdr, cap, pl, ifx = wl.frames(d * n, n)
            ores, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
            assert np.array_equal(gres, ores), (epoch, d)
        for i in range(epoch, keys.shape[0], 5):  # an incremental commit: deletes and rewrites
            kb = keys[i].tobytes()
            if i % 2:
                assert clf.delete_rc(infw.LpmIpKeySt.from_buffer_copy(kb)) == m.delete(kb)
            else:
                vb = tmpl[(i * 7 + epoch) % tmpl.shape[0]].tobytes()
                assert clf.update_rc(infw.LpmIpKeySt.from_buffer_copy(kb),
                                     infw.RulesValSt.from_buffer_copy(vb)) == m.update(kb, vb)
        clf.commit()
        assert clf.info()["commit_mode"] in (infw.COMMIT_INCREMENTAL, infw.COMMIT_REUPLOAD)
        assert clf.info()["n_device_slots"] == 4
