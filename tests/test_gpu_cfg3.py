"""configs[3] on the device (BASELINE.json configs[3]: a 1B-packet batch sharded over 8 GPUs, replicated tables, the
per-rule statistics all-reduced).  One MI355X here; the sharding and the counter sum are what the 8-GPU run rests on,
so they are checked at the full job size:

(a) bench.py's own job — `--gpus 1 --spawn --global-packets 2^30`: one rank process, an RCCL (nccl) process group of
    one, the 1,073,741,824 packets generated in HBM from their global index and classified in one launch, the
    counter block through StatsExchange's all-reduce — reports a stats_digest D;
(b) the same job as 8 shards `shard_range(G, g, 8)` (what rank g of 8 classifies) one after another in one process:
    the sum of the 8 shards' counter blocks has digest D, and the first and last 64k packets of every shard are
    bit-exact against the oracle (result words and verdicts), so the shard edges neither drop nor repeat packets;
(c) a context over eight device slots (devices=[0]*8 — the per-CPU slots of the reference's PERCPU stats map,
    kernel.c:36-41, become device slots) built by importing (b)'s compiled image, shard g classified on slot g: slot g's
    counters equal shard g's, and summing the slots rule by rule with infw_stats_read — the read statistics.go:126-157
    does per rule over the per-CPU values — gives digest D again.
"""
import hashlib
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
from parity import oracle_for

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = 1 << 30     # configs[3]: 1B packets
K = 8           # ranks of the 8-GPU node
EDGE = 1 << 16  # packets checked against the oracle at each end of every shard


def shard_range(global_n, rank, world):  # bench.py shard_range
    return global_n * rank // world, global_n * (rank + 1) // world


def digest(block):  # bench.py stats_digest: SHA-256 of the 1024 x 4 u64 counter block
    return hashlib.sha256(np.ascontiguousarray(np.asarray(block).astype("<u8").reshape(1024, 4)).tobytes()).hexdigest()


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.fixture(scope="module")
def bench_job():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--spawn", "--global-packets",
                        str(G), "--steps", "2", "--warmup", "1", "--no-cpu-baseline"], cwd=ROOT, env=e,
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.timeout(300)
def test_cfg3_bench_job_on_one_gpu(bench_job):
    line = bench_job
    assert line["rccl_world_size"] == 1 and line["scaling"] == "strong"
    assert line["config"]["global_batch"] == G and line["per_rank"][0]["packets_per_step"] == G
    assert line["config"]["packets_counted_in_stats"] > G // 2 * line["steps"]
    assert line["value"] > 0 and line["roofline"]["kernel_ms_avg"] > 0


@pytest.mark.timeout(600)
def test_cfg3_shards_and_device_slots(bench_job):
    want = bench_job["config"]["stats_digest"]
    dev = torch.device("cuda", 0)
    wl = W.Workload(W.CFG2_MIXED_1M)
    one = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(one, order=wl.shuffled_order())  # bench.py's table (same map in any order)
    one.commit()
    eight = infw.Classifier(devices=[0] * K, max_entries=wl.n_entries + 16)
    eight.import_image(one.export_image())
    assert eight.info()["n_device_slots"] == K and eight.info()["imported"] == 1
    eight.stats_reset()
    m = oracle_for(wl)

    nmax = max(b - a for a, b in (shard_range(G, g, K) for g in range(K)))
    buf = SoaBatch.empty(nmax, dev)
    res = torch.empty(nmax, dtype=torch.int32, device=dev)
    ver = torch.empty(nmax, dtype=torch.uint8, device=dev)
    total = np.zeros((1024, 4), np.uint64)
    per_shard = []
    ends = 0
    for g in range(K):
        a, b = shard_range(G, g, K)
        n = b - a
        batch = buf.slice(0, n)
        wl.gen_device(batch, start=a, dev_ordinal=0)
        # (b) the shard on the one-slot context, its own counter block
        blk = torch.zeros((1024, 4), dtype=torch.int64, device=dev)
        one.stats_bind(0, blk.data_ptr())
        one.classify(batch, results=res[:n], verdicts=ver[:n])
        torch.cuda.synchronize()
        one.stats_bind(0, None)
        c = blk.cpu().numpy().view(np.uint64).copy()
        per_shard.append(c)
        total += c
        for lo in (a, b - EDGE):  # shard edges against the oracle
            hdr, cap, pl, ifx = wl.frames(lo, EDGE)
            ores, over, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=16)
            gres = res[lo - a:lo - a + EDGE].cpu().numpy().view(np.uint32)
            gver = ver[lo - a:lo - a + EDGE].cpu().numpy()
            assert np.array_equal(gres, ores), (g, lo, np.nonzero(gres != ores)[0][:5])
            assert np.array_equal(gver, over), (g, lo)
            ends += 1
        # (c) the same shard on device slot g of the eight-slot context (the result words must agree too)
        res2 = torch.empty(n, dtype=torch.int32, device=dev)
        eight.classify(batch, results=res2, dev=g)
        torch.cuda.synchronize()
        assert torch.equal(res2, res[:n]), g
        del res2
    assert ends == 2 * K
    assert digest(total) == want, "sum of the 8 shards' counters != the 1B-packet job's all-reduced counters"
    # (the bench line counts the packets of all its timed steps)
    assert int(total[:, 0].sum() + total[:, 2].sum()) * bench_job["steps"] == bench_job["config"]["packets_counted_in_stats"]

    # per-slot counters: slot g holds shard g's; summed rule by rule (statistics.go:126-157) they give the job's
    slots = np.zeros((K, 1024, 4), np.uint64)
    for rule in range(1024):
        for s, st in enumerate(eight.stats_read(rule)):
            slots[s, rule] = (st.allow_packets, st.allow_bytes, st.deny_packets, st.deny_bytes)
    for g in range(K):
        assert np.array_equal(slots[g], per_shard[g]), g
    assert digest(slots.sum(axis=0, dtype=np.uint64)) == want
