"""Multi-process path on the CPU (gloo, world size 2): each rank classifies its own
contiguous shard of the global packet index range, step by step, and the per-rule
counters go through bench.py's own StatsExchange (double-buffered asynchronous
all-reduce, RCCL on the GPU box) — the totals equal a single-process run over the
whole range.

The per-rank classification here is the product's compiled-table walk on the host
(infw_debug_walk); on the GPU box the HIP kernel does it (tests/test_gpu_parity.py)."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_TOTAL = 1 << 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


STEPS = 4


def _classifier():
    import infw
    from infw import workloads as W
    from parity import stats_from_results
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    wl.load_into(c)
    c.commit()

    def stats_for(start, n):
        t = wl.tuples(start, n)
        return stats_from_results(c.debug_walk(t), t[:, 5])
    return stats_for


def _stats_for(start, n):
    return _classifier()(start, n)


def _worker(rank, world, port, out_path):
    sys.path[:0] = [os.path.dirname(os.path.abspath(__file__)),
                    os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ingress-node-firewall_amd"),
                    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bench import StatsExchange
    stats_for = _classifier()
    n = N_TOTAL // world
    m = n // STEPS
    ex = StatsExchange(lambda: torch.zeros((1024, 4), dtype=torch.int64), True)
    for k in range(STEPS):                    # bench.py's step loop: step k = packets [k·m, (k+1)·m) of the shard
        buf = ex.begin(k)
        buf.copy_(torch.from_numpy(stats_for(rank * n + k * m, m).view(np.int64)))
        ex.end(k)
    ex.drain()
    st = ex.total
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py: max-over-ranks timing
    if rank == 0:
        np.save(out_path, st.numpy().view(np.uint64))
        assert t.item() == world
    dist.destroy_process_group()


def test_two_rank_shards_allreduce_equal_single_process(tmp_path):
    out = str(tmp_path / "st.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, start_method="spawn")
    got = np.load(out)
    want = _stats_for(0, N_TOTAL)
    assert np.array_equal(got, want)
    assert got[:, 0].sum() + got[:, 2].sum() > N_TOTAL // 2


def _strong_worker(rank, world, port, n_total, out_path):
    """bench.py --global-packets: rank g classifies [g·N/k, (g+1)·N/k) of one fixed job; the all-reduced
    counters' digest is what the bench line reports."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.dirname(os.path.abspath(__file__)), root, os.path.join(root, "ingress-node-firewall_amd"),
                    os.path.join(root, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bench import StatsExchange, shard_range, stats_digest
    stats_for = _classifier()
    a, b = shard_range(n_total, rank, world)
    ex = StatsExchange(lambda: torch.zeros((1024, 4), dtype=torch.int64), True)
    for k in range(2):  # two steps over the same shard, as bench.py repeats its resident batch
        buf = ex.begin(k)
        if b > a:
            buf.copy_(torch.from_numpy(stats_for(a, b - a).view(np.int64)))
        ex.end(k)
    ex.drain()
    assert not bool((ex.total % 2).any())
    if rank == 0:
        with open(out_path, "w") as f:
            f.write(stats_digest((ex.total // 2).numpy()))
    dist.destroy_process_group()


def test_strong_scaling_digest_equal_across_world_sizes(tmp_path):
    """configs[3]'s invariant: a fixed job's all-reduced per-rule totals are identical at every
    GPU count — here k = 1, 2, 4 on gloo, with a job size that does not divide evenly — and equal the
    single-process counters (statistics.go:126-157 sums per-CPU slots the same way)."""
    from bench import stats_digest
    n_total = (1 << 15) + 7
    digests = {}
    for world in (1, 2, 4):
        out = str(tmp_path / f"d{world}.txt")
        mp.start_processes(_strong_worker, args=(world, _free_port(), n_total, out), nprocs=world,
                           start_method="spawn")
        digests[world] = open(out).read()
    assert len(set(digests.values())) == 1, digests
    assert digests[1] == stats_digest(_stats_for(0, n_total))
