"""Statistics polled while batches run (statistics.go:112-131 beside XDP, ebpfsyncer.go:81-88).

The reference's poller reads the per-CPU statistics map every period while the XDP program keeps counting on every
CPU; a lookup never waits for packets in flight.  Here one thread queues batches back to back on the legacy null
stream — the most blocking stream there is: work on it orders after every blocking stream — while a second thread
polls infw_stats_read for rules 1..99 every few ms, as statistics.go does.

  - every rule's four counters, poll after poll, never decrease (snapshots of monotone device counters);
  - once the batches are done, the read equals the oracle's counters for the batch times the launches;
  - a lookup does not wait for the queued batches: its latency stays far below the queue's GPU time (the readers copy
    on a non-blocking stream of their own; before round 6 every lookup was a hipDeviceSynchronize).
"""
import threading
import time

import numpy as np
import pytest
import torch

import infw
from infw import workloads as W
from infw.batch import SoaBatch
from parity import oracle_for, oracle_run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_stats_poll_beside_batches_on_the_null_stream():
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    dev = torch.device("cuda", 0)
    n = 8 << 20
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, start=0, dev_ordinal=0)
    _, _, want, _ = oracle_run(oracle_for(wl), wl, 0, n, threads=16)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    null = torch.cuda.default_stream(dev)  # stream 0: the legacy null stream
    assert null.cuda_stream == 0
    rounds, launches = 3, 600
    torch.cuda.synchronize()
    clf.stats_reset()

    stop = threading.Event()
    polls, lat, errors = [], [], []

    def poller():
        try:
            while not stop.is_set():
                snap = np.zeros((99, 4), np.uint64)
                for rule in range(1, 100):
                    t0 = time.perf_counter()
                    s = clf.stats_read(rule, wait=False)[0]
                    lat.append(time.perf_counter() - t0)
                    snap[rule - 1] = (s.allow_packets, s.allow_bytes, s.deny_packets, s.deny_bytes)
                polls.append(snap)
                time.sleep(0.003)
        except BaseException as e:  # surfaced below
            errors.append(e)

    th = threading.Thread(target=poller)
    th.start()
    gpu_ms = []
    try:
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(null)
            for _ in range(launches):
                clf.classify(batch, results=res, stream=null)
            e1.record(null)
            e1.synchronize()
            gpu_ms.append(e0.elapsed_time(e1))
    finally:
        stop.set()
        th.join()
    assert not errors, errors
    torch.cuda.synchronize()
    final = clf.stats_read_all(wait=False)
    assert np.array_equal(final, want * np.uint64(rounds * launches)), "counters after the batches != oracle x launches"
    assert len(polls) >= 5, len(polls)
    for a, b in zip(polls, polls[1:]):
        assert (b >= a).all(), "a rule's counter went down between two polls"
    assert polls[-1].sum() > polls[0].sum(), "the polls saw no progress"
    lat_ms = np.array(lat) * 1e3
    queue_ms = min(gpu_ms)
    print(f"[stats poll] {len(polls)} polls, lookup latency median {np.median(lat_ms):.3f} ms, "
          f"p99 {np.percentile(lat_ms, 99):.3f} ms, max {lat_ms.max():.3f} ms; queue of {launches} batches "
          f"{queue_ms:.1f} ms of GPU time")
    # a lookup that waited for the queued batches would take a good part of the queue's GPU time
    assert queue_ms > 50, queue_ms
    assert np.median(lat_ms) < 1.0 and np.percentile(lat_ms, 99) < 0.1 * queue_ms, (np.median(lat_ms), queue_ms)
