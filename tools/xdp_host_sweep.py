#!/usr/bin/env python3
"""infw_classify_xdp_host (the host-fed AF_XDP path) over packer threads x pipeline chunk, on the GPU box.

The bench line's setup (bench.py --xdp-ring host-packed): configs[2]'s full table, its frames at a 2048-B stride in
the process's own pageable private anonymous mapping (transparent huge pages requested), one RX descriptor ring per
interface; then one infw_classify_xdp_host call over all rings per measurement, best of --reps.  Every setting must
give the same result words as the first.  With --trace the library prints its per-call pipeline timing (option
trace & 8: coordinator waits on the packers / on a host slot, drain; the packers' own packing and release-wait time).
  python tools/xdp_host_sweep.py [--frames 16777216] [--threads 4,8,16] [--chunks 131072,524288] [--trace]
                                 [--order ring|packet] [--no-thp]
"""
import argparse
import json
import mmap
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ingress-node-firewall_amd")]

STRIDE = 2048


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 24)
    ap.add_argument("--threads", default="1,2,4,8,12,14,15,16")
    ap.add_argument("--chunks", default="131072,524288,2097152")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--no-thp", action="store_true")
    ap.add_argument("--order", choices=("ring", "packet"), default="ring",
                    help="umem layout (bench.py --umem-order)")
    ap.add_argument("--per-call", default="",
                    help="comma-separated descriptors per call (summed over the rings: each call takes an equal "
                         "slice of every ring, as a daemon polling its sockets would): the per-call overhead sweep "
                         "at the default thread count and chunk, after the threads x chunk sweep")
    args = ap.parse_args()
    import numpy as np
    import torch
    import infw
    from infw import workloads as W

    n = args.frames
    wl = W.Workload(W.CFG2_MIXED_1M)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    t0 = time.perf_counter()
    hdr, cap, plen, ifx = wl.frames(0, n)
    mm = mmap.mmap(-1, n * STRIDE, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    try:
        mm.madvise(mmap.MADV_NOHUGEPAGE if args.no_thp else mmap.MADV_HUGEPAGE)
    except (AttributeError, OSError):
        pass
    umem = np.frombuffer(mm, dtype=np.uint8, count=n * STRIDE)
    ln = np.where(cap < hdr.shape[1], cap, plen).astype(np.uint32)
    rings, at = [], 0
    for v in np.unique(ifx):
        idx = np.nonzero(ifx == v)[0]
        d = np.zeros((idx.size, 4), np.uint32)
        # ring order: the ring's frames back to back (its own umem fed by a FIFO fill ring); packet: interleaved
        slots = idx.astype(np.uint64) if args.order == "packet" else np.arange(at, at + idx.size, dtype=np.uint64)
        at += idx.size
        umem.reshape(n, STRIDE)[slots.astype(np.int64), :hdr.shape[1]] = hdr[idx]
        a = slots * np.uint64(STRIDE)
        d[:, 0], d[:, 1], d[:, 2] = a & np.uint64(0xFFFFFFFF), a >> np.uint64(32), ln[idx]
        res = torch.empty(idx.size, dtype=torch.int32).pin_memory()
        rings.append((torch.from_numpy(umem), d, idx.size, int(v), res, None))
    del hdr
    setup_s = time.perf_counter() - t0
    print(json.dumps({"frames": n, "stride": STRIDE, "rings": len(rings), "setup_s": round(setup_s, 1),
                      "thp": not args.no_thp, "order": args.order, "cpus": os.cpu_count(),
                      "affinity": len(os.sched_getaffinity(0)),
                      "loadavg_1m": os.getloadavg()[0]}), flush=True)
    if args.trace:
        clf.set_option("trace", 8)
    ref = None
    for chunk in [int(c) for c in args.chunks.split(",")]:
        for t in [int(x) for x in args.threads.split(",")]:
            clf.set_option("host_threads", t)
            clf.classify_xdp_host(rings, chunk=chunk)  # warm: the pipe for this shape, page tables
            best = 1e30
            for _ in range(args.reps):
                s = time.perf_counter()
                clf.classify_xdp_host(rings, chunk=chunk)
                best = min(best, time.perf_counter() - s)
            words = np.concatenate([r[4].numpy() for r in rings])
            if ref is None:
                ref = words.copy()
            same = bool(np.array_equal(words, ref))
            print(json.dumps({"chunk": chunk, "threads": t, "ms": round(best * 1e3, 3),
                              "Mpps": round(n / best / 1e6, 1), "Mpps_per_thread": round(n / best / 1e6 / t, 1),
                              "h2d_GBps": round(n * 28 / best / 1e9, 2), "same_words": same,
                              "loadavg_1m": os.getloadavg()[0]}), flush=True)
            assert same
    for per in [int(x) for x in args.per_call.split(",") if x]:
        clf.set_option("host_threads", 0)
        q = max(1, per // len(rings))  # descriptors per ring per call

        def calls():
            for a in range(0, max(r[2] for r in rings), q):
                yield [(r[0], r[1][a:a + q], min(q, r[2] - a), r[3], r[4][a:a + q], None) for r in rings if a < r[2]]
        batches = list(calls())
        for b in batches[:4]:
            clf.classify_xdp_host(b)  # warm
        best = 1e30
        for _ in range(args.reps):
            s0 = time.perf_counter()
            for b in batches:
                clf.classify_xdp_host(b)
            best = min(best, time.perf_counter() - s0)
        words = np.concatenate([r[4].numpy() for r in rings])
        assert np.array_equal(words, ref)
        print(json.dumps({"per_call": per, "calls": len(batches), "ms": round(best * 1e3, 3),
                          "us_per_call": round(best / len(batches) * 1e6, 1), "Mpps": round(n / best / 1e6, 1),
                          "threads": clf.option("host_threads") or "auto", "same_words": True,
                          "loadavg_1m": os.getloadavg()[0]}), flush=True)


if __name__ == "__main__":
    main()
