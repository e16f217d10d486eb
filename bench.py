#!/usr/bin/env python3
"""Benchmark: Mpps classified at 1M prefixes x 99-100 rules (BASELINE.json metric).

One step = one pass of the hot path (parse -> LPM -> first-match scan ->
per-rule stats) over one resident batch of synthetic SoA packets per GPU, plus
(N > 1) the RCCL all-reduce of the 1024 x 4 u64 per-rule statistics.

  python bench.py [--gpus N --steps K --warmup W]

Launch: with --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts
N rank processes itself (torch.multiprocessing spawn; the parent never touches
the GPU) and they form an RCCL process group over 127.0.0.1.  Under
torch.distributed.run (WORLD_SIZE set) each process is one rank and --gpus, when
given, must equal WORLD_SIZE.  --spawn takes the spawn path at N = 1 too (an
RCCL group of one).  Rank 0 prints ONE JSON line; `rccl_world_size` is the
process group's size (null without one) and `per_rank` each rank's kernel time.

Workload (N=1 and per GPU at N>1):
BASELINE.json configs[2] — 1M mixed IPv4/IPv6 prefixes, BGP-like lengths,
4 ifindexes, 4096 interned 99-rule lists, Zipf(1.1) traffic — with a
128M-packet batch per GPU (configs[3]'s 1B-packet job is 8 x 128M).
Packets are generated on the device from their global index, so a rank's
shard is identical at any GPU count (weak scaling).  The table is compiled once
(rank 0) and handed to the other ranks as an image (infw_table_export/import).

  --global-packets G   configs[3]'s fixed job: G packets in total, rank g of k
                       takes [g*G/k, (g+1)*G/k) (strong scaling); the line's
                       stats_digest (SHA-256 of the all-reduced 1024 x 4 u64
                       counters of one step) is then identical for every k.
  --templates T        distinct rule lists (T >= prefixes: one 1200-B value per
                       key, configs[2]'s distinct-lists variant).
  --host-walk          TEST ONLY (tests/test_bench_launch.py): no GPU; each rank
                       walks its shard through the compiled host table image
                       (infw_debug_walk) and the counters go through the same
                       StatsExchange over gloo.  Checks the launcher, sharding
                       and exchange; the line says it is not a measurement.
  --in-process         the library's own multi-GPU shape: ONE process, ONE
                       context over N device slots (the table compiled once and
                       published to every slot), one host thread and HIP stream
                       per slot classifying its shard, the counters summed per
                       rule over the slots (infw_stats_read_all, the per-CPU
                       read of statistics.go:126-157).  --slots-on-gpu0 puts all
                       N slots on device 0 (a one-GPU rehearsal of the shape).
  --opt NAME=VALUE     a per-context option (include/infw.h infw_set_option) for
                       every context the bench creates (A/B runs of table forms).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "ingress-node-firewall_amd")]

ALGO_BYTES_PER_PKT = 36  # standard layout: 32 B SoA tuple in + 4 B result word out
# family-compact layout (infw_batch_soa_c): 4 address bytes per packet + 12 more per IPv6 packet, + 16 B of
# ifindex/pkt_len/meta/l4word in, + 4 B result word out = 24 + 12 * (IPv6 share) bytes per packet
HBM_PEAK_GBS = 8000.0    # MI355X HBM3E peak (MI355X_MICROARCH.md)
PCIE_H2D_GBS = 56.9      # dense pinned H2D copy rate, PCIe Gen5 x16 (tools/micro/pcie.hip, profiles/r06z/micro/pcie.jsonl)
HOST_FED = ("host-packed", "host-bursts")  # --xdp-ring feeds whose frames the library's host packer threads read
METRIC = "Mpps classified @1M prefixes x 100 rules, 1/2/4/8 GPUs; % HBM BW roofline"


class StatsExchange:
    """Per-step counter blocks (1024 x 4 u64, the stats map of kernel.c:36-41) and their exchange.

    Double-buffered: step k's counters go to buffer k & 1; with use_dist its all-reduce is issued
    asynchronously (RCCL: on the collective's own stream, so it overlaps step k + 1's classification)
    and settled — the launch stream waits for it, the host does not — before step k + 2 reuses the
    buffer, adding the reduced block to `total`.  Without use_dist the block is added directly.
    tests/test_dist_gloo.py drives this class on gloo with world size 2."""

    def __init__(self, make, use_dist):
        import torch.distributed as dist
        self._dist = dist
        self.bufs = [make(), make()]
        self.total = make()
        self.pending = [None, None]
        self.use_dist = use_dist

    def _settle(self, b):
        if self.pending[b] is not None:
            self.pending[b].wait()
            self.total.add_(self.bufs[b])
            self.pending[b] = None

    def begin(self, k):
        """The zeroed counter block step k classifies into."""
        b = k & 1
        self._settle(b)
        self.bufs[b].zero_()
        return self.bufs[b]

    def end(self, k):
        b = k & 1
        if self.use_dist:
            self.pending[b] = self._dist.all_reduce(self.bufs[b], async_op=True)  # 32 KiB of u64 over xGMI
        else:
            self.total.add_(self.bufs[b])

    def drain(self):
        self._settle(0)
        self._settle(1)


def shard_range(global_n, rank, world):
    """Packets [a, b) of rank `rank` in a fixed job of global_n packets."""
    return global_n * rank // world, global_n * (rank + 1) // world


def stats_digest(block):
    """SHA-256 of one step's all-reduced counter block: 1024 x {allow pkts, allow bytes, deny pkts, deny bytes}
    as little-endian u64 (the layout of ruleStatistics_st, ingress_node_firewall.h:45-54)."""
    import numpy as np
    a = np.ascontiguousarray(np.asarray(block).astype("<u8").reshape(1024, 4))
    return hashlib.sha256(a.tobytes()).hexdigest()


def usable_cores():
    """Host cores this process may run on: the CPU affinity set, capped by a cgroup v2 CPU quota if any."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def workload_key(cfg, templates, prefixes):
    """Names the workload a traffic / PMC summary belongs to (profiles/traffic_<key>.json)."""
    return (f"cfg{cfg}" + ("_distinct" if templates and templates >= (prefixes or 1000000) else "") +
            (f"_p{prefixes}" if prefixes else ""))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node: > 1 spawns the ranks unless launched by torch.distributed.run, "
                         "where it must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--spawn", action="store_true", help="take the spawn path (own RCCL process group) at N = 1 too")
    ap.add_argument("--host-walk", action="store_true",
                    help="TEST ONLY: no GPU, ranks walk the compiled host image over gloo (not a measurement)")
    ap.add_argument("--compile-per-rank", action="store_true",
                    help="every rank compiles the table itself instead of importing rank 0's image")
    ap.add_argument("--key-order", choices=("shuffled", "workload"), default="shuffled",
                    help="order of the table updates: seeded random like the reference's Go map range (default), "
                         "or the generator's popularity order (same map either way)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 27, help="packets per GPU per step")
    ap.add_argument("--cfg", type=int, default=2, choices=[1, 2, 4])
    ap.add_argument("--prefixes", type=int, default=0, help="override table size (0 = config default)")
    ap.add_argument("--templates", type=int, default=0,
                    help="distinct rule lists (0 = config default; >= prefixes: one list per key)")
    ap.add_argument("--uniform", action="store_true",
                    help="sources uniform over the prefixes instead of the config's Zipf(1.1) (cache-hostile variant)")
    ap.add_argument("--global-packets", type=int, default=0,
                    help="fixed job of this many packets sharded over the ranks (strong scaling, configs[3])")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="packets in the CPU-baseline sample (0: ~10-20 s of oracle work on the usable cores)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (0: every usable core)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-line-rates", action="store_true",
                    help="skip the in-process random-line / stream rate probe (and so random_line_model)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic summary (default profiles/traffic_<workload>.json when it matches the kernel)")
    ap.add_argument("--layout", default="standard", choices=["compact", "standard"],
                    help="batch address layout (include/infw.h): 16-B standard (default) or family-compact")
    ap.add_argument("--from-frames", type=int, default=0, metavar="STRIDE",
                    help="packer-fed step: raw frames resident in HBM at this stride (e.g. 128) -> infw_pack_frames_c "
                         "-> infw_classify_c, both timed (implies --layout compact)")
    ap.add_argument("--in-process", action="store_true",
                    help="one process, one context over N device slots, a host thread + stream per slot")
    ap.add_argument("--slots-on-gpu0", action="store_true",
                    help="with --in-process: every slot on device 0 (rehearsal of the N-slot shape on one GPU)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="per-context option (include/infw.h) for every context this bench creates")
    ap.add_argument("--xdp-ring", choices=("hbm", "host", "registered", "host-packed", "host-bursts"), default=None,
                    help="AF_XDP feed: the frames in a umem of 2048-B chunks (--from-frames sets another chunk size) "
                         "in HBM, in pinned host memory (hipHostMalloc) or in the process's own anonymous mapping "
                         "page-locked with infw_host_register (what a daemon's XDP_UMEM_REG memory is), read over "
                         "PCIe; one RX descriptor ring per interface, classified by infw_classify_xdp (implies --fused). "
                         "host-packed: umem and rings in the process's own pageable mapping, read by the library's "
                         "host packer threads, the packed tuples pipelined through the device "
                         "(infw_classify_xdp_host); result words into pinned host memory. host-bursts: the same frames "
                         "handed over DPDK-style, one pointer per frame with its data_len / pkt_len "
                         "(infw_classify_bursts_host, include/infw_host.h)")
    ap.add_argument("--burst-size", type=int, default=0,
                    help="with --xdp-ring host-bursts: frames per burst (e.g. 32, an rte_eth_rx_burst's; 0: one burst "
                         "per interface)")
    ap.add_argument("--umem-order", choices=("packet", "ring"), default=None,
                    help="AF_XDP umem layout: frames at their packet index (rings interleave: default for hbm/host/"
                         "registered) or each ring's frames back to back in arrival order (a socket's own umem fed by a "
                         "FIFO fill ring: default for host-packed)")
    ap.add_argument("--xdp-chunk", type=int, default=0,
                    help="with --xdp-ring host-packed: descriptors per pipeline chunk (0: the library's default)")
    ap.add_argument("--fused", action="store_true",
                    help="with --from-frames: one kernel classifies straight from the frames (infw_classify_frames), "
                         "no SoA batch written or read; checked untimed against the packer path's results")
    args = ap.parse_args(argv)
    if args.xdp_ring:
        args.from_frames = args.from_frames or 2048
        args.fused = True
        args.umem_order = args.umem_order or ("ring" if args.xdp_ring in HOST_FED else "packet")
        if args.batch == 1 << 27:
            args.batch = 1 << 24  # 16M frames x 2048 B = 32 GiB of umem
    args.options = {}
    for o in args.opt:
        name, _, val = o.partition("=")
        if not name or not val:
            ap.error(f"--opt {o!r}: NAME=VALUE")
        args.options[name] = int(val)
    return args


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def main(argv=None):
    """Launcher.  Under torch.distributed.run (WORLD_SIZE set) this process is one rank.  Otherwise --gpus N > 1
    (or --spawn) starts N rank processes with torch.multiprocessing's spawn start method: fresh interpreters, so
    nothing of the parent's state — which never touches the GPU — is inherited, and each rank binds its own GPU."""
    args = parse(argv)
    if args.in_process:
        if args.host_walk:
            return run_in_process_host_walk(args, args.gpus or 1)
        return run_in_process(args, args.gpus or 1)
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree")
        return run_rank(args)
    n = args.gpus or 1
    if n > 1 or args.spawn:
        return spawn_ranks(args, n)
    return run_rank(args)


def spawn_ranks(args, n):
    import torch.multiprocessing as mp
    if not args.host_walk:
        import torch
        have = torch.cuda.device_count()  # counts devices without initialising one (the parent never does)
        if n > have:
            sys.exit(f"bench.py: --gpus {n} but {have} HIP device(s) are visible")
    mp.start_processes(_rank_entry, args=(args, n, free_port()), nprocs=n, start_method="spawn", join=True)


def _rank_entry(i, args, n, port):
    os.environ.update(RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run_rank(args)


def share_tables(args, clf, wl, rank, world, use_dist, log):
    """The rule table on this rank's context: compiled once by rank 0 and imported by the others
    (infw_table_export -> a /dev/shm file -> infw_table_import: no other rank compiles), or compiled by every rank
    with --compile-per-rank.  Returns (how, seconds)."""
    import mmap
    import torch.distributed as dist
    t0 = time.time()
    # the reference loader updates keys in Go map order (loader.go:158-208), i.e. at random: list ids — and so
    # where each list's decision lines sit — follow first-update order, and the generator lists prefixes in
    # popularity order, which would place the hot lists together (--key-order workload)
    order = wl.shuffled_order() if args.key_order == "shuffled" else None
    if not use_dist or world == 1 or args.compile_per_rank:
        wl.load_into(clf, order=order)
        clf.commit()
        return "compiled", time.time() - t0
    path = [None]
    if rank == 0:
        wl.load_into(clf, order=order)
        clf.commit()
        size = clf.export_size()
        # shared memory when it has room (a container's /dev/shm may be small), else the temp directory; the file
        # is allocated up front (posix_fallocate fails cleanly, where writing a mapping past a full tmpfs would
        # SIGBUS) and nothing else is tried if neither has room: every rank then compiles
        import tempfile
        for d in ("/dev/shm", tempfile.gettempdir()):
            try:
                st = os.statvfs(d)
                if st.f_bavail * st.f_frsize < size + (64 << 20):
                    continue
                p = os.path.join(d, f"infw_bench_{os.getpid()}_{os.environ.get('MASTER_PORT', '0')}.img")
                with open(p, "w+b") as f:
                    path[0] = p
                    import atexit
                    atexit.register(lambda q=p: os.path.exists(q) and os.unlink(q))  # also if a rank fails
                    os.posix_fallocate(f.fileno(), 0, size)
                    with mmap.mmap(f.fileno(), size) as mm:
                        import ctypes as C
                        buf = (C.c_char * size).from_buffer(mm)
                        clf.export_into(C.addressof(buf), size)
                        del buf
                break
            except OSError as e:
                log(f"[bench] table image export to {d} failed ({e})")
                if path[0]:
                    os.unlink(path[0])
                    path[0] = None
        if path[0] is None:
            log("[bench] no room for the table image: every rank compiles its own tables")
    dist.broadcast_object_list(path, src=0)
    how = "compiled"
    if rank != 0:
        if path[0] is None:
            wl.load_into(clf, order=order)
            clf.commit()
        else:
            import ctypes as C
            with open(path[0], "rb") as f:
                size = os.fstat(f.fileno()).st_size
                # a private (copy-on-write) mapping: ctypes needs a writable buffer, and nothing writes it
                with mmap.mmap(f.fileno(), size, access=mmap.ACCESS_COPY) as mm:
                    buf = (C.c_char * size).from_buffer(mm)
                    clf.import_image((C.addressof(buf), size))
                    del buf
            how = "imported"
    dist.barrier()
    if rank == 0 and path[0]:
        os.unlink(path[0])
    return how, time.time() - t0


def gather_ranks(values, world, use_dist, dev=None):
    """Every rank's `values` (a list of floats), in rank order."""
    if not use_dist:
        return [list(values)]
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def host_counters(results, pkt_len):
    """Per-rule counters implied by result words (kernel.c:441-456, :376-387) — the host walk's stand-in for the
    kernel's device counters."""
    import numpy as np
    out = np.zeros((1024, 4), np.uint64)
    act, key = results & 0xFF, (results >> 8) & 0xFFFF
    for a, col in ((2, 0), (1, 2)):  # XDP_PASS allow, XDP_DROP deny
        sel = (act == a) & (key < 1024)
        np.add.at(out[:, col], key[sel], np.uint64(1))
        np.add.at(out[:, col + 1], key[sel], pkt_len[sel].astype(np.uint64))
    return out


def run_host_walk(args, world, rank, use_dist, log):
    """TEST ONLY (--host-walk): the launcher, sharding, table sharing and StatsExchange of run_rank on a CPU box —
    gloo instead of RCCL, and each step's classification is infw_debug_walk over the compiled host image (the
    kernel's lookup code run on the host), not the HIP kernel.  The JSON line says it is no measurement."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import infw
    from infw import workloads as W
    if use_dist:
        dist.init_process_group("gloo")
    wl = W.Workload(args.cfg, n_prefixes=args.prefixes or 20000, n_templates=args.templates or 64)
    clf = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16, options=args.options)
    how, setup_s = share_tables(args, clf, wl, rank, world, use_dist, log)
    if args.global_packets:
        start, end = shard_range(args.global_packets, rank, world)
        n = end - start
    else:
        n = min(args.batch, 1 << 16)
        start = rank * n
    tuples = wl.tuples(start, n) if n else np.zeros((0, 8), np.uint32)
    ex = StatsExchange(lambda: torch.zeros((1024, 4), dtype=torch.int64), use_dist)

    def step(k):
        buf = ex.begin(k)
        if n:
            buf.copy_(torch.from_numpy(host_counters(clf.debug_walk(tuples), tuples[:, 5]).view(np.int64)))
        ex.end(k)

    for k in range(args.warmup):
        step(k)
    ex.drain()
    ex.total.zero_()
    if use_dist:
        dist.barrier()
    ts = time.perf_counter()
    for k in range(args.steps):
        step(k)
    ex.drain()
    if use_dist:
        dist.barrier()
    per_rank = gather_ranks([time.perf_counter() - ts, 0.0, setup_s, 1.0 if how == "imported" else 0.0, 0.0,
                             float(n)], world, use_dist)
    elapsed = max(r[0] for r in per_rank)
    assert not bool((ex.total % max(args.steps, 1)).any()), "steps' counters differ"
    digest = stats_digest((ex.total // max(args.steps, 1)).numpy())
    job = args.global_packets if args.global_packets else n * world
    if rank == 0:
        print(json.dumps({
            "metric": METRIC + " [host-walk selftest: not a measurement]", "value": round(job * args.steps / elapsed / 1e6, 4),
            "unit": "Mpps", "valid_measurement": False, "n_gpus": 0, "rccl_world_size": dist.get_world_size() if use_dist
            else None, "backend": "gloo" if use_dist else None, "steps": args.steps, "warmup": args.warmup,
            "scaling": "strong" if args.global_packets else "weak", "build_id": infw.build_id(),
            "config": {"workload_key": workload_key(args.cfg, args.templates, args.prefixes), "prefixes": wl.n_entries,
                       "global_batch": job, "packets_counted_in_stats": int(ex.total[:, 0].sum() + ex.total[:, 2].sum())
                       // max(args.steps, 1), "stats_digest": digest},
            "per_rank": [{"rank": r, "tables": "imported" if v[3] else "compiled", "packets_per_step": int(v[5])}
                         for r, v in enumerate(per_rank)]}), flush=True)
    if use_dist:
        dist.destroy_process_group()


def run_rank(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    import infw
    from infw import workloads as W
    from infw.batch import SoaBatch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = "WORLD_SIZE" in os.environ  # launched by torch.distributed.run or spawned (any N, 1 included)

    def log(*a):
        if rank == 0:
            print(*a, file=sys.stderr, flush=True)

    if args.host_walk:
        return run_host_walk(args, world, rank, use_dist, log)
    if use_dist:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    # ---- tables: compiled once (rank 0, imported by the other ranks), replicated on every GPU
    wl = W.Workload(args.cfg, n_prefixes=args.prefixes, n_templates=args.templates)
    if args.uniform:
        wl.uniform_sources()
    clf = infw.Classifier(devices=[local], max_entries=wl.n_entries + 16, options=args.options)
    how, setup_s = share_tables(args, clf, wl, rank, world, use_dist, log)
    commit_s = setup_s
    info = clf.info()
    log(f"[bench] cfg{args.cfg}: {wl.n_entries} entries, tables {how} in {setup_s:.1f}s "
        f"(compile/parse {info['compile_ms']:.0f} ms, upload {info['upload_ms']:.0f} ms, "
        f"{info['device_bytes'] / 2**20:.0f} MiB/GPU, lists={info['n_lists']}, levels={info['n_long_levels']})")

    # ---- resident input shard, generated on the device by global packet index
    if args.global_packets:  # configs[3]: a fixed job, rank g takes [g·N/k, (g+1)·N/k)
        start, end = shard_range(args.global_packets, rank, world)
        n = end - start
    else:                    # weak scaling: a fixed batch per GPU, rank g takes [g·n, (g+1)·n)
        n = args.batch
        start = rank * n
    if args.from_frames:
        args.layout = "compact"
        stride = args.from_frames
        frames = torch.empty(max(n, 1) * stride, dtype=torch.uint8, device=dev)
        f_lin, f_len, f_ifx = (torch.empty(max(n, 1), dtype=torch.int32, device=dev) for _ in range(3))
        if n:
            wl.gen_frames_device(frames, stride, f_lin[:n], f_len[:n], f_ifx[:n], start=start, dev_ordinal=local)
        from infw.batch import SoaBatchC
        batch_c = SoaBatchC.empty(max(n, 1), dev)
        batch = None
    else:
        batch = SoaBatch.empty(max(n, 1), dev).slice(0, n)
        if n:
            wl.gen_device(batch, start=start, dev_ordinal=local)
    if args.from_frames:  # one untimed pack prices the compact tuple by the batch's IPv6 share
        clf.pack_frames_c(frames, f_lin[:n], f_ifx[:n], batch_c, pkt_len=f_len[:n], stride=stride)
        n6 = int(((batch_c.meta[:n] & 0xFFFF) == 0x86DD).sum().item())
        algo_bytes = 24 + 12 * n6 / max(n, 1)
    elif args.layout == "compact":  # the packer's production layout (infw_pack_frames_c); converted untimed here
        batch_c = clf.compact(batch, dev=0)
        n6 = int(((batch.meta & 0xFFFF) == 0x86DD).sum().item())
        algo_bytes = 24 + 12 * n6 / max(n, 1)
    else:
        algo_bytes = ALGO_BYTES_PER_PKT
    results = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
    fused_check = None
    if args.fused:
        assert args.from_frames, "--fused needs --from-frames STRIDE"
        if n:  # untimed: the fused kernel's result words == the packer path's (counters: the digest below)
            ref = torch.empty_like(results)
            clf.classify_c(batch_c, results=ref)
            clf.classify_frames(frames, f_lin[:n], f_ifx[:n], n, results=results, pkt_len=f_len[:n], stride=stride)
            torch.cuda.synchronize()
            fused_check = bool(torch.equal(ref, results))
            assert fused_check, "classify_frames differs from pack_frames_c + classify_c"
            del ref
            clf.stats_reset()
        args.layout = "frames"
        algo_bytes = 27 + 12 * n6 / max(n, 1)  # frame bytes kernel.c reads (11 B IPv4, 23 B IPv6) + 12 B lengths/ifindex + result
    rings, perm = [], None
    if args.xdp_ring and n:
        # one AF_XDP RX ring per interface (a socket is bound to one interface queue): descriptor {addr, len} of
        # every frame of that interface, in arrival order; len = the frame's linear length when its linear part ends
        # inside the 80-B snapshot, else its frame length (single-buffer frames)
        ifx_h = f_ifx[:n].cpu().numpy().view(np.uint32)
        lin_h = f_lin[:n].cpu().numpy().view(np.uint32)
        len_h = np.where(lin_h < 80, lin_h, f_len[:n].cpu().numpy().view(np.uint32))
        # umem order: "packet" — every frame at its packet index (the interfaces' rings interleave in one umem, so a
        # ring's addresses ascend with gaps); "ring" — each ring's frames back to back in arrival order, as a socket's
        # own umem holds them in steady state when its fill ring returns chunks in the order they were consumed
        order, ring_addrs, at = [], [], 0
        for ifv in np.unique(ifx_h):
            idx = np.nonzero(ifx_h == ifv)[0]
            d = np.zeros((len(idx), 4), np.uint32)
            slots = idx.astype(np.uint64) if args.umem_order == "packet" else np.arange(at, at + len(idx), dtype=np.uint64)
            a = slots * np.uint64(stride)
            ring_addrs.append(a)
            d[:, 0], d[:, 1], d[:, 2] = a & np.uint64(0xFFFFFFFF), a >> np.uint64(32), len_h[idx]
            rings.append([int(ifv), len(idx), torch.from_numpy(d.view(np.int32))])
            order.append(idx)
            at += len(idx)
        perm = torch.from_numpy(np.concatenate(order)).to(dev)
        if args.umem_order == "ring":  # frame k of the umem = packet perm[k]
            frames = frames.view(-1, stride)[:n][perm].reshape(-1)
            torch.cuda.synchronize()
        if args.xdp_ring == "host":  # umem and rings in pinned host memory: the kernel reads them over PCIe
            umem = torch.empty(frames.numel(), dtype=torch.uint8, pin_memory=True)
            umem.copy_(frames)
            del frames
            frames = umem
            for r in rings:
                r[2] = r[2].pin_memory()
        elif args.xdp_ring == "registered":  # the daemon's own memory (an anonymous mapping), page-locked for the GPU
            import mmap
            registered = []

            def own(nbytes):
                mm = mmap.mmap(-1, max(nbytes, 4096))
                arr = np.frombuffer(mm, dtype=np.uint8, count=nbytes)
                clf.host_register(arr)
                registered.append((mm, arr))
                return torch.from_numpy(arr)
            umem = own(frames.numel())
            umem.copy_(frames)
            del frames
            frames = umem
            for r in rings:
                t = own(r[2].numel() * 4).view(torch.int32)
                t.copy_(r[2].view(-1))
                r[2] = t
        elif args.xdp_ring in HOST_FED:
            # the daemon's own pageable memory (an anonymous mapping, huge pages requested as AF_XDP umems commonly
            # are), never registered: the library's packer threads read it on the CPU; the rings stay pageable too
            import mmap
            # private (not shared) anonymous memory: transparent huge pages apply to it, as to a daemon's umem
            mm = mmap.mmap(-1, max(frames.numel(), 4096), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            try:
                mm.madvise(mmap.MADV_HUGEPAGE)
            except (AttributeError, OSError):
                pass
            umem = torch.from_numpy(np.frombuffer(mm, dtype=np.uint8, count=frames.numel()))
            umem.copy_(frames)
            del frames
            frames = umem
            host_res = [torch.empty(max(r[1], 1), dtype=torch.int32).pin_memory()[:r[1]] for r in rings]
            ring_args = [(frames, d, nr, ifv, hr, None) for (ifv, nr, d), hr in zip(rings, host_res)]
            if args.xdp_ring == "host-bursts":
                # DPDK-style: per frame its address (rte_pktmbuf_mtod), data_len (the linear part) and pkt_len, cut
                # into bursts of --burst-size frames of one port each (0: one burst per interface)
                flen_h = f_len[:n].cpu().numpy().view(np.uint32)
                base = np.uint64(frames.data_ptr())
                bursts = []
                for (ifv, nr, d), hr, idx, a in zip(rings, host_res, order, ring_addrs):
                    ptrs, hres = base + a, hr.numpy().view(np.uint32)
                    bs = args.burst_size or max(nr, 1)
                    for lo in range(0, nr, bs):
                        hi = min(nr, lo + bs)
                        bursts.append(infw.Burst(ptrs[lo:hi], lin_h[idx[lo:hi]], flen_h[idx[lo:hi]], ifv,
                                                 results=hres[lo:hi]))
                bursts = infw.BurstArray(bursts)  # the C array a daemon would hand over, built once (untimed)

            def host_call():
                if args.xdp_ring == "host-bursts":
                    clf.classify_bursts_host(bursts, chunk=args.xdp_chunk)
                else:
                    clf.classify_xdp_host(ring_args, chunk=args.xdp_chunk)
        else:
            for r in rings:
                r[2] = r[2].to(dev)
        algo_bytes = 11 + 12 * n6 / max(n, 1) + 16 + 4  # frame bytes read + the 16-B descriptor + the result word
        # untimed: the rings' result words, back in packet order, == the packer path's (counters: the digest below)
        ref = torch.empty_like(results)
        clf.classify_c(batch_c, results=ref)
        off = 0
        if args.xdp_ring in HOST_FED:
            host_call()
            results.copy_(torch.cat(host_res).to(dev))
        else:
            for ifv, nr, d in rings:
                clf.classify_xdp(frames, d, nr, ifv, results=results[off:off + nr])
                off += nr
        got = torch.empty_like(results)
        got[perm] = results
        torch.cuda.synchronize()
        fused_check = bool(torch.equal(ref, got))
        assert fused_check, "classify_xdp differs from pack_frames_c + classify_c"
        del ref, got
        clf.stats_reset()
    ex = StatsExchange(lambda: torch.zeros((1024, 4), dtype=torch.int64, device=dev), use_dist)
    # the device's random-line and stream rates, measured in this process just before the timed loop (same lease,
    # same device): what random_line_model prices the kernel's PMC line counts with (~0.3 s, untimed)
    rates = None if args.no_line_rates else probe_line_rates(W, local, log)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)

    step_wall = []

    def step(k, ev=None):
        stats = ex.begin(k)
        clf.stats_bind(0, stats.data_ptr())
        if ev is not None:
            ev[0].record(stream)
        if args.xdp_ring in HOST_FED:  # synchronous: pack || H2D || classify || D2H inside the library
            if ev is not None:
                ev[2].record(stream)
            t0 = time.perf_counter()
            host_call()
            step_wall.append(time.perf_counter() - t0)
        elif args.xdp_ring:
            if ev is not None:
                ev[2].record(stream)
            off = 0
            for ifv, nr, d in rings:  # one launch per interface ring
                clf.classify_xdp(frames, d, nr, ifv, results=results[off:off + nr], stream=stream)
                off += nr
        elif args.fused:
            if ev is not None:
                ev[2].record(stream)
            clf.classify_frames(frames, f_lin[:n], f_ifx[:n], n, results=results, pkt_len=f_len[:n], stride=stride,
                                stream=stream)
        elif args.from_frames:
            clf.pack_frames_c(frames, f_lin[:n], f_ifx[:n], batch_c, pkt_len=f_len[:n], stride=stride, stream=stream)
            if ev is not None:
                ev[2].record(stream)
            clf.classify_c(batch_c, results=results, stream=stream)
        elif args.layout == "compact":
            clf.classify_c(batch_c, results=results, stream=stream)
        else:
            clf.classify(batch, results=results, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        ex.end(k)

    for k in range(args.warmup):
        step(k)
    ex.drain()
    # the all-reduced counters of one step (every step classifies the same batch): the cross-k invariant
    digest_block = None
    if args.warmup:
        assert not bool((ex.total % args.warmup).any()), "warmup steps' counters differ"
        digest_block = ex.total // args.warmup
    ex.total.zero_()
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3 if args.from_frames else 2))
           for _ in range(args.steps)]
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for k in range(args.steps):
        step(k, evs[k])
    ex.drain()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - ts
    if args.xdp_ring in HOST_FED:  # the library's own streams: the step's wall time stands for the kernel's
        kern_ms = [w * 1e3 for w in step_wall[-args.steps:]]
    elif args.from_frames:  # ev[0] -> pack -> ev[2] -> classify -> ev[1]
        pack_ms = [e[0].elapsed_time(e[2]) for e in evs]
        kern_ms = [e[2].elapsed_time(e[1]) for e in evs]
    else:
        kern_ms = [e[0].elapsed_time(e[1]) for e in evs]
    avg_kern_ms = sum(kern_ms) / len(kern_ms)
    import resource
    peak_rss_gib = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20  # ru_maxrss: KiB on Linux
    mine = [elapsed, avg_kern_ms, setup_s, 1.0 if how == "imported" else 0.0, peak_rss_gib, float(n)]
    per_rank = gather_ranks(mine, world, use_dist, dev)
    elapsed = max(r[0] for r in per_rank)  # max over ranks

    job_pkts = args.global_packets if args.global_packets else n * world
    total_pkts = job_pkts * args.steps
    mpps = total_pkts / elapsed / 1e6
    achieved = algo_bytes * n / (avg_kern_ms * 1e-3) / 1e9
    total = ex.total
    counted = int(total[:, 0].sum().item() + total[:, 2].sum().item())
    if digest_block is None:
        assert not bool((total % args.steps).any()), "timed steps' counters differ"
        digest_block = total // args.steps
    else:
        assert torch.equal(total, digest_block * args.steps), "a timed step's counters differ from the warmup's"
    digest = stats_digest(digest_block.cpu().numpy())
    # the registry name of the instantiation(s) this line ran (infw_classify_variant: the library's own selector)
    kernel = clf.variant(infw.INPUT_COMPACT if args.xdp_ring in HOST_FED else infw.INPUT_XDP if args.xdp_ring else
                         {"standard": infw.INPUT_SOA, "compact": infw.INPUT_COMPACT,
                          "frames": infw.INPUT_FRAMES}[args.layout])
    host_feed = None
    if args.xdp_ring in HOST_FED:
        # per step over PCIe, as infw_classify_xdp_host cuts the rings: chunks of at most C descriptors running on
        # from one ring into the next (chunk 0: 512K, or a quarter of a call under four of those, >= 32K); a chunk of
        # n descriptors is one H2D copy of 28 B x S (S = n rounded up to 64: saddr4, pkt_len, meta, l4word and the
        # groups' whole 768-B v6tail blocks), 32 B x S when its rings carry several ifindexes; result words back
        C = ((args.xdp_chunk or (1 << 19)) + 511) // 512 * 512
        total = sum(nr for _, nr, _ in rings)
        if not args.xdp_chunk and total < 4 * C:
            C = min(C, max(32768, ((total + 3) // 4 + 4095) // 4096 * 4096))
        h2d, fill, ifs = 0, 0, set()
        for ifv, nr, _ in rings:
            a = 0
            while a < nr:
                take = min(C - fill, nr - a)
                ifs.add(ifv)
                fill, a = fill + take, a + take
                if fill == C:
                    h2d += (32 if len(ifs) > 1 else 28) * C
                    fill, ifs = 0, set()
        if fill:
            h2d += (32 if len(ifs) > 1 else 28) * (-(-fill // 64) * 64)
        step_s = sum(kern_ms) / len(kern_ms) / 1e3
        threads = clf.option("host_threads") or min(usable_cores(), 16)
        host_feed = {"host_threads": threads, "usable_cores": usable_cores(), "chunk": C,
                     "pcie_h2d_bytes_per_step": h2d, "pcie_h2d_GBps": round(h2d / step_s / 1e9, 2),
                     "pcie_d2h_GBps": round(4 * n / step_s / 1e9, 2),
                     "pcie_h2d_bytes_per_packet": round(h2d / max(n, 1), 2),
                     "pcie_h2d_peak_GBps": PCIE_H2D_GBS, "pcie_h2d_frac": round(h2d / step_s / 1e9 / PCIE_H2D_GBS, 3),
                     # the calling thread packs too (it packs whenever it would otherwise wait for the packers)
                     "Mpps_per_host_thread": round(n / step_s / 1e6 / (threads + 1), 1),
                     # the packers share the host with whatever else runs on it: the spread of the timed steps and the
                     # host's load average say how much of the step the CPUs were really ours
                     "step_ms_min": round(min(kern_ms), 3), "step_ms_median": round(float(np.median(kern_ms)), 3),
                     "step_ms_max": round(max(kern_ms), 3), "host_loadavg_1m": round(os.getloadavg()[0], 1)}
    if args.xdp_ring:
        extra_pipe = {"xdp_ring": {"umem": args.xdp_ring, "umem_order": args.umem_order, "chunk": stride,
                                   "rings": len(rings),
                                   "frames_per_ring": [r[1] for r in rings],
                                   "results_equal_packer_path": fused_check,
                                   "note": "umem and descriptor rings in " + {
                                       "host": "pinned host memory (hipHostMalloc), read by the kernel over PCIe "
                                               "(PCIe-inclusive rate)",
                                       "registered": "the process's own anonymous mapping page-locked with "
                                                     "infw_host_register, read by the kernel over PCIe "
                                                     "(PCIe-inclusive rate)",
                                       "host-packed": "the process's own pageable anonymous mapping, read by the "
                                                      "library's packer threads on the CPU; packed tuples to the "
                                                      "device and result words back over PCIe (PCIe-inclusive "
                                                      "rate; kernel_ms_avg is the step's wall time)",
                                       "host-bursts": "the process's own pageable anonymous mapping, handed over "
                                                      "as DPDK-style bursts (a pointer, data_len and pkt_len per "
                                                      "frame) and read by the library's packer threads; packed "
                                                      "tuples to the device and result words back over PCIe "
                                                      "(PCIe-inclusive rate; kernel_ms_avg is the step's wall time)",
                                       "hbm": "HBM"}[args.xdp_ring],
                                   **({"bursts": bursts.n, "burst_size": args.burst_size or None}
                                      if args.xdp_ring == "host-bursts" else {}),
                                   **({"host_feed": host_feed} if host_feed else {})}}
    elif args.fused:
        extra_pipe = {"from_frames": {"frame_stride": stride, "fused": True,
                                      "results_equal_packer_path": fused_check}}
    elif args.from_frames:
        # packer: the frame bytes kernel.c reads (ethertype, L3 proto, source address, first L4 word: 11 B IPv4 /
        # 23 B IPv6) + linear length, frame length, ifindex (12 B) in; the compact tuple (algo_bytes - 4) out
        s6 = (algo_bytes - 24) / 12
        pack_bytes = 11 + 12 * s6 + 12 + (algo_bytes - 4)
        avg_pack = sum(pack_ms) / len(pack_ms)
        extra_pipe = {"from_frames": {
            "frame_stride": stride, "pack_kernel_ms_avg": round(avg_pack, 4),
            "pack_algorithmic_bytes_per_packet": round(pack_bytes, 3),
            "pack_achieved_GBps": round(pack_bytes * n / (avg_pack * 1e-3) / 1e9, 1),
            "pipeline_algorithmic_bytes_per_packet": round(pack_bytes + algo_bytes, 3),
            "pipeline_kernel_ms_avg": round(avg_pack + sum(kern_ms) / len(kern_ms), 4)}}
    else:
        extra_pipe = {}
    wkey = workload_key(args.cfg, args.templates, args.prefixes) + ("_uniform" if args.uniform else "") + (
        "_frames" if args.from_frames else "") + ("_fused" if args.fused else "") + (
        f"_xdp{args.xdp_ring}" if args.xdp_ring else "") + (
        "_compact" if args.layout == "compact" and not args.from_frames else "")

    traffic = None
    traffic_from = None
    line_model = None
    extra = {}
    tpath = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{wkey}.json")
    tj = json.load(open(tpath)) if os.path.exists(tpath) else None
    build_id = infw.build_id()
    if tj is not None and (tj.get("build_id") != build_id or tj.get("kernel") != kernel or
                           tj.get("layout", "standard") != args.layout):
        log(f"[bench] {tpath} was profiled on build {tj.get('build_id')} {tj.get('kernel')!r} "
            f"({tj.get('layout', 'standard')}), not build {build_id} {kernel!r} ({args.layout}): traffic figures omitted")
        tj = None
    if tj is not None:
        try:
            traffic = tj.get("hbm_bytes_per_packet", None)
            traffic = None if traffic is None else round(traffic * n)
            traffic_from = (f"profiles/{tj.get('tag')}/summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, {wkey}, "
                            f"build {tj.get('build_id')})")
            # random-line model: the kernel's PMC L2 hits and misses per packet (the profile of this
            # build) priced at the rates this process measured on this device before the timed loop: table hits at
            # the L2-hit rate, table misses at the random-miss rate, and the streamed bytes (tuples in, result words
            # out; for raw frames each frame's whole 128-B line) at the stream bandwidth — the stream's own lines
            # are taken out of the L2 misses, not priced as random misses.  frac = that bound / the kernel time.
            if rates and "l2_hits_per_packet" in tj:
                h, m = tj["l2_hits_per_packet"], tj["l2_misses_per_packet"]
                side = 16.0 if args.xdp_ring else 12.0  # per frame: the descriptor, or lengths + ifindex
                stream_in = {"standard": 32.0, "compact": algo_bytes - 4, "frames": side + 128.0}[args.layout]
                s_lines = (side / 128 + 1.0) if args.layout == "frames" else stream_in / 128
                tm = max(0.0, m - s_lines)
                per_pkt_s = (h / (rates["l2_hit_G_per_s"] * 1e9) + tm / (rates["l2_miss_G_per_s"] * 1e9) +
                             (stream_in + 4) / (rates["stream_GB_per_s"] * 1e9))
                bound_ms = n * per_pkt_s * 1e3
                line_model = {"l2_hits_per_packet": round(h, 3), "l2_misses_per_packet": round(m, 3),
                              "stream_lines_per_packet": round(s_lines, 3), "table_misses_per_packet": round(tm, 3),
                              "stream_bytes_per_packet": round(stream_in + 4, 2),
                              "bound_ms": round(bound_ms, 3), "frac": round(bound_ms / avg_kern_ms, 3),
                              "counters_from": tj.get("tag"), "rates": "line_rates (this process, same device)"}
            # SURVEY.md §8d's side figures: fabric-side line traffic (one TCC_EA0_RDREQ per 128-B line, stream and
            # gathers alike) as GB/s at this run's kernel time, and the LDS bank-conflict rate
            if "ea_rdreq_per_packet" in tj:
                extra["line_traffic_GBps_at_128B"] = round(tj["ea_rdreq_per_packet"] * 128 * n / (avg_kern_ms * 1e-3)
                                                           / 1e9, 1)
                if rates:  # the fabric's line traffic against the stream bandwidth this process measured
                    extra["line_traffic_frac_of_stream"] = round(extra["line_traffic_GBps_at_128B"] /
                                                                 rates["stream_GB_per_s"], 3)
                    # the one bound the line counts give: at this build's lines per packet the kernel can run at
                    # most this much faster before its 128-B lines fill the measured stream bandwidth
                    extra["headroom_at_current_lines"] = round(1.0 / max(extra["line_traffic_frac_of_stream"], 1e-9), 3)
                extra["fetch_size_GBps"] = round(traffic / (avg_kern_ms * 1e-3) / 1e9, 1) if traffic else None
            if "lds_bank_conflict_rate" in tj:
                extra["lds_bank_conflict_rate"] = round(tj["lds_bank_conflict_rate"], 4)
        except (KeyError, TypeError, ValueError):
            traffic = None

    out = {
        "metric": METRIC,
        "value": round(mpps, 2),
        "unit": "Mpps",
        "n_gpus": world,
        "rccl_world_size": dist.get_world_size() if use_dist else None,
        "build_id": build_id,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.global_packets else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": {1: "cfg1: 10k IPv4 /16-/32 prefixes x 10 rules",
                         2: "cfg2: 1M mixed IPv4/IPv6 prefixes (BGP-like lengths) x 99 rules/target, "
                            f"{info['n_lists']} " + ("distinct" if "_distinct" in wkey else "interned")
                            + " lists, 4 ifindexes, " + ("uniform" if args.uniform else "Zipf(1.1)") + " sources",
                         4: "cfg4: adversarial /128 + last-slot ICMPv6"}[args.cfg]
                        + (f"; configs[3] job of {args.global_packets} packets sharded over {world} GPU(s)"
                           if args.global_packets else ""),
            "workload_key": wkey,
            "prefixes": wl.n_entries,
            "rule_lists": info["n_lists"],
            "packets_per_gpu_per_step": n,
            "global_batch": job_pkts,
            "parallelism": f"dp{world} (packet shards, replicated tables, RCCL all-reduce of stats)",
            "packets_counted_in_stats": counted,
            "stats_digest": digest,
            "tables": {"device_bytes_per_image": info["device_bytes"], "images_per_gpu": 2,
                       "dt_parts": info["dt_parts"], "d16_words": bool(info["d16"]), "key_order": args.key_order,
                       "setup_s": round(commit_s, 2), "rank0": how,
                       "compile_ms": round(info["compile_ms"], 1), "upload_ms": round(info["upload_ms"], 1),
                       # peak host RSS of rank 0 (table compile + workload); the others import its image
                       "host_peak_rss_gib": round(peak_rss_gib, 2)},
        },
        # every rank: its own wall time of the K steps, average kernel time (HIP events on its launch stream),
        # table setup and whether it compiled or imported rank 0's image, peak host RSS, packets per step
        "per_rank": [{"rank": r, "elapsed_s": round(v[0], 5), "kernel_ms_avg": round(v[1], 4),
                      "tables_setup_s": round(v[2], 2), "tables": "imported" if v[3] else "compiled",
                      "host_peak_rss_gib": round(v[4], 2), "packets_per_step": int(v[5])}
                     for r, v in enumerate(per_rank)],
        # host-packed: the path runs at the host packers' and the link's rate, so its bound is PCIe (the packed
        # tuples' H2D bytes against the measured dense H2D rate), not HBM
        "roofline": {
            "bound": "pcie" if host_feed else "hbm",
            "achieved": host_feed["pcie_h2d_GBps"] if host_feed else round(achieved, 2),
            "peak": PCIE_H2D_GBS if host_feed else HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": host_feed["pcie_h2d_frac"] if host_feed else round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic,
            "traffic_from": traffic_from,
            "kernel": kernel,
            "kernel_ms_avg": round(avg_kern_ms, 4),
            "algorithmic_bytes_per_packet": round(algo_bytes, 3),
            "layout": args.layout,
            "random_line_model": line_model,
            "line_rates": rates,
            **extra,
            **extra_pipe,
        },
        "cpu_baseline": None,
    }

    # ---- CPU baseline: the oracle (plain C restatement of kernel.c) on host cores, rank 0, N=1 only
    if world == 1 and rank == 0 and not args.no_cpu_baseline and n:
        if perm is not None:  # the rings' results back into packet order
            in_order = torch.empty_like(results)
            in_order[perm] = results
            results = in_order
        out["cpu_baseline"] = cpu_baseline(args, wl, results, n, start)

    if rank == 0:
        print(json.dumps(out), flush=True)
    clf.stats_bind(0, None)
    if use_dist:
        dist.destroy_process_group()


def probe_line_rates(W, ordinal, log):
    """The device's random-line and stream rates (workload.hip), or None when the probe cannot allocate its 2-GiB
    buffers beside the tables (a rank whose device is full reports no random_line_model, not a crash)."""
    import infw
    try:
        return W.line_rates(ordinal)
    except infw.InfwError as e:
        log(f"[bench] line-rate probe skipped: {e}")
        return None


def _slot_shard(args, s, n_slots):
    """Packets [start, start + n) of slot s: a fixed job's shard_range, or a fixed batch per slot (weak)."""
    if args.global_packets:
        a, b = shard_range(args.global_packets, s, n_slots)
        return a, b - a
    return s * args.batch, args.batch


def run_in_process(args, n_slots):
    """The library's own multi-GPU shape (how a cgo daemon would drive it): one context over N device
    slots — the table compiled once and published to every slot by infw_table_commit (one host thread per slot) —
    and one host thread with its own HIP stream per slot classifying that slot's shard, K steps back to back.  Each
    slot's counters land in its own statistics slot (kernel.c:36-41's per-CPU slots); the reader sums them per rule
    with infw_stats_read_all (statistics.go:126-157), so no collective is involved.  The timed region is bracketed
    by a thread barrier and a synchronize of every device; value = packets of all slots / that time."""
    import threading

    import numpy as np
    import torch

    import infw
    from infw import workloads as W
    from infw.batch import SoaBatch

    def log(*a):
        print(*a, file=sys.stderr, flush=True)

    have = torch.cuda.device_count()
    devices = [0] * n_slots if args.slots_on_gpu0 else list(range(n_slots))
    if max(devices) >= have:
        sys.exit(f"bench.py --in-process: {n_slots} slots need {max(devices) + 1} device(s), {have} visible")
    wl = W.Workload(args.cfg, n_prefixes=args.prefixes, n_templates=args.templates)
    if args.uniform:
        wl.uniform_sources()
    clf = infw.Classifier(devices=devices, max_entries=wl.n_entries + 16, options=args.options)
    t0 = time.time()
    wl.load_into(clf, order=wl.shuffled_order() if args.key_order == "shuffled" else None)
    clf.commit()
    info = clf.info()
    setup_s = time.time() - t0
    log(f"[bench] in-process: {n_slots} slot(s) on device(s) {devices}, {wl.n_entries} entries, tables compiled once "
        f"and published to every slot in {setup_s:.1f}s (slowest slot {info['device_ms_max']:.0f} ms)")
    shards = [_slot_shard(args, s, n_slots) for s in range(n_slots)]
    batches, results, streams = [], [], []
    for s, (start, n) in enumerate(shards):
        dev = torch.device("cuda", devices[s])
        b = SoaBatch.empty(max(n, 1), dev).slice(0, n)
        if n:
            wl.gen_device(b, start=start, dev_ordinal=devices[s])
        batches.append(b)
        results.append(torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n])
        streams.append(torch.cuda.Stream(device=dev))
    for d in set(devices):
        torch.cuda.synchronize(d)
    evs = [[tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(args.steps)]
           for _ in range(n_slots)]
    errors = []

    def slot_thread(s, steps, gate, timed):
        try:
            torch.cuda.set_device(devices[s])
            gate.wait()
            for k in range(steps):
                if timed:
                    evs[s][k][0].record(streams[s])
                if shards[s][1]:
                    clf.classify(batches[s], results=results[s], dev=s, stream=streams[s])
                if timed:
                    evs[s][k][1].record(streams[s])
        except BaseException as e:  # surfaced by the main thread
            errors.append(e)
            gate.abort()

    def run(steps, timed):
        gate = threading.Barrier(n_slots + 1)
        th = [threading.Thread(target=slot_thread, args=(s, steps, gate, timed)) for s in range(n_slots)]
        for t in th:
            t.start()
        for d in set(devices):
            torch.cuda.synchronize(d)
        gate.wait()
        ts = time.perf_counter()
        for t in th:
            t.join()
        for d in set(devices):
            torch.cuda.synchronize(d)
        if errors:
            raise errors[0]
        return time.perf_counter() - ts

    clf.stats_reset()
    run(args.warmup, False)
    warm = clf.stats_read_all()
    clf.stats_reset()
    elapsed = run(args.steps, True)
    total = clf.stats_read_all()  # summed per rule over the slots (infw_stats_read_all)
    if args.warmup:
        assert not (warm % args.warmup).any(), "warmup steps' counters differ"
        digest_block = warm // args.warmup
        assert np.array_equal(total, digest_block * args.steps), "a timed step's counters differ from the warmup's"
    else:
        assert not (total % max(args.steps, 1)).any(), "timed steps' counters differ"
        digest_block = total // max(args.steps, 1)
    job = sum(n for _, n in shards)
    kern = [sum(e[0].elapsed_time(e[1]) for e in evs[s]) / max(args.steps, 1) for s in range(n_slots)]
    out = {
        "metric": METRIC, "value": round(job * args.steps / elapsed / 1e6, 2), "unit": "Mpps",
        "n_gpus": len(set(devices)), "mode": "in-process", "device_slots": n_slots, "rccl_world_size": None,
        "build_id": infw.build_id(), "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / max(args.steps, 1) * 1e3, 3), "higher_is_better": True,
        "scaling": "strong" if args.global_packets else "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic",
        "config": {"workload_key": workload_key(args.cfg, args.templates, args.prefixes), "prefixes": wl.n_entries,
                   "rule_lists": info["n_lists"], "global_batch": job,
                   "parallelism": f"{n_slots} device slot(s) of one context on device(s) {sorted(set(devices))}, "
                                  "one host thread + stream each, counters summed per rule over slots",
                   # over the timed steps, as the rank path counts them
                   "packets_counted_in_stats": int(total[:, 0].sum() + total[:, 2].sum()),
                   "stats_digest": stats_digest(digest_block),
                   "tables": {"setup_s": round(setup_s, 2), "device_ms_max": round(info["device_ms_max"], 1),
                              "n_device_slots": info["n_device_slots"]}},
        "kernel": clf.variant(infw.INPUT_SOA),
        "per_slot": [{"slot": s, "device": devices[s], "packets_per_step": shards[s][1],
                      "kernel_ms_avg": round(kern[s], 4)} for s in range(n_slots)],
    }
    print(json.dumps(out), flush=True)
    clf.close()


def run_in_process_host_walk(args, n_slots):
    """TEST ONLY (--in-process --host-walk): the in-process shape on a CPU box — one host-only context, one host
    thread per slot walking its shard through the compiled host image (infw_debug_walk, which may run on many
    threads at once), the slots' counters summed per rule.  The digest equals the rank path's for the same job."""
    import threading

    import numpy as np

    import infw
    from infw import workloads as W
    wl = W.Workload(args.cfg, n_prefixes=args.prefixes or 20000, n_templates=args.templates or 64)
    clf = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16, options=args.options)
    wl.load_into(clf, order=wl.shuffled_order() if args.key_order == "shuffled" else None)
    clf.commit()
    shards = []
    for s in range(n_slots):
        if args.global_packets:
            a, b = shard_range(args.global_packets, s, n_slots)
            shards.append((a, b - a))
        else:
            shards.append((s * min(args.batch, 1 << 16), min(args.batch, 1 << 16)))
    slots = [np.zeros((1024, 4), np.uint64) for _ in range(n_slots)]
    errors = []

    def slot_thread(s):
        try:
            start, n = shards[s]
            if n:
                t = wl.tuples(start, n)
                for _ in range(max(args.steps, 1)):
                    slots[s] += host_counters(clf.debug_walk(t), t[:, 5])
        except BaseException as e:
            errors.append(e)

    th = [threading.Thread(target=slot_thread, args=(s,)) for s in range(n_slots)]
    ts = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    elapsed = time.perf_counter() - ts
    if errors:
        raise errors[0]
    total = sum(slots)
    assert not (total % max(args.steps, 1)).any()
    block = total // max(args.steps, 1)
    job = sum(n for _, n in shards)
    print(json.dumps({
        "metric": METRIC + " [host-walk selftest: not a measurement]", "value": round(job * args.steps / elapsed / 1e6, 4),
        "unit": "Mpps", "valid_measurement": False, "n_gpus": 0, "mode": "in-process", "device_slots": n_slots,
        "steps": args.steps, "scaling": "strong" if args.global_packets else "weak", "build_id": infw.build_id(),
        "config": {"workload_key": workload_key(args.cfg, args.templates, args.prefixes), "prefixes": wl.n_entries,
                   "global_batch": job, "packets_counted_in_stats": int(block[:, 0].sum() + block[:, 2].sum()),
                   "stats_digest": stats_digest(block)},
        "per_slot": [{"slot": s, "packets_per_step": shards[s][1]} for s in range(n_slots)]}), flush=True)


def cpu_baseline(args, wl, results, n, start=0):
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    m = orc.OracleMap(max_entries=wl.n_entries + 16)
    for k, v in wl.entries():
        m.update(k, v)
    cores = usable_cores()
    threads = args.cpu_threads or cores
    # ~0.6 Mpps per thread at 1M prefixes: about 15 s of classify work on the usable cores
    s = min(args.cpu_sample or max(8 << 20, ((threads * 6 << 20) >> 23) << 23), n)
    # bounded sample, in chunks of 8M frame snapshots (80 B each) so host memory stays ~0.7 GB;
    # only the oracle's classify calls are timed (frame synthesis is not CPU-path work)
    secs, parity, chunk, examined, ex_n = 0.0, True, 8 << 20, 0, 0
    for off in range(0, s, chunk):
        c = min(chunk, s - off)
        hdr, cap, pl, ifx = wl.frames(start + off, c)
        res, _, _, dt = m.classify_frames(hdr, cap, pl, ifx, nthreads=threads)
        secs += dt
        if off == 0:  # the reference's scan work on the first 1M packets (single thread, not timed)
            ex_n = min(c, 1 << 20)
            examined = m.rules_examined(hdr[:ex_n], cap[:ex_n], pl[:ex_n], ifx[:ex_n])
        gpu = results[off:off + c].cpu().numpy().view(np.uint32)
        parity = parity and bool(np.array_equal(gpu, res))
        del hdr, cap, pl, ifx, res
    return {
        "value": round(s / secs / 1e6, 3),
        "unit": "Mpps",
        "cores": cores,
        "threads": threads,
        "affinity_cpus": len(os.sched_getaffinity(0)),
        "kind": "port",
        "sample": f"first {s} packets of rank 0's cfg{args.cfg} batch, {threads} pthreads on {cores} usable cores "
                  f"(affinity set, cgroup quota), oracle/infw_oracle.c "
                  f"(frame parse + hash-per-length LPM + 100-slot scan), {secs:.2f}s of classify wall time",
        "gpu_results_bitexact_on_sample": parity,
        # bytes of rule records the reference's in-order loop examines per packet (12 B per valid
        # rule up to and including the first match); the GPU path reads one 64-B decision line instead
        "reference_rule_bytes_examined_per_packet": round(12 * examined / max(ex_n, 1), 2),
    }


if __name__ == "__main__":
    main()
