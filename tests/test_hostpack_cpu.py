"""The host packer of infw_classify_xdp_host on the CPU (infw_pack_xdp_host, csrc/infw_hostpack.h).

An AF_XDP RX ring (linux/if_xdp.h struct xdp_desc) over a umem of 2048-B chunks in ordinary host memory, in aligned
mode (frames at chunk + headroom, chunks in a shuffled order, as a fill ring recycles them) and in unaligned mode (the
offset in address bits 48..63).  Two checks, no device needed:
  - the packed family-compact streams, turned back into tuples, classified by the compiled host image
    (infw_debug_walk: the kernel's lookup code on the host) give the oracle's result words for the same frames
    (oracle/infw_oracle.c, which restates kernel.c:95-457 from the frame bytes);
  - edge frames (every truncation length 0..60, non-IP ethertypes, both families) pack to the fields kernel.c reads,
    restated here byte by byte from the fixed offsets (:104-166, :204, :291, :423-439).
The device path (pipelined chunks through the GPU) is tests/test_gpu_xdp_host.py.
"""
import numpy as np
import pytest

import infw
from frames import frame
from infw import workloads as W
from parity import oracle_for

CHUNK, HEADROOM = 2048, 256


def ring(hdrs, lens, mode, rng):
    """umem bytes and descriptors (n x 4 u32) for the frames."""
    n = len(hdrs)
    chunks = rng.permutation(n + 5)[:n]
    umem = np.zeros((n + 5) * CHUNK, np.uint8)
    desc = np.zeros((n, 4), np.uint32)
    for i in range(n):
        if mode == "aligned":
            base, off = int(chunks[i]) * CHUNK + HEADROOM, 0
        else:  # base in bits 0..47, offset in 48..63, frame at base + offset
            base, off = int(chunks[i]) * CHUNK, int(rng.integers(0, CHUNK - 96))
        h = np.frombuffer(bytes(hdrs[i]), np.uint8)
        umem[base + off: base + off + h.size] = h
        addr = base | (off << 48)
        desc[i, 0], desc[i, 1], desc[i, 2] = addr & 0xFFFFFFFF, addr >> 32, lens[i]
    return umem, desc


def fields_ref(f: bytes, length: int):
    """kernel.c's reads of one frame of linear length `length`: (saddr words, meta, l4word)."""
    b = lambda o: f[o] if o < length and o < len(f) else 0  # noqa: E731 — bytes past data_end read as 0
    et = (b(12) << 8 | b(13)) if length >= 14 else 0
    proto, soff, slen, l4off = 0, 0, 0, 0
    if et == 0x0800:
        proto, soff, slen, l4off = b(23), 26, 4, 34
    elif et == 0x86DD:
        proto, soff, slen, l4off = b(20), 22, 16, 54
    sb = bytes(b(soff + k) if k < slen else 0 for k in range(16))
    s = np.frombuffer(sb, "<u4")
    l4 = int.from_bytes(bytes(b(l4off + k) for k in range(4)), "little") if l4off else 0
    return s, et | proto << 16 | min(length, 255) << 24, l4


@pytest.mark.parametrize("mode", ["aligned", "unaligned"])
def test_packed_ring_walks_to_oracle(mode):
    rng = np.random.default_rng(3)
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    n = 3 * 64 + 29  # ragged last group
    hdr, cap, pl, ifx = wl.frames(4242, n)
    ring_if = int(np.bincount(ifx).argmax())
    want, _, _, _ = oracle_for(wl).classify_frames(hdr, pl.astype(cap.dtype), pl, np.full(n, ring_if, np.uint32),
                                                   nthreads=4)
    umem, desc = ring(hdr, pl, mode, rng)
    c = infw.pack_xdp_host(umem, desc, ring_if)
    assert (c["ifindex"] == ring_if).all() and np.array_equal(c["pkt_len"], pl)
    clf = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    got = clf.debug_walk(infw.compact_to_tuples(c))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (mode, bad[:5], got[bad[:5]], want[bad[:5]])
    assert ((c["meta"] & 0xFFFF) == 0x86DD).mean() > 0.2 and (want & 0xFF).astype(bool).mean() > 0.3


def test_edge_frames_pack_to_kernel_fields():
    base = [frame("10.1.2.3", "192.0.2.9", "tcp", dport=8080, length=64),
            frame("2001:db8::5", "2001:db8::1", "udp", dport=53, length=80),
            frame("10.9.9.9", proto="icmp", icmp_type=8, icmp_code=0),
            frame("2001:db8::7", proto="icmpv6", icmp_type=128, icmp_code=0),
            frame("10.1.1.1", proto="gre"),
            frame("10.1.1.1", "192.0.2.9", "tcp", dport=22, ethertype=0x8100),   # VLAN: not parsed
            frame("10.1.1.1", "192.0.2.9", "tcp", dport=22, ethertype=0x0806)]   # ARP
    frames, lens = [], []
    for f in base:
        for L in list(range(0, 61)) + [len(f), 1514]:
            frames.append(f)
            lens.append(L)
    rng = np.random.default_rng(5)
    for mode in ("aligned", "unaligned"):
        umem, desc = ring(frames, lens, mode, rng)
        c = infw.pack_xdp_host(umem, desc, 9)
        t = infw.compact_to_tuples(c)
        for i, (f, L) in enumerate(zip(frames, lens)):
            s, meta, l4 = fields_ref(f, L)
            assert t[i, 6] == meta and t[i, 7] == l4 and t[i, 5] == L and t[i, 4] == 9, (mode, i, L)
            assert t[i, 0] == s[0], (mode, i, L)
            if (meta & 0xFFFF) == 0x86DD:
                assert np.array_equal(t[i, 1:4], s[1:4]), (mode, i, L)


def test_pack_arguments():
    umem = np.zeros(4096, np.uint8)
    desc = np.zeros((0, 4), np.uint32)
    c = infw.pack_xdp_host(umem, desc, 1)  # an empty ring packs nothing
    assert c["meta"].size == 0
    import ctypes as C
    from infw import _native as N
    o = N.BatchSoaC(None, None, None, None, None, None)
    d = np.zeros((1, 4), np.uint32)
    assert N.lib.infw_pack_xdp_host(umem.ctypes.data, d.ctypes.data, 1, 1, C.byref(o)) == -22


@pytest.mark.parametrize("mode", ["aligned", "unaligned"])
def test_host_events_equal_oracle_samples(mode):
    """infw_xdp_host_events (include/infw_host.h): the deny-event perf samples of a ring from its frames in host memory
    and its result words equal the oracle's (kernel.c:392-399: orc_collect_events + orc_perf_sample over the same
    umem at the descriptors' offsets) byte for byte — header fields, the first min(len, 256) frame bytes, the pad —
    in ring order; a capacity below the event count keeps the count (perf's lost samples)."""
    rng = np.random.default_rng(11)
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    m = oracle_for(wl)
    hdr, cap, pl, ifx = wl.frames(5000, 12000)
    ifindex = int(np.bincount(ifx).argmax())  # one ring = one interface: that interface's frames
    hdr, pl = hdr[ifx == ifindex], pl[ifx == ifindex]
    big = pl.astype(np.uint32)  # frames up to their full length (> 256 B), 80-B snapshots padded with zeros
    umem, desc = ring(hdr, big, mode, rng)
    addr = desc[:, 0].astype(np.uint64) | desc[:, 1].astype(np.uint64) << np.uint64(32)
    offs = (addr & np.uint64((1 << 48) - 1)) + (addr >> np.uint64(48))
    recs, want = m.collect_event_samples(umem, offs, big, big, np.full(len(offs), ifindex, np.uint32))
    assert len(recs) > 100
    # the result words the oracle gives the same frames (what infw_classify_xdp_host returns for this ring)
    res, _, _, _ = m.classify_frames(np.stack([umem[o:o + 80] for o in offs.astype(np.int64)]), np.minimum(big, 80),
                                     big, np.full(len(offs), ifindex, np.uint32), nthreads=8)
    got, k = infw.xdp_host_events(umem, desc, ifindex, res, len(recs) + 5)
    assert k == len(recs)
    assert np.array_equal(got[:k], want), np.nonzero((got[:k] != want).any(axis=1))[0][:5]
    assert not got[k:].any()
    small, k2 = infw.xdp_host_events(umem, desc, ifindex, res, 10)
    assert k2 == len(recs) and np.array_equal(small, want[:10])


def _burst_of(hdr, linear, pkt_len, ifindex, stride=2048):
    """A DPDK-style burst: each frame's snapshot at its own place in a buffer (zeros after it), one pointer per frame."""
    n = len(hdr)
    buf = np.zeros(n * stride + 512, np.uint8)
    for i in range(n):
        h = np.frombuffer(bytes(hdr[i]), np.uint8)
        buf[i * stride: i * stride + h.size] = h
    ptrs = buf.ctypes.data + np.arange(n, dtype=np.uint64) * np.uint64(stride)
    return buf, infw.Burst(ptrs, linear, pkt_len, ifindex), np.arange(n, dtype=np.uint64) * np.uint64(stride)


def test_burst_packs_walk_to_oracle():
    """infw_pack_burst_host: frames behind pointers with linear lengths below their frame lengths (multi-segment mbufs)
    pack to tuples that the compiled host image walks to the oracle's result words for the same frames."""
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    n = 5 * 64 + 13
    hdr, cap, pl, ifx = wl.frames(777, n)
    port = int(np.bincount(ifx).argmax())
    # first segments of 60 / 64 / 128 B (the rest of the frame in other segments), a few cut inside the headers
    rng = np.random.default_rng(19)
    cap = np.minimum(cap, rng.choice(np.array([60, 64, 128, 20, 41, 9000], np.uint32), n,
                                     p=[.3, .3, .2, .05, .05, .1])).astype(np.uint32)
    want, _, _, _ = oracle_for(wl).classify_frames(hdr, cap, pl, np.full(n, port, np.uint32), nthreads=4)
    assert (cap < pl).mean() > 0.5  # linear part shorter than the frame for most of them
    buf, b, _ = _burst_of(hdr, cap, pl, port)
    c = infw.pack_burst_host(b)
    assert (c["ifindex"] == port).all() and np.array_equal(c["pkt_len"], pl)
    clf = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    got = clf.debug_walk(infw.compact_to_tuples(c))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bad[:5], got[bad[:5]], want[bad[:5]])


def test_burst_edge_frames_pack_to_kernel_fields():
    """Every truncation 0..60 of several protocols as the linear part of a 1514-B frame: the packed fields are the
    bytes kernel.c reads within the linear part, pkt_len the whole frame's."""
    base = [frame("10.1.2.3", "192.0.2.9", "tcp", dport=8080, length=64),
            frame("2001:db8::5", "2001:db8::1", "udp", dport=53, length=80),
            frame("2001:db8::7", proto="icmpv6", icmp_type=128, icmp_code=0),
            frame("10.1.1.1", "192.0.2.9", "tcp", dport=22, ethertype=0x0806)]
    frames, lens = [], []
    for f in base:
        for L in range(0, 61):
            frames.append(np.frombuffer(bytes(f).ljust(80, b"\0")[:80], np.uint8))
            lens.append(L)
    lens = np.array(lens, np.uint32)
    buf, b, _ = _burst_of(frames, lens, np.full(len(lens), 1514, np.uint32), 3)
    t = infw.compact_to_tuples(infw.pack_burst_host(b))
    for i, L in enumerate(lens):
        s, meta, l4 = fields_ref(bytes(frames[i]), int(L))
        assert t[i, 6] == meta and t[i, 7] == l4 and t[i, 5] == 1514 and t[i, 0] == s[0], (i, L)
        if (meta & 0xFFFF) == 0x86DD:
            assert np.array_equal(t[i, 1:4], s[1:4]), (i, L)


def test_burst_events_equal_oracle_samples():
    """infw_burst_host_events: the perf samples of a burst's denied frames equal the oracle's — captured =
    min(pkt_len, 256) with zeros past the linear part — and the count survives a small capacity."""
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    m = oracle_for(wl)
    hdr, cap, pl, ifx = wl.frames(9000, 8000)
    port = int(np.bincount(ifx).argmax())
    hdr, cap, pl = hdr[ifx == port], cap[ifx == port], pl[ifx == port]
    cap = np.minimum(cap, np.where(np.arange(cap.size) % 3 == 0, 64, 9000)).astype(np.uint32)  # some 64-B first segments
    buf, b, offs = _burst_of(hdr, cap, pl, port)
    recs, want = m.collect_event_samples(buf, offs, cap, pl, np.full(len(offs), port, np.uint32))
    res, _, _, _ = m.classify_frames(hdr, cap, pl, np.full(len(offs), port, np.uint32), nthreads=8)
    assert len(recs) > 50
    got, k = infw.burst_host_events(b, res, len(recs) + 3)
    assert k == len(recs) and np.array_equal(got[:k], want) and not got[k:].any()
    small, k2 = infw.burst_host_events(b, res, 7)
    assert k2 == k and np.array_equal(small, want[:7])
