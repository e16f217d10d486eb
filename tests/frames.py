"""Build Ethernet/IPv4/IPv6/L4 frames for golden vectors (test infrastructure).

Header sizes follow the structs the reference program reads
(bpf/headers/vmlinux.h: ethhdr 14, iphdr 20, ipv6hdr 40, tcphdr 20, udphdr 8,
sctphdr 12, icmphdr 8, icmp6hdr 8).
"""
from __future__ import annotations

import ipaddress
import struct

import numpy as np

PROTO = {"tcp": 6, "udp": 17, "sctp": 132, "icmp": 1, "icmpv6": 58, "gre": 47}


def frame(src: str, dst: str | None = None, proto="tcp", dport: int = 0, sport: int = 40000, icmp_type: int = 0,
          icmp_code: int = 0, length: int | None = None, ethertype: int | None = None, ihl: int = 5,
          truncate: int | None = None) -> bytes:
    """One frame.  src decides the family.  length pads with zeros; truncate cuts the bytes."""
    s = ipaddress.ip_address(src)
    v4 = s.version == 4
    d = ipaddress.ip_address(dst) if dst else ipaddress.ip_address("192.0.2.1" if v4 else "2001:db8::1")
    p = PROTO[proto] if isinstance(proto, str) else int(proto)
    et = ethertype if ethertype is not None else (0x0800 if v4 else 0x86DD)
    eth = bytes.fromhex("020000000001020000000002") + struct.pack("!H", et)
    if p in (6, 17, 132):
        if p == 6:
            l4 = struct.pack("!HHIIBBHHH", sport, dport, 1, 0, 0x50, 0x02, 65535, 0, 0)
        elif p == 17:
            l4 = struct.pack("!HHHH", sport, dport, 8, 0)
        else:
            l4 = struct.pack("!HHII", sport, dport, 0, 0)
    elif p in (1, 58):
        l4 = struct.pack("!BBHHH", icmp_type, icmp_code, 0, 1, 1)
    else:
        l4 = b"\x00\x00\x08\x00"
    if v4:
        ip = struct.pack("!BBHHHBBH4s4s", 0x40 | ihl, 0, 20 + len(l4), 1, 0, 64, p, 0, s.packed, d.packed)
        ip += b"\x00" * (4 * (ihl - 5)) if ihl > 5 else b""
    else:
        ip = struct.pack("!IHBB16s16s", 0x60000000, len(l4), p, 64, s.packed, d.packed)
    f = eth + ip + l4
    if length is not None and length > len(f):
        f += b"\x00" * (length - len(f))
    if truncate is not None:
        f = f[:truncate]
    return f


def snapshots(frames, width: int = 80):
    """Frames -> (hdr n x width, caplen, pkt_len) arrays for the batch APIs."""
    n = len(frames)
    hdr = np.zeros((n, width), np.uint8)
    cap = np.zeros(n, np.uint32)
    for i, f in enumerate(frames):
        b = np.frombuffer(f[:width], np.uint8)
        hdr[i, :b.size] = b
        cap[i] = len(f)
    return hdr, cap, cap.copy()


def http_targets(doc, tc):
    """TestSyncInterfaceIngressRulesWithHTTP (ebpfsyncer_test.go:41-445): (frame, ifindex, expected XDP action) for
    each connection of a test case — a TCP SYN from the netns peer 192.0.2.{4i+2} to 192.0.2.{4i+1}:port on dummy{i}."""
    out = []
    for target, ok in tc["targetResult"].items():
        ip, port = target.split(":")
        last = int(ip.split(".")[-1])
        i = (last - 1) // 4                       # 192.0.2.{4i+1} is dummy{i}
        peer = f"192.0.2.{4 * i + 2}"
        out.append((frame(peer, ip, "tcp", int(port)), doc["ifindex"][f"dummy{i}"], 2 if ok else 1))
    return out
