"""Deny-event consumer: perf samples -> the daemon's syslog lines.

Host-side mirror of ingressNodeFwEvents (pkg/ebpf/ingress_node_firewall_events.go:24-170) over the samples
infw_events_capture writes (include/infw.h: one 272-B slot per event-ring record, perf's u32 raw size followed by
the raw sample = event_hdr_st + min(len, 256) frame bytes + alignment pad, kernel.c:392-399).

  read_samples      perf.Reader.Read() -> Record.RawSample             events.go:64-75
  decode_sample     header / packet parse, iface lookup, syslog lines   events.go:77-166
  gopacket_layers   gopacket.NewPacket(packet, LayerTypeEthernet, gopacket.Default) for the layers the consumer logs

gopacket v1.1.19 (the reference's go.mod pin; vendored at vendor/github.com/google/gopacket) is a third-party
dependency; gopacket_layers restates the decoders the consumer depends on — layers/ethernet.go decodeEthernet,
ip4.go decodeIPv4 / IPv4.DecodeFromBytes / NextLayerType, ip6.go decodeIPv6 / IPv6.DecodeFromBytes, tcp.go decodeTCP,
udp.go decodeUDP, sctp.go decodeSCTP, icmp4.go / icmp6.go via base.go decodingLayerDecoder, packet.go
eagerPacket.NextDecoder — and keeps their quirks: IPv4, IPv6, TCP, UDP and SCTP layers are added even when their
decode fails (zero ports / nil addresses then), the ICMP layers only on success; IPv4 payloads are cut to the
header's total length and fragments stop at a Fragment layer.  Not restated (decoding stops there, "parity
unpinned" for such packets): IPv6 extension headers (hop-by-hop, routing, fragment, ...), IP protocols other than
TCP/UDP/SCTP/ICMP/ICMPv6/IPv4/IPv6, and application layers behind UDP ports (a VXLAN/Geneve/GTP payload would
add inner layers in gopacket).  Those packets are denied only by protocol-0 rules.
"""
from __future__ import annotations

import ipaddress
import struct
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

SAMPLE_BYTES = 272     # INFW_EVENT_SAMPLE_BYTES
XDP_DENY, XDP_ALLOW = 1, 2  # loader.go:30-31


def convert_xdp_action_to_string(action: int) -> str:
    """convertXdpActionToString (events.go:172-181)."""
    if action == XDP_DENY:
        return "Drop"
    if action == XDP_ALLOW:
        return "Allow"
    return f"Invalid action {action}"


def go_ip_string(ip: Optional[bytes]) -> str:
    """net.IP.String(): nil -> "<nil>", 4 bytes or IPv4-mapped 16 bytes -> dotted quad, else RFC 5952."""
    if ip is None or len(ip) == 0:
        return "<nil>"
    if len(ip) == 4:
        return ".".join(str(b) for b in ip)
    if len(ip) == 16:
        if ip[:10] == bytes(10) and ip[10:12] == b"\xff\xff":
            return ".".join(str(b) for b in ip[12:])
        return str(ipaddress.IPv6Address(bytes(ip)))  # longest zero run >= 2 groups, first on ties, lower hex
    return "?" + ip.hex()


def read_samples(samples: np.ndarray, count: int) -> Tuple[List[bytes], int]:
    """RawSample of each record written (min(count, capacity) slots) and the number of lost records (the perf
    ring's lost-sample count: events beyond the ring's capacity)."""
    s = np.asarray(samples, dtype=np.uint8).reshape(-1, SAMPLE_BYTES)
    k = min(int(count), s.shape[0])
    out = []
    for r in range(k):
        size = int(s[r, :4].view("<u4")[0])
        out.append(bytes(s[r, 4:4 + size]))
    return out, int(count) - k


def gopacket_layers(data: bytes) -> Dict[str, dict]:
    """The first layer of each logged type gopacket's eager decode of an Ethernet frame produces."""
    layers: Dict[str, dict] = {}

    def add(kind, **fields):
        layers.setdefault(kind, fields)  # Packet.Layer(t) returns the first layer of type t

    def ipv4(d):  # decodeIPv4: the layer is added before the error check
        if len(d) < 20:
            add("ipv4", src=None, dst=None)
            return
        flagsfrags = struct.unpack(">H", d[6:8])[0]
        ihl, length, proto = d[0] & 0x0F, struct.unpack(">H", d[2:4])[0], d[9]
        add("ipv4", src=bytes(d[12:16]), dst=bytes(d[16:20]))
        if length == 0:  # TSO: the actual length is the data's
            length = len(d) & 0xFFFF
        if length < 20 or ihl < 5 or ihl * 4 > length:
            return
        if len(d) > length:
            d = d[:length]
        elif len(d) < length and ihl * 4 > len(d):
            return
        opts = d[20:ihl * 4]
        while opts:  # IPv4.DecodeFromBytes option walk: its errors end the decode
            t = opts[0]
            if t == 0:
                break
            if t == 1:
                opts = opts[1:]
                continue
            if len(opts) < 2 or len(opts) < opts[1] or opts[1] <= 2:
                return
            opts = opts[opts[1]:]
        if (flagsfrags >> 13) & 0x1 or flagsfrags & 0x1FFF:  # IPv4MoreFragments / FragOffset: Fragment layer
            return
        nxt(proto, d[ihl * 4:])

    def ipv6(d):
        if len(d) < 40:
            add("ipv6", src=None, dst=None)
            return
        add("ipv6", src=bytes(d[8:24]), dst=bytes(d[24:40]))
        length, nh = struct.unpack(">H", d[4:6])[0], d[6]
        if nh == 0:  # hop-by-hop / jumbogram handling: not restated
            return
        if length == 0:
            return
        nxt(nh, d[40:40 + length])

    def nxt(proto, payload):  # eagerPacket.NextDecoder: an empty payload ends the decode
        if not payload:
            return
        if proto == 6:  # decodeTCP
            if len(payload) < 20:
                add("tcp", sport=0, dport=0)
            else:
                add("tcp", sport=struct.unpack(">H", payload[0:2])[0], dport=struct.unpack(">H", payload[2:4])[0])
        elif proto == 17:  # decodeUDP
            if len(payload) < 8:
                add("udp", sport=0, dport=0)
            else:
                add("udp", sport=struct.unpack(">H", payload[0:2])[0], dport=struct.unpack(">H", payload[2:4])[0])
        elif proto == 132:  # decodeSCTP
            if len(payload) < 12:
                add("sctp", sport=0, dport=0)
            else:
                add("sctp", sport=struct.unpack(">H", payload[0:2])[0], dport=struct.unpack(">H", payload[2:4])[0])
        elif proto == 1:  # decodingLayerDecoder(ICMPv4): added only when >= 8 bytes
            if len(payload) >= 8:
                add("icmpv4", type=payload[0], code=payload[1])
        elif proto == 58:  # ICMPv6: >= 4 bytes
            if len(payload) >= 4:
                add("icmpv6", type=payload[0], code=payload[1])
        elif proto == 4:
            ipv4(payload)
        elif proto == 41:
            ipv6(payload)

    if len(data) < 14:  # "Ethernet packet too small": no layer
        return layers
    et = struct.unpack(">H", data[12:14])[0]
    if et == 0x0800:
        ipv4(data[14:]) if len(data) > 14 else None
    elif et == 0x86DD:
        ipv6(data[14:]) if len(data) > 14 else None
    return layers


def decode_sample(raw: bytes, if_name: Callable[[int], Optional[str]]) -> Tuple[List[str], List[str]]:
    """One perf record -> (syslog lines, daemon log lines), events.go:77-166."""
    if len(raw) < 8:
        return [], ["Parsing perf event header err: unexpected EOF"]
    if_id, rule_id, action, _pad, pkt_length = struct.unpack("<HHBBH", raw[:8])
    body = raw[8:]
    if len(body) < pkt_length:  # binary.Read of PktLength bytes
        return [], ["Parsing perf event packet header : " + ("EOF" if not body else "unexpected EOF")]
    packet = body[:pkt_length]
    name = if_name(if_id)  # net.InterfaceByIndex
    if name is None:
        return [], [f"lookup network iface {if_id}: route ip+net: no such network interface"]
    lines = [f"ruleId {rule_id} action {convert_xdp_action_to_string(action)} len {pkt_length} if {name}\n"]
    ly = gopacket_layers(packet)
    if "ipv4" in ly:
        lines.append(f"\tipv4 src addr {go_ip_string(ly['ipv4']['src'])} dst addr {go_ip_string(ly['ipv4']['dst'])}\n")
    if "ipv6" in ly:
        lines.append(f"\tipv6 src addr {go_ip_string(ly['ipv6']['src'])} dst addr {go_ip_string(ly['ipv6']['dst'])}\n")
    if "tcp" in ly:
        lines.append(f"\ttcp srcPort {ly['tcp']['sport']} dstPort {ly['tcp']['dport']}\n")
    if "udp" in ly:
        lines.append(f"\tudp srcPort {ly['udp']['sport']} dstPort {ly['udp']['dport']}\n")
    if "sctp" in ly:
        lines.append(f"\tsctp srcPort {ly['sctp']['sport']} dstPort {ly['sctp']['dport']}\n")
    if "icmpv4" in ly:
        lines.append(f"\ticmpv4 type {ly['icmpv4']['type']} code {ly['icmpv4']['code']}\n")
    if "icmpv6" in ly:
        lines.append(f"\ticmpv6 type {ly['icmpv6']['type']} code {ly['icmpv6']['code']}\n")
    return lines, []


def drain(samples: np.ndarray, count: int, if_name: Callable[[int], Optional[str]]) -> Tuple[List[str], List[str]]:
    """Every record of one capture, in ring order: the syslog lines and the daemon's log lines (a lost-samples
    line first when the ring overflowed, like perf's PERF_RECORD_LOST record, events.go:78-81)."""
    raws, lost = read_samples(samples, count)
    sys_lines: List[str] = []
    log: List[str] = [f"Perf event ring buffer full, dropped {lost} samples"] if lost else []
    for raw in raws:
        a, b = decode_sample(raw, if_name)
        sys_lines += a
        log += b
    return sys_lines, log
