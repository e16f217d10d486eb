"""Independent Python restatement of the Go encoders the reference writes the
table map with (test infrastructure; the product's encoders live in
csrc/controlplane.cpp and are checked against these):
  BuildEBPFKey            pkg/ebpf/ingress_node_firewall_loader.go:530-547
  makeIngressFwRulesMap   pkg/ebpf/ingress_node_firewall_loader.go:435-515
  utils.GetPort/GetRange  pkg/utils/utils.go:20-60
"""
from __future__ import annotations

import ipaddress
import struct

XDP_DENY, XDP_ALLOW = 1, 2
PROTO = {"TCP": 6, "UDP": 17, "SCTP": 132, "ICMP": 1, "ICMPv6": 58}


def build_key(if_id: int, cidr: str) -> bytes:
    addr, mask = cidr.split("/")
    ip = ipaddress.ip_address(addr)
    bits = 32 if ip.version == 4 else 128
    m = int(mask)
    assert 0 <= m <= bits
    if ip.version == 4:
        data = ip.packed
    elif ip.ipv4_mapped is not None:           # ip.To4() != nil
        data = ip.ipv4_mapped.packed
    else:
        data = ip.packed
    return struct.pack("<II", m + 32, if_id) + data.ljust(16, b"\0")


def rule_bytes(rule_id, proto, ps, pe, it, ic, action) -> bytes:
    return struct.pack("<IBHHBBB", rule_id, proto, ps, pe, it, ic, action)


def make_value(rules) -> bytes:
    """rules: dicts {order, protocol, ports, icmp_type, icmp_code, action} (CRD form)."""
    slots = [rule_bytes(0, 0, 0, 0, 0, 0, 0)] * 100
    for r in rules:
        o = r["order"]
        proto = PROTO.get(r.get("protocol", ""), 0)
        ps = pe = it = ic = 0
        if proto in (6, 17, 132):
            p = str(r["ports"])
            if "-" in p:
                a, b = p.split("-", 1)
                ps, pe = int(a), int(b)
                assert 0 < ps < pe <= 65535
            else:
                ps = int(p)
                assert 0 < ps <= 65535
        elif proto in (1, 58):
            it, ic = r.get("icmp_type", 0), r.get("icmp_code", 0)
        act = {"Allow": XDP_ALLOW, "Deny": XDP_DENY}[r["action"]]
        slots[o] = rule_bytes(o, proto, ps, pe, it, ic, act)
    return b"".join(slots)


def raw_value(rules) -> bytes:
    """rules: dicts {slot, ruleId, protocol, dstPortStart, dstPortEnd, icmpType, icmpCode, action} (map form)."""
    slots = [rule_bytes(0, 0, 0, 0, 0, 0, 0)] * 100
    for r in rules:
        slots[r["slot"]] = rule_bytes(r["ruleId"], r["protocol"], r["dstPortStart"], r["dstPortEnd"], r["icmpType"],
                                      r["icmpCode"], r["action"])
    return b"".join(slots)


def sync(map_obj, key_to_val: dict):
    """IngressNodeFwRulesLoader's map edits (loader.go:169-191): purge stale keys, then update all."""
    existing = list(map_obj.keys())
    for k in existing:
        if k not in key_to_val:
            map_obj.delete(k)
    for k, v in key_to_val.items():
        assert map_obj.update(k, v, 0) == 0


def desired(rules_by_iface, ifindex: dict) -> dict:
    out = {}
    for name, entries in (rules_by_iface or {}).items():
        for e in entries:
            val = make_value(e["rules"])
            for cidr in e["source_cidrs"]:
                out[build_key(ifindex[name], cidr)] = val
    return out
