"""The reference's e2e behavioural table (tests/golden/ref_e2e.json, transcribed from
test/e2e/functional/tests/e2e.go:176-831 and test/e2e/events/events.go by tests/golden/transcribe.py) as test
inputs: the node's merged rules per interface, the frames each reachability check sends, and the reference's own
drop-event matching (events.go extractEventsFromString / isEventInList) over the consumer's syslog text.
"""
from __future__ import annotations

import json
import os
import re

import numpy as np

from frames import frame

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DOC = json.load(open(os.path.join(GOLD, "ref_e2e.json")))
SPORT = 40000  # synthetic ephemeral source port (ref_e2e.json "assumptions")


def valid_rules(rules_by_iface: dict) -> dict:
    """The interfaces the loader programs: invalid names are skipped (loader.go:143-146)."""
    return {k: v for k, v in rules_by_iface.items() if k in DOC["ifindex"]}


def controller_rules(rules_by_iface: dict):
    import infw
    return {name: [infw.IngressNodeFirewallRules(e["source_cidrs"], [infw.ProtocolRule(**r) for r in e["rules"]])
                   for e in ents] for name, ents in rules_by_iface.items()}


def conn_frame(c: dict) -> bytes:
    proto = c["protocol"].lower()
    if proto in ("icmp", "icmpv6"):
        return frame(c["src"], c["dst"], proto, icmp_type=c["icmp_type"], icmp_code=c["icmp_code"])
    return frame(c["src"], c["dst"], proto, dport=c["dport"], sport=SPORT)


def case_frames(conns):
    """(frames, ifindex per frame) of a list of connections."""
    return [conn_frame(c) for c in conns], [DOC["ifindex"][c["interface"]] for c in conns]


def packed(frames):
    """Frames back to back: (buffer, offsets u64, lengths u32)."""
    offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
    buf = np.frombuffer(b"".join(frames), np.uint8).copy()
    return buf, offs, np.array([len(f) for f in frames], np.uint32)


def if_name(ifindex: int):
    for k, v in DOC["ifindex"].items():
        if v == ifindex:
            return k
    return None


def extract_events(text: str):
    """events.go extractEventsFromString with the reference's own regular expressions."""
    out = []
    rt = re.compile(DOC["event_regex"]["transport"])
    for m in rt.finditer(text):
        out.append({"InterfaceName": m.group("inf"), "SourceAddress": m.group("srcaddr"),
                    "DestinationAddress": m.group("dstaddr"), "Action": DOC["event_action"][m.group("action")],
                    "Protocol": DOC["event_protocol"][m.group("proto")], "DestinationPort": m.group("dstport"),
                    "IcmpType": 0, "IcmpCode": 0})
    ri = re.compile(DOC["event_regex"]["icmp"])
    for m in ri.finditer(text):
        out.append({"InterfaceName": m.group("inf"), "SourceAddress": m.group("srcaddr"),
                    "DestinationAddress": m.group("dstaddr"), "Action": DOC["event_action"][m.group("action")],
                    "Protocol": DOC["event_protocol"][m.group("proto")], "DestinationPort": "",
                    "IcmpType": int(m.group("type")), "IcmpCode": int(m.group("code"))})
    return out


def event_in_list(events, want) -> bool:
    """events.go isEventInList: every field equal."""
    return any(all(e[k] == want[k] for k in want) for e in events)
