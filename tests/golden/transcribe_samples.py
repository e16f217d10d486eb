"""Transcribe the reference's sample IngressNodeFirewall objects into tests/golden/ref_samples.json (run from
tests/golden/ in the build container, where /root/reference exists; the GPU box only reads the JSON).

Source: /root/reference/config/samples/ingressnodefirewall-demo-1.yaml, -demo-2.yaml, -demo-3.yaml (two objects),
-denyall.yaml — read as data with yaml.safe_load_all.  Each object's spec becomes {interfaces, ingress: [{source_cidrs,
rules}]} in the loader mirror's ProtocolRule form (a rule whose protocolConfig lacks the tcp/udp/sctp block keeps
ports None, exactly what the CR carries).  The node state is the operator's per-interface merge
(controllers/ingressnodefirewall_controller.go mergeRuleSet :371-405, restated as in transcribe.py).

The expectations are written here from the YAML and the reference's data path, not from the oracle:
  - kernel.c:222-258 (:306-340 for IPv6): the longest prefix's list only (no fallback to a shorter prefix), the first
    rule in slot order whose protocol matches, transport ports end-exclusive (dstPortStart <= p < dstPortEnd, or ==
    dstPortStart when dstPortEnd is 0), ICMP / ICMPv6 type and code both equal, a rule without protocol applies its
    action to every parsed packet; no match -> UNDEF (result word 0, XDP_PASS);
  - the key space is unified (BuildEBPFKey, loader.go:530-547): 0.0.0.0/0 and 0::0/0 are the same key {prefixLen 32,
    ifindex}, which covers IPv6 sources as well;
  - result word = ruleId << 8 | action (XDP_DROP 1 for Deny, XDP_PASS 2 for Allow), verdict = the action, else PASS.

demo-1 as written is not loadable: its last entry has a TCP rule without a tcp block.  The reference's admission
webhook refuses the object ("no port defined", pkg/webhook/webhook.go:285-299); without the webhook
makeIngressFwRulesMap would dereference the nil TCP block (pkg/ebpf/ingress_node_firewall_loader.go:441).  The fixture
records that (the loader mirror must refuse the whole sync and leave the map untouched) and adds "demo-1-admitted":
the same object with that rule given ports "1-65535", the smallest edit the webhook admits, to exercise its entries.
"""
import copy
import json

import yaml

SAMPLES = "/root/reference/config/samples"
IFINDEX = {"eth0": 2, "eth1": 3}
ALLOW, DENY = 2, 1


def rule_of(r):
    pc = r.get("protocolConfig") or {}
    proto = pc.get("protocol", "")
    out = {"order": r["order"], "protocol": proto, "ports": None, "icmp_type": 0, "icmp_code": 0,
           "action": r["action"]}
    blk = pc.get(proto.lower()) if proto else None
    if proto in ("TCP", "UDP", "SCTP") and blk is not None:
        out["ports"] = blk.get("ports")
    if proto in ("ICMP", "ICMPv6") and blk is not None:
        out["icmp_type"], out["icmp_code"] = blk.get("icmpType", 0), blk.get("icmpCode", 0)
    return out


def objects(fname):
    out = []
    for doc in yaml.safe_load_all(open(f"{SAMPLES}/{fname}")):
        if not doc:
            continue
        spec = doc["spec"]
        out.append({"name": doc["metadata"]["name"], "interfaces": spec["interfaces"],
                    "ingress": [{"source_cidrs": e["sourceCIDRs"], "rules": [rule_of(r) for r in e["rules"]]}
                                for e in spec["ingress"]]})
    return out


def merge_rule_set(a, b):  # mergeRuleSet + mergeFirewallProtocolRules (ingressnodefirewall_controller.go:371-425)
    for rb in b:
        for cidr in rb["source_cidrs"]:
            for ra in a:
                if ra["source_cidrs"][0] == cidr:
                    ra["rules"] = ra["rules"] + rb["rules"]
                    break
            else:
                a.append({"source_cidrs": [cidr], "rules": list(rb["rules"])})
    return a


def node_state(objs):
    st = {}
    for o in objs:
        for iface in o["interfaces"]:
            st[iface] = merge_rule_set(st.setdefault(iface, []), copy.deepcopy(o["ingress"]))
    return st


def probe(iface, src, proto, dport=0, icmp_type=0, icmp_code=0, rule=0, action=0, why=""):
    return {"interface": iface, "src": src, "protocol": proto, "dport": dport, "icmp_type": icmp_type,
            "icmp_code": icmp_code, "expect_result": (rule << 8 | action) if rule else 0,
            "expect_verdict": action if rule else ALLOW, "why": why}


demo1 = objects("ingressnodefirewall-demo-1.yaml")
demo1_admitted = copy.deepcopy(demo1)
bad = demo1_admitted[0]["ingress"][3]["rules"][0]
assert bad["protocol"] == "TCP" and bad["ports"] is None
bad["ports"] = "1-65535"

samples = [
    {"name": "demo-1", "file": "config/samples/ingressnodefirewall-demo-1.yaml", "objects": demo1,
     "loadable": False,
     "refusal": "ingress[3] rule order 10: protocol TCP without a tcp block — the webhook's 'no port defined' "
                "(pkg/webhook/webhook.go:285-299); makeIngressFwRulesMap would dereference the nil block "
                "(pkg/ebpf/ingress_node_firewall_loader.go:441)"},
    {"name": "demo-1-admitted", "file": "config/samples/ingressnodefirewall-demo-1.yaml",
     "edit": "ingress[3].rules[0] given ports '1-65535' (the webhook requires a tcp block)",
     "objects": demo1_admitted, "loadable": True,
     # 1.1.1.1/24, 100:1::1/64, 3.3.3.3/24, 10:10::1/64, and 0.0.0.0/0 + 0::0/0 as ONE key
     "expect_keys": [["eth0", "1.1.1.1/24"], ["eth0", "100:1::1/64"], ["eth0", "3.3.3.3/24"], ["eth0", "10:10::1/64"],
                     ["eth0", "0.0.0.0/0"]],
     "probes": [
         probe("eth0", "1.1.1.7", "tcp", 150, rule=10, action=ALLOW, why="TCP 100-200 Allow"),
         probe("eth0", "1.1.1.7", "tcp", 100, rule=10, action=ALLOW, why="range start inclusive"),
         probe("eth0", "1.1.1.7", "tcp", 199, rule=10, action=ALLOW, why="last port of the range"),
         probe("eth0", "1.1.1.7", "tcp", 200, why="range end exclusive (kernel.c:240)"),
         probe("eth0", "1.1.1.7", "udp", 8000, rule=20, action=ALLOW, why="UDP 8000 Allow"),
         probe("eth0", "1.1.1.7", "udp", 8001, why="exact port"),
         probe("eth0", "1.1.1.7", "tcp", 80, why="the /24's list only: no fallback to the /0 entry"),
         probe("eth0", "1.1.1.7", "icmp", icmp_type=3, icmp_code=1, why="no ICMP rule in the /24's list"),
         probe("eth0", "100:1::9", "tcp", 150, rule=10, action=ALLOW, why="IPv6 /64 of the same entry"),
         probe("eth0", "100:1::9", "udp", 8000, rule=20, action=ALLOW, why="IPv6 /64 UDP"),
         probe("eth0", "100:1::9", "sctp", 150, why="no SCTP rule"),
         probe("eth0", "3.3.3.9", "icmp", icmp_type=3, icmp_code=1, rule=10, action=ALLOW, why="ICMP 3/1 Allow"),
         probe("eth0", "3.3.3.9", "icmp", icmp_type=3, icmp_code=0, why="type and code must both match"),
         probe("eth0", "3.3.3.9", "icmp", icmp_type=8, icmp_code=0, why="echo request: no rule"),
         probe("eth0", "3.3.3.9", "tcp", 80, why="the /24's list holds only the ICMP rule"),
         probe("eth0", "10:10::5", "icmpv6", icmp_type=128, icmp_code=0, rule=10, action=DENY, why="ICMPv6 128 Deny"),
         probe("eth0", "10:10::5", "icmpv6", icmp_type=129, icmp_code=0, why="echo reply: no rule"),
         probe("eth0", "10:10::5", "tcp", 443, why="the /64's list holds only the ICMPv6 rule"),
         probe("eth0", "8.8.8.8", "tcp", 443, rule=10, action=ALLOW, why="0.0.0.0/0 TCP 1-65535 Allow"),
         probe("eth0", "8.8.8.8", "tcp", 65535, why="end exclusive at 65535"),
         probe("eth0", "8.8.8.8", "udp", 53, why="the /0 list is TCP only"),
         probe("eth0", "2001:db8::1", "tcp", 22, rule=10, action=ALLOW, why="::/0 is the same key as 0.0.0.0/0"),
         probe("eth0", "2001:db8::1", "icmpv6", icmp_type=128, why="::/0 list is TCP only"),
         probe("eth1", "1.1.1.7", "tcp", 150, why="no entries on eth1"),
         probe("eth1", "10:10::5", "icmpv6", icmp_type=128, why="no entries on eth1"),
     ]},
    {"name": "demo-2", "file": "config/samples/ingressnodefirewall-demo-2.yaml",
     "objects": objects("ingressnodefirewall-demo-2.yaml"), "loadable": True,
     "expect_keys": [["eth0", "172.16.0.0/12"], ["eth0", "fc00:f853:ccd:e793::0/64"]],
     "probes": [
         probe("eth0", "172.16.5.5", "icmp", icmp_type=8, icmp_code=0, rule=10, action=DENY, why="echo request Deny"),
         probe("eth0", "172.31.255.254", "icmp", icmp_type=8, icmp_code=1, why="icmpCode 0 only"),
         probe("eth0", "172.20.1.1", "tcp", 8000, rule=20, action=DENY, why="TCP 8000-9000 Deny"),
         probe("eth0", "172.20.1.1", "tcp", 8999, rule=20, action=DENY, why="last port of the range"),
         probe("eth0", "172.20.1.1", "tcp", 9000, why="end exclusive"),
         probe("eth0", "172.20.1.1", "udp", 8500, why="TCP only"),
         probe("eth0", "172.32.0.1", "icmp", icmp_type=8, why="outside the /12"),
         probe("eth0", "fc00:f853:ccd:e793::42", "icmpv6", icmp_type=128, rule=10, action=DENY, why="ICMPv6 Deny"),
         probe("eth0", "fc00:f853:ccd:e793::42", "icmp", icmp_type=8, why="ICMP (proto 1) on IPv6: no rule"),
         probe("eth0", "fc00:f853:ccd:e794::42", "icmpv6", icmp_type=128, why="outside the /64"),
     ]},
    {"name": "demo-3", "file": "config/samples/ingressnodefirewall-demo-3.yaml",
     "objects": objects("ingressnodefirewall-demo-3.yaml"), "loadable": True,
     "expect_keys": [["eth0", "172.20.0.0/24"], ["eth1", "172.20.0.0/24"]],
     "probes": [
         probe("eth0", "172.20.0.9", "icmp", icmp_type=8, rule=10, action=DENY, why="demo-3-a on eth0"),
         probe("eth0", "172.20.0.9", "tcp", 8080, rule=20, action=DENY, why="demo-3-a TCP range"),
         probe("eth1", "172.20.0.9", "icmp", icmp_type=8, why="demo-3-b on eth1 has no ICMP rule"),
         probe("eth1", "172.20.0.9", "tcp", 8080, rule=20, action=DENY, why="demo-3-b TCP range"),
         probe("eth1", "172.20.1.9", "tcp", 8080, why="outside the /24"),
     ]},
    {"name": "denyall", "file": "config/samples/ingressnodefirewall-demo-denyall.yaml",
     "objects": objects("ingressnodefirewall-demo-denyall.yaml"), "loadable": True,
     "expect_keys": [["eth0", "0.0.0.0/0"]],
     "probes": [
         probe("eth0", "8.8.8.8", "tcp", 443, rule=20, action=DENY, why="a rule without protocol matches every packet"),
         probe("eth0", "8.8.8.8", "udp", 53, rule=20, action=DENY, why="any protocol"),
         probe("eth0", "8.8.8.8", "sctp", 9, rule=20, action=DENY, why="any protocol"),
         probe("eth0", "8.8.8.8", "icmp", icmp_type=0, rule=20, action=DENY, why="any protocol"),
         probe("eth0", "2001:db8::7", "tcp", 22, rule=20, action=DENY,
               why="the 0.0.0.0/0 key {32, ifindex} covers IPv6 sources too (unified key space)"),
         probe("eth0", "2001:db8::7", "icmpv6", icmp_type=128, rule=20, action=DENY, why="IPv6 ICMPv6"),
         probe("eth0", "8.8.8.8", "gre", why="unknown L4 protocol: UNDEF before the lookup (kernel.c:117-172)"),
         probe("eth1", "8.8.8.8", "tcp", 443, why="eth1 has no entries"),
     ]},
]
for s in samples:
    s["node_state"] = node_state(s["objects"])

json.dump({"source": "pbmoses/ingress-node-firewall config/samples/*.yaml, transcribed by "
                     "tests/golden/transcribe_samples.py (expectations written from the YAML and kernel.c)",
           "ifindex": IFINDEX, "samples": samples}, open("ref_samples.json", "w"), indent=1)
print(f"wrote ref_samples.json: {len(samples)} samples, {sum(len(s.get('probes', [])) for s in samples)} probes")
