"""Transcribes reference test cases and survey probe records into this directory's JSON fixtures.

Sources (pbmoses/ingress-node-firewall @ 2025-01-14, read as text):
  pkg/ebpfsyncer/ebpfsyncer_test.go:41-445   TestSyncInterfaceIngressRulesWithHTTP  -> ref_ebpfsyncer_http.json
  pkg/ebpfsyncer/ebpfsyncer_test.go:727-987  TestVerifyBPFKeysAfter...Update         -> ref_ebpfsyncer_keys.json
  pkg/ebpf/ingress_node_firewall_loader_test.go:19-89  TestAddOrUpdateRules          -> ref_loader_keys.json
  SURVEY.md [probe] records (reference XDP object under BPF_PROG_TEST_RUN)          -> survey_probes.json
Run: python transcribe.py   (deterministic; rewrites the JSON files)
"""
import json

P1, P2 = "12345", "12346"   # ebpfsyncer_test.go:29-30


def tcp(order, port, action):
    return {"order": order, "protocol": "TCP", "ports": port, "action": action}


def ent(cidr, rules):
    return {"source_cidrs": [cidr], "rules": rules}


NO = {"192.0.2.1:12345": True, "192.0.2.1:12346": True, "192.0.2.5:12345": True, "192.0.2.5:12346": True}
tcs = [
    {"name": "TC0 reset back to no rules", "rules": None, "isDelete": False, "targetResult": NO},
    {"name": "TC1 single rule and default drop", "rules": {"dummy0": [ent("192.0.2.0/24", [tcp(10, P1, "Deny")])]},
     "isDelete": False, "targetResult": {"192.0.2.1:12345": False, "192.0.2.1:12346": True, "192.0.2.5:12345": True,
                                         "192.0.2.5:12346": True}},
    {"name": "TC2 open another port",
     "rules": {"dummy0": [ent("192.0.2.0/24", [tcp(10, P1, "Deny"), tcp(20, P2, "Allow")])]}, "isDelete": False,
     "targetResult": {"192.0.2.1:12345": False, "192.0.2.1:12346": True, "192.0.2.5:12345": True,
                      "192.0.2.5:12346": True}},
    {"name": "TC3 reset back to no rules", "rules": None, "isDelete": False, "targetResult": NO},
    {"name": "TC4 open both ports on dummy0",
     "rules": {"dummy0": [ent("192.0.2.0/24", [tcp(10, P1, "Allow"), tcp(20, P2, "Allow")])]}, "isDelete": False,
     "targetResult": NO},
    {"name": "TC5 reset back to no rules", "rules": None, "isDelete": False, "targetResult": NO},
    {"name": "TC5b /24 on dummy0 and dummy1", "rules": {
        "dummy0": [ent("192.0.2.0/24", [tcp(10, P1, "Deny"), tcp(20, P2, "Allow")])],
        "dummy1": [ent("192.0.2.0/24", [tcp(10, P1, "Allow"), tcp(20, P2, "Deny")])]}, "isDelete": False,
     "targetResult": {"192.0.2.1:12345": False, "192.0.2.1:12346": True, "192.0.2.5:12345": True,
                      "192.0.2.5:12346": False}},
    {"name": "TC6 delete object", "rules": None, "isDelete": True, "targetResult": NO},
    {"name": "TC7 no rules", "rules": None, "isDelete": False, "targetResult": NO},
    {"name": "TC8 /30 per interface", "rules": {
        "dummy0": [ent("192.0.2.0/30", [tcp(10, P1, "Deny"), tcp(20, P2, "Allow")])],
        "dummy1": [ent("192.0.2.4/30", [tcp(10, P1, "Allow"), tcp(20, P2, "Deny")])]}, "isDelete": False,
     "targetResult": {"192.0.2.1:12345": False, "192.0.2.1:12346": True, "192.0.2.5:12345": True,
                      "192.0.2.5:12346": False}},
    {"name": "TC9 /30 per interface swapped", "rules": {
        "dummy0": [ent("192.0.2.0/30", [tcp(10, P1, "Allow"), tcp(20, P2, "Deny")])],
        "dummy1": [ent("192.0.2.4/30", [tcp(10, P1, "Deny"), tcp(20, P2, "Allow")])]}, "isDelete": False,
     "targetResult": {"192.0.2.1:12345": True, "192.0.2.1:12346": False, "192.0.2.5:12345": False,
                      "192.0.2.5:12346": True}},
]
json.dump({
    "source": "pbmoses/ingress-node-firewall pkg/ebpfsyncer/ebpfsyncer_test.go:41-445 "
              "(TestSyncInterfaceIngressRulesWithHTTP), transcribed",
    "topology": "veth dummy{i} in the root netns holds 192.0.2.{4i+1}/30, its peer in netns 'dummy' 192.0.2.{4i+2}/30 "
                "(ebpfsyncer_test.go:1236-1317); connecting to 192.0.2.{4i+1}:port sends TCP SYNs from 192.0.2.{4i+2} "
                "that arrive on dummy{i}, where the XDP program runs. targetResult true = the connection succeeds = "
                "the SYN gets XDP_PASS; false = XDP_DROP.",
    "ifindex": {"dummy0": 10, "dummy1": 11, "dummy2": 12},
    "ifindex_note": "the test resolves real ifindexes at run time; any distinct values stand in",
    "test_cases": tcs}, open("ref_ebpfsyncer_http.json", "w"), indent=1)

ktcs = [
    {"name": "TC0 2 CIDRs same interface", "isDelete": False,
     "rules": {"dummy0": [ent("10.0.0.0/8", [tcp(10, P1, "Allow")]), ent("0.0.0.0/0", [tcp(10, P1, "Deny")])]},
     "expectedKeys": [["dummy0", "10.0.0.0/8"], ["dummy0", "0.0.0.0/0"]]},
    {"name": "TC1 delete", "isDelete": True, "rules": None, "expectedKeys": []},
    {"name": "TC2 all rules to interface 1", "isDelete": False,
     "rules": {"dummy1": [ent("10.0.0.0/8", [tcp(10, P1, "Allow")]), ent("0.0.0.0/0", [tcp(10, P1, "Deny")])]},
     "expectedKeys": [["dummy1", "10.0.0.0/8"], ["dummy1", "0.0.0.0/0"]]},
    {"name": "TC3 remove default", "isDelete": False, "rules": {"dummy1": [ent("10.0.0.0/8", [tcp(10, P1, "Allow")])]},
     "expectedKeys": [["dummy1", "10.0.0.0/8"]]},
    {"name": "TC4 move to interface 0 with 2 CIDRs", "isDelete": False,
     "rules": {"dummy0": [{"source_cidrs": ["10.0.0.0/8", "0.0.0.0/0"], "rules": [tcp(10, P1, "Allow")]}]},
     "expectedKeys": [["dummy0", "10.0.0.0/8"], ["dummy0", "0.0.0.0/0"]]},
    {"name": "TC5 empty", "isDelete": False, "rules": {}, "expectedKeys": []},
    {"name": "TC6 same CIDR on 2 interfaces", "isDelete": False,
     "rules": {"dummy0": [ent("10.0.0.0/8", [tcp(10, P1, "Deny"), tcp(20, P2, "Allow")])],
               "dummy1": [ent("10.0.0.0/8", [tcp(10, P1, "Allow"), tcp(20, P2, "Deny")])]},
     "expectedKeys": [["dummy0", "10.0.0.0/8"], ["dummy1", "10.0.0.0/8"]]},
]
json.dump({"source": "pkg/ebpfsyncer/ebpfsyncer_test.go:727-987 (TestVerifyBPFKeysAfterInterfaceIngressRulesUpdate), "
                     "transcribed; expected keys are BuildEBPFKey(ifindex(iface), cidr)",
           "ifindex": {"dummy0": 10, "dummy1": 11}, "test_cases": ktcs}, open("ref_ebpfsyncer_keys.json", "w"), indent=1)

json.dump({"source": "pkg/ebpf/ingress_node_firewall_loader_test.go:19-89 (TestAddOrUpdateRules), transcribed",
           "test_cases": [
               {"keys": [[100, "10.0.0.0/8"], [100, "192.0.2.0/24"]], "rule": {"ruleId": 10, "action": 1},
                "expected_n_keys": 2},
               {"keys": [[100, "10.0.0.0/8"], [100, "10.0.0.0/16"]], "rule": {"ruleId": 10, "action": 1},
                "expected_n_keys": 2},
               {"keys": [[100, "10.0.0.0/8"], [101, "10.0.0.0/8"]], "rule": {"ruleId": 10, "action": 1},
                "expected_n_keys": 2}]},
          open("ref_loader_keys.json", "w"), indent=1)

# --- SURVEY.md [probe] observations: the reference's own XDP object run under
# BPF_PROG_TEST_RUN by the survey.  Each case
# restates the observed table, packet and outcome (retval + per-rule counter
# change).  "derived" fields follow from kernel.c source, not from a probe.
def rule(slot, rid, proto, ps=0, pe=0, it=0, ic=0, action=2):
    return {"slot": slot, "ruleId": rid, "protocol": proto, "dstPortStart": ps, "dstPortEnd": pe,
            "icmpType": it, "icmpCode": ic, "action": action}
def key(ifx, cidr): return {"ifindex": ifx, "cidr": cidr}
probes = [
 {"name": "ipv6 packet hits the IPv4 entry 10.0.0.0/8 (unified key space)", "cite": "SURVEY.md §0 finding 2 [probe]",
  "table": [{"key": key(1, "10.0.0.0/8"), "rules": [rule(5, 5, 0, action=1)]}],
  "packets": [{"src": "a00::1", "proto": "tcp", "dport": 80, "ifindex": 1, "expect": {"retval": 1, "stats": [[5, "deny"]]}}]},
 {"name": "0101:0100::1 hits 1.1.1.0/24", "cite": "SURVEY.md §0 finding 2 [probe]",
  "table": [{"key": key(1, "1.1.1.0/24"), "rules": [rule(10, 10, 6, 100, 200, action=2)]}],
  "packets": [{"src": "101:100::1", "proto": "tcp", "dport": 150, "ifindex": 1, "expect": {"retval": 2, "stats": [[10, "allow"]]}}]},
 {"name": "port range is end-exclusive", "cite": "SURVEY.md §0 finding 3 [probe]; kernel.c:241",
  "table": [{"key": key(1, "1.1.1.0/24"), "rules": [rule(10, 10, 6, 100, 200, action=2)]}],
  "packets": [{"src": "1.1.1.7", "proto": "tcp", "dport": 200, "ifindex": 1, "expect": {"retval": 2, "stats": []}},
              {"src": "1.1.1.7", "proto": "tcp", "dport": 199, "ifindex": 1, "expect": {"retval": 2, "stats": [[10, "allow"]]}},
              {"src": "1.1.1.7", "proto": "tcp", "dport": 100, "ifindex": 1, "expect": {"retval": 2, "stats": [[10, "allow"]]}},
              {"src": "1.1.1.7", "proto": "tcp", "dport": 99, "ifindex": 1, "expect": {"retval": 2, "stats": []}}]},
 {"name": "no fallback from a /32 to its /24 when no rule of the /32 matches", "cite": "SURVEY.md §0 finding 4 [probe]",
  "table": [{"key": key(1, "7.7.7.0/24"), "rules": [rule(1, 1, 0, action=1)]},
            {"key": key(1, "7.7.7.7/32"), "rules": [rule(2, 2, 17, 53, 0, action=2)]}],
  "packets": [{"src": "7.7.7.7", "proto": "tcp", "dport": 80, "ifindex": 1, "expect": {"retval": 2, "stats": []}},
              {"src": "7.7.7.8", "proto": "tcp", "dport": 80, "ifindex": 1, "expect": {"retval": 1, "stats": [[1, "deny"]]}},
              {"src": "7.7.7.7", "proto": "udp", "dport": 53, "ifindex": 1, "expect": {"retval": 2, "stats": [[2, "allow"]]}}]},
 {"name": "statistics only for keys < 1024", "cite": "SURVEY.md Appendix A.6 [probe]; kernel.c:40,376",
  "table": [{"key": key(1, "9.9.9.0/24"), "rules": [rule(1, 1024, 0, action=1)]}],
  "packets": [{"src": "9.9.9.9", "proto": "udp", "dport": 1, "ifindex": 1, "expect": {"retval": 1, "stats": []}}]},
 {"name": "rule id truncated to u16 for the stats key (derived: ingress_node_firewall.h:20)", "cite": "ingress_node_firewall.h:20, kernel.c:441",
  "table": [{"key": key(1, "9.9.8.0/24"), "rules": [rule(1, 65537, 0, action=2)]}],
  "packets": [{"src": "9.9.8.1", "proto": "udp", "dport": 1, "ifindex": 1, "expect": {"retval": 2, "stats": [[1, "allow"]]}}]},
 {"name": "non-IP ethertypes pass without lookup (ARP, VLAN)", "cite": "SURVEY.md Appendix A.1 [probe]; kernel.c:436-438",
  "table": [{"key": key(1, "0.0.0.0/0"), "rules": [rule(1, 1, 0, action=1)]}],
  "packets": [{"src": "1.2.3.4", "proto": "tcp", "dport": 80, "ifindex": 1, "ethertype": 2054, "expect": {"retval": 2, "stats": []}},
              {"src": "1.2.3.4", "proto": "tcp", "dport": 80, "ifindex": 1, "ethertype": 33024, "expect": {"retval": 2, "stats": []}},
              {"src": "1.2.3.4", "proto": "tcp", "dport": 80, "ifindex": 1, "expect": {"retval": 1, "stats": [[1, "deny"]]}}]},
 {"name": "IPv4 IHL is ignored: L4 read at fixed offset 34", "cite": "SURVEY.md Appendix A.3 [probe]; kernel.c:104",
  "table": [{"key": key(1, "5.5.5.0/24"), "rules": [rule(3, 3, 6, 0, 0, action=1)]}],
  "packets": [{"src": "5.5.5.5", "proto": "tcp", "dport": 443, "ifindex": 1, "ihl": 6, "expect": {"retval": 1, "stats": [[3, "deny"]]},
               "note": "with IHL=6 the 4 option bytes sit at offset 34, so the program reads dport 0 from the options (exact port 0 rule matches)"}]},
 {"name": "truncated L4 header: UNDEF, pass, no stats", "cite": "SURVEY.md Appendix A.3 [probe]; kernel.c:121-124",
  "table": [{"key": key(1, "0.0.0.0/0"), "rules": [rule(1, 1, 0, action=1)]}],
  "packets": [{"src": "1.2.3.4", "proto": "tcp", "dport": 80, "ifindex": 1, "truncate": 53, "expect": {"retval": 2, "stats": []}},
              {"src": "1.2.3.4", "proto": "tcp", "dport": 80, "ifindex": 1, "truncate": 54, "expect": {"retval": 1, "stats": [[1, "deny"]]}},
              {"src": "1.2.3.4", "proto": "udp", "dport": 80, "ifindex": 1, "truncate": 41, "expect": {"retval": 2, "stats": []}},
              {"src": "2001:db8::5", "proto": "icmpv6", "ifindex": 1, "truncate": 61, "expect": {"retval": 2, "stats": []}},
              {"src": "1.2.3.4", "proto": "gre", "ifindex": 1, "expect": {"retval": 2, "stats": []}}]},
 {"name": "ICMP/ICMPv6 rules are family-gated", "cite": "SURVEY.md Appendix A.4 [probe]; kernel.c:247,329",
  "table": [{"key": key(1, "0.0.0.0/0"), "rules": [rule(1, 1, 58, it=128, ic=0, action=1), rule(2, 2, 1, it=8, ic=0, action=1)]}],
  "packets": [{"src": "1.2.3.4", "proto": 58, "icmp_type": 128, "ifindex": 1, "expect": {"retval": 2, "stats": []}},
              {"src": "::1.2.3.4", "proto": 1, "icmp_type": 8, "ifindex": 1, "expect": {"retval": 2, "stats": []}},
              {"src": "1.2.3.4", "proto": "icmp", "icmp_type": 8, "ifindex": 1, "expect": {"retval": 1, "stats": [[2, "deny"]]}},
              {"src": "::1.2.3.4", "proto": "icmpv6", "icmp_type": 128, "ifindex": 1, "expect": {"retval": 1, "stats": [[1, "deny"]]}},
              {"src": "::1.2.3.4", "proto": "icmpv6", "icmp_type": 128, "icmp_code": 1, "ifindex": 1, "expect": {"retval": 2, "stats": []}}]},
 {"name": "first match with an action outside {1,2} stops the scan: pass, no stats", "cite": "SURVEY.md Appendix A.4 [probe]; kernel.c:444-456",
  "table": [{"key": key(1, "4.4.4.0/24"), "rules": [rule(1, 1, 0, action=7), rule(2, 2, 0, action=1)]}],
  "packets": [{"src": "4.4.4.4", "proto": "udp", "dport": 9, "ifindex": 1, "expect": {"retval": 2, "stats": [], "result": 263}}]},
 {"name": "slots with ruleId 0 are skipped; a miss on another ifindex", "cite": "kernel.c:225-227; SURVEY.md Appendix A.2",
  "table": [{"key": key(1, "8.8.0.0/16"), "rules": [rule(0, 0, 0, action=1), rule(4, 4, 17, 53, 0, action=2)]}],
  "packets": [{"src": "8.8.8.8", "proto": "udp", "dport": 53, "ifindex": 1, "expect": {"retval": 2, "stats": [[4, "allow"]]}},
              {"src": "8.8.8.8", "proto": "udp", "dport": 53, "ifindex": 2, "expect": {"retval": 2, "stats": []}}]},
 {"name": "identical-key v4 0.0.0.0/0 and v6 ::/0: one entry, last writer wins", "cite": "SURVEY.md §0 finding 2, Appendix A.2",
  "table": [{"key": key(3, "0.0.0.0/0"), "rules": [rule(1, 1, 0, action=1)]},
            {"key": key(3, "::/0"), "rules": [rule(2, 2, 0, action=2)]}],
  "expect_entries": 1,
  "packets": [{"src": "1.2.3.4", "proto": "tcp", "dport": 1, "ifindex": 3, "expect": {"retval": 2, "stats": [[2, "allow"]]}},
              {"src": "2001::1", "proto": "tcp", "dport": 1, "ifindex": 3, "expect": {"retval": 2, "stats": [[2, "allow"]]}}]},
 {"name": "IPv4-mapped CIDR keeps 4 bytes and a 128-bit mask length", "cite": "loader.go:537-544; SURVEY.md Appendix A.2",
  "table": [{"key": key(1, "::ffff:6.6.6.0/120"), "rules": [rule(9, 9, 0, action=1)]}],
  "packets": [{"src": "6.6.6.1", "proto": "tcp", "dport": 1, "ifindex": 1, "expect": {"retval": 2, "stats": []}},
              {"src": "606:600::", "proto": "tcp", "dport": 1, "ifindex": 1, "expect": {"retval": 1, "stats": [[9, "deny"]]}}]},
]
json.dump({"source": "SURVEY.md [probe] observations of the reference XDP object under BPF_PROG_TEST_RUN, restated; "
           "cases marked derived follow from the cited source lines", "frame_len_default": 0,
           "cases": probes}, open("survey_probes.json", "w"), indent=1)

# --- test/e2e/functional/tests/e2e.go:176-831: the reference's behavioural table.  Each entry's INF objects are
# generated the way the harness does it (e2e.go:879-945: source CIDRs = each pod's IP /32 and /128, rule orders
# from nextSourceCIDRsOrder), merged into the node's InterfaceIngressRules as the operator does
# (controllers/ingressnodefirewall_controller.go:329-347 mergeRuleSet :371-405, mergeFirewallProtocolRules
# :409-425), and the expected connectivity comes from the entry's `reachables` (connectivity false after the
# policy, e2e.go:971-975; true before it, :872-876), per protocol and family as reachabilityCheck (:1535-1621)
# checks it: IPv4 for every protocol but ICMPv6, IPv6 (dual stack) for every protocol but ICMP, ICMP echo
# requests type 8 / 128 code 0, transport connections to the reachable's port.  The deny events each blocked
# connection must produce are GetTransportTestEvent / GetICMPTestEvent (test/e2e/events/events.go), matched by the
# reference's own syslog regular expressions (events.go extractEventsFromString), copied here as data.
# Assumptions, stated: a dual-stack cluster with ENABLE_SCTP=true (e2e.go:111-116, :158-164); the pod IPs, the
# node interface's ifindex and the ephemeral source ports are synthetic (the cluster assigns them at run time).
POD_IPS = {  # synthetic pod IPs (KinD's default dual-stack pod CIDRs 10.244.0.0/16, fd00:10:244::/56)
    "e2e-inf-client-one": ("10.244.1.11", "fd00:10:244:1::b"), "e2e-inf-client-two": ("10.244.1.12", "fd00:10:244:1::c"),
    "e2e-inf-client-three": ("10.244.1.13", "fd00:10:244:1::d"), "e2e-inf-client-four": ("10.244.1.14", "fd00:10:244:1::e"),
    "e2e-inf-server-one": ("10.244.2.21", "fd00:10:244:2::15"), "e2e-inf-server-two": ("10.244.2.22", "fd00:10:244:2::16"),
}
C1, C2, C3, C4 = "e2e-inf-client-one", "e2e-inf-client-two", "e2e-inf-client-three", "e2e-inf-client-four"
S1, S2 = "e2e-inf-server-one", "e2e-inf-server-two"
SERVER_ONE_PORT, ALLOWED_PORT, SERVER_TWO_PORT, SERVER_ONE_RANGE = "80", "40000", "8080", "79-81"  # e2e.go:137-140
TRANSPORT = ["TCP", "UDP", "SCTP"]     # e2e.go:154, :158-160 (SCTP with ENABLE_SCTP)
ICMPS = ["ICMP", "ICMPv6"]             # e2e.go:155, :162-164 (ICMPv6 when not single stack)


def block_port(port):                  # infwutils.GetTransportProtocolBlockPortRule (ingress-node-firewall.go:208-219)
    return lambda proto, order: {"order": order, "protocol": proto, "ports": port, "action": "Deny"}


def block_echo(proto, order):          # the e2e entries' ICMP closures + GetICMPBlockRule (:221-250)
    return {"order": order, "protocol": proto, "icmp_type": 8 if proto == "ICMP" else 128, "icmp_code": 0,
            "action": "Deny"}


def block_port_or_echo(port):          # e2e.go:448-462: transport -> block port, ICMP -> block echo request
    return lambda proto, order: (block_port(port)(proto, order) if proto in TRANSPORT else block_echo(proto, order))


E2E = [  # (it, e2e.go line, testINFs [(interfaces, [(pods, protoRules)])], reachables [(src, dst, port)], protocols)
    ("block a port with a single rule defining the destinations port", 191,
     [(["eth0"], [([C1], [block_port(SERVER_ONE_PORT)])])], [(C1, S1, SERVER_ONE_PORT)], TRANSPORT),
    ("block a port using a range when multiple source CIDRs exist", 228,
     [(["eth0"], [([C1, C2], [block_port(SERVER_ONE_RANGE)])])], [(C1, S1, SERVER_ONE_PORT), (C2, S1, SERVER_ONE_PORT)],
     TRANSPORT),
    ("block multiple ports", 275,
     [(["eth0"], [([C1], [block_port(SERVER_ONE_PORT), block_port(SERVER_TWO_PORT)])])],
     [(C1, S1, SERVER_ONE_PORT), (C1, S2, SERVER_TWO_PORT)], TRANSPORT),
    ("block port when rules for a source CIDR are located in multiple IngressNodeFirewall objects", 325,
     [(["eth0"], [([C1], [block_port(ALLOWED_PORT)])]), (["eth0"], [([C1], [block_port(SERVER_ONE_PORT)])])],
     [(C1, S1, SERVER_ONE_PORT)], TRANSPORT),
    ("merges transport protocol rules when source CIDRs overlap in multiple IngressNodeFirewalls and the count of "
     "source CIDRs for each policy is different", 375,
     [(["eth0"], [([C1], [block_port(ALLOWED_PORT)])]), (["eth0"], [([C1, C2], [block_port(SERVER_ONE_PORT)])])],
     [(C1, S1, SERVER_ONE_PORT), (C2, S1, SERVER_ONE_PORT)], TRANSPORT),
    ("merges multiple IngressNodeFirewalls which contain multiple ingress entries with protocol rules for all "
     "protocols", 440,
     [(["eth0"], [([C1], [block_port_or_echo(SERVER_ONE_PORT)]), ([C2], [block_port_or_echo(SERVER_ONE_PORT)])]),
      (["eth0"], [([C3], [block_port_or_echo(SERVER_ONE_PORT)]), ([C4], [block_port_or_echo(SERVER_ONE_PORT)])])],
     [(C1, S1, SERVER_ONE_PORT), (C2, S1, SERVER_ONE_PORT), (C3, S1, SERVER_ONE_PORT), (C4, S1, SERVER_ONE_PORT)],
     TRANSPORT + ICMPS),
    ("block port when rules for a source CIDR are located in multiple IngressNodeFirewall objects (2)", 585,
     [(["eth0"], [([C1], [block_port(ALLOWED_PORT)])]), (["eth0"], [([C1], [block_port(SERVER_ONE_PORT)])])],
     [(C1, S1, SERVER_ONE_PORT)], TRANSPORT),
    ("merges transport protocol rules when source CIDRs overlap in multiple IngressNodeFirewalls but the number of "
     "source CIDRs in each policy is different", 635,
     [(["eth0"], [([C1], [block_port(ALLOWED_PORT)])]), (["eth0"], [([C1, C2], [block_port(SERVER_ONE_PORT)])])],
     [(C1, S1, SERVER_ONE_PORT), (C2, S1, SERVER_ONE_PORT)], TRANSPORT),
    ("block ICMP echo request", 697, [(["eth0"], [([C1], [block_echo])])], [(C1, S1, SERVER_ONE_PORT)], ICMPS),
    ("non existent interface name doesn't block application of IngressNodeFirewall policy for valid interface", 744,
     [(["doesntexist", "eth0"], [([C1], [block_port(SERVER_ONE_PORT)])])], [(C1, S1, SERVER_ONE_PORT)], ["TCP"]),
    ("non existent interface name in unrelated IngressNodeFirewall doesn't block application of new "
     "IngressNodeFirewalls policies", 781,
     [(["doesntexist"], [([C1], [block_port(ALLOWED_PORT)])]), (["eth0"], [([C1], [block_port(SERVER_ONE_PORT)])])],
     [(C1, S1, SERVER_ONE_PORT)], ["TCP"]),
]


def harness_infs(test_infs, protocols):
    """e2e.go:879-945: INF objects from the templates; orders continue per source CIDR across objects."""
    next_order = {}
    infs = []
    for interfaces, test_rules in test_infs:
        ingress = []
        for pods, proto_fns in test_rules:
            cidrs = []
            for pod in pods:
                for ip, bits in ((POD_IPS[pod][0], 32), (POD_IPS[pod][1], 128)):   # v4SubnetLen / v6SubnetLen
                    c = f"{ip}/{bits}"           # already canonical, so net.ParseCIDR's cidr.String() is the same text
                    next_order.setdefault(c, 1)
                    cidrs.append(c)
            order = max([0] + [next_order[c] for c in cidrs])
            rules = []
            for proto in protocols:
                for fn in proto_fns:
                    rules.append(fn(proto, order))
                    order += 1
            for c in cidrs:
                next_order[c] = order
            ingress.append({"source_cidrs": cidrs, "rules": rules})
        infs.append({"interfaces": interfaces, "ingress": ingress})
    return infs


def merge_rule_set(a, b):
    """mergeRuleSet (controllers/ingressnodefirewall_controller.go:371-405) + mergeFirewallProtocolRules (:409-425)."""
    for rb in b:
        for cidr in rb["source_cidrs"]:
            for ra in a:
                if ra["source_cidrs"][0] == cidr:
                    orders = [r["order"] for r in ra["rules"]]
                    for r in rb["rules"]:
                        assert r["order"] not in orders, "duplicate order: the operator reports a sync error"
                        orders.append(r["order"])
                    ra["rules"] = ra["rules"] + rb["rules"]
                    break
            else:
                a.append({"source_cidrs": [cidr], "rules": list(rb["rules"])})
    return a


def node_state(infs):
    """buildNodeStates (:267-350) for one node: every INF's ingress merged per interface, in object order."""
    st = {}
    for inf in infs:
        for iface in inf["interfaces"]:
            st[iface] = merge_rule_set(st.setdefault(iface, []), inf["ingress"])
    return st


def connections(reachables, protocols):
    """reachabilityCheck (e2e.go:1535-1621): the packets one check sends, with the drop event it expects."""
    out = []
    for src, dst, port in reachables:
        for proto in protocols:
            for fam in (4, 6):
                if (fam == 4 and proto == "ICMPv6") or (fam == 6 and proto == "ICMP"):
                    continue
                s, d = POD_IPS[src][fam == 6], POD_IPS[dst][fam == 6]
                c = {"src": s, "dst": d, "family": fam, "protocol": proto, "interface": "eth0",
                     "event": {"InterfaceName": "eth0", "SourceAddress": s, "DestinationAddress": d, "Action": "Deny",
                               "Protocol": proto}}
                if proto in TRANSPORT:
                    c["dport"] = int(port)
                    c["event"].update(DestinationPort=port, IcmpType=0, IcmpCode=0)
                else:  # GetICMPTestEvent(proto, inf, src, dst, 0, 8 | 128): icmpCode 0, icmpType 8 / 128
                    c["icmp_type"], c["icmp_code"] = (8 if fam == 4 else 128), 0
                    c["event"].update(DestinationPort="", IcmpType=c["icmp_type"], IcmpCode=0)
                out.append(c)
    return out


e2e_cases = []
for it, line, tinfs, reach, protos in E2E:
    infs = harness_infs(tinfs, protos)
    e2e_cases.append({"it": it, "cite": f"test/e2e/functional/tests/e2e.go:{line}", "protocols": protos,
                      "infs": infs, "interface_ingress_rules": node_state(json.loads(json.dumps(infs))),
                      "connections": connections(reach, protos),
                      "expect_before_policy": "reachable (XDP_PASS)", "expect_after_policy": "blocked (XDP_DROP)"})
json.dump({
    "source": "pbmoses/ingress-node-firewall test/e2e/functional/tests/e2e.go:176-831 (the IngressNodeFirewall table), "
              ":1205-1352 (daemon metrics) and test/e2e/events/events.go (expected drop events), transcribed by "
              "tests/golden/transcribe.py",
    "assumptions": "dual-stack cluster, ENABLE_SCTP=true; synthetic pod IPs; the node interface eth0 has ifindex 2 and "
                   "'doesntexist' is not a valid interface (loader.go:143-146 skips it); ephemeral source port 40000",
    "ifindex": {"eth0": 2},
    "event_regex": {  # events.go extractEventsFromString: the syslog lines a drop must produce
        "transport": "ruleId\\s([0-9]+)\\saction\\s(?P<action>\\w+).*if\\s(?P<inf>\\w+)\n.*\\ssrc\\saddr\\s"
                     "(?P<srcaddr>[0-9.:a-z]+)\\sdst\\saddr\\s(?P<dstaddr>[0-9.:a-z]+)\n.*(?P<proto>tcp|udp|sctp)"
                     "\\ssrcPort\\s\\d+\\sdstPort\\s(?P<dstport>\\d+)",
        "icmp": "ruleId\\s([0-9]+)\\saction\\s(?P<action>\\w+).*if\\s(?P<inf>\\w+)\\n.*\\s(ipv4|ipv6)\\ssrc\\saddr\\s"
                "(?P<srcaddr>[0-9.:a-z]+)\\sdst\\saddr\\s(?P<dstaddr>[0-9.:a-z]+)\\n.*(?P<proto>icmpv4|icmpv6)\\stype"
                "\\s(?P<type>\\d+)\\scode\\s(?P<code>\\d+)"},
    "event_protocol": {"tcp": "TCP", "udp": "UDP", "sctp": "SCTP", "icmpv4": "ICMP", "icmpv6": "ICMPv6"},
    "event_action": {"Drop": "Deny", "Allow": "Allow"},
    "cases": e2e_cases,
    "metrics": {  # e2e.go:1205-1352 "should expose daemon metrics"
        "cite": "test/e2e/functional/tests/e2e.go:1249-1260, 1284-1299, 1331-1341",
        "rules": [{"source_cidrs": [f"{POD_IPS[C1][0]}/32", f"{POD_IPS[C1][1]}/128"],
                   "rules": [block_echo("ICMP", 1), block_echo("ICMPv6", 2)]}],
        "pings": [{"src": POD_IPS[C1][0], "dst": POD_IPS[S1][0], "protocol": "ICMP", "icmp_type": 8},
                  {"src": POD_IPS[C1][1], "dst": POD_IPS[S1][1], "protocol": "ICMPv6", "icmp_type": 128}],
        "note": "one `ping -c 1` per family (test/e2e/icmp: ping -4/-6 -c 1), both blocked",
        "expect": {"ingressnodefirewall_node_packet_deny_total": 2}},
}, open("ref_e2e.json", "w"), indent=1)
