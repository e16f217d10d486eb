"""Golden vectors from the reference's own tests and the survey's probe records.

Each vector runs through (1) the oracle (pins the oracle) and (2) the
product's control plane + table compiler on a host-only context, walking the
compiled GPU table image on the CPU (infw_debug_walk).  The reference's syncer
vectors run through the HIP kernel in test_gpu_golden.py, the survey probes in
test_gpu_parity.py (test_survey_probes_on_device).
"""
import json
import os

import numpy as np
import pytest

import goenc
import infw
import orc
from frames import frame, http_targets, snapshots
from infw import workloads as W

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return json.load(open(os.path.join(GOLD, name)))


def probe_frames(case):
    fr, ifx = [], []
    for p in case["packets"]:
        fr.append(frame(p["src"], proto=p.get("proto", "tcp"), dport=p.get("dport", 0),
                        icmp_type=p.get("icmp_type", 0), icmp_code=p.get("icmp_code", 0),
                        ethertype=p.get("ethertype"), ihl=p.get("ihl", 5), truncate=p.get("truncate")))
        ifx.append(p["ifindex"])
    return fr, ifx


def expected_stats(case, frames):
    st = np.zeros((1024, 4), np.uint64)
    for p, f in zip(case["packets"], frames):
        for rid, kind in p["expect"]["stats"]:
            c = 0 if kind == "allow" else 2
            st[rid, c] += 1
            st[rid, c + 1] += len(f)
    return st


@pytest.mark.parametrize("case", load("survey_probes.json")["cases"], ids=lambda c: c["name"][:50])
def test_survey_probes_oracle(case):
    m = orc.OracleMap()
    for e in case["table"]:
        assert m.update(goenc.build_key(e["key"]["ifindex"], e["key"]["cidr"]), goenc.raw_value(e["rules"])) == 0
    if "expect_entries" in case:
        assert len(m) == case["expect_entries"]
    frames, ifx = probe_frames(case)
    stats = np.zeros((1024, 4), np.uint64)
    for p, f, i in zip(case["packets"], frames, ifx):
        act, res, _ = m.run(f, i, stats=stats)
        assert act == p["expect"]["retval"], (p, act, hex(res))
        if "result" in p["expect"]:
            assert res == p["expect"]["result"]
    assert np.array_equal(stats, expected_stats(case, frames))


@pytest.mark.parametrize("case", load("survey_probes.json")["cases"], ids=lambda c: c["name"][:50])
def test_survey_probes_compiled_tables(case):
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    for e in case["table"]:
        c.update(infw.build_ebpf_key(e["key"]["ifindex"], e["key"]["cidr"]),
                 infw.RulesValSt.from_buffer_copy(goenc.raw_value(e["rules"])))
    c.commit()
    if "expect_entries" in case:
        assert c.count() == case["expect_entries"]
    frames, ifx = probe_frames(case)
    hdr, cap, pl = snapshots(frames)
    res = c.debug_walk(W.pack_frames(hdr, cap, pl, np.array(ifx, np.uint32)))
    tuples = W.pack_frames(hdr, cap, pl, np.array(ifx, np.uint32))
    ver = infw.verdicts_from_results(res, tuples[:, 6])
    for p, v, r in zip(case["packets"], ver, res):
        assert v == p["expect"]["retval"], (p, v, hex(r))
        if "result" in p["expect"]:
            assert r == p["expect"]["result"]
    # counters implied by the result words equal the probe's counters
    from parity import stats_from_results
    assert np.array_equal(stats_from_results(res, pl), expected_stats(case, frames))


def test_ebpfsyncer_http_oracle():
    """TestSyncInterfaceIngressRulesWithHTTP: sync sequence + connection verdicts, on the oracle."""
    doc = load("ref_ebpfsyncer_http.json")
    m = orc.OracleMap()
    for tc in doc["test_cases"]:
        goenc.sync(m, {} if tc["isDelete"] else goenc.desired(tc["rules"], doc["ifindex"]))
        for f, ifx, want in http_targets(doc, tc):
            act, res, _ = m.run(f, ifx)
            assert act == want, (tc["name"], ifx, hex(res))


def test_ebpfsyncer_http_product_controller():
    """The same sequence through the product's loader mirror (IngNodeFwController over the C ABI)."""
    doc = load("ref_ebpfsyncer_http.json")
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    ctl = infw.IngNodeFwController(c, if_indices=lambda name: [doc["ifindex"][name]])
    for tc in doc["test_cases"]:
        if tc["isDelete"]:
            ctl.reset_all()
        else:
            rules = {name: [infw.IngressNodeFirewallRules(e["source_cidrs"], [infw.ProtocolRule(**r) for r in
                                                                            e["rules"]]) for e in ents]
                     for name, ents in (tc["rules"] or {}).items()}
            ctl.ingress_node_fw_rules_loader(rules)
        tg = http_targets(doc, tc)
        hdr, cap, pl = snapshots([t[0] for t in tg])
        tuples = W.pack_frames(hdr, cap, pl, np.array([t[1] for t in tg], np.uint32))
        ver = infw.verdicts_from_results(c.debug_walk(tuples), tuples[:, 6])
        assert list(ver) == [t[2] for t in tg], tc["name"]


def test_loader_partial_failure_publishes_applied_updates():
    """A load that fails part-way (ENOSPC on a full map, loader.go:200-208 returns the error) still publishes the
    updates made before the failure — the reference's per-key map writes are live at once — instead of leaving them
    pending for an unrelated later commit."""
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=2)
    ctl = infw.IngNodeFwController(c, if_indices=lambda name: [7])
    deny = [infw.ProtocolRule(order=1, protocol="TCP", ports="80", action="Deny")]
    with pytest.raises(OSError):
        ctl.ingress_node_fw_rules_loader({"eth0": [infw.IngressNodeFirewallRules(
            ["10.0.0.0/8", "11.0.0.0/8", "12.0.0.0/8"], deny)]})
    assert c.count() == 2
    frames = [frame(src, proto="tcp", dport=80) for src in ("10.1.2.3", "11.1.2.3", "12.1.2.3")]
    hdr, cap, pl = snapshots(frames)
    tuples = W.pack_frames(hdr, cap, pl, np.full(3, 7, np.uint32))
    ver = infw.verdicts_from_results(c.debug_walk(tuples), tuples[:, 6])
    assert list(ver) == [1, 1, 2]  # the two applied keys are in the published epoch (XDP_DROP), the third is not


def partial_ifindex_case():
    """A table with keys shorter than the ifindex and packets from interfaces with and without entries of their own:
    (entries [(key bytes, rule id)], values {rule id: 1200 B}, hdr, cap, pl, ifindex array, tuples)."""
    import struct
    rng = np.random.default_rng(3)
    entries = [(goenc.build_key(1, "10.0.0.0/8"), 3), (goenc.build_key(0x102, "10.1.0.0/16"), 4),
               (goenc.build_key(0x102, "2001:db8::/32"), 5), (goenc.build_key(0x102, "2001:db8:1::/48"), 6),
               (goenc.build_key(2, "0.0.0.0/0"), 7),
               (struct.pack("<II", 0, 0) + bytes(16), 8),                              # every ifindex
               (struct.pack("<II", 8, 0x02) + bytes(16), 9),                           # low byte 0x02
               (struct.pack("<II", 16, 0x0102) + bytes(16), 10),                       # low bytes 02 01
               (struct.pack("<II", 31, 0x00000702) + bytes(16), 11)]
    vals = {rid: goenc.raw_value([{"slot": 1, "ruleId": rid, "protocol": 0, "dstPortStart": 0, "dstPortEnd": 0,
                                   "icmpType": 0, "icmpCode": 0, "action": 1 + rid % 2}]) for _, rid in entries}
    ifxs = [1, 2, 3, 0x102, 0x202, 0x10102, 0x702, 0x703, 0x8702, 7]
    frames, fifx = [], []
    for k in range(3000):
        src = rng.choice(["10.%d.%d.%d" % tuple(rng.integers(0, 256, 3)), "11.1.2.3",
                          "2001:db8:%x::%x" % (rng.integers(0, 3), rng.integers(0, 999)), "2002::1"])
        frames.append(frame(src, proto="tcp", dport=80))
        fifx.append(ifxs[k % len(ifxs)])
    hdr, cap, pl = snapshots(frames)
    fifx = fifx
    return entries, vals, hdr, cap, pl, fifx, W.pack_frames(hdr, cap, pl, fifx)


def test_partial_ifindex_prefixes():
    """Keys shorter than the ifindex (prefixLen < 32; lpm_trie accepts them, BuildEBPFKey never writes one): they
    match every interface whose ifindex bytes (little-endian, as in the key) start with their bits, below every
    entry of the interface itself — including interfaces with no entries at all.  Compiled host tables vs the
    oracle, in both short-table forms, and a later full commit without them.  On the GPU:
    test_gpu_parity.py::test_partial_ifindex_prefixes_on_device."""
    entries, vals, hdr, cap, pl, fifx, tup = partial_ifindex_case()
    for mode in ("dir24", "compressed"):
        c = infw.Classifier(flags=infw.F_HOST_ONLY, options={"short_table": {"dir24": 0, "compressed": 1}[mode]})
        m = orc.OracleMap()
        for kb, rid in entries:
            assert c.update_rc(infw.LpmIpKeySt.from_buffer_copy(kb), infw.RulesValSt.from_buffer_copy(vals[rid])) == 0
            assert m.update(kb, vals[rid]) == 0
        c.commit()
        want, _, _, _ = m.classify_frames(hdr, cap, pl, fifx, nthreads=2)
        got = c.debug_walk(tup)
        assert np.array_equal(got, want), mode
        assert len({int(r) >> 8 for r in want}) >= 6  # defaults, own entries and unknown ifindexes all seen
        assert [bytes(k) for k, _ in c.iterate()] == list(m.keys())
        # delete the partial prefixes: the next commit (full) drops the defaults
        for kb, rid in entries[5:]:
            assert c.delete_rc(infw.LpmIpKeySt.from_buffer_copy(kb)) == m.delete(kb) == 0
        c.commit()
        assert c.info()["commit_mode"] == infw.COMMIT_FULL
        want, _, _, _ = m.classify_frames(hdr, cap, pl, fifx, nthreads=2)
        assert np.array_equal(c.debug_walk(tup), want), mode


def test_ebpfsyncer_key_sets():
    """TestVerifyBPFKeysAfterInterfaceIngressRulesUpdate: the map's key set after each sync."""
    doc = load("ref_ebpfsyncer_keys.json")
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    ctl = infw.IngNodeFwController(c, if_indices=lambda name: [doc["ifindex"][name]])
    m = orc.OracleMap()
    for tc in doc["test_cases"]:
        if tc["isDelete"]:
            ctl.reset_all()
            goenc.sync(m, {})
        else:
            rules = {name: [infw.IngressNodeFirewallRules(e["source_cidrs"], [infw.ProtocolRule(**r) for r in
                                                                            e["rules"]]) for e in ents]
                     for name, ents in (tc["rules"] or {}).items()}
            ctl.ingress_node_fw_rules_loader(rules)
            goenc.sync(m, goenc.desired(tc["rules"], doc["ifindex"]))
        want = {goenc.build_key(doc["ifindex"][i], cidr) for i, cidr in tc["expectedKeys"]}
        got = set(ctl.get_bpf_map_content_for_test().keys())
        assert got == want, tc["name"]
        assert set(m.keys()) == want, tc["name"]


def test_loader_key_identity():
    """TestAddOrUpdateRules: distinct (ifindex, prefix) pairs are distinct keys."""
    for tc in load("ref_loader_keys.json")["test_cases"]:
        c = infw.Classifier(flags=infw.F_HOST_ONLY)
        m = orc.OracleMap()
        val = goenc.raw_value([{"slot": 0, "ruleId": tc["rule"]["ruleId"], "protocol": 0, "dstPortStart": 0,
                                "dstPortEnd": 0, "icmpType": 0, "icmpCode": 0, "action": tc["rule"]["action"]}])
        for ifx, cidr in tc["keys"]:
            k = infw.build_ebpf_key(ifx, cidr)
            assert bytes(k) == goenc.build_key(ifx, cidr)
            c.update(k, infw.RulesValSt.from_buffer_copy(val))
            assert m.update(bytes(k), val) == 0
        assert c.count() == tc["expected_n_keys"] == len(m)


def test_demo1_sample():
    """configs[0]: config/samples/ingressnodefirewall-demo-1.yaml ingress[0] (TCP 100-200 Allow, UDP 8000 Allow)."""
    m = orc.OracleMap()
    rules = [{"order": 10, "protocol": "TCP", "ports": "100-200", "action": "Allow"},
             {"order": 20, "protocol": "UDP", "ports": 8000, "action": "Allow"}]
    for cidr in ("1.1.1.1/24", "100:1::1/64"):
        assert m.update(goenc.build_key(1, cidr), goenc.make_value(rules)) == 0
    cases = [("1.1.1.9", "tcp", 100, 2, (10 << 8) | 2), ("1.1.1.9", "tcp", 199, 2, (10 << 8) | 2),
             ("1.1.1.9", "tcp", 200, 2, 0), ("1.1.1.9", "udp", 8000, 2, (20 << 8) | 2),
             ("1.1.1.9", "udp", 8001, 2, 0), ("1.1.2.9", "tcp", 150, 2, 0),
             ("100:1::77", "tcp", 150, 2, (10 << 8) | 2), ("100:1:0:1::77", "tcp", 150, 2, 0),
             ("100:1::77", "icmpv6", 0, 2, 0)]
    for src, proto, port, act, res in cases:
        a, r, _ = m.run(frame(src, proto=proto, dport=port), 1)
        assert (a, r) == (act, res), (src, proto, port)


def test_rules_examined_oracle():
    """SURVEY.md §8d "rule bytes examined": valid rules the in-order loop looks at, up to and including the match
    (kernel.c:222-258); ruleId-0 slots are skipped and not counted, a lookup miss or a parse failure examines none."""
    from frames import snapshots
    m = orc.OracleMap()
    rules = [{"order": 1, "protocol": "TCP", "ports": "100-200", "action": "Allow"},
             {"order": 5, "protocol": "UDP", "ports": 53, "action": "Allow"},
             {"order": 10, "protocol": "", "action": "Deny"}]
    assert m.update(goenc.build_key(1, "10.0.0.0/8"), goenc.make_value(rules)) == 0
    cases = [(frame("10.1.2.3", proto="tcp", dport=150), 1), (frame("10.1.2.3", proto="udp", dport=53), 2),
             (frame("10.1.2.3", proto="icmp"), 3), (frame("10.1.2.3", proto="tcp", dport=7), 3),
             (frame("11.1.2.3", proto="tcp", dport=150), 0), (frame("10.1.2.3", proto="gre"), 0)]
    for f, want in cases:
        hdr, cap, pl = snapshots([f])
        assert m.rules_examined(hdr, cap, pl, np.array([1], np.uint32)) == want
    hdr, cap, pl = snapshots([f for f, _ in cases])
    assert m.rules_examined(hdr, cap, pl, np.ones(len(cases), np.uint32)) == sum(w for _, w in cases)


def test_debug_lookup_keys_oracle():
    """The dbg-map key of each probe packet (kernel.c:205-216, :291-299): only packets whose L4 header was
    extracted insert; IPv4 keys are {64, ifindex, saddr, 12 zero bytes}, IPv6 keys {160, ifindex, saddr}."""
    import struct
    need = {6: 20, 17: 8, 132: 12, 1: 8, 58: 8}
    for case in load("survey_probes.json")["cases"]:
        frames, ifx = probe_frames(case)
        hdr, cap, pl = snapshots(frames)
        keys, _ = orc.debug_map_after(hdr, cap, pl, np.array(ifx, np.uint32))
        want = []
        for f, i in zip(frames, ifx):
            et = f[12] << 8 | f[13] if len(f) >= 14 else None
            if et == 0x0800 and len(f) > 23 and f[23] in need and len(f) >= 34 + need[f[23]]:
                k = struct.pack("<II", 64, i) + f[26:30] + bytes(12)
            elif et == 0x86DD and len(f) > 20 and f[20] in need and len(f) >= 54 + need[f[20]]:
                k = struct.pack("<II", 160, i) + f[22:38]
            else:
                continue
            if k not in want:
                want.append(k)
        assert keys == want, case["name"]


# ---- the reference's e2e behavioural table (tests/golden/ref_e2e.json, e2e.go:176-831): TCP, UDP, SCTP, ICMP and
# ICMPv6 block rules, a port range, multiple ports, multiple source CIDRs, multi-object merges, an invalid interface

def _e2e_cases():
    from e2e_ref import DOC
    return DOC["cases"]


@pytest.mark.parametrize("case", _e2e_cases(), ids=lambda c: c["cite"].split(":")[-1])
def test_e2e_table_oracle(case):
    """Oracle: every reachability check passes before the policy and is dropped after it, and each drop's perf
    sample, through the consumer (events.go:77-166), yields the event the reference's e2e expects (events.go regex
    + isEventInList)."""
    from infw import events as E
    from e2e_ref import DOC, case_frames, event_in_list, extract_events, if_name, packed, valid_rules
    frames, ifx = case_frames(case["connections"])
    m = orc.OracleMap()
    assert [m.run(f, i)[0] for f, i in zip(frames, ifx)] == [2] * len(frames)   # initial connectivity
    goenc.sync(m, goenc.desired(valid_rules(case["interface_ingress_rules"]), DOC["ifindex"]))
    assert [m.run(f, i)[0] for f, i in zip(frames, ifx)] == [1] * len(frames)   # blocked
    buf, offs, lens = packed(frames)
    recs, samples = m.collect_event_samples(buf, offs, lens, lens, np.array(ifx, np.uint32))
    assert recs.shape[0] == len(frames)
    lines, log = E.drain(samples, recs.shape[0], if_name)
    assert not log
    got = extract_events("".join(lines))
    for c in case["connections"]:
        assert event_in_list(got, c["event"]), (c, lines)


@pytest.mark.parametrize("case", _e2e_cases(), ids=lambda c: c["cite"].split(":")[-1])
def test_e2e_table_product_controller(case):
    """The same checks through the product's loader mirror (IngNodeFwController over the C ABI, the invalid
    interface skipped as loader.go:143-146 does) and the compiled table image walked on the host."""
    from e2e_ref import DOC, case_frames, controller_rules
    from parity import stats_from_results
    frames, ifx = case_frames(case["connections"])
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    ctl = infw.IngNodeFwController(c, if_indices=lambda name: [DOC["ifindex"][name]],
                                   is_valid_interface=lambda name: name in DOC["ifindex"])
    hdr, cap, pl = snapshots(frames)
    tuples = W.pack_frames(hdr, cap, pl, np.array(ifx, np.uint32))
    assert list(infw.verdicts_from_results(c.debug_walk(tuples), tuples[:, 6])) == [2] * len(frames)
    ctl.ingress_node_fw_rules_loader(controller_rules(case["interface_ingress_rules"]))
    res = c.debug_walk(tuples)
    assert list(infw.verdicts_from_results(res, tuples[:, 6])) == [1] * len(frames)
    st = stats_from_results(res, pl)
    assert int(st[:, 2].sum()) == len(frames) and int(st[:, 0].sum()) == 0


def test_e2e_metrics_oracle():
    """e2e.go:1205-1352: one blocked ping per family -> packet_deny_total 2 (statistics.go:126-157 over rules 1..99)."""
    from e2e_ref import DOC, conn_frame
    doc = DOC["metrics"]
    m = orc.OracleMap()
    goenc.sync(m, goenc.desired({"eth0": doc["rules"]}, DOC["ifindex"]))
    stats = np.zeros((1024, 4), np.uint64)
    for p in doc["pings"]:
        f = conn_frame(dict(p, icmp_code=0))
        assert m.run(f, DOC["ifindex"]["eth0"], stats=stats)[0] == 1
    assert int(stats[1:100, 2].sum()) == doc["expect"]["ingressnodefirewall_node_packet_deny_total"]
