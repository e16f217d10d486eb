"""The HIP classifier against reference-held and frozen vectors, on the device.

- TestSyncInterfaceIngressRulesWithHTTP (pkg/ebpfsyncer/ebpfsyncer_test.go:41-445, tests/golden/ref_ebpfsyncer_http.json):
  the sync sequence through the product's loader mirror (IngNodeFwController over the C ABI) on a GPU context, every
  connection's XDP verdict from infw_classify — the reference's own expected verdicts, no oracle involved.
- TestVerifyBPFKeysAfterInterfaceIngressRulesUpdate (:727-987, ref_ebpfsyncer_keys.json): the map's key set after
  each sync, and a packet from every expected key's prefix classified on the device (checked against the oracle,
  which the CPU suite pins to the same file).
- Frozen digests (tests/golden/digests.json, written once from the oracle by tests/golden/make_digests.py): result
  words, verdicts and per-rule counters of the reduced BASELINE workloads and of the configs[4] swap sequence,
  checked by SHA-256 with no oracle loaded.
"""
import ipaddress
import json
import os

import numpy as np
import pytest
import torch

import infw
from frames import frame, http_targets, snapshots
from golden.make_digests import CASES, SWAP, record, swap_edits
from infw import workloads as W
from infw.batch import SoaBatch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
DIG = json.load(open(os.path.join(GOLD, "digests.json")))["cases"]


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _device_classify(clf, frames, ifx):
    """Frames -> (result words, verdicts) through the packer's tuple format and infw_classify on cuda:0."""
    hdr, cap, pl = snapshots(frames)
    tuples = W.pack_frames(hdr, cap, pl, np.array(ifx, np.uint32))
    dev = torch.device("cuda", 0)
    n = len(frames)
    b = SoaBatch.from_tuples(tuples, dev)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    ver = torch.empty(n, dtype=torch.uint8, device=dev)
    clf.classify(b, results=res, verdicts=ver)
    torch.cuda.synchronize()
    return res.cpu().numpy().view(np.uint32), ver.cpu().numpy()


def _controller_rules(tc):
    return {name: [infw.IngressNodeFirewallRules(e["source_cidrs"], [infw.ProtocolRule(**r) for r in e["rules"]])
                   for e in ents] for name, ents in (tc["rules"] or {}).items()}


def test_ebpfsyncer_http_verdicts_on_device():
    doc = json.load(open(os.path.join(GOLD, "ref_ebpfsyncer_http.json")))
    clf = infw.Classifier(devices=[0])
    ctl = infw.IngNodeFwController(clf, if_indices=lambda name: [doc["ifindex"][name]])
    for tc in doc["test_cases"]:
        if tc["isDelete"]:
            ctl.reset_all()
        else:
            ctl.ingress_node_fw_rules_loader(_controller_rules(tc))
        tg = http_targets(doc, tc)
        _, ver = _device_classify(clf, [t[0] for t in tg], [t[1] for t in tg])
        assert list(ver) == [t[2] for t in tg], tc["name"]


def test_ebpfsyncer_key_sets_on_device():
    import goenc
    import orc
    doc = json.load(open(os.path.join(GOLD, "ref_ebpfsyncer_keys.json")))
    clf = infw.Classifier(devices=[0])
    ctl = infw.IngNodeFwController(clf, if_indices=lambda name: [doc["ifindex"][name]])
    m = orc.OracleMap()
    for tc in doc["test_cases"]:
        if tc["isDelete"]:
            ctl.reset_all()
            goenc.sync(m, {})
        else:
            ctl.ingress_node_fw_rules_loader(_controller_rules(tc))
            goenc.sync(m, goenc.desired(tc["rules"], doc["ifindex"]))
        want = {goenc.build_key(doc["ifindex"][i], cidr) for i, cidr in tc["expectedKeys"]}
        assert set(ctl.get_bpf_map_content_for_test().keys()) == want, tc["name"]
        frames, ifx = [], []
        for iface, cidr in tc["expectedKeys"] + [["dummy0", "10.1.2.3/32"], ["dummy1", "2001:db8::9/128"]]:
            net = ipaddress.ip_network(cidr, strict=False)
            for host in (net.network_address, net.broadcast_address):
                for port in (12345, 12346, 80):
                    frames.append(frame(str(host), proto="tcp", dport=port))
                    ifx.append(doc["ifindex"][iface])
        res, _ = _device_classify(clf, frames, ifx)
        hdr, cap, pl = snapshots(frames)
        ores, _, _, _ = m.classify_frames(hdr, cap, pl, np.array(ifx, np.uint32), nthreads=1)
        assert np.array_equal(res, ores), tc["name"]


def _gpu_record(clf, wl, start, n):
    dev = torch.device("cuda", 0)
    b = SoaBatch.empty(n, dev)
    wl.gen_device(b, start, 0)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    ver = torch.empty(n, dtype=torch.uint8, device=dev)
    st = torch.zeros((1024, 4), dtype=torch.int64, device=dev)
    clf.stats_bind(0, st.data_ptr())
    clf.classify(b, results=res, verdicts=ver)
    torch.cuda.synchronize()
    clf.stats_bind(0, None)
    return record(res.cpu().numpy().view(np.uint32), ver.cpu().numpy(), st.cpu().numpy().view(np.uint64))


@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_kernel_matches_frozen_digests(case):
    name, cfg, npfx, ntmpl, start, n = case
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    got = _gpu_record(clf, wl, start, n)
    assert got == {k: DIG[name][k] for k in got}, name


def test_kernel_matches_frozen_swap():
    name, cfg, npfx, ntmpl, n = SWAP
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    a = _gpu_record(clf, wl, 0, n)
    for e in swap_edits(wl):
        if e[0] == "delete":
            clf.delete_rc(infw.LpmIpKeySt.from_buffer_copy(e[1]))
        else:
            clf.update(infw.LpmIpKeySt.from_buffer_copy(e[1]), infw.RulesValSt.from_buffer_copy(e[2]))
    clf.commit()  # incremental: the live swap between two batches
    b = _gpu_record(clf, wl, n, n)
    assert a == DIG[name]["batch_a"] and b == DIG[name]["batch_b"]


def test_e2e_table_on_device():
    """The reference's e2e behavioural table (e2e.go:176-831, tests/golden/ref_e2e.json) on the device, no oracle:
    for each entry the node's merged rules go through the loader mirror, the entry's reachability checks
    (TCP/UDP/SCTP to the blocked port or range, ICMP and ICMPv6 echo requests, both families) are classified
    straight from their frames in HBM (infw_classify_frames_ex) — all XDP_PASS before the policy, all XDP_DROP
    after — and every drop's perf sample (infw_events_capture) through the consumer must yield the drop event the
    reference's e2e looks for with its own regular expressions (test/e2e/events/events.go)."""
    import ctypes as C
    from infw import _native as N
    from infw import events as E
    from e2e_ref import DOC, case_frames, controller_rules, event_in_list, extract_events, if_name, packed
    dev = torch.device("cuda", 0)
    t32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)
    clf = infw.Classifier(devices=[0])
    ctl = infw.IngNodeFwController(clf, if_indices=lambda name: [DOC["ifindex"][name]],
                                   is_valid_interface=lambda name: name in DOC["ifindex"])
    for case in DOC["cases"]:
        frames, ifx = case_frames(case["connections"])
        n = len(frames)
        buf, offs, lens = packed(frames)
        dbuf = torch.from_numpy(buf).to(dev)
        doffs = torch.from_numpy(offs.view(np.int64)).to(dev)
        for phase, want in (("before", 2), ("after", 1)):
            if phase == "before":
                ctl.reset_all()
            else:
                ctl.ingress_node_fw_rules_loader(controller_rules(case["interface_ingress_rules"]))
            ev = torch.zeros(n * C.sizeof(N.EventRec), dtype=torch.uint8, device=dev)
            cnt = torch.zeros(1, dtype=torch.int64, device=dev)
            res = torch.empty(n, dtype=torch.int32, device=dev)
            ver = torch.empty(n, dtype=torch.uint8, device=dev)
            clf.classify_frames(dbuf, t32(lens), t32(ifx), n, results=res, verdicts=ver, offsets=doffs,
                                events=ev, events_count=cnt)
            smp = torch.zeros(n * N.EVENT_SAMPLE_BYTES, dtype=torch.uint8, device=dev)
            clf.events_capture(dbuf, t32(lens), t32(ifx), n, ev, cnt, smp, offsets=doffs)
            torch.cuda.synchronize()
            assert list(ver.cpu().numpy()) == [want] * n, (case["it"], phase)
            k = int(cnt.item())
            assert k == (n if want == 1 else 0), (case["it"], phase)
            if k:
                lines, log = E.drain(smp.cpu().numpy(), k, if_name)
                assert not log
                got = extract_events("".join(lines))
                for c in case["connections"]:
                    assert event_in_list(got, c["event"]), (case["it"], c)


def test_e2e_metrics_on_device():
    """e2e.go:1205-1352: one blocked ping per family, then Statistics.update_metrics (statistics.go:112-167) over
    the device's counters reports packet_deny_total == 2."""
    from e2e_ref import DOC, case_frames, controller_rules
    doc = DOC["metrics"]
    clf = infw.Classifier(devices=[0])
    ctl = infw.IngNodeFwController(clf, if_indices=lambda name: [DOC["ifindex"][name]])
    ctl.ingress_node_fw_rules_loader(controller_rules({"eth0": doc["rules"]}))
    conns = [dict(p, icmp_code=0, interface="eth0") for p in doc["pings"]]
    frames, ifx = case_frames(conns)
    _, ver = _device_classify(clf, frames, ifx)
    assert list(ver) == [1, 1]
    m = infw.Statistics(clf).update_metrics()
    assert m["ingressnodefirewall_node_packet_deny_total"] == doc["expect"]["ingressnodefirewall_node_packet_deny_total"]
    assert m["ingressnodefirewall_node_packet_allow_total"] == 0
    # resetAll drops the statistics map with the objects (ebpfsyncer.go:170): the next poll reads zero
    ctl.reset_all()
    assert all(v == 0 for v in infw.Statistics(clf).update_metrics().values())
