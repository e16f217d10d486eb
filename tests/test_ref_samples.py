"""The reference's own sample IngressNodeFirewall objects (config/samples/*.yaml, transcribed into
tests/golden/ref_samples.json by tests/golden/transcribe_samples.py) as golden fixtures.

demo-1 as written carries a TCP rule without ports: the loader mirror refuses the whole sync with -EINVAL and leaves
the map untouched (the reference's webhook refuses the object; its loader would dereference the nil block).
demo-1-admitted (that rule given ports 1-65535), demo-2, demo-3 (two objects on eth0 / eth1) and denyall are loaded
through the loader mirror (IngNodeFwController over the C ABI) and every probe — ICMP 3/1 Allow, ICMPv6 128 Deny,
TCP to 0.0.0.0/0 == ::/0 (one key), a protocol-less deny-all that also covers IPv6 sources, misses, other interfaces
— is checked against the expectations written from the YAML, against the oracle (goenc's loader restatement + the
C restatement of kernel.c), and on the device (-m gpu) through both batch kernels: infw_classify on packed tuples
and infw_classify_frames on the raw frames, result words, verdicts and per-rule counters.
"""
import json
import os

import numpy as np
import pytest

import goenc
import infw
import orc
from frames import frame, snapshots
from infw import workloads as W

DOC = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_samples.json")))
IFX = DOC["ifindex"]
LOADABLE = [s for s in DOC["samples"] if s["loadable"]]


def _rules(node_state):
    return {name: [infw.IngressNodeFirewallRules(e["source_cidrs"], [infw.ProtocolRule(**r) for r in e["rules"]])
                   for e in ents] for name, ents in node_state.items()}


def _controller(sample, clf):
    ctl = infw.IngNodeFwController(clf, if_indices=lambda name: [IFX[name]])
    ctl.ingress_node_fw_rules_loader(_rules(sample["node_state"]))
    return ctl


def _frames(sample):
    fr = [frame(p["src"], None, p["protocol"], dport=p["dport"], icmp_type=p["icmp_type"], icmp_code=p["icmp_code"])
          for p in sample["probes"]]
    return fr, np.array([IFX[p["interface"]] for p in sample["probes"]], np.uint32)


def _expect(sample):
    return (np.array([p["expect_result"] for p in sample["probes"]], np.uint32),
            np.array([p["expect_verdict"] for p in sample["probes"]], np.uint8))


def _check(sample, res, ver, label):
    want_r, want_v = _expect(sample)
    for i, p in enumerate(sample["probes"]):
        assert res[i] == want_r[i] and ver[i] == want_v[i], (label, sample["name"], p, hex(res[i]), ver[i])


def test_demo1_as_written_is_refused():
    s = next(x for x in DOC["samples"] if x["name"] == "demo-1")
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    with pytest.raises(infw.InfwError) as e:
        _controller(s, c)
    assert e.value.errno == 22
    assert c.count() == 0  # a bad rule fails the load before the map is touched (loader.go:158-162)


@pytest.mark.parametrize("sample", LOADABLE, ids=[s["name"] for s in LOADABLE])
def test_sample_keys_and_verdicts_on_host(sample):
    """Key set (0.0.0.0/0 and 0::0/0 are one key), the oracle and the product's compiled host image against the
    expectations written from the YAML."""
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    ctl = _controller(sample, c)
    content = ctl.get_bpf_map_content_for_test()
    assert set(content) == {goenc.build_key(IFX[i], cidr) for i, cidr in sample["expect_keys"]}
    fr, ifx = _frames(sample)
    hdr, cap, pl = snapshots(fr)
    # oracle: the reference loader's map edits restated (goenc) + kernel.c restated
    m = orc.OracleMap()
    goenc.sync(m, goenc.desired(sample["node_state"], IFX))
    assert set(m.keys()) == set(content)
    ores, over, _, _ = m.classify_frames(hdr, cap, pl, ifx)
    _check(sample, ores, over, "oracle")
    tup = W.pack_frames(hdr, cap, pl, ifx)
    res = c.debug_walk(tup)
    _check(sample, res, infw.verdicts_from_results(res, tup[:, 6]), "host image")


@pytest.mark.gpu
@pytest.mark.parametrize("sample", LOADABLE, ids=[s["name"] for s in LOADABLE])
def test_sample_verdicts_on_device(sample):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from e2e_ref import packed
    from infw.batch import SoaBatch
    from parity import stats_from_results
    dev = torch.device("cuda", 0)
    clf = infw.Classifier(devices=[0])
    _controller(sample, clf)
    fr, ifx = _frames(sample)
    n = len(fr)
    hdr, cap, pl = snapshots(fr)
    tup = W.pack_frames(hdr, cap, pl, ifx)
    # packed tuples -> infw_classify
    b = SoaBatch.from_tuples(tup, dev)
    res = torch.empty(n, dtype=torch.int32, device=dev)
    ver = torch.empty(n, dtype=torch.uint8, device=dev)
    clf.stats_reset()
    clf.classify(b, results=res, verdicts=ver)
    torch.cuda.synchronize()
    gres, gver = res.cpu().numpy().view(np.uint32), ver.cpu().numpy()
    _check(sample, gres, gver, "infw_classify")
    want_r, _ = _expect(sample)
    got_stats = clf.stats_read_all()
    assert np.array_equal(got_stats, stats_from_results(want_r, pl)), sample["name"]
    # raw frames back to back -> infw_classify_frames (the packer's semantics in the kernel)
    buf, offs, lens = packed(fr)
    t_buf = torch.from_numpy(buf).to(dev)
    t_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    t_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    t_ifx = torch.from_numpy(ifx.view(np.int32)).to(dev)
    res2 = torch.empty(n, dtype=torch.int32, device=dev)
    ver2 = torch.empty(n, dtype=torch.uint8, device=dev)
    clf.classify_frames(t_buf, t_len, t_ifx, n, results=res2, verdicts=ver2, offsets=t_off)
    torch.cuda.synchronize()
    _check(sample, res2.cpu().numpy().view(np.uint32), ver2.cpu().numpy(), "infw_classify_frames")
