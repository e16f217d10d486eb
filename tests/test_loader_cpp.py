"""The C++ host side above the C ABI (ingress-node-firewall_amd/host/infw_loader.hpp: pkg/ebpf IngNodeFwController
and pkg/metrics in C++, the form a daemon links where the reference's Go is absent), driven through
tests/c/loader_test.cpp on a host-only context (and, -m gpu, on the MI355X).  Checked against the reference's own expectations (the key sets of
ebpfsyncer_test.go:727-987) and, map content byte for byte, against the Python mirror (infw/controller.py) over
the reference's sync sequences — which test_golden.py pins to the reference's verdicts."""
import os
import subprocess

import pytest

import goenc
import infw
from conftest import run_make
from test_golden import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "ingress-node-firewall_amd", "lib", "infw_loader_test")
# the same driver and loader linked against the AddressSanitizer/UBSan build of the whole host side (make asan-host):
# the reference sync sequences, the e2e rule sets and the Go error paths run through it too (CPU only)
ASAN_DRIVER = os.path.join(ROOT, "ingress-node-firewall_amd", "build", "asan", "infw_loader_test")
DRIVERS = pytest.mark.parametrize("drv", [DRIVER, ASAN_DRIVER], ids=["lib", "asan"])


@pytest.fixture(scope="module", autouse=True)
def driver():
    if not os.path.exists(DRIVER):  # built by `make` (the GPU box gets it with the libraries)
        r = run_make(os.path.relpath(DRIVER, ROOT), timeout=600)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert os.path.exists(DRIVER)


@pytest.fixture(scope="module")
def asan_driver():
    import shutil
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    r = run_make("asan-host")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return ASAN_DRIVER


def _driver(drv, request):
    if drv == ASAN_DRIVER:
        if os.environ.get("INFW_SKIP_ASAN"):
            pytest.skip("INFW_SKIP_ASAN set")
        request.getfixturevalue("asan_driver")
    return drv


def run(script: str, with_results=False, drv=DRIVER):
    r = subprocess.run([drv], input=script, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out, dumps, syncs, results = r.stdout.splitlines(), [], [], []
    i = 0
    while i < len(out):
        f = out[i].split()
        if f[0] == "results":
            assert f[1] == "0", out[i]
            n = int(f[2])
            results.append([int(x, 16) for x in out[i + 1:i + 1 + n]])
            i += n
        elif f[0] == "dump":
            assert f[1] == "0"
            n = int(f[2])
            dumps.append({bytes.fromhex(e.split()[1]): bytes.fromhex(e.split()[2]) for e in out[i + 1:i + 1 + n]})
            i += n
        elif f[0] == "sync":
            syncs.append((int(f[1]), int(f[2])))
        i += 1
    if with_results:
        return r.stdout, dumps, syncs, results
    return r.stdout, dumps, syncs


def sync_lines(rules_by_iface) -> str:
    s = ["sync"]
    for name, ents in (rules_by_iface or {}).items():
        s.append(f"iface {name}")
        for e in ents:
            s.append("ruleset " + " ".join(e["source_cidrs"]))
            for r in e["rules"]:
                ports = r.get("ports")
                s.append(f"rule {r['order']} {r.get('protocol') or '-'} {'-' if ports is None else ports} "
                         f"{r.get('icmp_type', 0)} {r.get('icmp_code', 0)} {r.get('action', 'Allow')}")
    s.append("endsync")
    return "\n".join(s) + "\n"


def py_rules(rules_by_iface):
    return {name: [infw.IngressNodeFirewallRules(e["source_cidrs"], [infw.ProtocolRule(**r) for r in e["rules"]])
                   for e in ents] for name, ents in (rules_by_iface or {}).items()}


def test_known_answers():
    """addUInt64 (statistics.go:170-180) and strconv.Atoi (ENABLE_EBPF_LPM_LOOKUP_DBG, loader.go:72-83)."""
    out, _, _ = run("selftest\n")
    assert "selftest ok" in out
    out, _, _ = run("debug 1\nreset\n")
    assert "ctor 0" in out
    out, _, _ = run("debug yes\nreset\n")
    assert "ctor -22" in out


@DRIVERS
@pytest.mark.parametrize("doc_name", ["ref_ebpfsyncer_keys.json", "ref_ebpfsyncer_http.json"])
def test_reference_sync_sequences(doc_name, drv, request):
    """TestVerifyBPFKeysAfterInterfaceIngressRulesUpdate / TestSyncInterfaceIngressRulesWithHTTP: after every
    sync the C++ loader's map has the reference's expected keys (where the test states them) and exactly the
    Python mirror's keys and 1200-B values."""
    doc = load(doc_name)
    script = "".join(f"ifindex {n} {i}\n" for n, i in doc["ifindex"].items())
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    ctl = infw.IngNodeFwController(c, if_indices=lambda name: [doc["ifindex"][name]])
    want = []
    for tc in doc["test_cases"]:
        if tc["isDelete"]:
            script += "reset\n"
            ctl.reset_all()
        else:
            script += sync_lines(tc["rules"])
            ctl.ingress_node_fw_rules_loader(py_rules(tc["rules"]))
        script += "dump\n"
        want.append({k: bytes(v) for k, v in ctl.get_bpf_map_content_for_test().items()})
    out, dumps, syncs = run(script, drv=_driver(drv, request))
    assert all(rc == 0 and errs == 0 for rc, errs in syncs), out[-2000:]
    assert len(dumps) == len(doc["test_cases"])
    for tc, got, exp in zip(doc["test_cases"], dumps, want):
        assert got == exp, tc["name"]
        if "expectedKeys" in tc:
            assert set(got) == {goenc.build_key(doc["ifindex"][i], cidr) for i, cidr in tc["expectedKeys"]}, tc["name"]


@DRIVERS
def test_e2e_table_and_invalid_interfaces(drv, request):
    """The e2e behavioural table's rule sets (e2e.go:176-831, merged per node as the operator does) including an
    interface that does not exist — skipped as loader.go:143-146 does — equal the Python mirror's map."""
    from e2e_ref import DOC
    for case in DOC["cases"]:
        rules = case["interface_ingress_rules"]
        script = "".join(f"ifindex {n} {i}\n" for n, i in DOC["ifindex"].items())
        script += "".join(f"invalid {n}\n" for n in rules if n not in DOC["ifindex"])
        script += sync_lines(rules) + "dump\n"
        c = infw.Classifier(flags=infw.F_HOST_ONLY)
        ctl = infw.IngNodeFwController(c, if_indices=lambda name: [DOC["ifindex"][name]],
                                       is_valid_interface=lambda name: name in DOC["ifindex"])
        ctl.ingress_node_fw_rules_loader(py_rules(rules))
        out, dumps, syncs = run(script, drv=_driver(drv, request))
        assert syncs == [(0, 0)], out[-1000:]
        assert dumps[0] == {k: bytes(v) for k, v in ctl.get_bpf_map_content_for_test().items()}, case["cite"]
        assert dumps[0], case["cite"]


@DRIVERS
def test_errors_like_the_go_loader(drv, request):
    """A rule the Go code rejects fails the whole load before the map is touched (loader.go:158-162); an update
    that hits a full map (ENOSPC, loader.go:200-208) ends the load with the keys before it published; stale keys
    of the previous sync are purged; a bond's slaves each get the keys (loader.go:149)."""
    drv = _driver(drv, request)
    base = "ifindex eth0 7\nifindex bond0 8 9\n"
    ok = {"eth0": [{"source_cidrs": ["10.0.0.0/8"], "rules": [{"order": 1, "protocol": "TCP", "ports": "80",
                                                                "action": "Deny"}]}]}
    bad = {"eth0": [{"source_cidrs": ["11.0.0.0/8"], "rules": [{"order": 1, "protocol": "TCP", "ports": "200-100",
                                                                 "action": "Deny"}]}]}
    out, dumps, syncs = run(base + sync_lines(ok) + sync_lines(bad) + "dump\n", drv=drv)
    assert syncs[0] == (0, 0) and syncs[1][0] == -22
    assert set(dumps[0]) == {goenc.build_key(7, "10.0.0.0/8")}
    full = {"eth0": [{"source_cidrs": ["10.0.0.0/8", "11.0.0.0/8", "12.0.0.0/8"],
                      "rules": [{"order": 1, "protocol": "TCP", "ports": "80", "action": "Deny"}]}]}
    out, dumps, syncs = run("maxentries 2\n" + base + sync_lines(full) + "dump\n", drv=drv)
    assert syncs[0][0] == -28 and len(dumps[0]) == 2   # ENOSPC; the two applied keys are committed
    bond = {"bond0": [{"source_cidrs": ["1.1.1.0/24", "100:1::/64"], "rules": [{"order": 5, "protocol": "UDP",
                                                                                 "ports": "53", "action": "Allow"}]}]}
    out, dumps, syncs = run(base + sync_lines(ok) + sync_lines(bond) + "dump\n", drv=drv)
    assert syncs == [(0, 0), (0, 0)]
    assert set(dumps[0]) == {goenc.build_key(i, c) for i in (8, 9) for c in ("1.1.1.0/24", "100:1::/64")}
    assert all(v == goenc.make_value(bond["bond0"][0]["rules"]) for v in dumps[0].values())
    out, _, syncs = run(base + sync_lines({"ghost": ok["eth0"]}), drv=drv)
    assert syncs[0][0] == -19   # GetInterfaceIndices fails: the load returns its error


def _demo_workload(tmp_path):
    """configs[0]'s demo table (config/samples ingressnodefirewall-demo-1.yaml:12-27) as a sync script, a second
    interface with a deny-all ICMP rule and a UDP range, and 20k workload packets as a tuple file."""
    import numpy as np
    from infw import workloads as W
    rules = {"eth1": [{"source_cidrs": ["1.1.1.1/24", "100:1::1/64"],
                       "rules": [{"order": 10, "protocol": "TCP", "ports": "100-200", "action": "Allow"},
                                 {"order": 20, "protocol": "UDP", "ports": "8000", "action": "Allow"},
                                 {"order": 30, "protocol": "", "action": "Deny"}]}],
             "eth2": [{"source_cidrs": ["0.0.0.0/0", "::/0"],
                       "rules": [{"order": 5, "protocol": "ICMP", "icmp_type": 8, "action": "Deny"},
                                 {"order": 6, "protocol": "ICMPv6", "icmp_type": 128, "action": "Deny"},
                                 {"order": 7, "protocol": "UDP", "ports": "7000-9000", "action": "Allow"}]}]}
    wl = W.Workload(W.CFG0_DEMO)
    hdr, cap, pl, ifx = wl.frames(0, 20000)
    tup = np.ascontiguousarray(W.pack_frames(hdr, cap, pl, ifx), dtype=np.uint32)
    path = tmp_path / "tuples.bin"
    tup.tofile(path)
    ifmap = "ifindex eth1 1\nifindex eth2 2\n"
    return rules, ifmap, tup, str(path)


def test_cpp_loader_tables_walk_like_python(tmp_path):
    """The C++ loader's committed image, walked on the host, classifies 20k workload packets exactly like the
    Python mirror's (whose loader test_golden.py pins to the reference's verdicts)."""
    import numpy as np
    rules, ifmap, tup, path = _demo_workload(tmp_path)
    out, _, syncs, results = run(ifmap + sync_lines(rules) + f"walk {path}\n", with_results=True)
    assert syncs == [(0, 0)]
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    ctl = infw.IngNodeFwController(c, if_indices=lambda name: [{"eth1": 1, "eth2": 2}[name]])
    ctl.ingress_node_fw_rules_loader(py_rules(rules))
    want = c.debug_walk(tup)
    assert np.array_equal(np.array(results[0], np.uint32), want)
    assert len(set(results[0])) >= 4


@pytest.mark.gpu
def test_cpp_loader_on_device(tmp_path):
    """The C++ host side end to end on the MI355X: IngressNodeFwRulesLoader commits to the device, the packets go
    through infw_classify_host (host-resident batch, pipelined H2D), and UpdateMetrics reads the device's
    statistics slot — result words equal to the host walk of the same image, totals equal to the counters the
    result words imply (statistics.go:126-157 over rules 1..99)."""
    import numpy as np
    pytest.importorskip("torch")
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    rules, ifmap, tup, path = _demo_workload(tmp_path)
    out, _, syncs, results = run("device\n" + ifmap + sync_lines(rules) + f"classify {path}\nwalk {path}\nmetrics\n"
                                 "reset\nmetrics\n", with_results=True)
    assert syncs == [(0, 0)], out[-1000:]
    got, walk = np.array(results[0], np.uint32), np.array(results[1], np.uint32)
    assert np.array_equal(got, walk)
    act, rid, plen = got & 0xFF, (got >> 8) & 0xFFFF, tup[:, 5].astype(np.uint64)
    counted = (rid >= 1) & (rid < 100)
    want = [int(((act == 2) & counted).sum()), int(plen[(act == 2) & counted].sum()),
            int(((act == 1) & counted).sum()), int(plen[(act == 1) & counted].sum())]
    lines = [l.split() for l in out.splitlines() if l.startswith("metrics")]
    line = lines[0]
    assert line[1] == "0" and [int(x) for x in line[2:6]] == want and line[6] == "0", (line, want)
    assert want[0] > 0 and want[2] > 0
    # ResetAll drops the statistics with the table (ebpfsyncer.go:170): the next poll reads zero
    assert lines[1][1:] == ["0", "0", "0", "0", "0", "0"], lines[1]
