"""Control-plane encoders (csrc/controlplane.cpp) against an independent restatement
of the Go helpers (tests/goenc.py) and the Go error cases:
BuildEBPFKey (loader.go:530-547), makeIngressFwRulesMap (loader.go:429-515),
utils.GetPort / GetRange (utils.go:20-60)."""
import pytest

import goenc
import infw


@pytest.mark.parametrize("ifx,cidr", [
    (100, "10.0.0.0/8"), (100, "192.0.2.0/24"), (100, "10.0.0.0/16"), (101, "10.0.0.0/8"),  # loader_test.go:19-51
    (1, "1.1.1.1/24"), (1, "100:1::1/64"), (1, "3.3.3.3/24"), (1, "10:10::1/64"),          # demo-1 sample
    (1, "0.0.0.0/0"), (1, "0::0/0"), (7, "::ffff:1.2.3.4/120"), (7, "::ffff:1.2.3.4/24"),
    (2, "2001:db8::/32"), (2, "fe80::1:2:3:4/128"), (2, "255.255.255.255/32"), (3, "::/0"),
    (4, "1:2:3:4:5:6:7:8/127"), (4, "1::7:8/96"), (4, "::1.2.3.4/100"), (5, "10.0.0.1/008"),
])
def test_build_key_matches_go_restatement(ifx, cidr):
    assert bytes(infw.build_ebpf_key(ifx, cidr)) == goenc.build_key(ifx, cidr)


@pytest.mark.parametrize("cidr", ["10.0.0.0", "10.0.0.0/33", "::/129", "1.2.3/8", "01.2.3.4/8", "256.1.1.1/8",
                                  "1::2::3/64", "fe80::1%eth0/64", "1.2.3.4/-1", "1.2.3.4/", "/8", "1:2:3:4:5:6:7:8:9/64",
                                  "1.2.3.4/8x", "g::/8"])
def test_build_key_rejects_what_go_rejects(cidr):
    with pytest.raises(infw.InfwError):
        infw.build_ebpf_key(1, cidr)


RULE_CASES = [
    [{"order": 10, "protocol": "TCP", "ports": "100-200", "action": "Allow"},
     {"order": 20, "protocol": "UDP", "ports": 8000, "action": "Allow"}],
    [{"order": 1, "protocol": "SCTP", "ports": "1-65535", "action": "Deny"},
     {"order": 2, "protocol": "ICMP", "icmp_type": 3, "icmp_code": 1, "action": "Allow"},
     {"order": 3, "protocol": "ICMPv6", "icmp_type": 128, "action": "Deny"},
     {"order": 99, "protocol": "", "action": "Deny"}],
    [{"order": 5, "protocol": "TCP", "ports": "00080", "action": "Allow"}],
]


@pytest.mark.parametrize("rules", RULE_CASES)
def test_make_rules_matches_go_restatement(rules):
    val = infw.make_rules_val([infw.ProtocolRule(**r) for r in rules])
    assert bytes(val) == goenc.make_value(rules)


@pytest.mark.parametrize("proto,ports", [("TCP", "0"), ("TCP", "65536"), ("UDP", "200-100"), ("UDP", "100-100"),
                                         ("SCTP", "0-10"), ("TCP", "a"), ("TCP", ""), ("TCP", "1-2-3"),
                                         ("TCP", None), ("TCP", "+80"), ("UDP", "80-")])
def test_port_errors(proto, ports):
    with pytest.raises(infw.InfwError):
        infw.make_rules_val([infw.ProtocolRule(1, proto, ports, action="Allow")])


def test_action_and_order_errors():
    with pytest.raises(infw.InfwError):
        infw.make_rules_val([infw.ProtocolRule(1, "TCP", "80", action="Reject")])
    with pytest.raises(infw.InfwError) as e:  # Go would panic indexing Rules[100]
        infw.make_rules_val([infw.ProtocolRule(100, "TCP", "80", action="Allow")])
    assert e.value.errno == 7  # E2BIG


def test_same_order_twice_overlays_fields_like_go():
    """Two rules with one order write the same slot field by field (loader.go:437-514)."""
    val = infw.make_rules_val([infw.ProtocolRule(4, "TCP", "100-200", action="Allow"),
                               infw.ProtocolRule(4, "ICMP", icmp_type=8, action="Deny")])
    r = val.rules[4]
    assert (r.ruleId, r.protocol, r.dstPortStart, r.dstPortEnd, r.icmpType, r.action) == (4, 1, 100, 200, 8, 1)


def test_statistics_sum_and_overflow_rule():
    from infw.controller import add_uint64
    assert add_uint64(0, 5) == (5, True)
    assert add_uint64(2**64 - 1, 1) == (0, False)
    assert add_uint64(2**63, 2**62) == (2**63 + 2**62, True)


def test_debug_lookup_env_go_atoi():
    """ENABLE_EBPF_LPM_LOOKUP_DBG -> debug_lookup constant (loader.go:72-83): strconv.Atoi, uint32 wrap."""
    from infw.controller import IngNodeFwController, go_atoi
    assert go_atoi("1") == 1 and go_atoi("+7") == 7 and go_atoi("-1") == -1 and go_atoi("007") == 7
    for bad in ("", " 1", "1 ", "0x10", "1.0", "+", "٣", "9223372036854775808"):
        with pytest.raises(ValueError):
            go_atoi(bad)
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    IngNodeFwController(c, lambda n: [1], environ={"ENABLE_EBPF_LPM_LOOKUP_DBG": "1"})
    IngNodeFwController(c, lambda n: [1], environ={})
    with pytest.raises(ValueError):
        IngNodeFwController(c, lambda n: [1], environ={"ENABLE_EBPF_LPM_LOOKUP_DBG": "yes"})
    assert c.debug_keys() == []   # host-only context: no device sets
