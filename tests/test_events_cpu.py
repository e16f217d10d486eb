"""Deny-event payload and consumer on the CPU (§8f-1).

The oracle's perf samples (orc_perf_sample: kernel.c:392-399 + perf's raw-record sizing) and the product's
consumer (infw/events.py: events.go:77-166 over a restatement of the gopacket decoders it uses) on known-answer
frames.  Expected lines are written out by hand from the Go format strings; the reference holds no fixture for
them (its events path has no test), so they pin the restatement only as far as these cases go.
The device side (infw_events_capture vs the oracle's samples) is tests/test_gpu_parity.py::test_event_samples.
"""
import struct

import numpy as np

import goenc
import orc
from frames import frame
from infw import events as E

NAMES = {1: "eth0", 2: "bond0"}


def samples_for(frames, ifx, table, pkt_len=None):
    m = orc.OracleMap()
    for k, v in table:
        assert m.update(k, v) == 0
    buf = np.frombuffer(b"".join(frames), np.uint8)
    offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
    lin = np.array([len(f) for f in frames], np.uint32)
    pl = lin.copy() if pkt_len is None else np.asarray(pkt_len, np.uint32)
    return m.collect_event_samples(buf, offs, lin, pl, np.asarray(ifx, np.uint32))


def deny_all(ifindex, cidr, rule_id=7):
    return (goenc.build_key(ifindex, cidr),
            goenc.raw_value([{"slot": 1, "ruleId": rule_id, "protocol": 0, "dstPortStart": 0, "dstPortEnd": 0,
                              "icmpType": 0, "icmpCode": 0, "action": 1}]))


def test_perf_sample_layout():
    f = frame("10.1.2.3", "192.0.2.9", "tcp", dport=80, sport=1234, length=60)
    recs, s = samples_for([f], [1], [deny_all(1, "10.0.0.0/8")])
    assert recs.tolist() == [[0, 1, 7, 1, 60, 60]]
    size = int(s[0, :4].view("<u4")[0])
    assert size == 68 and (size + 4) % 8 == 0               # round_up(8 + 60 + 4, 8) - 4
    assert bytes(s[0, 4:12]) == struct.pack("<HHBBH", 1, 7, 1, 0, 60)
    assert bytes(s[0, 12:72]) == f and not s[0, 72:].any()


def test_decode_known_answers():
    frames = [frame("10.1.2.3", "192.0.2.9", "tcp", dport=80, sport=1234),
              frame("10.1.2.4", "198.51.100.7", "udp", dport=53, sport=5353),
              frame("10.1.2.5", "192.0.2.1", "icmp", icmp_type=8, icmp_code=0),
              frame("10.1.2.6", "192.0.2.1", "sctp", dport=3868, sport=2905),
              frame("2001:db8:0:0:1::5", "2001:db8::1", "icmpv6", icmp_type=128, icmp_code=0),
              frame("2001:db8::7", "::ffff:192.0.2.1", "tcp", dport=443, sport=50000)]
    recs, s = samples_for(frames, [1, 1, 1, 2, 2, 2], [deny_all(1, "10.0.0.0/8"), deny_all(2, "10.0.0.0/8", 9),
                                                        deny_all(2, "2001:db8::/32", 11)])
    assert recs.shape[0] == 6
    lines, log = E.drain(s, recs.shape[0], NAMES.get)
    assert log == []
    assert lines == [
        "ruleId 7 action Drop len 54 if eth0\n", "\tipv4 src addr 10.1.2.3 dst addr 192.0.2.9\n",
        "\ttcp srcPort 1234 dstPort 80\n",
        "ruleId 7 action Drop len 42 if eth0\n", "\tipv4 src addr 10.1.2.4 dst addr 198.51.100.7\n",
        "\tudp srcPort 5353 dstPort 53\n",
        "ruleId 7 action Drop len 42 if eth0\n", "\tipv4 src addr 10.1.2.5 dst addr 192.0.2.1\n",
        "\ticmpv4 type 8 code 0\n",
        "ruleId 9 action Drop len 46 if bond0\n", "\tipv4 src addr 10.1.2.6 dst addr 192.0.2.1\n",
        "\tsctp srcPort 2905 dstPort 3868\n",
        "ruleId 11 action Drop len 62 if bond0\n", "\tipv6 src addr 2001:db8::1:0:0:5 dst addr 2001:db8::1\n",
        "\ticmpv6 type 128 code 0\n",
        "ruleId 11 action Drop len 74 if bond0\n", "\tipv6 src addr 2001:db8::7 dst addr 192.0.2.1\n",
        "\ttcp srcPort 50000 dstPort 443\n"]


def test_decode_length_edges():
    """PktLength is the frame length (u16), not the captured size: a frame longer than the 256 captured bytes plus
    perf's 4 pad bytes fails binary.Read and logs nothing but the parse error; 257..260 still decodes."""
    table = [deny_all(1, "10.0.0.0/8")]
    frames = [frame("10.9.9.9", "192.0.2.2", "tcp", dport=22, length=258),
              frame("10.9.9.8", "192.0.2.2", "tcp", dport=22, length=300)]
    recs, s = samples_for(frames, [1, 1], table)
    assert [int(r[5]) for r in recs] == [256, 256]
    assert [int(x) for x in s[:, :4].copy().view("<u4")[:, 0]] == [268, 268]
    lines, log = E.drain(s, 2, NAMES.get)
    assert lines == ["ruleId 7 action Drop len 258 if eth0\n", "\tipv4 src addr 10.9.9.9 dst addr 192.0.2.2\n",
                     "\ttcp srcPort 40000 dstPort 22\n"]
    assert log == ["Parsing perf event packet header : unexpected EOF"]
    # multi-buffer frame: pkt_len 1000 over a 60-B linear part: 256 captured bytes, those past 60 zero
    f = frame("10.9.9.7", "192.0.2.3", "udp", dport=9, length=60)
    recs, s = samples_for([f], [1], table, pkt_len=[1000])
    assert recs[0, 4] == 1000 and recs[0, 5] == 256
    assert bytes(s[0, 12:72]) == f and not s[0, 72:].any()


def test_decode_gopacket_quirks():
    table = [deny_all(1, "10.0.0.0/8")]
    f = bytearray(frame("10.1.1.1", "192.0.2.4", "tcp", dport=80))
    frag = bytearray(f)
    frag[20:22] = b"\x20\x00"                          # IPv4 more-fragments: Fragment layer, no TCP line
    short = bytearray(f)
    short[16:18] = struct.pack("!H", 24)               # total length 24: 4 TCP bytes -> TCP layer with zero ports
    mapped_src = frame("::ffff:10.1.1.2", "2001:db8::9", "udp", dport=7)  # an IPv6 header with a v4-mapped source
    recs, s = samples_for([bytes(frag), bytes(short)], [1, 1], table)
    lines, _ = E.drain(s, 2, NAMES.get)
    assert lines == ["ruleId 7 action Drop len 54 if eth0\n", "\tipv4 src addr 10.1.1.1 dst addr 192.0.2.4\n",
                     "ruleId 7 action Drop len 54 if eth0\n", "\tipv4 src addr 10.1.1.1 dst addr 192.0.2.4\n",
                     "\ttcp srcPort 0 dstPort 0\n"]
    ly = E.gopacket_layers(mapped_src)
    assert E.go_ip_string(ly["ipv6"]["src"]) == "10.1.1.2" and ly["udp"] == {"sport": 40000, "dport": 7}
    # unknown interface: the record is skipped with the lookup error (events.go:98-102)
    recs, s = samples_for([frame("10.1.1.3", proto="tcp", dport=1)], [1], table)
    lines, log = E.drain(s, 1, {}.get)
    assert lines == [] and log[0].startswith("lookup network iface 1:")


def test_lost_samples_line():
    recs, s = samples_for([frame("10.1.1.%d" % i, proto="tcp", dport=1) for i in range(3)], [1] * 3,
                          [deny_all(1, "10.0.0.0/8")])
    lines, log = E.drain(s[:2], 5, NAMES.get)  # 5 events, a 2-slot ring
    assert log == ["Perf event ring buffer full, dropped 3 samples"] and len(lines) == 6
