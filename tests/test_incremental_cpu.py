"""Incremental commits on the CPU: the patched host image must
classify exactly like the oracle after every commit, and like a context that
recompiles every epoch (INFW_F_FULL_COMMIT).  infw_debug_walk runs the kernel's
lookup code over the committed host image — the bytes the devices receive.
"""
import ipaddress
import random
import struct

import numpy as np
import pytest

import infw
import orc
from infw import workloads as W
from frames import frame, snapshots
from test_compiler_cpu import _clustered_table, _val

PROTOS = ["tcp", "udp", "sctp", "icmp", "icmpv6", "gre"]


def _src_in(key: bytes, rng) -> str:
    """A source address inside the key's prefix (random host bits), in the family the key was written with."""
    plen, _ = struct.unpack("<II", key[:8])
    P = plen - 32
    ip = int.from_bytes(key[8:24], "big")
    v4 = ip & ((1 << 96) - 1) == 0 and P <= 32 and rng.random() < 0.8
    if v4:
        a = (ip >> 96) >> (32 - P) << (32 - P) if P else 0
        a |= rng.getrandbits(32 - P) if P < 32 else 0
        return str(ipaddress.IPv4Address(a))
    a = ip >> (128 - P) << (128 - P) if P else 0
    a |= rng.getrandbits(128 - P) if P < 128 else 0
    return str(ipaddress.IPv6Address(a))


def _packets_for(keys, rng, per_key=4):
    fr, ifx = [], []
    for k in keys:
        _, i = struct.unpack("<II", k[:8])
        for _ in range(per_key):
            fr.append(frame(_src_in(k, rng), proto=rng.choice(PROTOS), dport=rng.randrange(65536),
                            icmp_type=rng.randrange(256), icmp_code=rng.randrange(4), length=rng.randrange(60, 1500)))
            ifx.append(i)
    hdr, cap, pl = snapshots(fr)
    return hdr, cap, pl, np.array(ifx, np.uint32)


def _apply(ctxs, m, k, v):
    """v None = delete; the same edit on every context and on the oracle map, identical return codes."""
    if v is None:
        want = m.delete(k)
        for c in ctxs:
            assert c.delete_rc(infw.LpmIpKeySt.from_buffer_copy(k)) == want
    else:
        want = m.update(k, v)
        for c in ctxs:
            assert c.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v)) == want


def _check(ctxs, m, hdr, cap, pl, ifx, what):
    want, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=4)
    tup = W.pack_frames(hdr, cap, pl, ifx)
    for c in ctxs:
        got = c.debug_walk(tup)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (what, c.info()["commit_mode"], bad[:5], got[bad[:5]], want[bad[:5]])


@pytest.mark.parametrize("d16", ["0", "1"])
def test_incremental_churn_matches_oracle_and_full(monkeypatch, d16):
    """Random edit batches, each committed incrementally (or by the fallback) and fully: both images walk like
    the oracle, with and without /16 words in front of DIR-24-8 (re-derived for every /16 an edit covers,
    /8../32 edits)."""
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "d16", int(d16))
    rng = random.Random(23)
    entries, anchors = _clustered_table(rng, n_groups=30)
    inc = infw.Classifier(flags=infw.F_HOST_ONLY)
    full = infw.Classifier(flags=infw.F_HOST_ONLY | infw.F_FULL_COMMIT)
    m = orc.OracleMap()
    for k, v in entries:
        _apply((inc, full), m, k, v)
    inc.commit()
    full.commit()
    assert inc.info()["commit_mode"] == infw.COMMIT_FULL
    assert inc.info()["d16"] == full.info()["d16"] == int(d16)
    live = dict(entries)
    modes = []
    for step in range(12):
        touched = []
        for _ in range(rng.choice([1, 5, 40, 150])):
            r = rng.random()
            if r < 0.3 and live:                       # delete
                k = rng.choice(list(live))
                del live[k]
                _apply((inc, full), m, k, None)
            elif r < 0.6 and live:                     # new value for an existing key (new or shared list)
                k = rng.choice(list(live))
                live[k] = _val(rng, 7) if rng.random() < 0.5 else rng.choice(list(live.values()))
                _apply((inc, full), m, k, live[k])
            else:                                      # new key on a known ifindex
                ifx, top = rng.choice(anchors)
                if rng.random() < 0.5:                 # IPv6 long prefix in a known or a new /32 group
                    t = top if rng.random() < 0.6 else rng.getrandbits(32)
                    L = rng.choice([33, 48, 56, 64, 65, 100, 128])
                    ip = ((t << 96) | rng.getrandbits(96)).to_bytes(16, "big")
                else:                                  # <= /32: IPv4-written, nested under existing ones or not
                    L = rng.choice([8, 12, 16, 20, 23, 24, 25, 27, 30, 32])
                    a = top if rng.random() < 0.5 else rng.getrandbits(32)
                    ip = a.to_bytes(4, "big") + b"\0" * 12
                k = struct.pack("<II", L + 32, ifx) + ip
                live[k] = _val(rng, 9)
                _apply((inc, full), m, k, live[k])
            touched.append(k)
        inc.commit()
        full.commit()
        info = inc.info()
        modes.append((info["commit_mode"], info["full_reason"]))
        assert full.info()["commit_mode"] == infw.COMMIT_FULL
        assert info["n_entries"] == full.info()["n_entries"] == len(m)
        _check((inc, full), m, *_packets_for(touched, rng), f"step {step}: edited prefixes")
        _check((inc, full), m, *_packets_for(rng.sample(list(live), min(300, len(live))), rng), f"step {step}: all")
    assert sum(md == infw.COMMIT_INCREMENTAL for md, _ in modes) >= 4, modes


def test_incremental_on_workload_table():
    """configs[2] shape (100k prefixes): small edit batches stay incremental and bit-exact (300 mixed IPv4 / IPv6
    edits per commit: the IPv6 bucket phase runs on its own thread beside the short-table phase)."""
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=100000, n_templates=512)
    ents = list(wl.entries())
    inc = infw.Classifier(flags=infw.F_HOST_ONLY)
    m = orc.OracleMap()
    for k, v in ents:
        _apply((inc,), m, k, v)
    inc.commit()
    rng = random.Random(5)
    vals = [v for _, v in ents[:2000]]
    for step in range(4):
        touched = []
        for k, _ in rng.sample(ents, 300):
            v = None if rng.random() < 0.3 else (rng.choice(vals) if rng.random() < 0.7 else _val(rng, 3))
            _apply((inc,), m, k, v)
            touched.append(k)
        inc.commit()
        info = inc.info()
        assert info["commit_mode"] == infw.COMMIT_INCREMENTAL, info["full_reason"]
        assert info["compile_ms"] < 2000
        _check((inc,), m, *_packets_for(touched, rng, 2), f"step {step}: edited")
        hdr, cap, pl, ifx = wl.frames(step * 20000, 20000)
        _check((inc,), m, hdr, cap, pl, ifx, f"step {step}: workload")


def test_commit_reasons():
    """Layout changes fall back to a full compile and say why."""
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    v = _val(random.Random(1), 1)
    key = lambda ifx, cidr: infw.LpmIpKeySt.from_buffer_copy(__import__("goenc").build_key(ifx, cidr))
    val = infw.RulesValSt.from_buffer_copy(v)
    c.update(key(1, "10.0.0.0/8"), val)
    c.commit()
    c.update(key(1, "10.1.0.0/16"), val)
    c.commit()
    assert c.info()["commit_mode"] == infw.COMMIT_INCREMENTAL
    c.update(key(2, "10.1.0.0/16"), val)
    c.commit()
    assert c.info()["commit_mode"] == infw.COMMIT_FULL and c.info()["full_reason"] == "new ifindex"
    c.update(key(2, "2001:db8::/48"), val)
    c.commit()
    assert c.info()["full_reason"] == "first long prefix"
    c.commit()  # nothing pending
    assert c.info()["commit_mode"] == infw.COMMIT_INCREMENTAL and c.info()["patch_bytes"] == 0


def test_lists_past_the_part_count_table_stay_incremental():
    """An epoch compiled with per-list part counts (<= 4096 lists, INFW_DT_PL_LISTS) takes new rule lists past the
    table incrementally: they keep uniform value parts (infw_dt_parts_of), and the patched image classifies like
    the oracle (round 2 recompiled the whole epoch — 2 s at configs[2] — for one new list)."""
    import random
    from tools_commit import new_value
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=30000, n_templates=4096)
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 4096)
    wl.load_into(c)
    c.commit()
    n0 = c.info()["n_lists"]
    assert n0 > 4000
    m = orc.OracleMap(max_entries=wl.n_entries + 4096)
    for k, v in wl.entries():
        m.update(k, v)
    rng = random.Random(3)
    keys = [k for k, _ in wl.entries()]
    for rnd in range(3):
        touched = rng.sample(keys, 300)
        for k in touched:
            _apply([c], m, k, new_value(rng))
        c.commit()
        i = c.info()
        assert i["commit_mode"] == infw.COMMIT_INCREMENTAL, i["full_reason"]
        hdr, cap, pl, ifx = _packets_for(touched[:150], rng)
        tup = W.pack_frames(hdr, cap, pl, ifx)
        ro, _, _, _ = m.classify_frames(hdr, cap, pl, ifx)
        assert np.array_equal(c.debug_walk(tup), ro), rnd
    assert c.info()["n_lists"] > max(n0, 4096)
