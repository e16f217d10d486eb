"""Table compiler (host side of the GPU tables) against the oracle, on the CPU.

The product compiles the table map into DIR-24-8 + IPv6 /32 buckets +
Waldvogel overflow table + class-filtered rule lists; infw_debug_walk runs the
kernel's lookup code over that image on the host.  These tests compare it with
the oracle on the BASELINE workloads and on adversarial random tables.
"""
import os
import random
import struct

import numpy as np
import pytest

import infw
import orc
from infw import workloads as W


def walk_vs_oracle(entries, tuples_from, n=20000, seed=1):
    """entries: list of (key bytes, value bytes)."""
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    m = orc.OracleMap()
    for k, v in entries:
        rc = c.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v))
        assert rc == m.update(k, v)
    c.commit()
    hdr, cap, pl, ifx = tuples_from(n, seed)
    res, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=4)
    got = c.debug_walk(W.pack_frames(hdr, cap, pl, ifx))
    bad = np.nonzero(got != res)[0]
    assert bad.size == 0, (bad[:5], got[bad[:5]], res[bad[:5]])
    return c, res


@pytest.mark.parametrize("cfg,npfx,ntmpl", [(W.CFG0_DEMO, 0, 0), (W.CFG1_V4_10K, 0, 0), (W.CFG2_MIXED_1M, 100000, 512),
                                            (W.CFG4_ADVERSARIAL, 20000, 64)])
def test_workloads(cfg, npfx, ntmpl):
    """The host walk of the compiled image equals the oracle."""
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    walk_vs_oracle(list(wl.entries()), lambda n, s: wl.frames(s * n, n))


@pytest.mark.parametrize("cfg,npfx,ntmpl", [(W.CFG1_V4_10K, 0, 0), (W.CFG2_MIXED_1M, 100000, 512),
                                            (W.CFG4_ADVERSARIAL, 20000, 64)])
@pytest.mark.parametrize("d16", ["0", "1"])
def test_workloads_d16_words(monkeypatch, cfg, npfx, ntmpl, d16):
    """/16 words in front of DIR-24-8 forced off / on (INFW_D16): the host walk (which reads them like the
    kernel) equals the oracle either way."""
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "d16", int(d16))
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    c, _ = walk_vs_oracle(list(wl.entries()), lambda n, s: wl.frames(s * n, n), n=30000)
    info = c.info()
    assert info["d16"] == int(d16)
    assert d16 == "0" or info["d16_permille"] > 0


def test_d16_chosen_for_sparse_short_tables(monkeypatch):
    """The automatic choice: configs[1] (10k /16../32 prefixes, one per /16 mostly) gets /16 words; a /16 packed
    with many BGP-like prefixes of several lists does not."""
    monkeypatch.delitem(infw.DEFAULT_OPTIONS, "d16", raising=False)
    wl = W.Workload(W.CFG1_V4_10K)
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    for k, v in wl.entries():
        c.update(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v))
    c.commit()
    assert c.info()["d16"] == 1 and c.info()["d16_permille"] > 800
    rng = random.Random(3)
    ents = []
    for b in range(64):  # 64 /16s, each holding 40 /24s and /28s of 8 lists: 4+ runs per /16
        for j in range(40):
            L = rng.choice([24, 28])
            a = (10 << 24) | (b << 16) | (rng.randrange(256) << 8) | (rng.randrange(16) << 4)
            k = struct.pack("<II", L + 32, 5) + a.to_bytes(4, "big") + b"\0" * 12
            ents.append((k, _val(random.Random(j % 8), 1)))
    c2, _ = walk_vs_oracle(ents, lambda n, s: _v4_frames_in(ents, n, s))
    assert c2.info()["d16"] == 0 and c2.info()["d16_permille"] < 500


def _v4_frames_in(ents, n, seed):
    from frames import frame, snapshots
    rng = random.Random(seed)
    fr, ifx = [], []
    for _ in range(n):
        k, _ = rng.choice(ents)
        plen, i = struct.unpack("<II", k[:8])
        a = int.from_bytes(k[8:12], "big") | rng.getrandbits(32 - (plen - 32))
        fr.append(frame("%d.%d.%d.%d" % tuple(a.to_bytes(4, "big")), proto=rng.choice(["tcp", "udp"]),
                        dport=rng.randrange(65536), length=100))
        ifx.append(i)
    hdr, cap, pl = snapshots(fr)
    return hdr, cap, pl, np.array(ifx, np.uint32)


def test_distinct_lists_parallel_compile(monkeypatch):
    """configs[2]'s distinct-lists variant (one 1200-B value per key, loader.go:158-161) at 12k keys: the
    rule lists compile on host threads (>= 4096 lists) into thread-local pools that are rebased; the walk
    must equal the oracle, and the image must equal a single-threaded compile's (same walk, same counts)."""
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=12000, n_templates=12000)
    assert wl.n_templates == 12000 and len(set(wl.val_index().tolist())) == 12000
    ents = list(wl.entries())
    c, res = walk_vs_oracle(ents, lambda n, s: wl.frames(s * n, n), n=30000)
    info = c.info()
    assert info["n_lists"] >= 11900
    monkeypatch.setitem(infw.DEFAULT_OPTIONS, "compile_threads", int("1"))
    c1, res1 = walk_vs_oracle(ents, lambda n, s: wl.frames(s * n, n), n=30000)
    i1 = c1.info()
    for k in ("n_lists", "n_rules", "dt_parts", "n_tbl8_groups"):
        assert info[k] == i1[k], k


def _val(rng, rid_base):
    import goenc
    rules = []
    for slot in rng.sample(range(1, 100), 6):
        proto = rng.choice([0, 6, 17, 132, 1, 58, 47])
        ps = rng.randrange(0, 65536)
        pe = rng.choice([0, 0, min(65535, ps + rng.randrange(0, 300)), rng.randrange(0, 65536)])
        rules.append({"slot": slot, "ruleId": rng.choice([slot, slot + rid_base, 0, 1024, 65536 + slot]),
                      "protocol": proto, "dstPortStart": ps, "dstPortEnd": pe, "icmpType": rng.randrange(256),
                      "icmpCode": rng.randrange(4), "action": rng.choice([1, 2, 2, 1, 0, 3])})
    return goenc.raw_value(rules)


def _clustered_table(rng, n_groups=40):
    """IPv6 prefixes clustered under few /32s (overflow groups), nested lengths 0..128 on 3 ifindexes,
    cross-family aliases, plus IPv4 nesting — every LPM corner the layout has."""
    ents = []
    anchors = []
    for g in range(n_groups):
        ifx = rng.choice([3, 4, 70000])
        top = rng.getrandbits(32)
        anchors.append((ifx, top))
        for _ in range(rng.choice([1, 2, 3, 4, 9, 25])):   # > 3 -> overflow group
            L = rng.choice([33, 40, 47, 48, 56, 63, 64, 65, 96, 127, 128])
            addr = (top << 96) | rng.getrandbits(96)
            ents.append((ifx, L + 32, addr.to_bytes(16, "big")))
        for L in (0, 8, 16, 24, 30, 32):                     # short prefixes over the same bits (v6-written)
            ents.append((ifx, L + 32, ((top << 96) | rng.getrandbits(96)).to_bytes(16, "big")))
    for _ in range(300):                                      # IPv4 nesting
        ifx = rng.choice([3, 4])
        a = rng.getrandbits(32) & 0xFFFFFF00 if rng.random() < 0.5 else rng.getrandbits(32)
        for L in (8, 16, 20, 24, 25, 28, 32):
            if rng.random() < 0.4:
                ents.append((ifx, L + 32, a.to_bytes(4, "big") + b"\0" * 12))
    out = []
    for i, (ifx, plen, ip) in enumerate(ents):
        out.append((struct.pack("<II", plen, ifx) + ip, _val(rng, i)))
    return out, anchors


def clustered_packets(anchors, n, seed):
    """Frames aimed at a _clustered_table: sources under its /32 anchors (IPv6 and IPv4-aliased), some on other
    ifindexes, every protocol; (hdr, caplen, pkt_len, ifindex)."""
    import ipaddress
    from frames import frame, snapshots
    r = random.Random(seed)
    fr, ifx = [], []
    for _ in range(n):
        i, top = r.choice(anchors)
        if r.random() < 0.15:
            i = r.choice([3, 4, 5, 70000])
        if r.random() < 0.7:
            src = str(ipaddress.IPv6Address((top << 96) | r.getrandbits(96)))
        elif r.random() < 0.5:
            src = str(ipaddress.IPv4Address(top))
        else:
            src = str(ipaddress.IPv4Address(r.getrandbits(32)))
        proto = r.choice(["tcp", "udp", "sctp", "icmp", "icmpv6", 1, 58, "gre"])
        fr.append(frame(src, proto=proto, dport=r.randrange(65536), icmp_type=r.randrange(256),
                        icmp_code=r.randrange(4), length=r.randrange(60, 1500)))
        ifx.append(i)
    hdr, cap, pl = snapshots(fr)
    return hdr, cap, pl, np.array(ifx, np.uint32)


def test_clustered_overflow_groups():
    rng = random.Random(7)
    entries, anchors = _clustered_table(rng)
    c, res = walk_vs_oracle(entries, lambda n, seed: clustered_packets(anchors, n, seed), n=6000)
    info = c.info()
    assert info["n_v6_overflow"] > 0 and info["n_v6_groups"] > info["n_v6_overflow"]
    assert (res != 0).mean() > 0.3


def test_update_delete_churn_matches_oracle():
    """Random update/delete/commit churn: the compiled image tracks the map exactly."""
    rng = random.Random(11)
    entries, anchors = _clustered_table(rng, n_groups=15)
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    m = orc.OracleMap()
    from frames import frame, snapshots
    fr = [frame(str(__import__("ipaddress").IPv6Address((t << 96) | rng.getrandbits(96))), proto="udp",
                dport=rng.randrange(65536)) for _, t in anchors for _ in range(20)]
    ifx = np.array([i for i, _ in anchors for _ in range(20)], np.uint32)
    hdr, cap, pl = snapshots(fr)
    tup = W.pack_frames(hdr, cap, pl, ifx)
    for step in range(6):
        for k, v in rng.sample(entries, len(entries) // 3):
            if rng.random() < 0.4:
                assert c.delete_rc(infw.LpmIpKeySt.from_buffer_copy(k)) == m.delete(k)
            else:
                assert c.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v)) == \
                    m.update(k, v)
        c.commit()
        res, _, _, _ = m.classify_frames(hdr, cap, pl, ifx)
        assert np.array_equal(c.debug_walk(tup), res), step


def test_decision_tables_exhaustive_values():
    """Every 16-bit packet value for every packet class of random 100-slot rule lists: the compiled
    first-match decision tables (and, inside infw_debug_walk, the serial class-list scan) equal the
    oracle's scan of the raw rulesVal_st — compact (u8 result code) and u32 leaf forms alike."""
    rng = random.Random(3)
    import goenc
    from frames import frame, snapshots
    ents = []
    for t in range(6):
        rules = []
        for slot in range(1, 100):
            if rng.random() < 0.35:
                continue
            proto = rng.choice([6, 6, 17, 17, 132, 1, 58, 0, 47]) if slot > 60 or rng.random() < 0.97 else 0
            ps = rng.randrange(0, 65536)
            kind = rng.random()
            pe = 0 if kind < 0.4 else min(65535, ps + rng.randrange(1, 4000)) if kind < 0.9 else rng.randrange(0, 65536)
            # t < 4: what the control plane writes (ruleId = order, Allow/Deny) -> compact leaves;
            # t = 4: rule ids above 127, t = 5: actions outside {1, 2} -> u32 leaves
            rid = slot + (100000 if t == 4 else 0)
            act = rng.choice([0, 1, 2, 3, 200]) if t == 5 else rng.choice([1, 2])
            rules.append({"slot": slot, "ruleId": rid, "protocol": proto, "dstPortStart": ps, "dstPortEnd": pe,
                          "icmpType": rng.randrange(256), "icmpCode": rng.randrange(256),
                          "action": act})
        ents.append((goenc.build_key(9, f"10.{t}.0.0/16"), goenc.raw_value(rules)))
        ents.append((goenc.build_key(9, f"2001:db8:{t}::/48"), goenc.raw_value(rules)))
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    m = orc.OracleMap()
    for k, v in ents:
        c.update(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v))
        assert m.update(k, v) == 0
    c.commit()
    vals = np.arange(65536, dtype=np.uint32)
    for t in range(6):
        for src, proto in ((f"10.{t}.1.1", 6), (f"10.{t}.1.1", 17), (f"10.{t}.1.1", 132), (f"10.{t}.1.1", 1),
                           (f"10.{t}.1.1", 58), (f"2001:db8:{t}::9", 6), (f"2001:db8:{t}::9", 58),
                           (f"2001:db8:{t}::9", 1), (f"2001:db8:{t}::9", 132)):
            base = frame(src, proto=proto, dport=0, length=100)
            tup = np.repeat(W.pack_frames(*snapshots([base]), np.array([9], np.uint32)), 65536, axis=0)
            if proto in (1, 58):
                tup[:, 7] = (vals >> 8) | ((vals & 0xFF) << 8)          # l4word bytes 0,1 = type, code
            else:
                tup[:, 7] = ((vals >> 8) << 16) | ((vals & 0xFF) << 24)  # bytes 2,3 = dport (network order)
            got = c.debug_walk(tup)
            # oracle on the same 65536 frames
            hdr = np.repeat(snapshots([base])[0], 65536, axis=0)
            off = 34 if "." in src else 54
            if proto in (1, 58):
                hdr[:, off], hdr[:, off + 1] = vals >> 8, vals & 0xFF
            else:
                hdr[:, off + 2], hdr[:, off + 3] = vals >> 8, vals & 0xFF
            n = np.full(65536, 100, np.uint32)
            want, _, _, _ = m.classify_frames(hdr, n, n, np.full(65536, 9, np.uint32), nthreads=4)
            assert np.array_equal(got, want), (t, src, proto, np.nonzero(got != want)[0][:5])


def test_host_sanitizer_walk():
    """tools/asan_walk.cpp under AddressSanitizer/UBSan: the compiler and the shared
    host/device walk over random tables in every short-table form (incl. a DIR-24-8
    build with no <= /32 entry), decision tables checked against the serial scan."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    from conftest import run_make
    r = run_make("asan", timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]
    # the same harness with /16 words in front of DIR-24-8 forced on (built per compile, re-derived by every
    # patched commit; the harness passes the option to the compiler)
    env = dict(os.environ, ASAN_D16="1", ASAN_CHURN_ROUNDS="3")
    r = subprocess.run([os.path.join(root, "ingress-node-firewall_amd", "build", "asan_walk")], cwd=root, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]


def test_many_ifindexes_host_walk():
    """400 ifindexes (ifindex map outside the kernel's LDS copy, compressed short table chosen by size):
    the compiled image walked on the CPU equals the oracle (the GPU form is test_gpu_parity.test_many_ifindexes)."""
    import struct
    import orc
    from frames import snapshots  # noqa: F401
    from test_incremental_cpu import _packets_for
    rng = random.Random(400)
    ifs = rng.sample(range(1, 1 << 20), 400)
    ents = {}
    for i in range(6000):
        ifx = ifs[i % 400]
        if rng.random() < 0.6:
            L = rng.choice([0, 8, 16, 20, 24, 25, 28, 32])
            ip = rng.getrandbits(32).to_bytes(4, "big") + bytes(12)
        else:
            L = rng.choice([16, 32, 40, 48, 56, 64, 96, 128])
            ip = rng.getrandbits(128).to_bytes(16, "big")
        ents[struct.pack("<II", L + 32, ifx) + ip] = _val(rng, i)
    c = infw.Classifier(devices=[], max_entries=len(ents) + 16, flags=infw.F_HOST_ONLY)
    m = orc.OracleMap(max_entries=len(ents) + 16)
    for k, v in ents.items():
        assert c.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v)) == m.update(k, v)
    c.commit()
    hdr, cap, pl, ifx = _packets_for(rng.sample(list(ents), 2000), rng, 2)
    ifx[::7] = np.array([rng.randrange(1 << 20, 1 << 21) for _ in range(ifx[::7].size)], np.uint32)
    want, _, _, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=4)
    got = c.debug_walk(W.pack_frames(hdr, cap, pl, ifx))
    assert np.array_equal(got, want)
    assert c.info()["n_if_slots"] == 400
