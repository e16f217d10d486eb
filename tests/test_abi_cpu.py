"""C ABI on a CPU-only box: the library loads, exports every symbol include/*.h
declares, and its table-map semantics equal the oracle's LPM-trie map
(update flags / ENOSPC / delete / LPM lookup / get_next_key post-order)."""
import ctypes as C
import os
import random
import re
import struct

import pytest

import infw
import orc
from infw import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    """Every function include/*.h declares (infw.h, infw_host.h)."""
    inc = os.path.join(ROOT, "include")
    src = "\n".join(open(os.path.join(inc, f)).read() for f in sorted(os.listdir(inc)) if f.endswith(".h"))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*(infw_\w+)\s*\(", src, flags=re.M)))


def test_exports_every_declared_symbol():
    decl = header_functions()
    assert len(decl) >= 20
    assert sorted(N.ABI_SYMBOLS) == decl
    for name in decl:
        assert hasattr(N.lib, name), name
    assert N.lib.infw_abi_version() == 4


def test_struct_sizes_match_reference_abi():
    assert C.sizeof(infw.LpmIpKeySt) == 24 and C.sizeof(infw.RulesValSt) == 1200
    assert C.sizeof(infw.RuleTypeSt) == 12 and C.sizeof(infw.RuleStatisticsSt) == 32


def test_no_device_means_no_classifier():
    """Without a HIP device a classifying context cannot be created: there is no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(infw.InfwError) as e:
        infw.Classifier()
    assert e.value.errno == 19  # ENODEV
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    rc = N.lib.infw_classify(c._ctx, 0, C.byref(N.BatchSoa(1, 1, 1, 1, 1)), 1, None, None, None)
    assert rc == -19
    rc = N.lib.infw_classify_frames(c._ctx, 0, C.byref(N.FrameBatch(1, None, 64, 1, None, 1)), 1, None, None, None)
    assert rc == -19


def key(plen, ifx, ip: bytes):
    return struct.pack("<II", plen, ifx) + ip.ljust(16, b"\0")


VAL_A = bytes(1200)
VAL_B = struct.pack("<IBHHBBB", 7, 0, 0, 0, 0, 0, 1) * 100


def test_update_flags_and_errors_match_oracle():
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=3)
    m = orc.OracleMap(max_entries=3)
    K = infw.LpmIpKeySt.from_buffer_copy
    V = infw.RulesValSt.from_buffer_copy
    cases = [
        (key(56, 1, b"\x01\x01\x01\x07"), VAL_A, 0),        # new
        (key(56, 1, b"\x01\x01\x01\x99"), VAL_B, 1),        # same /24 prefix, other host bits: EEXIST
        (key(56, 1, b"\x01\x01\x01\x99"), VAL_B, 2),        # EXIST: replace
        (key(64, 1, b"\x02\x02\x02\x02"), VAL_A, 2),        # EXIST on a missing key: ENOENT
        (key(64, 1, b"\x02\x02\x02\x02"), VAL_A, 3),        # flags > BPF_EXIST: EINVAL
        (key(161, 1, b""), VAL_A, 0),                      # prefixLen > 160: EINVAL
        (key(64, 1, b"\x02\x02\x02\x02"), VAL_A, 0),
        (key(160, 9, bytes(range(16))), VAL_B, 0),
        (key(40, 3, b"\x0a"), VAL_A, 0),                    # 4th entry on a 3-entry map: ENOSPC
        (key(64, 1, b"\x02\x02\x02\x02"), VAL_B, 0),        # replace on a full map: allowed
    ]
    for k, v, f in cases:
        assert c.update_rc(K(k), V(v), f) == m.update(k, v, f), (k.hex(), f)
    assert c.count() == len(m) == 3
    # delete by exact prefix, host bits ignored; ENOENT when absent
    for k in (key(56, 1, b"\x01\x01\x01\x00"), key(56, 1, b"\x01\x01\x01\x00"), key(48, 1, b"\x01\x01")):
        assert c.delete_rc(K(k)) == m.delete(k)


def random_key(rng):
    ifx = rng.choice([1, 2, 0xFFFFFFFF])
    # prefixLen < 32: partial-ifindex prefixes (never written by BuildEBPFKey, accepted by the LPM trie)
    plen = rng.choice([0, 8, 16, 31, 32, 33, 40, 48, 56, 63, 64, 65, 80, 96, 128, 150, 159, 160])
    ip = bytes(rng.getrandbits(8) for _ in range(16))
    if rng.random() < 0.5:  # nested / shared prefixes
        ip = bytes([10, 20]) + ip[2:]
    return key(plen, ifx, ip)


def test_random_map_ops_match_oracle():
    rng = random.Random(5)
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=200)
    m = orc.OracleMap(max_entries=200)
    K = infw.LpmIpKeySt.from_buffer_copy
    vals = [bytes(rng.getrandbits(8) for _ in range(1200)) for _ in range(5)]
    keys = [random_key(rng) for _ in range(300)]
    for step in range(3000):
        k = rng.choice(keys)
        op = rng.random()
        if op < 0.5:
            v, f = rng.choice(vals), rng.choice([0, 0, 1, 2])
            assert c.update_rc(K(k), infw.RulesValSt.from_buffer_copy(v), f) == m.update(k, v, f)
        elif op < 0.7:
            assert c.delete_rc(K(k)) == m.delete(k)
        else:  # LPM lookup with an arbitrary prefixLen
            q = k[:4] if rng.random() < 0.5 else struct.pack("<I", rng.choice([8, 32, 64, 100, 160]))
            q = q + k[4:]
            got = c.lookup(K(q))
            want = m.lookup(q)
            assert (None if got is None else bytes(got)) == want, step
    # full iteration: identical key bytes in identical (post-)order
    assert [bytes(k) for k, _ in c.iterate()] == list(m.keys())
    # get_next_key of an absent key restarts at the first key
    absent = key(160, 77, b"\xff" * 16)
    assert bytes(c.next_key(K(absent))) == m.next_key(absent) == next(iter(m.keys()))


def test_key_order_through_churn_merges_and_commits():
    """get_next_key's lazily merged order (sorted keys + keys inserted since the last merge, removed keys skipped,
    tombstones dropped at commit) against the oracle's post-order, past the 4096-insert merge threshold."""
    rng = random.Random(11)
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=20000)
    m = orc.OracleMap(max_entries=20000)
    K = infw.LpmIpKeySt.from_buffer_copy
    vals = [bytes(rng.getrandbits(8) for _ in range(1200)) for _ in range(3)]
    keys = list({random_key(rng) for _ in range(9000)})
    for rnd in range(4):
        for k in rng.sample(keys, 5000):
            v = rng.choice(vals)
            assert c.update_rc(K(k), infw.RulesValSt.from_buffer_copy(v), 0) == m.update(k, v, 0)
        for k in rng.sample(keys, 2500):
            assert c.delete_rc(K(k)) == m.delete(k)
        if rnd % 2:
            c.commit()
        want = list(m.keys())
        assert c.count() == len(want)
        assert [bytes(k) for k, _ in c.iterate()] == want, rnd
        for _ in range(50):  # next_key from present keys
            i = rng.randrange(len(want))
            nxt = c.next_key(K(want[i]))
            assert (None if nxt is None else bytes(nxt)) == (want[i + 1] if i + 1 < len(want) else None)


def test_commit_epoch_counts():
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    e0 = c.info()["epoch"]
    c.update(infw.build_ebpf_key(1, "10.0.0.0/8"), infw.RulesValSt())
    c.commit()
    c.commit()
    assert c.info()["epoch"] == e0 + 2 and c.info()["n_entries"] == 1


def test_prefix_shorter_than_ifindex_accepted():
    """lpm_trie accepts prefixLen < 32 (a partial ifindex); so does the map — matching is tests/test_golden.py's."""
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    m = orc.OracleMap()
    k = key(24, 1, b"")
    assert c.update_rc(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt()) == m.update(k, bytes(1200)) == 0
    assert bytes(c.lookup(infw.LpmIpKeySt.from_buffer_copy(key(64, 1, b"\x0a\0\0\x01")))) == bytes(1200)
    c.commit()
