"""Compiled-epoch images (infw_table_export / infw_table_import) on the CPU: an imported context is the exporter's
committed epoch — the same key walk (get_next_key post-order), lookups, compiled host tables (debug walk over
packets of every key) — and keeps behaving like it under later incremental edits, which commit incrementally on the
import (the incremental-commit state travels with the image).  Error paths: import into a non-empty context,
a truncated or corrupted image, another build's image, export with uncommitted edits."""
import ctypes as C
import os
import random

import numpy as np
import pytest

import infw
import orc
from infw import _native as N
from infw import workloads as W
from test_incremental_cpu import _apply, _packets_for


def _wl_ctx(cfg=W.CFG2_MIXED_1M, npfx=20000, ntmpl=64):
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 4096)
    wl.load_into(c)
    c.commit()
    return wl, c


def _keys(c):
    out, k = [], c.next_key(None)
    while k is not None:
        out.append(bytes(k))
        k = c.next_key(k)
    return out


@pytest.mark.parametrize("cfg", [W.CFG1_V4_10K, W.CFG2_MIXED_1M, W.CFG4_ADVERSARIAL])
def test_import_equals_export(cfg):
    wl, a = _wl_ctx(cfg)
    img = a.export_image()
    assert len(img) == a.export_size()
    b = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 4096)
    b.import_image(img)
    ia, ib = a.info(), b.info()
    assert ib["imported"] == 1 and ib["full_reason"] == "imported"
    for f in ("n_entries", "n_lists", "n_rules", "n_tbl8_groups", "n_long_levels", "n_v6_groups", "dt_parts",
              "short_mode"):
        assert ia[f] == ib[f], f
    assert b.count() == a.count() > 0
    ka = _keys(a)
    assert ka == _keys(b)
    rng = random.Random(5)
    for k in rng.sample(ka, 200):
        lk = infw.LpmIpKeySt.from_buffer_copy(k)
        assert bytes(a.lookup(lk)) == bytes(b.lookup(lk))
    t = wl.tuples(0, 1 << 16)
    assert np.array_equal(a.debug_walk(t), b.debug_walk(t))
    assert b.export_image() == img  # the imported epoch exports the same bytes


def test_import_then_incremental_edits_track_the_exporter():
    wl, a = _wl_ctx(W.CFG2_MIXED_1M, 5000, 32)
    b = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 4096)
    b.import_image(a.export_image())
    m = orc.OracleMap(max_entries=wl.n_entries + 4096)
    for k, v in wl.entries():
        m.update(k, v)
    rng = random.Random(11)
    keys = [k for k, _ in wl.entries()]
    vals = [v for _, v in wl.entries()]
    for rnd in range(4):
        touched = []
        for _ in range(200):
            k = rng.choice(keys)
            _apply([a, b], m, k, None if rng.random() < 0.3 else rng.choice(vals))
            touched.append(k)
        a.commit()
        b.commit()
        assert b.info()["commit_mode"] == a.info()["commit_mode"] == infw.COMMIT_INCREMENTAL, b.info()["full_reason"]
        hdr, cap, pl, ifx = _packets_for(touched[:100], rng)
        tup = W.pack_frames(hdr, cap, pl, ifx)
        ra, rb = a.debug_walk(tup), b.debug_walk(tup)
        ro, _, _, _ = m.classify_frames(hdr, cap, pl, ifx)
        assert np.array_equal(ra, rb) and np.array_equal(rb, ro), rnd
    assert _keys(a) == _keys(b)


def test_import_errors():
    wl, a = _wl_ctx(W.CFG1_V4_10K, 2000, 16)
    img = a.export_image()
    b = infw.Classifier(flags=infw.F_HOST_ONLY)
    k = infw.build_ebpf_key(7, "10.0.0.0/8")
    b.update(k, infw.RulesValSt())
    with pytest.raises(infw.InfwError) as e:  # not empty
        b.import_image(img)
    assert e.value.errno == 16  # EBUSY
    assert b.count() == 1       # untouched
    for bad in (img[:-1], img[:100], b"x" * 200, img + b"\0"):
        c = infw.Classifier(flags=infw.F_HOST_ONLY)
        with pytest.raises(infw.InfwError) as e:
            c.import_image(bad)
        assert e.value.errno == 22 and c.count() == 0
    forged = bytearray(img)
    forged[16:32] = b"0" * 16   # another build id
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    with pytest.raises(infw.InfwError) as e:
        c.import_image(bytes(forged))
    assert e.value.errno == 22 and "another build" in N.last_error()
    small = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=10)
    with pytest.raises(infw.InfwError) as e:
        small.import_image(img)
    assert e.value.errno == 28  # ENOSPC
    a.update(k, infw.RulesValSt())  # uncommitted edit
    n = C.c_uint64(0)
    assert N.lib.infw_table_export(a._ctx, None, 0, C.byref(n)) == -16
    a.commit()
    assert N.lib.infw_table_export(a._ctx, None, 0, C.byref(n)) == 0
    assert N.lib.infw_table_export(a._ctx, C.create_string_buffer(16), 16, C.byref(n)) == -28 and n.value > 16


def test_build_id():
    bid = infw.build_id()
    assert len(bid) == 16 and int(bid, 16) >= 0


# ---- round 4: a self-verifying image (XXH64 payload hash + structural checks of the compiled tables)

HDR = 72  # magic 8, format 4, abi 4, build id 32, element sizes 16, payload XXH64 8 (image.cpp Header)
# (name, kind, element size) in image.cpp's order: the entry set, tables_io(), tbl8_of, then the IncState
_TABLES = [("if_keys", "v", 4), ("if_slot", "v", 4), ("if_mult", "p", 4), ("if_shift", "p", 4), ("n_slots", "p", 4),
           ("l16", "v", 4), ("nodes", "v", 64), ("vpool", "v", 4), ("n_tbl8_groups", "p", 8), ("tbl24", "v", 8),
           ("tbl8", "v", 4), ("short_mode", "p", 4), ("ltab", "v", 32), ("btab", "v", 64),
           ("n_buckets", "p", 8), ("n_overflow_groups", "p", 8), ("wild", "v", 4), ("n_wild", "p", 4),
           ("levels", "v", 1), ("desc", "v", 8), ("rules", "v", 8), ("dte", "v", 64), ("dtl", "v", 64),
           ("dt_plog2", "p", 4), ("dt_pl", "v", 4), ("d16", "v", 8),
           ("d16_on", "p", 4), ("d16_permille", "p", 4), ("dt_half", "p", 4), ("n_lists", "p", 4), ("n_entries", "p", 8),
           ("n_long_entries", "p", 8)]


def image_sections(img: bytes):
    """{name: (offset, bytes)} of every field of a table image (image.cpp write_image)."""
    out, o = {}, HDR
    u64 = lambda at: int.from_bytes(img[at:at + 8], "little")
    nv = u64(o)
    out["values"] = (o + 8, nv * 1200)
    o += 8 + nv * 1200
    nn = u64(o)
    out["entries"] = (o + 8, nn * 48)
    o += 8 + nn * 48
    for name, kind, sz in _TABLES:
        if kind == "p":
            out[name] = (o, sz)
            o += sz
        else:
            n = u64(o)
            out[name] = (o + 8, n * sz)
            o += 8 + n * sz
    for name, pair, kind in (("tbl8_of", 12, "m"), ("inc_valid", 1, "p"), ("slot_of", 8, "m"),
                             ("list_of_vid", 8, "m"), ("list_refs", 8, "v"), ("dead_lists", 8, "p")):
        if kind == "p":
            out[name] = (o, pair)
            o += pair
        else:
            n = u64(o)
            out[name] = (o + 8, n * pair)
            o += 8 + n * pair
    assert o == len(img), (o, len(img))
    return out


def rehash(img: bytearray) -> bytes:
    import xxhash
    img[64:72] = xxhash.xxh64(bytes(img[HDR:]), seed=0).intdigest().to_bytes(8, "little")
    return bytes(img)


def _one_if_ctx(cfg, npfx, ntmpl):
    """A committed host-only context holding the workload's entries of its first interface only (one 128-MiB
    DIR-24-8 slot: the corruption tests copy and hash the image many times)."""
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    ents = list(wl.entries())
    ifx = ents[0][0][4:8]
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16)
    for k, v in ents:
        if k[4:8] == ifx:
            c.update(infw.LpmIpKeySt.from_buffer_copy(k), infw.RulesValSt.from_buffer_copy(v))
    c.commit()
    assert c.info()["n_if_slots"] == 1
    return c


def _refused(img, why=None):
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    with pytest.raises(infw.InfwError) as e:
        if isinstance(img, bytearray):  # no copy: the caller flips bytes in place
            buf = (C.c_char * len(img)).from_buffer(img)
            c.import_image((C.addressof(buf), len(img)))
        else:
            c.import_image(img)
    assert e.value.errno == 22, N.last_error()
    if why:
        assert why in N.last_error(), N.last_error()
    assert c.count() == 0 and c.info()["epoch"] == 0  # nothing installed
    return N.last_error()


def test_payload_hash_is_xxh64():
    import xxhash
    _, a = _wl_ctx(W.CFG1_V4_10K, 2000, 16)
    img = a.export_image()
    assert int.from_bytes(img[64:72], "little") == xxhash.xxh64(img[HDR:]).intdigest()
    assert rehash(bytearray(img)) == img


@pytest.mark.parametrize("cfg", [W.CFG2_MIXED_1M, W.CFG4_ADVERSARIAL])
def test_one_flipped_byte_per_section_refused(cfg):
    """A same-length image with one byte flipped in any section — the entry set, every compiled table, the
    incremental-commit state — is refused with -EINVAL by the payload hash, and nothing is installed."""
    img = bytearray(_one_if_ctx(cfg, 3000, 32).export_image())
    secs = image_sections(img)
    flipped = 0
    for name, (off, n) in secs.items():
        if n == 0:
            continue
        for at in {off, off + n // 2, off + n - 1}:
            img[at] ^= 0x10
            assert "payload hash" in _refused(img), name
            img[at] ^= 0x10
            flipped += 1
    assert flipped > 3 * 30
    for at in range(HDR):  # and every header byte (magic, format, ABI, build id, element sizes, the hash itself)
        img[at] ^= 0x01
        _refused(img)
        img[at] ^= 0x01


def _u(img, secs, name, i, sz, val=None):
    off = secs[name][0] + i * sz
    if val is None:
        return int.from_bytes(img[off:off + sz], "little")
    img[off:off + sz] = int(val).to_bytes(sz, "little")


def _structural_cases(img: bytes):
    """(label, corrupted image with a valid hash, expected message part): what a faulty exporter could write."""
    import struct
    secs = image_sections(img)
    n_lists = _u(img, secs, "n_lists", 0, 4)
    n_slots = _u(img, secs, "n_slots", 0, 4)
    cases = []

    def case(label, why, edit):
        b = bytearray(img)
        edit(b)
        cases.append((label, rehash(b), why))

    # a DIR-24-8 word naming a tbl8 group past the groups, or a list id past the lists
    ngrp = _u(img, secs, "n_tbl8_groups", 0, 8)
    case("tbl24 group index", "DIR-24-8 word", lambda b: _u(b, secs, "tbl24", 12345, 8, (1 << 63) | (ngrp + 7)))
    case("tbl24 list id", "DIR-24-8 word", lambda b: _u(b, secs, "tbl24", 777, 8, n_lists + 1))
    case("tbl8 value", "tbl8 value", lambda b: _u(b, secs, "tbl8", 3, 4, n_lists + 5))
    # the tables' size fields disagree with their buffers (same image length)
    case("n_slots", "", lambda b: _u(b, secs, "n_slots", 0, 4, n_slots + 1))
    case("n_tbl8_groups", "tbl8 size", lambda b: _u(b, secs, "n_tbl8_groups", 0, 8, ngrp + 100))
    case("dt_plog2", "", lambda b: _u(b, secs, "dt_plog2", 0, 4, 5))
    case("n_lists", "", lambda b: _u(b, secs, "n_lists", 0, 4, n_lists + 1000))
    # an ifindex map slot past the slots
    ifs = [i for i in range(secs["if_slot"][1] // 4) if _u(img, secs, "if_slot", i, 4) != 0xFFFFFFFF]
    case("if_slot", "ifindex slot", lambda b: _u(b, secs, "if_slot", ifs[0], 4, n_slots + 3))
    # a decision root selecting leaf lines past the leaf pool
    ndtl = secs["dtl"][1] // 64

    def root(b):
        off = secs["dte"][0]
        b[off:off + 64] = struct.pack("<16I", 0x80000000 | (ndtl - 1), *([0x00020001] * 15))
    case("dte root", "decision root", root)
    # an IPv6 record naming a list past the lists; an IPv6 bucket table with no free bucket (endless probes)
    btab_off, btab_n = secs["btab"][0], secs["btab"][1] // 64
    used = [i for i in range(btab_n) if int.from_bytes(img[btab_off + 64 * i:btab_off + 64 * i + 4], "little")]
    if used:
        def rec(b):
            at = btab_off + 64 * used[0] + 16 + 12  # record 0's meta
            meta = int.from_bytes(b[at:at + 4], "little")
            b[at:at + 4] = ((meta & ~0x1FFFFFF) | (n_lists + 9)).to_bytes(4, "little")
        case("v6 record list id", "IPv6 record", rec)

    def full(b):
        for i in range(btab_n):
            at = btab_off + 64 * i
            if not int.from_bytes(b[at:at + 4], "little"):
                b[at:at + 16] = struct.pack("<4I", 1, 0xFFFFFFF0 - i, 0, 0)  # a group of no records
    case("btab full", "free bucket", full)
    # the incremental-commit state's list ids
    if secs["list_of_vid"][1]:
        case("list_of_vid", "value -> list", lambda b: _u(b, secs, "list_of_vid", 1, 4, n_lists + 2))
    return cases


@pytest.mark.parametrize("cfg", [W.CFG2_MIXED_1M, W.CFG4_ADVERSARIAL])
def test_structural_checks_with_valid_hash(cfg):
    """Images whose hash is right but whose compiled tables would send the kernel (or the host walk) outside a buffer
    or into an endless probe — a faulty exporter, not a torn file — are refused with -EINVAL before anything is
    installed or uploaded; a size field changed in an otherwise valid image too."""
    img = _one_if_ctx(cfg, 3000, 32).export_image()
    cases = _structural_cases(img)
    assert len(cases) >= 11
    for label, bad, why in cases:
        msg = _refused(bad, why or None)
        assert "corrupt table image" in msg or "truncated" in msg or "trailing" in msg, (label, msg)


def test_import_into_emptied_context():
    """A context whose entries were all removed and committed counts as empty: the import succeeds."""
    wl, a = _wl_ctx(W.CFG1_V4_10K, 2000, 16)
    img = a.export_image()
    b = infw.Classifier(flags=infw.F_HOST_ONLY)
    k = infw.build_ebpf_key(7, "10.0.0.0/8")
    b.update(k, infw.RulesValSt())
    b.commit()
    b.delete(k)
    with pytest.raises(infw.InfwError) as e:  # the delete is not committed yet
        b.import_image(img)
    assert e.value.errno == 16
    b.commit()
    b.import_image(img)
    assert b.export_image() == img and b.count() == a.count()


def _dup_values_image(img: bytes) -> bytes:
    """The image with its second interned value overwritten by its first (a valid hash): the entry set then names
    two equal values, which the importer must refuse before it touches the map."""
    b = bytearray(img)
    secs = image_sections(img)
    off, n = secs["values"]
    assert n >= 2400
    b[off + 1200:off + 2400] = b[off:off + 1200]
    return rehash(b)


def test_refused_import_changes_nothing():
    """a refused import leaves the context as it was.
    - A populated context with committed entries and uncommitted edits: busy is decided before the image is read,
      so a corrupt image gets -EBUSY too and the pending edits survive; they commit and walk like the oracle.
    - An emptied context (its entries removed and committed; its compiled lists still map value ids): imports
      refused for too many entries (-ENOSPC), a torn payload and duplicate values (-EINVAL) keep its value pool, so
      the next update + incremental commit classifies with the new value's own rules, as the oracle does."""
    wl, a = _wl_ctx(W.CFG1_V4_10K, 2000, 16)
    img = a.export_image()
    torn = bytearray(img)
    torn[len(torn) // 2] ^= 1
    rng = random.Random(3)
    vals = [bytes(v) for _, v in wl.entries()][:64]
    v1 = next(v for v in vals if v != vals[0])
    # populated
    b = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=4096)
    m = orc.OracleMap()
    keys = [bytes(infw.build_ebpf_key(3, f"10.{i}.0.0/16")) for i in range(8)]
    for k in keys[:4]:
        _apply([b], m, k, vals[0])
    b.commit()
    for k in keys[4:]:
        _apply([b], m, k, v1)  # uncommitted
    for bad in (img, bytes(torn), _dup_values_image(img)):
        with pytest.raises(infw.InfwError) as e:
            b.import_image(bad)
        assert e.value.errno == 16
        assert b.count() == 8
    b.commit()
    hdr, cap, pl, ifx = _packets_for(keys, rng)
    tup = W.pack_frames(hdr, cap, pl, ifx)
    want, _, _, _ = m.classify_frames(hdr, cap, pl, ifx)
    assert np.array_equal(b.debug_walk(tup), want)
    # emptied
    for bad, errno in ((img, 28), (bytes(torn), 22), (_dup_values_image(img), 22)):
        e_ctx = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=16 if errno == 28 else 4096)
        m = orc.OracleMap()
        k0, k1 = keys[0], keys[1]
        _apply([e_ctx], m, k0, vals[0])
        e_ctx.commit()
        _apply([e_ctx], m, k0, None)
        e_ctx.commit()
        with pytest.raises(infw.InfwError) as e:
            e_ctx.import_image(bad)
        assert e.value.errno == errno, N.last_error()
        assert e_ctx.count() == 0
        _apply([e_ctx], m, k1, v1)
        e_ctx.commit()
        assert e_ctx.info()["commit_mode"] == infw.COMMIT_INCREMENTAL
        hdr, cap, pl, ifx = _packets_for([k0, k1], rng, per_key=300)
        tup = W.pack_frames(hdr, cap, pl, ifx)
        want, _, _, _ = m.classify_frames(hdr, cap, pl, ifx)
        assert np.array_equal(e_ctx.debug_walk(tup), want), errno
        assert (want != 0).any()


ASAN_ABI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ingress-node-firewall_amd",
                        "build", "asan", "asan_abi")


def test_host_sanitizer_abi_and_images(tmp_path):
    """tools/asan_abi.cpp against the AddressSanitizer/UBSan build of libinfw.so's host sources (make asan-host):
    the C ABI's host-only paths and image export / import / re-export with flipped bytes; then every structurally
    corrupt image above (valid hash) through infw_table_import under the sanitizers."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    root = os.path.dirname(ASAN_ABI)
    from conftest import run_make
    r = run_make("asan-host")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    r = subprocess.run([ASAN_ABI], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-3000:]
    for cfg in (W.CFG2_MIXED_1M, W.CFG4_ADVERSARIAL):
        img = _one_if_ctx(cfg, 3000, 32).export_image()
        for i, (label, bad, why) in enumerate(_structural_cases(img) + [("clean", img, None)]):
            p = tmp_path / "img.bin"
            p.write_bytes(bad)
            r = subprocess.run([ASAN_ABI, "import", str(p)], capture_output=True, text=True, timeout=300)
            assert r.returncode == 0, (label, r.stdout[-1000:] + r.stderr[-3000:])
            if label == "clean":
                assert r.stdout.startswith("rc=0 count=") and not r.stdout.startswith("rc=0 count=0"), r.stdout
            else:
                assert r.stdout.startswith("rc=22 count=0"), (label, r.stdout)
