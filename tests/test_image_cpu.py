"""Compiled-epoch images (infw_table_export / infw_table_import) on the CPU: an imported context is the exporter's
committed epoch — the same key walk (get_next_key post-order), lookups, compiled host tables (debug walk over
packets of every key) — and keeps behaving like it under later incremental edits, which commit incrementally on the
import (the incremental-commit state travels with the image).  Error paths: import into a non-empty context,
a truncated or corrupted image, another build's image, export with uncommitted edits."""
import ctypes as C
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
