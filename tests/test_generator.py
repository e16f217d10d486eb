"""Synthetic workload generator: packet i is a pure function of (seed, i); the host
frame builder + packer and the tuple generator agree; shards are independent of
the shard split (what makes the multi-GPU totals GPU-count invariant)."""
import numpy as np

from infw import workloads as W


def test_pack_equals_generated_tuples_all_configs():
    for cfg, kw in ((W.CFG0_DEMO, {}), (W.CFG1_V4_10K, {}), (W.CFG2_MIXED_1M, dict(n_prefixes=20000, n_templates=64)),
                    (W.CFG4_ADVERSARIAL, dict(n_prefixes=5000, n_templates=16))):
        wl = W.Workload(cfg, **kw)
        hdr, cap, pl, ifx = wl.frames(12345, 50000)
        assert np.array_equal(W.pack_frames(hdr, cap, pl, ifx), wl.tuples(12345, 50000)), cfg


def test_shard_invariance():
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    whole = wl.tuples(0, 40000)
    parts = np.concatenate([wl.tuples(a, 10000) for a in (0, 10000, 20000, 30000)])
    assert np.array_equal(whole, parts)
    wl2 = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    assert np.array_equal(wl2.tuples(777, 1000), whole[777:1777])


def test_workload_mix_is_as_specified():
    wl = W.Workload(W.CFG0_DEMO)
    t = wl.tuples(0, 200000)
    et = t[:, 6] & 0xFFFF
    v4, v6 = (et == 0x0800).mean(), (et == 0x86DD).mean()
    assert 0.45 < v4 < 0.55 and 0.45 < v6 < 0.55
    proto = (t[:, 6] >> 16) & 0xFF
    assert 0.55 < (proto == 6).mean() < 0.65
    assert ((t[:, 6] >> 24) < 54).mean() > 0.001        # some truncated frames
    assert (t[:, 5] >= 54).mean() > 0.99                  # frame lengths U[54, 1514]


def test_uniform_sources_flattens_the_head():
    """bench.py --uniform: sources uniform over the prefixes (no Zipf head), tables unchanged."""
    z = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    u = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    u.uniform_sources()
    assert np.array_equal(z.keys_bytes(), u.keys_bytes())
    top = lambda wl: np.sort(np.unique(wl.tuples(0, 50000)[:, 0], return_counts=True)[1])[-2]  # [-1]: word 0 of non-IP
    assert top(z) > 20 * top(u)


def test_shuffled_key_order_builds_the_same_map():
    """bench.py's default table load (--key-order shuffled: the reference loader's Go map order, at random) keeps,
    per LPM entry, its last update of the workload order — value and host bits — so the committed map and every
    classification equal the workload-order load's; duplicate keys (configs[4]'s identical v4 / v6 /0 keys,
    generator repeats, host-bit variants) are where a plain shuffle would differ."""
    import infw
    for cfg, kw in ((W.CFG4_ADVERSARIAL, dict(n_prefixes=20000, n_templates=64)),
                    (W.CFG2_MIXED_1M, dict(n_prefixes=30000, n_templates=30000)), (W.CFG1_V4_10K, {})):
        wl = W.Workload(cfg, **kw)
        a = infw.Classifier(flags=infw.F_HOST_ONLY)
        wl.load_into(a)
        a.commit()
        order = wl.shuffled_order()
        assert len(order) < wl.n_entries and len(set(order.tolist())) == len(order)
        assert not np.array_equal(np.sort(order), order)
        b = infw.Classifier(flags=infw.F_HOST_ONLY)
        wl.load_into(b, order=order)
        b.commit()
        assert sorted((bytes(k), bytes(v)) for k, v in a.iterate()) == sorted((bytes(k), bytes(v)) for k, v in b.iterate())
        hdr, cap, pl, ifx = wl.frames(0, 30000)
        tup = W.pack_frames(hdr, cap, pl, ifx)
        assert np.array_equal(a.debug_walk(tup), b.debug_walk(tup)), cfg
