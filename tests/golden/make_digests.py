"""Frozen result digests of the reduced BASELINE workloads (golden/cfg0_demo1, v4_10k, mixed_100k,
swap), generated from the oracle (oracle/infw_oracle.c) over the deterministic workload generator.

For each case: table spec + packet range, the SHA-256 of the per-packet result words (u32 LE), of the XDP verdicts
(u8) and of the 1024 x 4 u64 LE per-rule counters, the counter totals, and the first 16 result words in clear.
tests/test_golden_digests.py checks the oracle against this file on the CPU; tests/test_gpu_golden.py checks the
HIP classifier against it on the GPU without loading the oracle — so a later change to either side (or a shared
misreading introduced after the freeze) shows as a digest mismatch.

Run: python tests/golden/make_digests.py   (rewrites tests/golden/digests.json; deterministic)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "ingress-node-firewall_amd"), os.path.join(ROOT, "oracle"),
                os.path.dirname(HERE)]

import numpy as np  # noqa: E402

# name, cfg, n_prefixes, n_templates, first packet, packets
CASES = [
    ("cfg0_demo1", 0, 0, 0, 0, 1 << 20),
    ("v4_10k", 1, 0, 0, 0, 1 << 20),
    ("mixed_100k", 2, 100000, 512, 0, 1 << 20),
    ("mixed_100k_distinct", 2, 100000, 100000, 0, 1 << 19),
    ("adversarial_20k", 4, 20000, 64, 0, 1 << 19),
]
SWAP = ("swap_adversarial_20k", 4, 20000, 64, 1 << 18)  # batch A = [0, n) on epoch 1, batch B = [n, 2n) on epoch 2


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def record(res, ver, stats):
    res = np.asarray(res, "<u4")
    st = np.asarray(stats, "<u8").reshape(1024, 4)
    return {"results_sha256": sha(res), "verdicts_sha256": sha(np.asarray(ver, np.uint8)),
            "stats_sha256": sha(st), "allow_packets": int(st[:, 0].sum()), "deny_packets": int(st[:, 2].sum()),
            "allow_bytes": int(st[:, 1].sum()), "deny_bytes": int(st[:, 3].sum()),
            "first_results": [int(x) for x in res[:16]]}


def swap_edits(wl):
    """The live table swap of configs[4] (test_epoch_swap_between_batches): delete every 3rd key, rewrite every 5th
    with another template.  Yields ("delete", key) / ("update", key, value) in order."""
    keys = wl.keys_bytes().reshape(-1, 24)
    tmpl = wl.templates_bytes().reshape(-1, 1200)
    for i in range(0, keys.shape[0], 3):
        yield ("delete", keys[i].tobytes())
    for i in range(1, keys.shape[0], 5):
        yield ("update", keys[i].tobytes(), tmpl[(i * 7) % tmpl.shape[0]].tobytes())


def oracle_case(cfg, npfx, ntmpl, start, n):
    from infw import workloads as W
    from parity import oracle_for
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    m = oracle_for(wl)
    hdr, cap, pl, ifx = wl.frames(start, n)
    res, ver, stats, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    return record(res, ver, stats)


def oracle_swap():
    from infw import workloads as W
    from parity import oracle_for
    _, cfg, npfx, ntmpl, n = SWAP
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    m = oracle_for(wl)
    hdr, cap, pl, ifx = wl.frames(0, n)
    ra, va, sa, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    for e in swap_edits(wl):
        m.delete(e[1]) if e[0] == "delete" else m.update(e[1], e[2])
    hdr, cap, pl, ifx = wl.frames(n, n)
    rb, vb, sb, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
    return {"batch_a": record(ra, va, sa), "batch_b": record(rb, vb, sb), "stats_after_both": record(
        np.zeros(0, np.uint32), np.zeros(0, np.uint8), sa + sb)}


def main():
    out = {"generator": "tests/golden/make_digests.py (oracle/infw_oracle.c over ingress-node-firewall_amd/csrc/"
                        "infw_gen.h packets)", "cases": {}}
    for name, cfg, npfx, ntmpl, start, n in CASES:
        out["cases"][name] = dict({"cfg": cfg, "n_prefixes": npfx, "n_templates": ntmpl, "start": start, "n": n},
                                  **oracle_case(cfg, npfx, ntmpl, start, n))
        print(name, out["cases"][name]["results_sha256"][:16], flush=True)
    name, cfg, npfx, ntmpl, n = SWAP
    out["cases"][name] = dict({"cfg": cfg, "n_prefixes": npfx, "n_templates": ntmpl, "n": n}, **oracle_swap())
    json.dump(out, open(os.path.join(HERE, "digests.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
