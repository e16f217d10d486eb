#!/usr/bin/env python3
"""Commit latency at configs[2] scale (1M prefixes): incremental vs full commits.

Loads the cfg2 table, commits it (full), then applies edit batches of growing
size — a mix of value changes (existing and new rule lists), deletes and
re-adds — and commits each one incrementally; then repeats the largest batch
with INFW_F_FULL_COMMIT for comparison.  One JSON line per commit:
host patch/compile ms, device copy ms, bytes copied to the device.
  python tools/commit_latency.py [--host-only] [--slots N]
--slots N: a context over N device slots of GPU 0 (devices=[0]*N, one host thread per slot at commit); the line
also reports the slowest slot's device time.
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ingress-node-firewall_amd")]


def new_value(rng) -> bytes:
    """A fresh 100-slot rule list (ruleId = order, TCP/UDP ranges, Allow/Deny) packed like rulesVal_st."""
    import struct
    slots = [b"\0" * 12] * 100
    for o in rng.sample(range(1, 100), 12):
        ps = rng.randrange(1, 60000)
        slots[o] = struct.pack("<IBHHBBB", o, rng.choice([6, 17]), ps, ps + rng.randrange(0, 2000), 0, 0,
                               rng.choice([1, 2]))
    return b"".join(slots)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host-only", action="store_true")
    ap.add_argument("--sizes", default="1,10,100,1000,10000")
    ap.add_argument("--slots", type=int, default=1)
    args = ap.parse_args()
    import infw
    from infw import workloads as W
    wl = W.Workload(W.CFG2_MIXED_1M)
    keys = wl.keys_bytes().reshape(-1, 24)
    tmpl = wl.templates_bytes().reshape(-1, 1200)
    flags = infw.F_HOST_ONLY if args.host_only else 0
    devs = None if args.host_only else [0] * args.slots
    rng = random.Random(1)

    def run(c, label, size):
        for i in rng.sample(range(keys.shape[0]), size):
            kb = infw.LpmIpKeySt.from_buffer_copy(keys[i].tobytes())
            r = rng.random()
            if r < 0.2:
                c.delete_rc(kb)
            elif r < 0.9:
                c.update(kb, infw.RulesValSt.from_buffer_copy(tmpl[rng.randrange(tmpl.shape[0])].tobytes()))
            else:
                c.update(kb, infw.RulesValSt.from_buffer_copy(new_value(rng)))
        t = time.perf_counter()
        c.commit()
        wall = (time.perf_counter() - t) * 1e3
        i = c.info()
        print(json.dumps({"commit": label, "edits": size, "mode": ["full", "incremental", "reupload"][i["commit_mode"]],
                          "wall_ms": round(wall, 2), "host_ms": round(i["compile_ms"], 2),
                          "device_ms": round(i["upload_ms"], 2), "device_bytes_copied": i["patch_bytes"],
                          "slots": i["n_device_slots"], "slowest_slot_ms": round(i["device_ms_max"], 2),
                          "full_reason": i["full_reason"]}), flush=True)

    c = infw.Classifier(devices=devs, max_entries=wl.n_entries + 65536, flags=flags)
    wl.load_into(c)
    run(c, "initial", 0)
    sizes = [int(x) for x in args.sizes.split(",")]
    for s in sizes:
        run(c, "incremental", s)
    c.close()
    f = infw.Classifier(devices=devs, max_entries=wl.n_entries + 65536, flags=flags | infw.F_FULL_COMMIT)
    wl.load_into(f)
    f.commit()
    run(f, "forced-full", sizes[-1])


if __name__ == "__main__":
    main()
