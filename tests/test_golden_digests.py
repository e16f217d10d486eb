"""Frozen digests (tests/golden/digests.json, written by tests/golden/make_digests.py from the oracle) on the CPU:
the oracle must still produce them, and so must the product's compiled table image walked on the host
(infw_debug_walk).  tests/test_gpu_golden.py checks the HIP kernel against the same file without the oracle."""
import json
import os

import numpy as np
import pytest

import infw
from golden.make_digests import CASES, SWAP, oracle_case, oracle_swap, record, swap_edits
from infw import workloads as W

DIG = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "digests.json")))["cases"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_oracle_reproduces_frozen_digests(case):
    name, cfg, npfx, ntmpl, start, n = case
    got = oracle_case(cfg, npfx, ntmpl, start, n)
    want = {k: v for k, v in DIG[name].items() if k in got}
    assert got == want, name


def test_oracle_reproduces_frozen_swap():
    got = oracle_swap()
    assert got == {k: DIG[SWAP[0]][k] for k in got}


def _host_walk(clf, wl, start, n):
    t = wl.tuples(start, n)
    res = clf.debug_walk(t)
    from parity import stats_from_results
    return record(res, infw.verdicts_from_results(res, t[:, 6]), stats_from_results(res, t[:, 5]))


@pytest.mark.parametrize("case", CASES[:3] + CASES[4:], ids=lambda c: c[0])
def test_compiled_tables_match_frozen_digests(case):
    name, cfg, npfx, ntmpl, start, n = case
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    clf = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    n = min(n, 1 << 18)  # the host walk is serial: the first 256k packets, checked against the first results
    got = _host_walk(clf, wl, start, n)
    assert got["first_results"] == DIG[name]["first_results"], name


def test_compiled_tables_match_frozen_swap():
    name, cfg, npfx, ntmpl, n = SWAP
    wl = W.Workload(cfg, n_prefixes=npfx, n_templates=ntmpl)
    clf = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    a = _host_walk(clf, wl, 0, n)
    for e in swap_edits(wl):
        if e[0] == "delete":
            clf.delete_rc(infw.LpmIpKeySt.from_buffer_copy(e[1]))  # duplicate keys: -ENOENT, as the oracle
        else:
            clf.update(infw.LpmIpKeySt.from_buffer_copy(e[1]), infw.RulesValSt.from_buffer_copy(e[2]))
    clf.commit()
    b = _host_walk(clf, wl, n, n)
    assert a == DIG[name]["batch_a"] and b == DIG[name]["batch_b"]
