"""The kernel-variant registry and the launches that reach each entry (shared by tests/test_variants_cpu.py and
tests/test_gpu_variants.py).

The library launches exactly the classify_kernel instantiations of its registry (classify.hip kVariants,
infw_kernel_variant_name) and picks one per launch with one selector from the epoch's kind, the batch form, the
launch shape and the sidebands (infw_classify_variant answers which, without launching).  A scenario here is one
such launch: a table kind (the per-context options that make the compiler build that kind of epoch), the two-phase
switch, a launch shape, an input form and the sidebands.  scenarios() enumerates them all; every registry entry
must be the answer of at least one, and no answer may be outside the registry.
"""
from __future__ import annotations

import itertools

import infw

# table kinds: per-context options (include/infw.h infw_set_option) -> the epoch the compiler builds
KINDS = {
    "full": dict(short_table=1, d16=0, dt_adapt=1, dt_half=0),       # compressed short table: not lean
    "full.nopl": dict(short_table=1, d16=0, dt_adapt=0, dt_half=0),
    "lean": dict(short_table=0, d16=0, dt_adapt=0, dt_half=0),
    "lean.pl": dict(short_table=0, d16=0, dt_adapt=1, dt_half=0),
    "lean.pl.d16": dict(short_table=0, d16=1, dt_adapt=1, dt_half=0),
    "lean.d16": dict(short_table=0, d16=1, dt_adapt=0, dt_half=0),
    "lean.d16.half": dict(short_table=0, d16=1, dt_adapt=0, dt_half=1),
}
# every launch shape infw_set_launch accepts: (block, scan_group, blocks_per_cu)
SHAPES = [(768, 0, 2), (512, 0, 2), (512, 0, 3), (512, 0, 4), (256, 0, 6),
          (512, 1, 3), (512, 4, 3), (512, 8, 3), (256, 1, 6), (256, 4, 6), (256, 8, 6)]
INPUTS = {"soa": infw.INPUT_SOA, "compact": infw.INPUT_COMPACT, "frames": infw.INPUT_FRAMES, "xdp": infw.INPUT_XDP}
# a small configs[2]-shaped table: 16 value parts (so per-list part counts exist), IPv4 and IPv6 entries
TABLE = dict(n_prefixes=20000, n_templates=64)


def scenarios():
    """(kind, split, shape, input name, events, debug) of every launch worth asking about."""
    for kind, split, shape, inp, ev, dbg in itertools.product(KINDS, (0, 1), SHAPES, INPUTS, (False, True),
                                                              (False, True)):
        if inp in ("compact", "xdp") and ev:
            continue  # infw_classify_c and infw_classify_xdp have no event stream
        yield kind, split, shape, inp, ev, dbg


def registry():
    """Every classify_kernel instantiation (the decide kernel of the two-phase form is listed last)."""
    return infw.kernel_variants()


def names_of(answer: str):
    """The registry names of one infw_classify_variant answer ("a" or "a+decide.512")."""
    return answer.split("+")
