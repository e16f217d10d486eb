"""The kernel-variant registry against the selector, on the CPU (no device: host-only contexts answer
infw_classify_variant from their committed image).  Every launch of tests/variants.py's scenarios must name
registered instantiations only, and every registered instantiation must be the answer of some launch — so the
device test (tests/test_gpu_variants.py) that runs one launch per registry entry against the oracle runs every
instantiation the production dispatcher can reach, and nothing unreachable is compiled into the library."""
import pytest

import infw
from infw import workloads as W

import variants as V


def _ctx(kind):
    wl = W.Workload(W.CFG2_MIXED_1M, **V.TABLE)
    c = infw.Classifier(flags=infw.F_HOST_ONLY, max_entries=wl.n_entries + 16, options=V.KINDS[kind])
    wl.load_into(c)
    c.commit()
    return c


def reach():
    """{registry name: first scenario answering it} and every answer seen."""
    first, answers = {}, set()
    for kind in V.KINDS:
        c = _ctx(kind)
        info = c.info()
        lean = info["short_mode"] != 1
        assert lean == kind.startswith("lean"), (kind, info["short_mode"])
        assert info["d16"] == V.KINDS[kind]["d16"] and info["dt_half_reads"] == V.KINDS[kind]["dt_half"], kind
        for kind_, split, shape, inp, ev, dbg in V.scenarios():
            if kind_ != kind:
                continue
            c.set_option("split", split)
            c.set_launch(*shape)
            c.debug_lookup(1 if dbg else 0)
            a = c.variant(V.INPUTS[inp], events=ev)
            answers.add(a)
            for name in V.names_of(a):
                first.setdefault(name, (kind, split, shape, inp, ev, dbg))
        c.close()
    return first, answers


def test_registry_names_are_distinct():
    reg = V.registry()
    assert len(reg) == len(set(reg)) >= 30
    assert reg[-1] == "decide.512"


def test_every_answer_registered_and_every_entry_reached():
    reg = set(V.registry())
    first, answers = reach()
    unregistered = {a for a in answers if "(unregistered)" in a or not set(V.names_of(a)) <= reg}
    assert not unregistered, sorted(unregistered)
    unreached = reg - set(first)
    assert not unreached, sorted(unreached)


def test_default_launch_per_epoch_kind():
    """The production path (default shape, SoA batch, no sidebands) per table kind — the instantiations the bench
    lines run."""
    want = {
        "full": "soa.768.w6.g0.c12.b9",
        "lean": "soa.768.w6.g0.c12.b9.lean",
        "lean.pl": "soa.768.w6.g0.c12.b9.lean.pl",
        "lean.pl.d16": "soa.768.w6.g0.c12.b9.lean.pl.d16",
        "lean.d16": "soa.768.w6.g0.c13.b8.lean.d16",
        "lean.d16.half": "soa.768.w6.g0.c13.b8.lean.d16.half",
    }
    for kind, name in want.items():
        c = _ctx(kind)
        assert c.variant() == name, kind
        c.set_option("split", 1)
        a = c.variant()
        assert a.endswith("+decide.512") == kind.startswith("lean"), (kind, a)
        c.close()


def test_launch_shape_validation():
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    for shape in V.SHAPES:
        c.set_launch(*shape)
        assert c.launch() == shape
    for bad in [(768, 0, 3), (640, 0, 3), (512, 2, 3), (512, 1, 4), (1024, 0, 1), (768, 4, 2), (64, 0, 16)]:
        with pytest.raises(infw.InfwError) as e:
            c.set_launch(*bad)
        assert e.value.errno == 22
        assert c.launch() == V.SHAPES[-1]  # unchanged


def test_options_validated():
    """infw_set_option: every listed option reads back its default and takes values in range; unknown names and
    out-of-range values are refused with -EINVAL and change nothing."""
    c = infw.Classifier(flags=infw.F_HOST_ONLY)
    names = infw.option_names()
    assert names == ["short_table", "d16", "dt_half", "dt_parts", "dt_adapt", "dt_budget_mb", "compile_threads",
                     "split", "split_min_mb", "stat_flush_tiles", "trace", "host_threads"]
    defaults = {n: c.option(n) for n in names}
    assert defaults == {"short_table": -1, "d16": -1, "dt_half": -1, "dt_parts": 0, "dt_adapt": 1, "dt_budget_mb": 2048,
                        "compile_threads": 0, "split": -1, "split_min_mb": 1024, "stat_flush_tiles": 1024, "trace": 0,
                        "host_threads": 0}
    for name, bad in [("nope", 0), ("dt_parts", 3), ("dt_parts", 32), ("split", 2), ("short_table", 2),
                      ("stat_flush_tiles", 0), ("stat_flush_tiles", 1025), ("dt_budget_mb", 1), ("trace", 16),
                      ("host_threads", -1), ("host_threads", 65)]:
        with pytest.raises(infw.InfwError) as e:
            c.set_option(name, bad)
        assert e.value.errno == 22
    assert {n: c.option(n) for n in names} == defaults
    c.set_option("dt_parts", 4)
    assert c.option("dt_parts") == 4


def test_library_reads_no_environment():
    """The shipping library names no getenv (include/infw.h: everything is a per-context option)."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", infw.LIB_PATH], capture_output=True, text=True).stdout
    assert "getenv" not in out and "secure_getenv" not in out


def test_variant_arguments_validated():
    """infw_classify_variant: inputs past INFW_INPUT_XDP, unknown flags and an event stream on the family-compact
    or AF_XDP forms (infw_classify_c / infw_classify_xdp have none) are -EINVAL; the AF_XDP form names its own
    instantiations (xdp.*), the frames form its own (frames.*)."""
    c = _ctx("lean.pl")
    assert c.variant(infw.INPUT_XDP).startswith("xdp.768.")
    assert c.variant(infw.INPUT_FRAMES).startswith("frames.768.")
    for inp, ev in [(infw.INPUT_XDP, True), (infw.INPUT_COMPACT, True), (4, False), (-1, False)]:
        with pytest.raises(infw.InfwError) as e:
            c.variant(inp, events=ev)
        assert e.value.errno == 22, (inp, ev)
    c.close()
