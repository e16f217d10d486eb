"""The C ABI's threading contract (include/infw.h "threads") under ThreadSanitizer, on the CPU.

The reference keeps classifying on every CPU while its syncer edits and reloads the maps under e.mu
(pkg/ebpfsyncer/ebpfsyncer.go:62, 72-73).  tools/tsan_abi.cpp runs that shape on a host-only context against the
TSan build of libinfw.so's host sources (make tsan-host): a control-plane thread commits a sequence of epochs —
batched and single edits, deletes, full and incremental commits, option and launch-shape changes — while three
threads walk a fixed packet set through the committed host image (every walk must equal exactly one epoch's results)
and two more read the table info, statistics, kernel-variant answers, options, launch shape and debug keys.
A data race in the instrumented code fails the run (TSan's exit status); the GPU form of the same contract is
tests/test_gpu_threads.py."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TSAN_ABI = os.path.join(ROOT, "ingress-node-firewall_amd", "build", "tsan", "tsan_abi")
TSAN_POOL = os.path.join(ROOT, "ingress-node-firewall_amd", "build", "tsan", "tsan_hostpool")


def test_threading_contract_under_tsan():
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    from conftest import run_make
    r = run_make("tsan-host")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1")
    r = subprocess.run([TSAN_ABI], capture_output=True, text=True, timeout=900, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-3000:]
    walks = int(r.stdout.split("epochs, ")[1].split()[0])
    assert walks > 0  # the walkers really ran beside the commits


def test_host_packer_pool_under_tsan():
    """The packer threads of infw_classify_xdp_host (csrc/hostfeed.cpp) without a device: tools/tsan_hostpool.cpp
    plays the coordinator — waits for each ragged chunk, checks the slot against the packer run on its own thread,
    releases the next chunk into the freed slot — for 1-8 threads and three chunk sizes, jobs back to back on one
    pool and aborted half-way, under ThreadSanitizer."""
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    from conftest import run_make
    r = run_make("tsan-host")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1")
    r = subprocess.run([TSAN_POOL], capture_output=True, text=True, timeout=900, env=env)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0 and r.stdout.startswith("tsan_hostpool OK"), r.stdout[-2000:] + r.stderr[-3000:]
