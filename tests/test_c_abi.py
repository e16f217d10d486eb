"""The C-ABI boundary driven from plain C (tests/c/abi_demo.c), the way a cgo build of
pkg/ebpf binds it: no Python or torch between the caller and lib/libinfw.so.

CPU: the demo compiles against include/infw.h alone, links against the library, and its
host-only mode (INFW_F_HOST_ONLY: map API, -ENODEV from classify, tests-only host walk) passes.
GPU: the same binary classifies a host-resident batch through infw_classify_host and reads
the per-rule counters back (loader.go:130-194, kernel.c:459-462, statistics.go:126-157)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(ROOT, "ingress-node-firewall_amd", "lib")


def build_demo(tmp_path):
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path / "abi_demo")
    cmd = [cc, "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "c", "abi_demo.c"), "-o", exe,
           "-L", LIB_DIR, "-linfw", "-Wl,-rpath," + LIB_DIR]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def build_xdp_demo(tmp_path):
    """tests/c/xdp_demo.c: plain C against include/infw.h, plus the HIP runtime's C header for the stream sync a
    daemon does after infw_classify_xdp."""
    cc = shutil.which("gcc") or shutil.which("cc")
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    if cc is None or not os.path.exists(os.path.join(rocm, "include", "hip", "hip_runtime_api.h")):
        pytest.skip("no C compiler or HIP headers")
    exe = str(tmp_path / "xdp_demo")
    cmd = [cc, "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I",
           os.path.join(ROOT, "include"), "-I", os.path.join(rocm, "include"),
           os.path.join(ROOT, "tests", "c", "xdp_demo.c"), "-o", exe, "-L", LIB_DIR, "-linfw",
           "-L", os.path.join(rocm, "lib"), "-lamdhip64", "-Wl,-rpath," + LIB_DIR + ":" + os.path.join(rocm, "lib")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_xdp_caller_host_only(tmp_path):
    exe = build_xdp_demo(tmp_path)
    out = subprocess.run([exe, "host"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("xdp_demo OK (host)")


@pytest.mark.gpu
def test_c_xdp_caller_on_device(tmp_path):
    """A daemon's own (registered) umem, ring and result arrays through infw_classify_xdp, two interface rings; the
    same memory unregistered refused by it (-EFAULT) and classified by the host-fed path (infw_classify_xdp_host)."""
    exe = build_xdp_demo(tmp_path)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "allow 2 (600 B), deny 1 (100 B); pageable memory refused" in out.stdout


def test_c_caller_host_only(tmp_path):
    exe = build_demo(tmp_path)
    out = subprocess.run([exe, "host"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("abi_demo OK (host)")


@pytest.mark.gpu
def test_c_caller_on_device(tmp_path):
    exe = build_demo(tmp_path)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "allow 2 (600 B), deny 1 (100 B)" in out.stdout
