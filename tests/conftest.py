"""pytest configuration: import paths and the `gpu` marker.

-m "not gpu" runs on a CPU-only box: oracle vs golden vectors, host logic,
table compiler (host walk) vs oracle, C-ABI load/exports, gloo multi-process.
-m gpu runs the parity tests proper through the C ABI on a MI355X.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ingress-node-firewall_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def run_make(*targets, timeout=900):
    """`make -s -C ROOT targets` under an exclusive lock on build/.make.lock: tests in parallel workers (pytest -n)
    that build the same sanitizer targets must not write the same objects at once."""
    import fcntl
    import subprocess
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        return subprocess.run(["make", "-s", "-C", ROOT, *targets], capture_output=True, text=True, timeout=timeout)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP classifier")
