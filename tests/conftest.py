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


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP classifier")
