"""Rule values for commit tests: tools/commit_latency.py's generator of fresh 100-slot rule lists."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from commit_latency import new_value  # noqa: E402,F401
