"""Diagnostic (GPU): bench.py's probe_with_gets leg on its own (for rocprofv3 kernel traces)."""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

print(json.dumps(bench.probe_with_gets(0)))
