#!/bin/bash
# Round 6, session 5: partitions planned around a live resident reader (31 workgroups per XCD):
# the concurrent-gets leg, the reader tests, and the C2 bench (no reader: unchanged plans).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PBF_TESTS="tests/test_gpu_dropin.py tests/test_gpu_parity.py" bash tools/gpu_session.sh pytest_new bench_c1 bench
