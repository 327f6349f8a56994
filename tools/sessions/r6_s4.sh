#!/bin/bash
# Round 6, session 4: the resident reader's single-store answers (no L2 write-back per answer):
# its tests, and the per-key / concurrent-gets legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PBF_TESTS="tests/test_gpu_dropin.py tests/test_gpu_lsm_get.py" bash tools/gpu_session.sh pytest_new bench_c1
