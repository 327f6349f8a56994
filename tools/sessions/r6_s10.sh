#!/bin/bash
# Round 6, session 10: the wave-local length sort of variable-length keys (C3 partition), A/B
# against the unsorted hash (PBF_VAR_SORT=0), parity of the variable-length paths first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PBF_TESTS="tests/test_gpu_parity.py tests/test_gpu_device_resident.py" bash tools/gpu_session.sh pytest_new || exit $?
bash tools/gpu_session.sh ab_c3_2 prof_var_c3 prof_c3
