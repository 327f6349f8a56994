#!/bin/bash
# Round 6, session 3: attribution A/B of the ring partition changes (build store phase 1 vs 0;
# readfirstlane'd group count vs not) with kernel profiles, and the per-key path after the Python
# trims.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh profab ab1 bench_c1
