#!/bin/bash
# Round 6 final records C (final sources, C5 in one pipeline): the C5 line again (it carries the
# one-pipeline traffic recomputed from record B's PMC passes), C5mixed and SSTable legs, C3 / C4 /
# C5 kernel profiles, the simulated rank of the 8-GPU C5 key layout, self-launched rehearsals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh bench_c5 bench_c5mixed bench_sst prof_c3 prof_c4_serial prof_c5 c5sim8 selflaunch
