#!/bin/bash
# Round 6, session 2: the one-round-trip resident reader (inline request heads) and the build
# partition's desynchronised store phase: GPU suite, C1 per-key latency, C2 bench + profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh pytest bench_c1 bench prof
