#!/bin/bash
# Round 6 final records B (final sources): PMC traffic of C3 / C4 / C5 (copied into profiles/),
# then the C3 / C4 / C5 bench lines that carry it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh traffic_c3 traffic_c4 traffic_c5 || exit $?
for c in c3 c4 c5; do cp gpurun_out/traffic_$c.json profiles/traffic_$c.json || exit 1; done
bash tools/gpu_session.sh bench_c3 bench_c4 bench_c5
