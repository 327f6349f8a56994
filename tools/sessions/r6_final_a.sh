#!/bin/bash
# Round 6 final records A (final sources): smoke, GPU suite, C2 PMC traffic (copied into
# profiles/ so the bench line carries it), C2 bench + rocprofv3 profile, C1 per-key legs, C2 PMC
# issue passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh smoke pytest traffic || exit $?
cp gpurun_out/traffic_c2.json profiles/traffic_c2.json || exit 1
bash tools/gpu_session.sh bench prof bench_c1 pmcall
