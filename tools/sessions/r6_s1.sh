#!/bin/bash
# Round 6, session 1: the suite on the new sources (replication, digest, per-key fast path, >4 GiB
# ring regions, small-tile DMA), C2 bench, C1 per-key latency, the C2 store-phase A/B, C5 keys
# layout with replication (simulated rank 0 of 8; gloo 2-rank rehearsal), C3 instruction counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh smoke pytest bench bench_c1 ab c5sim8 sl_c5 pmc_c3_insts
