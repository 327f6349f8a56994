#!/bin/bash
# Run tools/gpu_session.sh steps on the GPU box (fresh gpurun_out/), retrying transient
# infrastructure failures (exit 3 / "transient") up to 3 times.  Usage: tools/gpu.sh STEP...
cd "$(dirname "$0")/.."
for attempt in 1 2 3; do
  rm -rf gpurun_out/*
  /usr/local/graft/bin/gpurun --timeout 1200 -- "bash tools/gpu_session.sh $*" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if grep -q "status=transient\|no box\|stopped responding" /tmp/gpurun_last.log; then
    echo "transient failure (attempt $attempt), retrying in 30s"; sleep 30; continue
  fi
  break
done
grep "^\[gpurun\]" /tmp/gpurun_last.log | tail -3
cat gpurun_out/session.log 2>/dev/null | grep "rc="
exit $rc
