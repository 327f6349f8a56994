#!/bin/bash
# Run tools/gpu_session.sh steps on the GPU box (fresh gpurun_out/), waiting out transient
# infrastructure failures (honouring gpurun's "retry in Ns").  Usage: tools/gpu.sh STEP...
cd "$(dirname "$0")/.."
for attempt in 1 2 3 4; do
  rm -rf gpurun_out/*
  /usr/local/graft/bin/gpurun --timeout 1200 -- "bash tools/gpu_session.sh $*" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if grep -q "status=transient\|no box\|stopped responding\|backing off" /tmp/gpurun_last.log || [ $rc -eq 3 ]; then
    wait_s=$(grep -o "retry in [0-9]*s" /tmp/gpurun_last.log | tail -1 | grep -o "[0-9]*")
    wait_s=${wait_s:-60}
    echo "transient failure (attempt $attempt), waiting $((wait_s + 15))s"; sleep $((wait_s + 15)); continue
  fi
  break
done
grep "^\[gpurun\]" /tmp/gpurun_last.log | tail -3
cat gpurun_out/session.log 2>/dev/null | grep "rc="
exit $rc
