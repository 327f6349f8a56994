#!/bin/bash
# gpurun with waits on transient pool failures (no box free, box lost while being prepared).
# Usage: tools/gpurun_retry.sh 'remote command'   (log: /tmp/gpurun_last.log)
cd "$(dirname "$0")/.."
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-20}); do
  rm -rf gpurun_out/*
  /usr/local/graft/bin/gpurun --timeout 1200 -- "$1" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" /tmp/gpurun_last.log; then
    wait_s=$(grep -o "retry in [0-9]*s" /tmp/gpurun_last.log | tail -1 | grep -o "[0-9]*")
    wait_s=${wait_s:-120}
    echo "transient failure (attempt $attempt), waiting $((wait_s + 30))s"; sleep $((wait_s + 30)); continue
  fi
  break
done
grep "^\[gpurun\]" /tmp/gpurun_last.log | tail -3
cat gpurun_out/session.log 2>/dev/null | grep "rc="
exit $rc
