#!/bin/bash
# Dev helper: run a command on the GPU box via gpurun; re-submit only when the
# box could not be prepared ("status=transient": nothing ran, nothing charged).
for attempt in 1 2 3 4 5 6 7 8 9 10; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1)
  echo "$out"
  if echo "$out" | grep -q "status=transient"; then sleep 60; continue; fi
  break
done
