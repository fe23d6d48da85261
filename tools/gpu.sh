#!/bin/bash
# Dev helper: run a command on the GPU box via gpurun; re-submit only when the
# box could not be prepared ("status=transient" / exit 3: nothing ran, nothing
# charged), waiting as long as gpurun's back-off asks ("retry in Ns").
for attempt in $(seq 1 40); do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out"
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | tail -1 | grep -o "[0-9]*")
    sleep $(( ${w:-60} + 5 )); continue
  fi
  exit $rc
done
exit 3
