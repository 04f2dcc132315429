#!/bin/bash
# waits for a free GPU slot (gpurun exit 3 = nothing charged) and runs the command once
LOG="$1"; shift   # usage: tools/gpuq.sh <log> <gpurun args...> (CPU-side helper, never run on the box)
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then echo "rc=$rc" >> "$LOG"; exit $rc; fi
  sleep 120
done
