#!/bin/bash
# GPU clock / power while a bench leg runs (GPU box): samples rocm-smi every ~0.3 s
#   tools/clock_probe.sh [bench args...]  -> gpurun_out/clock_probe.log
set -u
mkdir -p gpurun_out
OUT=gpurun_out/clock_probe.log
: > $OUT
timeout -k 10 300 python bench.py "$@" > gpurun_out/clock_bench.log 2>&1 &
BP=$!
for i in $(seq 1 400); do
  kill -0 $BP 2>/dev/null || break
  echo "t=$i $(rocm-smi --showclocks --showpower --csv 2>/dev/null | grep -v '^device' | head -2 | tr '\n' ' ')" >> $OUT
  sleep 0.3
done
wait $BP
tail -1 gpurun_out/clock_bench.log | cut -c1-300
grep -c . $OUT
