#!/bin/bash
# sigma A/B (GPU box): sigma / enc / merge GPU tests, then the with-sigma side measurement with the
# default column expansion and with the round-1 one (PVAC_SIGMA_PATH=copies), alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "sigma or enc or merge" > gpurun_out/pytest_sab.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sab.log
[ $rc -ne 0 ] && exit $rc
for v in new old new old; do
  if [ $v = old ]; then export PVAC_SIGMA_PATH=copies; else unset PVAC_SIGMA_PATH; fi
  timeout -k 10 300 python bench.py --only sigma > gpurun_out/sig_$v.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/sig_$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); s=d.get("extras",d); print(json.dumps(s)[:400])')"
done
