#!/bin/bash
# cfg-4 kernel-trace stats (GPU box) for the product library and each lib/exp/libpvac_hip_<name>.so
# given (tools/chain_stats.sh per variant; "env:NAME=VALUE" runs the product library with it)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
L=pvac_hfhe_cppbyv_amd/lib
cp $L/libpvac_hip.so /tmp/lib_new.so || exit 1
rc=0
for v in new "$@"; do
  envv=""
  if [ $v = new ] || [ "${v#env:}" != "$v" ]; then cp /tmp/lib_new.so $L/libpvac_hip.so; else cp $L/exp/libpvac_hip_$v.so $L/libpvac_hip.so; fi
  [ "${v#env:}" != "$v" ] && envv="${v#env:}"
  tag=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
  echo "== $v"
  env $envv bash tools/chain_stats.sh "$tag" 2>&1 | grep -v Traceback | grep -E "k_large|\[" | head -12 || { rc=1; break; }
done
cp /tmp/lib_new.so $L/libpvac_hip.so
exit $rc
