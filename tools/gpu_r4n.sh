#!/bin/bash
set -o pipefail
R="$GRAFT_REPO_ROOT"
bash "$R/tools/gpu_quick4.sh" r4n || exit 1
bash "$R/tools/gpu_streams_sweep.sh" || exit 1
