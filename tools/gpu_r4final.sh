#!/bin/bash
# round-4 final: full GPU suite + smoke + default bench line (tools/gpu_quick4.sh), then the profiles
# (cfg-4 kernel trace with its timed window, the chain's PMC of the timed chain, the headline trace)
set -o pipefail
R="$GRAFT_REPO_ROOT"
bash "$R/tools/gpu_quick4.sh" r4final || exit 1
CHAIN_INPUTS=4096 bash "$R/tools/gpu_r4prof.sh" || exit 1
