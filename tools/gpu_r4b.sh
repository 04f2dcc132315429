#!/bin/bash
# round 4: chain API + direct mode: gpu tests (chain first), then the cfg-4 leg alone
set -o pipefail
D=gpurun_out/${1:-r4b}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest_chain.log 2>&1 || { tail -40 $D/pytest_chain.log; exit 1; }
tail -3 $D/pytest_chain.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 600 python bench.py --only chain --chain-compare-streams > $D/chain.log 2>&1 || { tail -20 $D/chain.log; exit 1; }
tail -c 2500 $D/chain.log
