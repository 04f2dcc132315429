set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --only chain "$@" > gpurun_out/chain.log 2>&1 && tail -1 gpurun_out/chain.log
