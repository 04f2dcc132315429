set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --pairs 2097152 --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/b21.log 2>&1 && tail -1 gpurun_out/b21.log
