set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/final/prof_headline" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-extras > "$GRAFT_REPO_ROOT/gpurun_out/final/prof_headline.log" 2>&1) || exit $?
tail -1 gpurun_out/final/prof_headline.log | cut -c1-300
