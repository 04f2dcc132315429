#!/bin/bash
# round-end rehearsal on the GPU box: gpu tests, smoke(), default bench, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest.log 2>&1 || { tail -20 gpurun_out/final/pytest.log; exit 1; }
tail -1 gpurun_out/final/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final/bench.log 2>&1 || { tail -20 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.log | cut -c1-600
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/final/prof" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/final/prof.log" 2>&1) || exit $?
echo prof ok
# the headline command alone (no side legs): rocprof's average for k_ct_mul_fresh3 is then the
# bench line's avg_kernel_ms
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/final/prof_headline" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-extras > "$GRAFT_REPO_ROOT/gpurun_out/final/prof_headline.log" 2>&1) || exit $?
echo prof headline ok
# N>1 rehearsal (2 gloo ranks on cuda:0) and one rank at the N>1 shard size (2^21 pairs)
# (bench.py starts the two ranks itself; sharing cuda:0 must be asked for explicitly)
PVAC_BENCH_BACKEND=gloo PVAC_BENCH_ALLOW_SHARED=1 timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 \
  --pairs 262144 > gpurun_out/final/dist2.log 2>&1 || { tail -20 gpurun_out/final/dist2.log; exit 1; }
grep '^{' gpurun_out/final/dist2.log | cut -c1-400
timeout -k 10 300 python bench.py --pairs 2097152 --steps 3 --warmup 1 --no-cpu --no-extras > gpurun_out/final/bench_2p21.log 2>&1 || { tail -20 gpurun_out/final/bench_2p21.log; exit 1; }
tail -1 gpurun_out/final/bench_2p21.log | cut -c1-400
