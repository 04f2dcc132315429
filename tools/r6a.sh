set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6a/pytest.log 2>&1 || { tail -30 gpurun_out/r6a/pytest.log; exit 1; }
tail -3 gpurun_out/r6a/pytest.log
