set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 tests/cpp/build/test_adapter --time 32768 > gpurun_out/rt.log 2>&1; rc=$?; cat gpurun_out/rt.log; exit $rc
