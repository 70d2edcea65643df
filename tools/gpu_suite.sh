#!/bin/bash
# the full GPU suite (as the driver runs it), then optionally the default bench
#   gpurun --timeout 1200 -- 'bash tools/gpu_suite.sh r05e [bench]'
set -o pipefail
TAG=${1:?tag}
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; grep -E "FAILED|Error|error" $O/${TAG}_gpu_tests.log | head -20; tail -5 $O/${TAG}_gpu_tests.log; exit 1; }
tail -2 $O/${TAG}_gpu_tests.log
if [ "$2" = bench ]; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/${TAG}_bench.log 2>&1 || { echo "BENCH FAILED"; tail -5 $O/${TAG}_bench.log; exit 1; }
  tail -c 600 $O/${TAG}_bench.log
fi
