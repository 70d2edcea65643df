#!/bin/bash
# GPU box: the -m gpu suite (optionally a -k filter as $1), then (optional) the bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
fi
tail -5 gpurun_out/gpu_tests.log
