#!/bin/bash
# Iteration loop for kernel work: GPU test suite, then the k_gst_encode counter passes.
#   gpurun -- 'bash tools/gpu_iter.sh TAG'
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
bash tools/gpu_gst_pmc.sh ${TAG}_pmc 10000 2
