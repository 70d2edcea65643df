#!/bin/bash
# Single-instance (rps 0) study: pool / round tests, a verbose bench step, and a kernel trace
# (per-dispatch CSV kept) of a short single-instance run for the round timeline.
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=$PWD/gpurun_out
R=$PWD
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pools.py tests/test_gpu_rounds.py $EXTRA_TESTS -x -q --timeout 300 \
  --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
Q="--rps 0 --no-cpu --no-single --no-pcie --no-cliff --configs= --no-checks --no-exact"
PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py $Q --steps 1 > $O/${TAG}_single.log 2>&1 || { echo SINGLE FAILED; tail -20 $O/${TAG}_single.log; exit 1; }
python3 tools/line_summary.py $O/${TAG}_single.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/${TAG}_tr -o tr --output-format csv -- python3 $R/bench.py $Q \
  --records ${TREC:-1200} --steps 1 --warmup 0 > $O/${TAG}_tr.log 2>&1 || { echo TRACE FAILED; exit 1; }
gzip -f $(find $O/${TAG}_tr -name '*kernel_trace.csv')
echo DONE
