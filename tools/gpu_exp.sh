#!/bin/bash
# One GPU call for an experiment: getitem / span tests, a quick headline bench line, an
# optional PX_PSA_ROUND_MAX sweep (ROUNDS="40000000 80000000"), and a kernel trace.
#   gpurun -- 'ROUNDS="..." bash tools/gpu_exp.sh r03n'
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=$PWD/gpurun_out
R=$PWD
mkdir -p $O
TESTS=${TESTS:-tests/test_gpu_spans.py tests/test_gpu_getitem_overlap.py tests/test_gpu_golden.py}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/${TAG}_tests.log; exit 1; }
  tail -2 $O/${TAG}_tests.log
fi
Q="--no-cpu --no-single --no-pcie --no-cliff --configs="
timeout -k 10 300 python -u bench.py $Q --steps 3 > $O/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/${TAG}_bench.log; exit 1; }
python3 tools/line_summary.py $O/${TAG}_bench.log
for RM in $ROUNDS; do
  PX_PSA_ROUND_MAX=$RM PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py $Q --no-checks --no-exact --steps 2 \
    > $O/${TAG}_rm$RM.log 2>&1 || { echo "BENCH RM $RM FAILED"; tail -20 $O/${TAG}_rm$RM.log; exit 1; }
  echo "round max $RM:"; python3 tools/line_summary.py $O/${TAG}_rm$RM.log
done
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${TAG}_ks -o ks --output-format csv -- python3 $R/bench.py $Q \
    --no-checks --no-exact --steps 1 --warmup 0 > $O/${TAG}_ks.log 2>&1 || { echo KTRACE FAILED; exit 1; }
  find $O/${TAG}_ks -name '*kernel_trace.csv' -delete
  python3 $R/tools/ks_top.py $(find $O/${TAG}_ks -name '*kernel_stats.csv' | head -1) 25
fi
