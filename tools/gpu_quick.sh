#!/bin/bash
# One GPU call for an encode-stage change: the headline bench (no CPU / single / PCIe /
# cliff legs), a kernel-trace summary of one headline step, and (TESTS=...) some GPU tests.
#   gpurun -- 'bash tools/gpu_quick.sh r04f'
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=$PWD/gpurun_out
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1 \
    || { echo TESTS FAILED; tail -20 $O/${TAG}_tests.log; exit 1; }
  tail -2 $O/${TAG}_tests.log
fi
timeout -k 10 300 python -u bench.py --no-cpu --no-single --no-pcie --no-cliff --configs "${CONFIGS:-}" --steps 2 \
  ${BENCH_ARGS:-} > $O/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -5 $O/${TAG}_bench.log; exit 1; }
R=$PWD
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${TAG}_ks -o ks --output-format csv -- python3 $R/bench.py \
  --no-cpu --no-single --no-pcie --no-cliff --no-exact --no-checks --configs "" --steps 1 --warmup 0 ${BENCH_ARGS:-} \
  > $O/${TAG}_ks.log 2>&1 || { echo KTRACE FAILED; tail -5 $O/${TAG}_ks.log; exit 1; }
find $O/${TAG}_ks -name '*kernel_stats.csv' | head -1
