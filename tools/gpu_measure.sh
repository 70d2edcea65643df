#!/bin/bash
# One GPU call: the headline bench (PSA verbose), the single instance (rps 0), the
# suffix-array / pool / round tests (plus $EXTRA_TESTS), and a kernel trace of one bench
# step.   gpurun -- 'bash tools/gpu_measure.sh r03f'
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=$PWD/gpurun_out
mkdir -p $O
PX_PSA_VERBOSE=1 timeout -k 10 240 python -u bench.py --no-cpu --no-single --no-pcie --configs "" --steps 2 \
  > $O/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -5 $O/${TAG}_bench.log; exit 1; }
timeout -k 10 240 python -u bench.py --rps 0 --no-cpu --no-single --no-pcie --no-cliff --no-checks --configs "" --steps 1 \
  > $O/${TAG}_single.log 2>&1 || { echo SINGLE FAILED; tail -5 $O/${TAG}_single.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_psa.py tests/test_gpu_pools.py tests/test_gpu_rounds.py $EXTRA_TESTS \
  -x -q --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -20 $O/${TAG}_tests.log; exit 1; }
R=$PWD
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/${TAG}_prof -o prof -- python3 $R/bench.py --no-cpu \
  --no-single --no-pcie --no-cliff --no-exact --no-checks --configs "" --steps 1 --warmup 0 > $O/${TAG}_prof.log 2>&1
if [ "$SPROF" = 1 ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/${TAG}_sprof -o prof -- python3 $R/bench.py --rps 0 --no-cpu \
    --no-single --no-pcie --no-cliff --no-exact --no-checks --configs "" --steps 1 --warmup 0 > $O/${TAG}_sprof.log 2>&1
fi
