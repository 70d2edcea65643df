#!/bin/bash
# kernel traces of one headline bench step and of one single-instance (rps 0) step
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=$PWD/gpurun_out
R=$PWD
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py -x -q --timeout 200 --timeout-method thread \
  > $O/${TAG}_facade.log 2>&1 || { echo FACADE FAILED; tail -20 $O/${TAG}_facade.log; exit 1; }
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/${TAG}_prof -o prof -- python3 $R/bench.py --no-cpu \
  --no-single --no-pcie --no-exact --no-checks --configs "" --steps 1 --warmup 0 > $O/${TAG}_prof.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/${TAG}_sprof -o prof -- python3 $R/bench.py --rps 0 --no-cpu \
  --no-single --no-pcie --no-exact --no-checks --configs "" --steps 1 --warmup 0 > $O/${TAG}_sprof.log 2>&1
