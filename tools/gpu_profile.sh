#!/bin/bash
# One GPU call: GPU test suite, the default bench line (with the CPU baseline), a
# rocprofv3 kernel-trace summary of the same bench, and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE) that bench.py's roofline.traffic reads.
#   gpurun --timeout 1200 -- 'bash tools/gpu_profile.sh r01b'
# Outputs land in gpurun_out/<tag>_*; copy the ones to keep into profiles/.
set -o pipefail
TAG=${1:?tag}
SKIP_TESTS=${SKIP_TESTS:-0}
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/${TAG}_gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
  tail -2 $O/${TAG}_gpu_tests.log
fi
timeout -k 10 300 python -u bench.py > $O/${TAG}_bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/${TAG}_bench.log; exit 1; }
tail -1 $O/${TAG}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_ks -o ks --output-format csv \
  -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/${TAG}_ks.log 2>&1 || { echo "KTRACE FAILED"; tail -20 $O/${TAG}_ks.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/${TAG}_pmc_f -o f --output-format csv \
  -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/${TAG}_pmc_f.log 2>&1 || { echo "PMC FETCH FAILED"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/${TAG}_pmc_w -o w --output-format csv \
  -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/${TAG}_pmc_w.log 2>&1 || { echo "PMC WRITE FAILED"; exit 1; }
find $O/${TAG}_ks $O/${TAG}_pmc_f $O/${TAG}_pmc_w -name '*.csv' | sort
echo DONE
