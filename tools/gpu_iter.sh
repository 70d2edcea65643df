#!/bin/bash
# One iteration on the suffix-array path: its parity tests, the headline bench line, the
# single instance (rps 0, verbose rounds), and a kernel trace of a short single-instance run.
#   gpurun -- 'bash tools/gpu_iter.sh r03r'
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=$PWD/gpurun_out
R=$PWD
mkdir -p $O
T=${TESTS:-tests/test_gpu_psa.py tests/test_gpu_pools.py tests/test_gpu_rounds.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py}
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1 \
  || { echo TESTS FAILED; tail -30 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
Q="--no-cpu --no-single --no-pcie --no-cliff --configs="
PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py $Q --steps 3 > $O/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 $O/${TAG}_bench.log; exit 1; }
python3 tools/line_summary.py $O/${TAG}_bench.log
PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py $Q --rps 0 --no-checks --no-exact --steps 1 > $O/${TAG}_single.log 2>&1 || { echo SINGLE FAILED; tail -20 $O/${TAG}_single.log; exit 1; }
python3 tools/line_summary.py $O/${TAG}_single.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/${TAG}_tr -o tr --output-format csv -- python3 $R/bench.py $Q \
  --rps 0 --no-checks --no-exact --records ${TREC:-1200} --steps 1 --warmup 0 > $O/${TAG}_tr.log 2>&1 || { echo TRACE FAILED; exit 1; }
gzip -f $(find $O/${TAG}_tr -name '*kernel_trace.csv')
python3 $R/tools/round_timeline.py $(find $O/${TAG}_tr -name '*kernel_trace.csv.gz')
