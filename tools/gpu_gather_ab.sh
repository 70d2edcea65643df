#!/bin/bash
# A/B of the gather kernel variants (PX_GATHER_W8) and head shares: bench lines + kernel stats
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
O=$PWD/gpurun_out
R=$PWD
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_spans.py tests/test_gpu_getitem_overlap.py -x -q --timeout 200 \
  --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/${TAG}_tests.log; exit 1; }
PX_GATHER_W8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_spans.py -x -q --timeout 200 \
  --timeout-method thread >> $O/${TAG}_tests.log 2>&1 || { echo TESTS W8 FAILED; tail -30 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
Q="--no-cpu --no-single --no-pcie --no-cliff --configs= --no-checks"
for V in "0 24" "1 24" "0 63" "1 63"; do
  set -- $V
  PX_GATHER_W8=$1 PX_GET_HEAD64=$2 timeout -k 10 300 python -u bench.py $Q --steps 4 > $O/${TAG}_w$1_h$2.log 2>&1 || { echo "BENCH $V FAILED"; exit 1; }
  echo "w8=$1 head=$2:"; python3 tools/line_summary.py $O/${TAG}_w$1_h$2.log | head -1
done
cd /tmp
for W in 0 1; do
  PX_GATHER_W8=$W PX_GET_HEAD64=63 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${TAG}_ks$W -o ks --output-format csv -- python3 $R/bench.py $Q \
    --no-exact --steps 2 --warmup 0 > $O/${TAG}_ks$W.log 2>&1 || { echo KTRACE FAILED; exit 1; }
  find $O/${TAG}_ks$W -name '*kernel_trace.csv' -delete
  echo "w8=$W"; python3 $R/tools/ks_top.py $(find $O/${TAG}_ks$W -name '*kernel_stats.csv' | head -1) 60 | grep -i "gather\|total"
done
