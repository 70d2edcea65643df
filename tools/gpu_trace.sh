#!/bin/bash
# one config-3 bench step under a kernel trace; keeps the dispatch sequence of the
# suffix-array pipeline (tools/trace_seq.py) and the stats summary
#   gpurun -- 'bash tools/gpu_trace.sh r05f [extra bench args]'
set -o pipefail
TAG=${1:?tag}
shift
O=$PWD/gpurun_out
R=$PWD
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu \
  --no-single --no-pcie --no-cliff --no-exact --no-checks --configs= --steps 1 --warmup 0 "$@" > $O/${TAG}_kt.log 2>&1 || { echo TRACE FAILED; tail -5 $O/${TAG}_kt.log; exit 1; }
T=$(find $O/${TAG}_kt -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_seq.py "$T" > $O/${TAG}_seq.txt
python3 $R/tools/trace_seq.py "$T" '.' > $O/${TAG}_seq_all.txt
find $O/${TAG}_kt -name '*kernel_trace.csv' -delete
echo DONE
