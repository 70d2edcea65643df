#!/bin/bash
# set batch phase clock (PX_SET_VERBOSE): where the span build's 20 ms go, host and device
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
PX_SET_VERBOSE=1 timeout -k 10 200 python -u bench.py $B > $O/r05s9_verbose.log 2>&1 || { echo BENCH FAILED; tail -3 $O/r05s9_verbose.log; exit 1; }
grep -c . $O/r05s9_verbose.log
