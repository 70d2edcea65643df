#!/bin/bash
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 60 ./tools/ubench/gload > $O/r05j_gload.txt 2>&1 || { echo GLOAD FAILED; cat $O/r05j_gload.txt; exit 1; }
cat $O/r05j_gload.txt
PX_SET_VERBOSE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-exact --no-checks > $O/r05j_setphases.log 2>&1 || { echo BENCH FAILED; exit 1; }
echo DONE
