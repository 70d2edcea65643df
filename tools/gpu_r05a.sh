#!/bin/bash
# round 5: the driver's headline flags, old trim policy (retain 8 GiB) vs the adaptive one
set -o pipefail
O=gpurun_out
mkdir -p $O
ARGS="--steps 20 --warmup 5 --configs= --no-cpu --no-single --no-pcie --no-cliff"
timeout -k 10 300 python -u bench.py $ARGS --retain-mb 8192 > $O/r05a_retain8g.log 2>&1 || { echo A FAILED; tail -5 $O/r05a_retain8g.log; exit 1; }
timeout -k 10 300 python -u bench.py $ARGS > $O/r05a_adaptive.log 2>&1 || { echo B FAILED; tail -5 $O/r05a_adaptive.log; exit 1; }
echo DONE
