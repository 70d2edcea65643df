#!/bin/bash
# host phases of one set batch per config (PX_SET_VERBOSE=1): gpurun -- 'bash tools/set_phases.sh 4'
mkdir -p gpurun_out
CFG=${1:-4}
PX_SET_VERBOSE=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-pcie --no-checks --no-exact --configs= --config $CFG > gpurun_out/phases_c$CFG.log 2>&1
tail -40 gpurun_out/phases_c$CFG.log | grep -v '^{'
