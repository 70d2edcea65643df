#!/bin/bash
# host phases of getitem batches (PX_GET_VERBOSE=1): gpurun -- 'bash tools/get_phases.sh 4'
mkdir -p gpurun_out
CFG=${1:-4}
PX_GET_VERBOSE=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-pcie --no-checks --no-exact --configs= --config $CFG > gpurun_out/getphases_c$CFG.log 2>&1
grep -v '^{' gpurun_out/getphases_c$CFG.log | tail -24
