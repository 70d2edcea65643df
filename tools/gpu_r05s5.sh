#!/bin/bash
# waves of the compat piece decode (PX_SPAN_WAVES): 28 resident per CU = 7,168 on 256 CUs
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
for V in ${VARS:-7168 14336 16384 32768 7168 14336 16384 32768}; do
  PX_SPAN_WAVES=$V timeout -k 10 200 python -u bench.py $B > $O/r05s5_$V.log 2>&1 || { echo BENCH $V FAILED; tail -3 $O/r05s5_$V.log; exit 1; }
  tail -1 $O/r05s5_$V.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('$V', l['setitem_MBps'], l['getitem_path']['span_build_ms'], l['kernel_ms']['encode_stage'], l['ms_per_step'])"
done
