#!/bin/bash
# LDS lane-stack depth again, now that deeper frames spill to scratch instead of going serial (VARS)
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
for V in ${VARS:-d6 d8 d10 d6 d8 d10}; do
  L=$PWD/pixiu_amd/libpixiu_amd.so; [ $V != d10 ] && L=$PWD/pixiu_amd/libpixiu_amd_$V.so
  PIXIU_AMD_LIB=$L timeout -k 10 200 python -u bench.py $B > $O/r05s3_$V.log 2>&1 || { echo BENCH $V FAILED; tail -3 $O/r05s3_$V.log; exit 1; }
  tail -1 $O/r05s3_$V.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('$V', l['setitem_MBps'], l['getitem_path']['span_build_ms'], l['kernel_ms']['encode_stage'], l['ms_per_step'])"
done
