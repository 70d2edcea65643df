#!/bin/bash
# lane-stack depth of the decoder (PX_LANE_DEPTH builds): the span build and getitem
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-exact"
for L in "" pixiu_amd/libpixiu_amd_ld6.so pixiu_amd/libpixiu_amd_ld8.so; do
  PIXIU_AMD_LIB=$L timeout -k 10 300 python -u bench.py $B > $O/r05k_$(basename ${L:-base}).log 2>&1 || { echo BENCH $L FAILED; tail -3 $O/r05k_$(basename ${L:-base}).log; exit 1; }
  tail -1 $O/r05k_$(basename ${L:-base}).log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('${L:-base}', l['setitem_MBps'], l['getitem_path']['span_build_ms'], l['kernel_ms'], l['parity_counts'])"
done
timeout -k 10 60 ./tools/ubench/gload > $O/r05k_gload.txt 2>&1 && cat $O/r05k_gload.txt
