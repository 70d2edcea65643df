#!/bin/bash
# Debug aid: k_decode timing of variant libraries (pixiu_amd/libpixiu_amd_v<NAME>.so,
# built beside the product library) on one config-3 batch; the product library is
# restored afterwards.   gpurun -- 'bash tools/gpu_var_run.sh NAME...'
set -o pipefail
export TMPDIR=/tmp
cp pixiu_amd/libpixiu_amd.so /tmp/keep.so
timeout -k 10 120 python -u tools/decode_run.py 3 10000 2 0 > gpurun_out/var_base.log 2>&1 || exit 1
for v in "$@"; do
  cp pixiu_amd/libpixiu_amd_v$v.so pixiu_amd/libpixiu_amd.so
  timeout -k 10 120 python -u tools/decode_run.py 3 10000 2 0 > gpurun_out/var_$v.log 2>&1 || { cp /tmp/keep.so pixiu_amd/libpixiu_amd.so; exit 1; }
done
cp /tmp/keep.so pixiu_amd/libpixiu_amd.so
for v in base "$@"; do echo "$v: $(grep waves gpurun_out/var_$v.log)"; done
