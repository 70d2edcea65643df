#!/bin/bash
# GPU box: k_decode time for each decoder build variant (pixiu_amd/libpixiu_amd_d*.so) at
# records_per_shard 2 and 64 (config 3).
mkdir -p gpurun_out
for L in pixiu_amd/libpixiu_amd.so pixiu_amd/libpixiu_amd_d*.so; do
  for R in 2 64; do
    echo "== $L rps $R"
    PIXIU_AMD_LIB=$PWD/$L timeout -k 10 120 python -u tools/decode_run.py 3 10000 $R 0 2>&1 | grep waves || exit 1
  done
done
