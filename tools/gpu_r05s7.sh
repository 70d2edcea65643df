#!/bin/bash
# LCE text positions per thread (PX_LCE_SPAN 8 against the default 16): batch shards and the
# single instance
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 2 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
for R in 139 0; do
for V in 8 16 8 16; do
  PX_LCE_SPAN=$V timeout -k 10 200 python -u bench.py $B --rps $R > $O/r05s7_${R}_$V.log 2>&1 || { echo BENCH $V FAILED; tail -3 $O/r05s7_${R}_$V.log; exit 1; }
  tail -1 $O/r05s7_${R}_$V.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('rps $R span $V', l['setitem_MBps'], l['kernel_ms']['encode_stage'], l['encode_stage'].get('psa_split_ms'), l['ms_per_step'])"
done
done
