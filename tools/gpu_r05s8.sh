#!/bin/bash
# span-table piece size (PX_SPAN_PIECE) again, with the decoder's spilled lane stack
set -o pipefail
O=gpurun_out
mkdir -p $O
B="--steps 3 --warmup 1 --configs= --no-cpu --no-single --no-pcie --no-cliff --no-checks --no-exact --config 3"
for V in 2048 4096 8192 2048 4096 8192; do
  PX_SPAN_PIECE=$V timeout -k 10 200 python -u bench.py $B > $O/r05s8_$V.log 2>&1 || { echo BENCH $V FAILED; tail -3 $O/r05s8_$V.log; exit 1; }
  tail -1 $O/r05s8_$V.log | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print('piece $V', l['setitem_MBps'], l['getitem_MBps'], l['getitem_path']['span_build_ms'], l['getitem_path']['span_entries'], l['ms_per_step'])"
done
