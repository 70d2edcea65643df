#!/bin/bash
# A/B of the decoder's XCD-aware order on one config: PX_DEC_XCD=0 vs 1, bench lines
# into gpurun_out/ab_*.log.   gpurun -- 'bash tools/ab_decode.sh 3'
set -o pipefail
CFG=${1:-3}
mkdir -p gpurun_out
export TMPDIR=/tmp
for X in 0 1; do
  PX_DEC_XCD=$X timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-pcie --no-checks --configs= --config $CFG \
    > gpurun_out/ab_xcd${X}_c$CFG.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/ab_xcd${X}_c$CFG.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_xcd${X}_c$CFG.log') if l.startswith('{')][-1])
print('xcd=$X', 'get', d['getitem_MBps'], 'exact', d['getitem_exact_MBps'], 'k_decode', d['kernel_ms']['getitem_stage'], d['kernel_ms']['getitem_stage_exact'], d.get('getitem_path'), 'set', d['setitem_MBps'])"
done
