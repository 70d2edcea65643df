#!/bin/bash
# GPU box: bench.py config 3 over shard sizes (no CPU leg, no other configs).
#   gpurun -- 'bash tools/rps_sweep.sh "2 16 64 128"'
# (PX_PSA_VERBOSE=1 keeps the per-round lines flowing into the logs, so a long shard size
# does not look hung)
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in ${1:-2 16 64 128}; do
  PX_PSA_VERBOSE=1 timeout -k 10 300 python -u bench.py --rps $R --configs= --no-cpu --no-pcie --steps 3 --warmup 1 ${2:-} > gpurun_out/rps_$R.log 2>&1 || { echo "rps $R FAILED"; grep -v "psa: step" gpurun_out/rps_$R.log | tail -20; exit 1; }
  python3 -c "
import json; d = json.loads([l for l in open('gpurun_out/rps_$R.log') if l.startswith('{')][-1])
print($R, 'value', d['value'], 'set', d['setitem_MBps'], 'get', d['getitem_MBps'], 'ratio', d['compression_ratio'], 'enc', d['kernel_ms'], d['encode_stage'], 'parity', d.get('parity_counts'))"
done
