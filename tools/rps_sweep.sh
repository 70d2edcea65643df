#!/bin/bash
# GPU box: bench.py config 3 over shard sizes (no CPU leg, no other configs).
#   gpurun -- 'bash tools/rps_sweep.sh "2 16 64 128"'
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in ${1:-2 16 64 128}; do
  timeout -k 10 300 python -u bench.py --rps $R --configs= --no-cpu --no-pcie --steps 3 --warmup 1 ${2:-} > gpurun_out/rps_$R.log 2>&1 || { echo "rps $R FAILED"; tail -20 gpurun_out/rps_$R.log; exit 1; }
  python3 -c "
import json; d = json.loads(open('gpurun_out/rps_$R.log').read().strip().splitlines()[-1])
print($R, 'value', d['value'], 'set', d['setitem_MBps'], 'get', d['getitem_MBps'], 'ratio', d['compression_ratio'], 'enc', d['kernel_ms'], d['encode_stage'], 'parity', d.get('parity_counts'))"
done
