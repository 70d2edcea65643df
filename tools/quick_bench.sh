#!/bin/bash
# one bench line per config (3 steps), summary printed: gpurun -- 'bash tools/quick_bench.sh 3 2 4'
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in "$@"; do
  L=gpurun_out/qb_c$C.log
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-pcie --no-checks --configs= --config $C > $L 2>&1 || { echo "BENCH FAILED"; tail -20 $L; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$L') if l.startswith('{')][-1])
print('cfg $C set', d['setitem_MBps'], 'get', d['getitem_MBps'], 'exact', d['getitem_exact_MBps'], 'ratio', d['compression_ratio'], d['kernel_ms'], d['getitem_split_ms'])"
done
