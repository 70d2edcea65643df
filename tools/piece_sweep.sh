#!/bin/bash
# k_gather piece size sweep (config 3 and 5): gpurun -- 'bash tools/piece_sweep.sh'
mkdir -p gpurun_out
for P in 256 512 1024 2048; do
  for C in 3 5; do
    L=gpurun_out/piece_${P}_c$C.log
    PX_GATHER_PIECE=$P timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pcie --no-checks --no-exact --configs= --config $C > $L 2>&1 || { echo FAIL; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('$L') if l.startswith('{')][-1])
print('piece $P cfg $C get', d['getitem_MBps'], d['kernel_ms']['getitem_stage'], d['getitem_split_ms'])"
  done
done
