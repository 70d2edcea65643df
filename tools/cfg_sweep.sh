#!/bin/bash
# GPU box: bench.py per config over shard sizes.  Args: "CFG:RPS CFG:RPS ..."
mkdir -p gpurun_out
export TMPDIR=/tmp
for CR in $1; do
  C=${CR%%:*}; R=${CR##*:}
  timeout -k 10 400 python -u bench.py --config $C --rps $R --configs= --no-cpu --no-pcie --steps 2 --warmup 1 > gpurun_out/cfg${C}_rps$R.log 2>&1 || { echo "cfg $C rps $R FAILED"; tail -20 gpurun_out/cfg${C}_rps$R.log; exit 1; }
  python3 -c "
import json; d = json.loads(open('gpurun_out/cfg${C}_rps$R.log').read().strip().splitlines()[-1])
print($C, $R, 'value', d['value'], 'set', d['setitem_MBps'], 'get', d['getitem_MBps'], 'ratio', d['compression_ratio'], 'enc_ms', d['kernel_ms']['encode_stage'], 'dec_ms', d['kernel_ms']['getitem_stage'], d['encode_stage']['psa_shards'], d['encode_stage']['walked_shards'], 'parity', d.get('parity_counts'))"
done
